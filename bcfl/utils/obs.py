"""Observability: per-phase timers, roctx ranges, metrics JSONL, reference-compatible telemetry.

The reference only measures wall clock from import to exit and samples ``psutil.cpu_percent`` /
RSS twice with swapped variable names, so its "Memory Usage" is start-minus-end and usually
negative (``src/Servercase/server_IID_IMDB.py:59-63,221-233``; ``-3.30 GB`` at
``serverless_cancer_classification_with_BioBERT.ipynb:705``). Here: phase timers
(``data, train, pack, comm, mix, eval_local, eval_global, ckpt, ledger, anomaly``), roctx ranges
so rocprofv3 timelines show the phases, one JSON record per (round, client), and the same
human-readable lines as the reference with the memory sign fixed and labelled.
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict
from typing import Any, Dict, Optional

import torch

try:
    import psutil
except Exception:  # pragma: no cover
    psutil = None


def _roctx_push(name: str):
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:
            pass


def _roctx_pop():
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_pop()
        except Exception:
            pass


class PhaseTimer:
    """Host monotonic timers per phase (optionally synchronising the device at boundaries)."""

    def __init__(self, sync_device: bool = False, roctx: bool = True):
        self.sync_device = sync_device and torch.cuda.is_available()
        self.roctx = roctx
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.roctx:
            _roctx_push(name)
        if self.sync_device:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if self.sync_device:
                torch.cuda.synchronize()
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1
            if self.roctx:
                _roctx_pop()

    def snapshot(self, reset: bool = True) -> Dict[str, float]:
        out = {f"t_{k}": v for k, v in self.totals.items()}
        if reset:
            self.totals.clear()
            self.counts.clear()
        return out


class MetricsWriter:
    def __init__(self, path: Optional[str], enabled: bool = True, append: bool = False):
        self.path = path if enabled else None
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            self._fh = open(self.path, "a" if append else "w")
        else:
            self._fh = None

    def write(self, rec: Dict[str, Any]):
        if self._fh:
            self._fh.write(json.dumps(rec, sort_keys=True, default=float) + "\n")
            self._fh.flush()

    def close(self):
        if self._fh:
            self._fh.close()
            self._fh = None


class Telemetry:
    """Start/end process telemetry (reference C17), sign-correct."""

    def __init__(self):
        self.t0 = time.time()
        self.proc = psutil.Process() if psutil else None
        self.cpu0 = psutil.cpu_percent() if psutil else 0.0
        self.rss0 = self.proc.memory_info().rss if self.proc else 0

    def finish(self) -> Dict[str, float]:
        cpu1 = psutil.cpu_percent() if psutil else 0.0
        rss1 = self.proc.memory_info().rss if self.proc else 0
        out = {
            "latency_min": (time.time() - self.t0) / 60.0,
            "cpu_overhead_pct": cpu1 - self.cpu0,
            "host_rss_delta_gb": (rss1 - self.rss0) / 1024 ** 3,
        }
        if torch.cuda.is_available():
            out["hbm_peak_gb"] = torch.cuda.max_memory_allocated() / 1024 ** 3
        return out

    @staticmethod
    def print_reference_lines(t: Dict[str, float], global_accuracies, model_size_gb: Optional[float]):
        if model_size_gb is not None:
            print("Model size in GB")
            print(model_size_gb)
        print(f"CPU Overhead: {t['cpu_overhead_pct']}%")
        print(f"Memory Usage (host RSS end-start): {t['host_rss_delta_gb']:.2f} GB")
        if "hbm_peak_gb" in t:
            print(f"HBM peak: {t['hbm_peak_gb']:.2f} GB")
        print(f"Latency: {t['latency_min']} min")
        print("global accuracies")
        print(list(global_accuracies))
