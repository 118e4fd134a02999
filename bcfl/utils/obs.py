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
    """Per-phase timers: host monotonic time, and (GPU) device time from HIP events.

    Host time ends when a phase has ISSUED its work; with asynchronous launches the device wait
    then shows up in whichever later phase first reads a result. The device timer records one
    HIP event on the issuing (main) stream at the end of every phase: phase k's device time is
    the interval from the previous phase's end event to its own, so the device phases of a round
    tile its device timeline exactly (an idle gap is charged to the phase that follows it) and
    sum to the round's device span. Work on side streams that the main stream never waits for
    (the overlapped global evaluation, mailbox posts) is reported separately as hidden time
    (``add_hidden``). Events are read back lazily (``resolve``) so timing never stalls a round."""

    def __init__(self, sync_device: bool = False, roctx: bool = True, device_events: bool = True):
        self.sync_device = sync_device and torch.cuda.is_available()
        self.roctx = roctx
        self.dev = device_events and torch.cuda.is_available()
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)
        self.hidden: Dict[str, float] = defaultdict(float)
        self._marks = []          # [(phase, end event)] of the current round
        self._last = None         # end event of the previous phase (device timeline anchor)
        self._pending = []        # [(record, start event, marks)] awaiting read-back
        self.on_resolve = None    # callback(record) once a round's device times are filled in

    def _mark(self, name: str):
        if not self.dev:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._marks.append((name, ev))
        self._last = ev

    def begin_round(self):
        """Anchor the round's device timeline at the previous phase's end event (first round:
        an event recorded now), so consecutive rounds tile the device timeline."""
        if not self.dev:
            return
        if self._last is None:
            self._last = torch.cuda.Event(enable_timing=True)
            self._last.record()
        self._start = self._last

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
            self._mark(name)
            if self.roctx:
                _roctx_pop()

    def add_hidden(self, name: str, seconds: float):
        """Device time of side-stream work the main stream does not wait for."""
        self.hidden[name] += float(seconds)

    def snapshot(self, reset: bool = True) -> Dict[str, float]:
        out = {f"t_{k}": v for k, v in self.totals.items()}
        if self.hidden:
            out.update({f"t_hidden_{k}": v for k, v in self.hidden.items()})
            out["t_overlap_hidden"] = sum(self.hidden.values())
        if reset:
            self.totals.clear()
            self.counts.clear()
            self.hidden.clear()
        return out

    def end_round(self, rec: Dict[str, Any]):
        """Queue the round's device phases for read-back into ``rec`` (``dev_t_*`` keys)."""
        if not self.dev:
            return
        self._mark("other")  # host work after the last phase (history, metrics)
        start = getattr(self, "_start", None)
        if start is not None and self._marks:
            self._pending.append((rec, start, self._marks))
        self._marks = []
        self._start = None
        self.resolve(block=False)

    def resolve(self, block: bool = False):
        """Fill ``dev_t_*`` of every queued round whose events have completed (all of them with
        ``block``; events complete in stream order, so stop at the first pending one)."""
        while self._pending:
            rec, start, marks = self._pending[0]
            if not (block or marks[-1][1].query()):
                break
            self._pending.pop(0)
            dev: Dict[str, float] = defaultdict(float)
            prev = start
            for name, ev in marks:
                dev[name] += prev.elapsed_time(ev) / 1000.0
                prev = ev
            rec.update({f"dev_t_{k}": v for k, v in dev.items()})
            rec["dev_t_round"] = sum(dev.values())
            if self.on_resolve is not None:
                self.on_resolve(rec)


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
