"""Client-drift correction for Non-IID federations (SCAFFOLD control variates in update space).

Why: with label-sharded Non-IID data (reference ``serverless_NonIID_IMDB.py:59-60`` shards the
label-sorted IMDB split contiguously, so each client sees essentially one class) every local epoch
pulls a client towards predicting ITS label; averaging / gossip cancels those pulls and the
federation oscillates around the majority rate (profiles/accuracy_sweep_federated.json). SCAFFOLD
(Karimireddy et al., 2020) removes the per-client bias with control variates: client ``i`` steps
along ``g - c_i + c`` where ``c_i`` is its own average update direction and ``c`` the federation's.

MI355X-first formulation — no extra communication and one fused term in the optimizer:

* the correction lives in UPDATE space (what AdamW applies per unit of lr), so it composes with the
  adaptive optimizer: each step is ``p -= lr * (adam_update + s * d_i)``; ``d_i = c - c_i`` is a
  flat fp32 buffer read by the multi-tensor AdamW kernel in the same pass (``corr`` argument of
  ``adamw_mt_kernel``, elementwise.hip) — no extra launch per step;
* ``d_i`` is derived from states the round already has. With ``L = sum of the round's local lrs``,
  ``x`` the round-start model, ``y_i`` the client's trained model and ``x'`` its model after
  aggregation (FedAvg result / gossip mix), SCAFFOLD option II gives
  ``c_i' = (x - y_i) / L - d_i`` and ``c' = mean_j c_j' = (x - x') / L``, so
  ``d_i' = c' - c_i' = (y_i - x') / L + d_i``: two axpby passes per client per round
  (:meth:`after_train`, :meth:`after_mix`), nothing on the wire. With a damping scale ``s`` the
  steps applied ``s * d_i``, so the carried term is ``s * d_i`` (still exactly ``c' - c_i'``).
  Under gossip with a partial topology ``x'`` is the neighbourhood mean, i.e. the neighbourhood
  estimate of ``c``.

Measured (CPU, tiny-bert, 8 one-class clients, 16 rounds, /tmp-free test in tests/test_fl.py):
without correction the global accuracy peaks near 0.95 and collapses back to 0.5; with it both
server FedAvg and serverless gossip reach >= 0.99 and stay there.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch

from .. import ops

MODES = ("none", "scaffold")
# partitions whose clients see skewed label distributions (bcfl/data/partition.py)
LABEL_SKEWED = ("label_shards", "ref_contiguous", "dirichlet")


def resolve_mode(mode: str, partition: str) -> str:
    """``auto``: SCAFFOLD where local optima disagree (label-skewed shards), off for IID splits,
    where the control variates only add noise (profiles/accuracy_curves_iid_mi355x.json)."""
    if mode == "auto":
        return "scaffold" if partition in LABEL_SKEWED else "none"
    return mode


class DriftCorrection:
    def __init__(self, mode: str, scale: float, clients: Iterable[int], numel: int, device):
        if mode not in MODES:
            raise ValueError(f"drift_correction must be one of {MODES}, got {mode!r}")
        self.mode, self.scale = mode, float(scale)
        self.enabled = mode != "none"
        self.buf: Dict[int, torch.Tensor] = {}
        self.ready: Dict[int, bool] = {}
        self.lr_sum: Dict[int, float] = {}
        if self.enabled:
            for c in clients:
                self.buf[c] = torch.zeros(numel, dtype=torch.float32, device=device)
                self.ready[c] = False

    def attach(self, opt, c: int) -> None:
        """Before client ``c``'s local steps: its optimizer applies ``d_c`` (round 0: nothing)."""
        if not self.enabled:
            return
        opt.corr = self.buf[c] if self.ready[c] else None
        opt.corr_scale = self.scale

    @staticmethod
    def detach(opt) -> None:
        opt.corr = None

    @torch.no_grad()
    def after_train(self, c: int, trained: torch.Tensor, lr_sum: float) -> None:
        """``buf <- y_c / L + s * d_c`` (stream-ordered after the client's last optimizer step)."""
        if not self.enabled or lr_sum <= 0:
            return
        self.lr_sum[c] = float(lr_sum)
        ops.axpby_(self.buf[c], trained, 1.0 / lr_sum, self.scale if self.ready[c] else 0.0)

    @torch.no_grad()
    def after_mix(self, c: int, aggregated: torch.Tensor) -> None:
        """``d_c' = buf - x'_c / L`` once the client's post-aggregation model is known."""
        if not self.enabled or c not in self.lr_sum:
            return
        ops.axpby_(self.buf[c], aggregated, -1.0 / self.lr_sum.pop(c), 1.0)
        self.ready[c] = True

    # ---- resume -------------------------------------------------------------------------
    def state_dict(self) -> Optional[dict]:
        if not self.enabled:
            return None
        return {"buf": {int(c): t.detach().cpu().clone() for c, t in self.buf.items()},
                "ready": {int(c): bool(v) for c, v in self.ready.items()}}

    @torch.no_grad()
    def load_state_dict(self, st: Optional[dict]) -> None:
        if not self.enabled or not st:
            return
        for c, t in st["buf"].items():
            self.buf[int(c)].copy_(t)
        for c, v in st["ready"].items():
            self.ready[int(c)] = bool(v)
