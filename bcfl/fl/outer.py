"""Outer (round-level) optimizer: SGD with (Nesterov) momentum on the round's pseudo-gradient.

The reference averages models and takes the average as the next round's model, i.e. an outer
SGD step of learning rate 1 without momentum on the pseudo-gradient ``g = x_prev - mean(y_k)``
(``serverless_NonIID_IMDB.py:296-297``, Flower FedAvg ``server_IID_IMDB.py:205-209``). That is
what ``outer_lr=1, outer_momentum=0`` (the default) keeps, bit for bit.

Why an option: the benchmarks train RANDOM-INIT models (no pretrained checkpoints here), and on
IID splits every client's Adam step in the plateau phase is mostly noise, which the average
cancels: 20 rounds x 4 local steps never leave the constant-prediction plateau (train loss 0.69
throughout, profiles/iid_stability_r4.json) while the accuracy on the draw flips between the
majority rate and ~0.99 with the bias term. Momentum on the round-level pseudo-gradient
(FedAvgM, Hsu et al. 2019; the outer Nesterov step of DiLoCo, Douillard et al. 2023) accumulates
the consistent component across rounds — the standard remedy for slow FedAvg progress.

    g = x_prev - x_agg;   v = mu v + g;   x_new = x_prev - lr (g + mu v)   (Nesterov)
                                           x_new = x_prev - lr v           (heavy ball)

Everything is in place on fp32 flat buffers (two axpby passes per client per round).
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch

from .. import ops


class OuterOptimizer:
    def __init__(self, lr: float, momentum: float, nesterov: bool, keys: Iterable[int],
                 numel: int, device):
        self.lr, self.mu, self.nesterov = float(lr), float(momentum), bool(nesterov)
        self.enabled = not (self.lr == 1.0 and self.mu == 0.0)
        self.prev: Dict[int, torch.Tensor] = {}
        self.mom: Dict[int, torch.Tensor] = {}
        if self.enabled:
            for k in keys:
                self.prev[k] = torch.zeros(numel, dtype=torch.float32, device=device)
                self.mom[k] = torch.zeros(numel, dtype=torch.float32, device=device)

    @torch.no_grad()
    def begin(self, k: int, x: torch.Tensor) -> None:
        """Round start: remember the model the round starts from."""
        if self.enabled:
            self.prev[k].copy_(x)

    @torch.no_grad()
    def step(self, k: int, x: torch.Tensor, param_out: Optional[torch.Tensor] = None,
             prev: Optional[torch.Tensor] = None) -> None:
        """``x`` holds the aggregated model (in place -> the outer-updated model). ``prev``
        overrides the recorded round start (server FedAvg: the global model itself)."""
        if not self.enabled:
            return
        g = self.prev[k]
        if prev is not None:
            g.copy_(prev)
        ops.axpby_(g, x, -1.0, 1.0)                       # g = x_prev - x_agg
        v = self.mom[k]
        ops.axpby_(v, g, 1.0, self.mu)                    # v = mu v + g
        # x_prev = x_agg + g
        if self.nesterov:                                  # x = x_agg + (1 - lr) g - lr mu v
            ops.axpby_(x, g, 1.0 - self.lr, 1.0)
            ops.axpby_(x, v, -self.lr * self.mu, 1.0)
        else:                                              # x = x_agg + g - lr v
            ops.axpby_(x, g, 1.0, 1.0)
            ops.axpby_(x, v, -self.lr, 1.0)
        if param_out is not None and param_out.data_ptr() != x.data_ptr():
            ops.cast_copy_(param_out, x)

    def state_dict(self) -> Optional[dict]:
        if not self.enabled:
            return None
        return {"mom": {int(k): t.detach().cpu().clone() for k, t in self.mom.items()}}

    @torch.no_grad()
    def load_state_dict(self, st: Optional[dict]) -> None:
        if not self.enabled or not st:
            return
        for k, t in st["mom"].items():
            self.mom[int(k)].copy_(t)
