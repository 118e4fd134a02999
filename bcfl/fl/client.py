"""Reference-compatible client API (``IMDBClient(fl.client.NumPyClient)``,
``src/Servercase/server_IID_IMDB.py:155-179`` and the serverless extension
``src/Serverlesscase/serverless_IID_IMDB.py:136-187``).

A user of the reference can keep writing ``client.fit(params, config)`` /
``client.evaluate(params, config)`` / ``client.train_model()`` / ``client.evaluate_model()``;
underneath, parameters are the flat device buffer (``get_parameters`` returns HF-ordered numpy
arrays only because that is the API contract, and ``set_parameters`` does NOT cast to fp32 via
``torch.Tensor(v)`` as the reference does — it writes the fp32 master and refreshes the bf16
compute copy).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ckpt import hf_layout
from .trainer import EvalResult


class Client:
    def __init__(self, fed, cid: int, round_idx: int = 0):
        self.fed, self.cid, self.round = fed, cid, round_idx
        self._layout = hf_layout(fed.model, fed.flat)

    # --- NumPyClient interface ------------------------------------------------------------
    def get_parameters(self, config: Optional[dict] = None) -> List[np.ndarray]:
        host = self.fed.flat.master.detach().cpu().numpy()
        return [host[o:o + int(np.prod(s))].reshape(s).copy() for _, o, s in self._layout]

    @torch.no_grad()
    def set_parameters(self, parameters: List[np.ndarray]):
        m = self.fed.flat.master
        if len(parameters) != len(self._layout):
            raise ValueError(f"expected {len(self._layout)} tensors, got {len(parameters)}")
        for (_, o, s), p in zip(self._layout, parameters):
            m[o:o + int(np.prod(s))].copy_(torch.as_tensor(np.asarray(p), dtype=torch.float32).reshape(-1))
        self.fed.flat.sync_param_from_master()

    def fit(self, parameters, config: Optional[dict] = None) -> Tuple[List[np.ndarray], int, dict]:
        self.set_parameters(parameters)
        st = self.train_model()
        return self.get_parameters(), int(st["examples"]), {"train_loss": st["train_loss"]}

    def evaluate(self, parameters, config: Optional[dict] = None) -> Tuple[float, int, Dict[str, float]]:
        self.set_parameters(parameters)
        loss, acc, n = self._eval()
        return float(loss), n, {"accuracy": float(acc), "loss": float(loss)}

    # --- serverless additions ----------------------------------------------------------------
    def train_model(self) -> Dict[str, float]:
        f = self.fed
        f.opt.reset()
        st = f._train_client(self.cid, self.round)
        st["train_loss"] = float(st["loss_t"].item()) / max(st["batches"], 1) if st["loss_t"] is not None else 0.0
        return st

    def evaluate_model(self) -> Tuple[float, float]:
        loss, acc, _ = self._eval()
        return loss, acc

    def _eval(self):
        f = self.fed
        e: EvalResult = f.trainer.evaluate(f.test_batches(self.cid, self.round))
        loss = e.ref_loss if f.cfg.compat_bad_test_loss else e.loss
        return loss, e.accuracy, e.count
