"""One contiguous buffer per client: parameters, fp32 master, gradients and AdamW state.

The reference serialises the model as 201 separate numpy arrays on every exchange
(``get_parameters`` -> ``[val.cpu().numpy() for ...]``, ``src/Servercase/server_IID_IMDB.py:161-162``)
and loads them back with ``torch.Tensor(v)`` + ``load_state_dict`` (``:164-167``). Here every
trainable parameter is a VIEW into one flat device buffer (each tensor start aligned to 64
elements = 128 B for bf16), so FedAvg is one RCCL all-reduce, a gossip exchange is one
send/recv per peer, AdamW is one multi-tensor kernel, and host round-trips disappear (K12).

Buffers (N = padded element count):
  ``param``  compute dtype (bf16 on MI355X) — what the model reads
  ``master`` fp32 master weights (aliases ``param`` when the compute dtype is fp32)
Gradients stay the tensors autograd produces (``p.grad`` is reset to None, so autograd hands
over its result without an accumulate kernel); the multi-tensor AdamW reads them in place.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .. import ops

ALIGN = 64


class FlatParams:
    def __init__(self, params: List[nn.Parameter], device=None, dtype: Optional[torch.dtype] = None,
                 names: Optional[List[str]] = None):
        if not params:
            raise ValueError("no trainable parameters")
        device = torch.device(device) if device is not None else params[0].device
        dtype = dtype or params[0].dtype
        self.device, self.dtype = device, dtype
        self.names = names or [f"p{i}" for i in range(len(params))]
        self.slots: List[Tuple[int, int, torch.Size]] = []
        off = 0
        for p in params:
            n = p.numel()
            self.slots.append((off, n, p.shape))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.num_params = sum(n for _, n, _ in self.slots)
        self.param = torch.zeros(self.numel, dtype=dtype, device=device)
        with torch.no_grad():
            for p, (o, n, shp) in zip(params, self.slots):
                self.param[o:o + n].copy_(p.data.reshape(-1).to(device=device, dtype=dtype))
        if dtype == torch.float32:
            self.master = self.param
        else:
            self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
            with torch.no_grad():
                for p, (o, n, shp) in zip(params, self.slots):
                    self.master[o:o + n].copy_(p.data.reshape(-1).to(device=device, dtype=torch.float32))
        self.params = params
        self._bind()

    def _bind(self):
        for p, (o, n, shp) in zip(self.params, self.slots):
            p.data = self.param[o:o + n].view(shp)
            p.grad = None

    @classmethod
    def from_model(cls, model: nn.Module, device=None, dtype=None) -> "FlatParams":
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        return cls([p for _, p in named], device, dtype, [n for n, _ in named])

    # ------------------------------------------------------------------------------------
    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def grads(self):
        """(grad tensors, flat offsets) of the parameters that received a gradient."""
        gs, offs = [], []
        for p, (o, n, shp) in zip(self.params, self.slots):
            if p.grad is not None:
                gs.append(p.grad)
                offs.append(o)
        return gs, offs

    def flat_grad(self) -> torch.Tensor:
        """Gradients gathered into one flat fp32 buffer (tests / diagnostics only)."""
        g = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        for p, (o, n, shp) in zip(self.params, self.slots):
            if p.grad is not None:
                g[o:o + n].copy_(p.grad.reshape(-1))
        return g

    @torch.no_grad()
    def sync_param_from_master(self):
        if self.master is not self.param:
            ops.cast_copy_(self.param, self.master)

    def rebind(self, master: torch.Tensor, param: torch.Tensor):
        """Point this replica at ANOTHER client's buffers (fp32 master + compute-dtype param of
        the same layout): the model's parameter views move, nothing is copied. Client lanes use
        this to train each hosted client in place on its own resident state."""
        if master.numel() != self.numel or param.numel() != self.numel or param.dtype != self.dtype:
            raise ValueError("rebind: buffers must match this FlatParams' layout and dtype")
        self.master, self.param = master, param
        self._bind()

    @torch.no_grad()
    def load_master(self, src: torch.Tensor):
        self.master.copy_(src)
        self.sync_param_from_master()

    def nbytes(self, which: str = "param") -> int:
        t = getattr(self, which)
        return t.numel() * t.element_size()

    def state_views(self, buf: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        buf = self.master if buf is None else buf
        return {nm: buf[o:o + n].view(shp) for nm, (o, n, shp) in zip(self.names, self.slots)}


class FlatAdamW:
    """Fused AdamW over a FlatParams (ONE kernel per step; K10).

    ``mode="hf"`` reproduces ``transformers.AdamW`` (4.35: eps outside the bias correction,
    ``correct_bias=True``) that the reference instantiates at ``server_IID_IMDB.py:109``;
    ``mode="torch"`` reproduces ``torch.optim.AdamW``. ``reset()`` = the reference's fresh
    optimizer per fit (C8)."""

    def __init__(self, flat: FlatParams, lr: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-6,
                 weight_decay: float = 0.0, mode: str = "hf", max_grad_norm: float = 0.0):
        self.flat = flat
        self.lr, self.betas, self.eps, self.wd, self.mode = lr, tuple(betas), eps, weight_decay, mode
        # global-norm gradient clipping (0 = off, the reference's plain loop); the coefficient
        # stays on the device (ops.grad_clip_coef) and scales the gradients inside the AdamW pass
        self.max_grad_norm = float(max_grad_norm)
        self.last_grad_norm: Optional[torch.Tensor] = None
        self.m = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.v = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.step_count = 0
        # drift correction (bcfl.fl.drift): flat fp32 update-space direction added to every step
        # as p -= lr * corr_scale * corr, fused into the AdamW kernel; None = off
        self.corr: Optional[torch.Tensor] = None
        self.corr_scale = 1.0

    def reset(self):
        self.m.zero_()
        self.v.zero_()
        self.step_count = 0

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, partner: Optional[FlatParams] = None):
        """One AdamW step. ``partner``: a micro-batch replica bound to the SAME buffers whose
        parameters hold the gradient of the other rows of the batch; both gradients are summed
        inside the multi-tensor kernel."""
        self.step_count += 1
        f = self.flat
        grads2 = None
        if partner is None:
            grads, offs = f.grads()
        else:
            grads, offs, grads2 = [], [], []
            for p, q, (o, n, shp) in zip(f.params, partner.params, f.slots):
                g1, g2 = p.grad, q.grad
                if g1 is None and g2 is None:
                    continue
                grads.append(g1 if g1 is not None else torch.zeros_like(g2))
                grads2.append(g2 if g2 is not None else torch.zeros_like(g1))
                offs.append(o)
        gscale = None
        if self.max_grad_norm > 0 and grads:
            # clip the TRUE gradient: grad_scale (loss-scale undo) applies before the norm
            gscale = ops.grad_clip_coef(grads, self.max_grad_norm / grad_scale, grads2)
            self.last_grad_norm = gscale[1:2] * grad_scale
        ops.adamw_multi_(f.master, grads, offs, self.m, self.v, self.step_count, self.lr,
                         self.betas[0], self.betas[1], self.eps, self.wd, self.mode,
                         param_out=None if f.master is f.param else f.param,
                         grad_scale=grad_scale, corr=self.corr,
                         corr_lr=self.lr * self.corr_scale, grads2=grads2, gscale=gscale)

    # ---- optimizer overlapped with the backward pass ---------------------------------------
    # A rank that trains ONE client (the 8-GPU layout) runs its AdamW pass after the last
    # gradient of the step otherwise (~0.7 ms of HBM-bound work per BERT-base step on the
    # critical path). With overlap, each layer's parameters are updated on a side stream as soon
    # as autograd has produced the layer's last gradient, while the backward pass continues
    # through the earlier layers (which never read the later layers' weights). The update is the
    # same element-wise AdamW, so results are bitwise those of step().
    @staticmethod
    def _group_key(name: str) -> str:
        parts = name.split(".")
        for i, t in enumerate(parts[:-1]):
            if t in ("layer", "layers") and parts[i + 1].isdigit():
                return ".".join(parts[:i + 2])
        return parts[0]

    def enable_overlap(self) -> bool:
        f = self.flat
        if f.device.type != "cuda" or getattr(self, "overlap", False):
            return getattr(self, "overlap", False)
        keys = [self._group_key(n) for n in f.names]
        self._groups, self._gid = [], []
        for i, k in enumerate(keys):
            if i == 0 or keys[i - 1] != k:
                self._groups.append([])
            self._groups[-1].append(i)
            self._gid.append(len(self._groups) - 1)
        self._astream = torch.cuda.Stream(device=f.device)
        self._live = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook(i))
                       for i, p in enumerate(f.params)]
        self.overlap = True
        return True

    def overlap_active(self) -> bool:
        return getattr(self, "overlap", False) and self.max_grad_norm <= 0

    def _hook(self, i: int):
        def fn(_p):
            if self._live:
                g = self._gid[i]
                self._left[g] -= 1
                if self._left[g] == 0:
                    self._launch(g)
        return fn

    def begin_overlapped(self, grad_scale: float = 1.0) -> None:
        """Before backward(): open the step (groups launch from the gradient hooks)."""
        self.step_count += 1
        self._left = [len(g) for g in self._groups]
        self._launched = [False] * len(self._groups)
        self._main = torch.cuda.current_stream(self.flat.device)
        self._gs = grad_scale
        self._live = True

    @torch.no_grad()
    def _launch(self, g: int) -> None:
        from ..ops import functional as _F
        self._launched[g] = True
        f = self.flat
        idx = [i for i in self._groups[g] if f.params[i].grad is not None]
        if not idx:
            return
        grads = [f.params[i].grad for i in idx]
        offs = [f.slots[i][0] for i in idx]
        a, main = self._astream, self._main
        a.wait_stream(main)
        side = _F._WG["side"].get((main.device_index, main.cuda_stream))
        if side is not None:   # side-stream weight gradients launched from this stream
            a.wait_stream(side)
        with torch.cuda.stream(a):
            for t in grads:
                t.record_stream(a)
            ops.adamw_multi_(f.master, grads, offs, self.m, self.v, self.step_count, self.lr,
                             self.betas[0], self.betas[1], self.eps, self.wd, self.mode,
                             param_out=None if f.master is f.param else f.param,
                             grad_scale=self._gs, corr=self.corr,
                             corr_lr=self.lr * self.corr_scale)

    def finish_overlapped(self) -> None:
        """After backward(): update what no hook launched, then the step's stream waits."""
        self._live = False
        for g in range(len(self._groups)):
            if not self._launched[g]:
                self._launch(g)
        self._main.wait_stream(self._astream)

    def state_dict(self):
        return {"m": self.m, "v": self.v, "step": self.step_count}

    def load_state_dict(self, st):
        self.m.copy_(st["m"])
        self.v.copy_(st["v"])
        self.step_count = int(st["step"])
