"""Shared model plumbing: parameter init, HF-name mapping, packed-batch helpers."""
from __future__ import annotations

import os
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..data.batching import PackedBatch, PaddedBatch


def new_param(shape, device=None, dtype=torch.float32, init: str = "normal", std: float = 0.02,
              requires_grad: bool = True) -> nn.Parameter:
    t = torch.empty(shape, device=device, dtype=dtype)
    if init == "normal":
        t.normal_(0.0, std)
    elif init == "zeros":
        t.zero_()
    elif init == "ones":
        t.fill_(1.0)
    else:
        raise KeyError(init)
    return nn.Parameter(t, requires_grad=requires_grad)


def check_positions(batch: PackedBatch, max_positions: int) -> None:
    """Host-side bound check before a position-table gather on the GPU: real rows use positions
    0..len-1 (filler rows use 0), so the longest real row must fit the table — an out-of-range
    position would be an out-of-bounds read in the embedding kernel and an out-of-bounds write in
    its backward."""
    n = int(batch.seq_lens.max()) if len(batch.seq_lens) else 0
    if n > max_positions:
        raise ValueError(f"sequence of {n} tokens exceeds the model's {max_positions} positions")


def padded_to_packed(b: PaddedBatch, device=None) -> PackedBatch:
    """Convert an HF-style padded batch (right padding) into a packed batch."""
    import numpy as np
    mask = b.attention_mask.bool()
    lens = mask.sum(1).cpu().numpy().astype(np.int64)
    cu = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=cu[1:])
    ids = b.input_ids[mask].to(torch.int32)
    pos = torch.cat([torch.arange(int(n), dtype=torch.int32) for n in lens]) if len(lens) else \
        torch.zeros(0, dtype=torch.int32)
    pb = PackedBatch(ids.cpu(), pos, torch.from_numpy(cu.astype(np.int32)),
                     b.labels.to(torch.int32).cpu(), int(lens.max()) if len(lens) else 0, lens, cu)
    return pb.to(device) if device is not None else pb


class SeqClassifierBase(nn.Module):
    """Interface every bcfl sequence classifier implements."""

    hf_architecture: str = ""
    hf_model_type: str = ""
    # The classifier reads one row per sequence ([CLS] / last token), so the last encoder layer
    # only computes those rows (same logits and gradients; tests compare against False).
    pooled_rows_only: bool = os.environ.get("BCFL_POOLED_ROWS", "1") == "1"

    def forward(self, batch: PackedBatch) -> torch.Tensor:  # logits [B, C]
        raise NotImplementedError

    def forward_padded(self, input_ids, attention_mask, labels=None) -> torch.Tensor:
        pb = padded_to_packed(PaddedBatch(input_ids.cpu(), attention_mask.cpu(),
                                          labels.cpu() if labels is not None else
                                          torch.zeros(input_ids.shape[0], dtype=torch.long)),
                              device=next(self.parameters()).device)
        return self.forward(pb)

    # --- HF-compatible naming -------------------------------------------------------------
    def hf_items(self) -> List[Tuple[str, Callable[[], torch.Tensor], Callable[[torch.Tensor], None]]]:
        """(hf_name, getter, setter) in HF state-dict order."""
        raise NotImplementedError

    def hf_state_dict(self) -> "OrderedDict[str, torch.Tensor]":
        return OrderedDict((n, g()) for n, g, _ in self.hf_items())

    @torch.no_grad()
    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> List[str]:
        missing = []
        for n, _, s in self.hf_items():
            if n in sd:
                s(sd[n])
            else:
                missing.append(n)
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:8]}{'...' if len(missing) > 8 else ''}")
        return missing

    def hf_config(self) -> Dict:
        raise NotImplementedError

    def trainable_parameters(self) -> List[nn.Parameter]:
        return [p for p in self.parameters() if p.requires_grad]


def row_slice(param: nn.Parameter, lo: int, hi: int):
    """getter/setter pair for rows [lo, hi) of a fused parameter (e.g. Wq inside Wqkv)."""
    def get():
        return param.data[lo:hi]

    def set_(t):
        param.data[lo:hi].copy_(t.to(param.dtype))
    return get, set_


def whole(param: nn.Parameter):
    def get():
        return param.data

    def set_(t):
        param.data.copy_(t.to(param.dtype).view_as(param.data))
    return get, set_
