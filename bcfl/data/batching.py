"""Packed (varlen) batches and the per-client loader.

The reference pads every batch to its longest row with ``DataCollatorWithPadding``
(``src/Servercase/server_IID_IMDB.py:89-99``) and moves each batch host->device inside the hot
loop (``serverless_IID_IMDB.py:162``). Here a batch is *packed*: the valid tokens of all rows
back to back plus ``cu_seqlens`` (row boundaries), so no kernel ever computes a pad position.
All int32 fields of an epoch are laid out in ONE pinned host buffer and moved with ONE
asynchronous H2D copy; batches are views into the device copy.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterator, List, Optional

import numpy as np
import torch

from .synthetic import TokenDataset

__all__ = ["PackedBatch", "PaddedBatch", "MicroBatches", "make_packed_batch", "make_padded_batch",
           "ClientLoader"]


@dataclass
class PackedBatch:
    input_ids: torch.Tensor     # [T] int32
    position_ids: torch.Tensor  # [T] int32
    cu_seqlens: torch.Tensor    # [B+1] int32
    labels: torch.Tensor        # [B] int32
    max_seqlen: int
    seq_lens: np.ndarray        # host copy of row lengths (real rows only)
    cu_host: np.ndarray         # host copy of cu_seqlens (incl. the filler row, if any)
    # optional [2, T] int32 stable sort orders (sorted keys | source rows) of input_ids and
    # position_ids, computed on the host with the batch (ClientLoader presort): the embedding
    # table gradients then need no device sort per step
    sort_ids: Optional[torch.Tensor] = None
    sort_pos: Optional[torch.Tensor] = None
    # optional [2, n] int32 attention work order (attn_schedule), staged with the batch
    attn_sched: Optional[torch.Tensor] = None

    def order(self):
        return (self.sort_ids, self.sort_pos) if self.sort_ids is not None else None

    @property
    def batch_size(self) -> int:
        """Number of REAL rows (a filler row added by :func:`pad_packed` is not counted)."""
        return int(self.seq_lens.shape[0])

    @property
    def n_seq(self) -> int:
        return self.batch_size

    @property
    def num_tokens(self) -> int:
        return int(self.cu_host[-1])

    @property
    def real_tokens(self) -> int:
        return int(self.cu_host[self.batch_size])

    def to(self, device, non_blocking: bool = True) -> "PackedBatch":
        mv = lambda t: None if t is None else t.to(device, non_blocking=non_blocking)  # noqa: E731
        return PackedBatch(mv(self.input_ids), mv(self.position_ids), mv(self.cu_seqlens),
                           mv(self.labels), self.max_seqlen, self.seq_lens, self.cu_host,
                           mv(self.sort_ids), mv(self.sort_pos), mv(self.attn_sched))


ATTN_BLOCK = 128  # rows per attention workgroup (attention.hip BLK)


def attn_schedule(cu_host: np.ndarray, blk: int = ATTN_BLOCK) -> torch.Tensor:
    """[2, n] int32 work order of the varlen attention kernels: one entry ``(b << 12) | block``
    per 128-row block of every sequence (filler row included), longest sequence first (LPT: the
    hardware dispatcher starts the long blocks at once and back-fills the short ones; in batch
    order a long sequence late in the batch would start last and set the kernel's tail).
    Row 0 orders query blocks (forward, dQ): within a sequence the last block first (the costliest
    under a causal mask). Row 1 orders key blocks (dK / dV): the first block first."""
    cu = np.asarray(cu_host, dtype=np.int64)
    lens = cu[1:] - cu[:-1]
    nb = (lens + blk - 1) // blk
    b = np.repeat(np.arange(len(lens), dtype=np.int64), nb)
    k = np.arange(int(nb.sum()), dtype=np.int64) - np.repeat(np.cumsum(nb) - nb, nb)
    L = lens[b]
    q_order = np.lexsort((-k, -L))   # by L desc, then block desc
    k_order = np.lexsort((k, -L))    # by L desc, then block asc
    enc = (b << 12) | k
    return torch.from_numpy(np.stack([enc[q_order], enc[k_order]]).astype(np.int32))


def _sort_order(keys: torch.Tensor) -> torch.Tensor:
    """[2, T] int32: stable ascending sort of ``keys`` (sorted keys | source positions) — the
    same order the device path's stable at::sort produces."""
    k = keys.numpy()
    perm = np.argsort(k, kind="stable")
    return torch.from_numpy(np.stack([k[perm], perm]).astype(np.int32))


def presort(b: PackedBatch) -> PackedBatch:
    return PackedBatch(b.input_ids, b.position_ids, b.cu_seqlens, b.labels, b.max_seqlen,
                       b.seq_lens, b.cu_host, _sort_order(b.input_ids), _sort_order(b.position_ids),
                       b.attn_sched)


def pad_packed(b: PackedBatch, multiple: int, pad_id: int = 0) -> PackedBatch:
    """Round the packed token count up to ``multiple`` with ONE filler row appended as its own
    sequence (attention never mixes it with real rows; pooling/loss only read the real rows).
    Bucketing T keeps the GEMM shapes (M = T) to a small set, so the BLAS algorithm choice and
    tuning results are reused batch after batch."""
    if multiple <= 1:
        return b
    T = b.num_tokens
    P = (-T) % multiple
    if P == 0:
        return b
    ids = torch.cat([b.input_ids, torch.full((P,), pad_id, dtype=torch.int32)])
    # filler positions are all 0: a filler row can be longer than the model's position table
    # (P < multiple = 256 > 128 positions of the tiny test models) and its values are never read
    pos = torch.cat([b.position_ids, torch.zeros(P, dtype=torch.int32)])
    cu = np.concatenate([b.cu_host, [T + P]])
    return PackedBatch(ids, pos, torch.from_numpy(cu.astype(np.int32)), b.labels,
                       max(b.max_seqlen, P), b.seq_lens, cu, attn_sched=attn_schedule(cu))


class MicroBatches(list):
    """One optimizer step's rows as k packed micro-batches (each padded on its own) that a
    :class:`bcfl.fl.trainer.LocalTrainer` with micro-batch replicas trains CONCURRENTLY on k HIP
    streams, summing the gradients into one AdamW step — how a GPU that hosts a single client
    (8 clients on 8 GPUs) keeps more than one kernel stream busy."""

    @property
    def batch_size(self) -> int:
        return sum(b.batch_size for b in self)

    @property
    def num_tokens(self) -> int:
        return sum(b.num_tokens for b in self)

    @property
    def real_tokens(self) -> int:
        return sum(b.real_tokens for b in self)

    @property
    def labels(self) -> torch.Tensor:
        return torch.cat([b.labels for b in self])


@dataclass
class PaddedBatch:
    input_ids: torch.Tensor       # [B, S] int64
    attention_mask: torch.Tensor  # [B, S] int64
    labels: torch.Tensor          # [B]


def _gather(ds: TokenDataset, idx: np.ndarray):
    lens = ds.lengths[idx]
    cu = np.zeros(len(idx) + 1, dtype=np.int64)
    np.cumsum(lens, out=cu[1:])
    starts = ds.offsets[idx]
    # flat gather index: start_of_row + position_in_row
    pos = np.arange(cu[-1], dtype=np.int64) - np.repeat(cu[:-1], lens)
    flat = np.repeat(starts, lens) + pos
    return ds.tokens[flat], pos, cu, lens


def make_packed_batch(ds: TokenDataset, idx: np.ndarray) -> PackedBatch:
    toks, pos, cu, lens = _gather(ds, np.asarray(idx, dtype=np.int64))
    return PackedBatch(torch.from_numpy(toks.astype(np.int32)),
                       torch.from_numpy(pos.astype(np.int32)),
                       torch.from_numpy(cu.astype(np.int32)),
                       torch.from_numpy(ds.labels[idx].astype(np.int32)),
                       int(lens.max()) if len(lens) else 0, lens, cu,
                       attn_sched=attn_schedule(cu))


def make_padded_batch(ds: TokenDataset, idx: np.ndarray, pad_id: int = 0) -> PaddedBatch:
    idx = np.asarray(idx, dtype=np.int64)
    lens = ds.lengths[idx]
    S = int(lens.max())
    ids = np.full((len(idx), S), pad_id, dtype=np.int64)
    mask = np.zeros((len(idx), S), dtype=np.int64)
    for r, i in enumerate(idx):
        row = ds.row(int(i))
        ids[r, : len(row)] = row
        mask[r, : len(row)] = 1
    return PaddedBatch(torch.from_numpy(ids), torch.from_numpy(mask),
                       torch.from_numpy(ds.labels[idx].astype(np.int64)))


class ClientLoader:
    """Epoch iterator over one client's rows (train: shuffled like ``DataLoader(shuffle=True)``)."""

    def __init__(self, ds: TokenDataset, indices: np.ndarray, batch_size: int = 32,
                 shuffle: bool = False, seed: int = 0, pad_multiple: int = 0, split: int = 1,
                 presort: bool = False):
        self.split = max(1, int(split))  # > 1: every batch as MicroBatches of ~equal row counts
        self.presort = presort           # training batches: host-side embedding sort orders
        self.ds = ds
        self.indices = np.asarray(indices, dtype=np.int64)
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.seed = seed
        self.pad_multiple = pad_multiple
        self.epoch = 0

    def __len__(self) -> int:  # number of batches (Flower's num_examples quirk uses this)
        return (len(self.indices) + self.batch_size - 1) // self.batch_size

    @property
    def num_examples(self) -> int:
        return int(len(self.indices))

    def _order(self, epoch: Optional[int] = None) -> np.ndarray:
        e = self.epoch if epoch is None else epoch
        if not self.shuffle:
            return self.indices
        r = np.random.default_rng([self.seed, e])
        return self.indices[r.permutation(len(self.indices))]

    def _one(self, idx: np.ndarray) -> PackedBatch:
        b = pad_packed(make_packed_batch(self.ds, idx), self.pad_multiple)
        return presort(b) if self.presort else b

    def _pack(self, idx: np.ndarray):
        if self.split <= 1 or len(idx) < 2:
            return self._one(idx)
        parts = [p for p in np.array_split(idx, min(self.split, len(idx))) if len(p)]
        return MicroBatches(self._one(p) for p in parts)

    def host_batches(self, epoch: Optional[int] = None) -> list:
        order = self._order(epoch)
        return [self._pack(order[i:i + self.batch_size]) for i in range(0, len(order), self.batch_size)]

    @staticmethod
    def _parts(b: PackedBatch):
        return [t for t in (b.input_ids, b.position_ids, b.cu_seqlens, b.labels, b.sort_ids,
                            b.sort_pos, b.attn_sched) if t is not None]

    def stage(self, epoch: Optional[int] = None, pin: bool = True):
        """Host half of :meth:`device_batches`: the epoch's packed batches and ONE (pinned)
        int32 buffer holding all of their index tensors. Pure host work (no device call), so it
        can run on a prefetch thread while the previous round trains."""
        hb = self.host_batches(epoch)
        self.epoch += 1
        if not pin:
            return hb, None
        flat = [x for b in hb for x in (b if isinstance(b, MicroBatches) else [b])]
        total = int(sum(t.numel() for b in flat for t in self._parts(b)))
        host = torch.empty(total, dtype=torch.int32, pin_memory=True)
        off = 0
        for b in flat:
            for t in self._parts(b):
                n = t.numel()
                host[off:off + n].copy_(t.reshape(-1))
                off += n
        return hb, host

    def device_batches(self, device, epoch: Optional[int] = None) -> List[PackedBatch]:
        """All batches of one epoch, staged with ONE pinned-buffer H2D copy."""
        dev = torch.device(device)
        return self.upload(self.stage(epoch, pin=dev.type == "cuda"), dev)

    def upload(self, staged, device) -> List[PackedBatch]:
        """Device half: one H2D copy of the staged buffer on the current stream, then views."""
        hb, host = staged
        dev = torch.device(device)
        if dev.type != "cuda":
            return hb
        parts = self._parts
        devbuf = host.to(dev, non_blocking=True)
        off = 0

        def view(b: PackedBatch) -> PackedBatch:
            nonlocal off
            views = []
            for t in parts(b):
                n = t.numel()
                views.append(devbuf[off:off + n].view(t.shape))
                off += n
            i = 4
            so = (None, None)
            if b.sort_ids is not None:
                so, i = (views[4], views[5]), 6
            sched = views[i] if b.attn_sched is not None else None
            return PackedBatch(views[0], views[1], views[2], views[3], b.max_seqlen, b.seq_lens,
                               b.cu_host, *so, attn_sched=sched)

        out = [MicroBatches(view(x) for x in b) if isinstance(b, MicroBatches) else view(b)
               for b in hb]
        self._keepalive = (host, devbuf)
        return out

    def __iter__(self) -> Iterator[PackedBatch]:
        yield from self.host_batches()
        self.epoch += 1
