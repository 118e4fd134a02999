"""Process-group runtime: one process per GPU (RCCL over xGMI) or per CPU worker (gloo).

Launch: ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...``
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the env). A run without those
env vars is a world of one and needs no process group at all.

Replaces the reference's Flower simulation over Ray (``fl.simulation.start_simulation`` with
``ray_init_args={"num_cpus": 1}``, ``src/Servercase/server_IID_IMDB.py:211-218``: clients run one
at a time and parameters travel as pickled numpy lists through the object store).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class Runtime:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str
    initialized_here: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


_RT: Optional[Runtime] = None


def init_runtime(device: str = "auto", backend: str = "auto", timeout_s: int = 600) -> Runtime:
    global _RT
    if _RT is not None:
        return _RT
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device == "auto":
        use_cuda = torch.cuda.is_available()
    else:
        use_cuda = device.startswith("cuda")
    if use_cuda:
        n = torch.cuda.device_count()
        dev = torch.device("cuda", local_rank % max(n, 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if backend == "auto":
        # BCFL_DIST_BACKEND=gloo: several ranks sharing ONE GPU (RCCL refuses duplicate devices)
        # — how the multi-rank bench path (hipIpc mailboxes between processes) is rehearsed on a
        # 1-GPU box; the 8-GPU job uses RCCL
        backend = os.environ.get("BCFL_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
    here = False
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
            kw["pg_options"] = _rccl_options()
        dist.init_process_group(**kw)
        here = True
    _RT = Runtime(rank, world, local_rank, dev, backend, here)
    return _RT


def _rccl_options():
    """Communicator options of the engine's RCCL process group:

    * the collectives run on a HIGH-PRIORITY stream: FedAvg / gossip transfers are issued while
      the next local step's kernels fill the CUs, and a low-priority communicator stream would
      queue behind them instead of overlapping;
    * channels: RCCL's own choice for MI355X unless ``BCFL_RCCL_CHANNELS`` pins both bounds
      (``NCCL_MIN_NCHANNELS`` / ``NCCL_MAX_NCHANNELS``: more channels spread one collective
      over more of the 7 xGMI links and more CUs)."""
    ch = os.environ.get("BCFL_RCCL_CHANNELS")
    if ch:
        os.environ.setdefault("NCCL_MIN_NCHANNELS", ch)
        os.environ.setdefault("NCCL_MAX_NCHANNELS", ch)
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):
        return None


def runtime() -> Runtime:
    return _RT if _RT is not None else init_runtime()


def shutdown():
    global _RT
    if _RT is not None and _RT.initialized_here and dist.is_initialized():
        dist.destroy_process_group()
    _RT = None


def set_runtime_for_tests(rt: Optional[Runtime]):
    global _RT
    _RT = rt


# ------------------------------------- collectives -------------------------------------------

def barrier():
    rt = runtime()
    if rt.distributed:
        if rt.backend == "nccl":
            dist.barrier(device_ids=[rt.device.index])
        else:
            dist.barrier()


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
    rt = runtime()
    if not rt.distributed:
        return None
    return dist.all_reduce(t, op=op, async_op=async_op)


def all_reduce_bf16_(x: torch.Tensor) -> int:
    """Sum a flat fp32 tensor over ranks with bf16 on the wire and fp32 accumulation.

    Reduce-scatter as an all-to-all of bf16 chunks (every rank receives all ranks' copy of ITS
    1/world chunk and sums them in fp32), then an all-gather of the bf16-rounded chunk sums:
    2 (world-1)/world x 2 B per element on the wire — half of a ring fp32 all-reduce — and only
    ONE bf16 rounding per element (a bf16 ring all-reduce would round at every hop). Meant for
    DELTAS (FedAvg: sum_k w_k (x_k - G)), whose bf16 rounding is relative to the update, not to
    the weights. Returns the bytes this rank put on the wire."""
    rt = runtime()
    if not rt.distributed:
        return 0
    from .. import ops
    W, n = rt.world, x.numel()
    per = -(-n // W)
    per = -(-per // 64) * 64                  # 128-byte aligned chunks for the vector kernels
    key = (W * per, x.device)
    bufs = _BF16_BUFS.get(key)
    if bufs is None:                          # persistent wire buffers (no per-call allocation)
        bufs = {"send": torch.zeros(W * per, dtype=torch.bfloat16, device=x.device),
                "recv": torch.empty(W * per, dtype=torch.bfloat16, device=x.device),
                "out": torch.empty(W * per, dtype=torch.bfloat16, device=x.device),
                "acc": torch.empty(per, dtype=torch.float32, device=x.device)}
        _BF16_BUFS.clear()
        _BF16_BUFS[key] = bufs
    send, recv, out, acc = bufs["send"], bufs["recv"], bufs["out"], bufs["acc"]
    ops.cast_copy_(send[:n], x.reshape(-1))
    dist.all_to_all_single(recv, send)        # every rank gets all ranks' copy of ITS chunk
    chunks = list(recv.view(W, per))
    acc.copy_(chunks[0])
    # fp32 sum of the W bf16 copies, written back as bf16 into this rank's slot of `out` (one
    # kernel), then the all-gather of the bf16 chunk sums
    mine = out.view(W, per)[rt.rank]
    ops.gossip_mix_(acc, chunks[1:], 1.0, [1.0] * (W - 1), mine)
    dist.all_gather_into_tensor(out, mine)
    ops.cast_copy_(x.reshape(-1), out[:n])
    return 2 * (W - 1) * per * 2


_BF16_BUFS: dict = {}


def broadcast_(t: torch.Tensor, src: int = 0):
    if runtime().distributed:
        dist.broadcast(t, src=src)


def all_gather_tensor(t: torch.Tensor) -> torch.Tensor:
    """[world, *t.shape] gather (same shape on every rank)."""
    rt = runtime()
    if not rt.distributed:
        return t.unsqueeze(0).clone()
    out = torch.empty((rt.world, *t.shape), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous())
    return out


def all_gather_object(obj: Any) -> List[Any]:
    rt = runtime()
    if not rt.distributed:
        return [obj]
    out = [None] * rt.world
    dist.all_gather_object(out, obj)
    return out


def max_over_ranks(x: float) -> float:
    rt = runtime()
    if not rt.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=rt.device if rt.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class P2PHandle:
    """Outstanding batched send/recv (RCCL runs it on its own stream, overlapping compute)."""

    def __init__(self, works):
        self.works = works or []
        self.done = not self.works

    def wait(self):
        if not self.done:
            for w in self.works:
                w.wait()
            self.done = True


def p2p_exchange(sends: Sequence[Tuple[torch.Tensor, int]],
                 recvs: Sequence[Tuple[torch.Tensor, int]]) -> P2PHandle:
    """Grouped point-to-point: ``ncclGroupStart; ncclSend...; ncclRecv...; ncclGroupEnd``.

    Returns immediately; the transfers run on the communicator's stream after the work already
    queued on the current stream (so a snapshot copy issued before is ordered correctly)."""
    rt = runtime()
    if not rt.distributed or (not sends and not recvs):
        return P2PHandle([])
    ops_ = [dist.P2POp(dist.isend, t, peer) for t, peer in sends]
    ops_ += [dist.P2POp(dist.irecv, t, peer) for t, peer in recvs]
    return P2PHandle(dist.batch_isend_irecv(ops_))
