"""Local training / evaluation on device (reference ``train()``/``test()``,
``src/Servercase/server_IID_IMDB.py:108-135``, and ``IMDBClient.train_model``/``evaluate_model``,
``src/Serverlesscase/serverless_IID_IMDB.py:156-187``).

Differences by design: batches are packed and pre-staged on the device (one H2D per client per
epoch instead of one per batch), the optimizer is the fused flat AdamW, and metrics accumulate
on the device so an epoch has exactly one host sync.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Sequence

import torch

from .. import ops
from ..data.batching import MicroBatches, PackedBatch
from ..parallel.flat import FlatAdamW, FlatParams


@dataclass
class EvalResult:
    correct: int
    count: int
    loss_sum: float        # sum over examples of per-example CE
    batch_mean_sum: float  # reference quirk: sum of per-batch mean losses

    @property
    def accuracy(self) -> float:
        return self.correct / max(self.count, 1)

    @property
    def loss(self) -> float:
        return self.loss_sum / max(self.count, 1)

    @property
    def ref_loss(self) -> float:
        """Reference ``test()``: Σ batch-mean losses ÷ dataset size."""
        return self.batch_mean_sum / max(self.count, 1)


# Backward on the calling thread: autograd's per-device worker thread hands every Python
# backward Function across threads (GIL hand-off per node), which made the one-client step's
# host issue 8.1 ms against 9.6 ms of device time, and the device idled wherever the host fell
# behind (loss head, optimizer launch, step boundary). On the caller thread the same step issues
# in 5.8 ms (scripts/host_step_timing.py, profiles/host_issue_r6.json). Streams are unchanged:
# each backward node still runs on the stream its forward ran on. BCFL_AUTOGRAD_THREAD=1 restores
# the worker thread (A/B runs).
_CALLER_THREAD_BACKWARD = os.environ.get("BCFL_AUTOGRAD_THREAD", "0") != "1"


def backward(loss: torch.Tensor) -> None:
    if _CALLER_THREAD_BACKWARD and loss.is_cuda:
        with torch.autograd.set_multithreading_enabled(False):
            loss.backward()
    else:
        loss.backward()


class MicroReplica:
    """A second model instance whose parameters are views of the trainer's OWN flat buffers
    (FlatParams.rebind), plus the HIP stream its micro-batch runs on."""

    def __init__(self, model, flat: FlatParams, stream):
        self.model, self.flat, self.stream = model, flat, stream


class LocalTrainer:
    def __init__(self, model, flat: FlatParams, opt: FlatAdamW, micro: "MicroReplica" = None):
        self.model, self.flat, self.opt = model, flat, opt
        self.micro = micro

    def _step_micro(self, mb: MicroBatches, loss_acc: torch.Tensor) -> None:
        """Two micro-batches of one optimizer step trained concurrently: rows [0, B1) on the
        current stream with this model, rows [B1, B) on the replica's stream with the replica
        (same weights). Each loss is weighted by its share of the rows, so the summed gradient
        is the full batch's mean-loss gradient; AdamW sums the two in its single pass."""
        rep = self.micro
        a, b = mb
        B = a.batch_size + b.batch_size
        main = torch.cuda.current_stream(self.flat.device) if self.flat.device.type == "cuda" else None
        if rep.flat.master is not self.flat.master or rep.flat.param is not self.flat.param:
            rep.flat.rebind(self.flat.master, self.flat.param)  # follow the main replica's rebinds
        self.model.train()
        rep.model.train()
        la = ops.cross_entropy(self.model(a), a.labels) * (a.batch_size / B)
        if main is not None:
            rep.stream.wait_stream(main)
            with torch.cuda.stream(rep.stream):
                lb = ops.cross_entropy(rep.model(b), b.labels) * (b.batch_size / B)
        else:
            lb = ops.cross_entropy(rep.model(b), b.labels) * (b.batch_size / B)
        backward(la)
        if main is not None:
            ops.join_wgrad(self.flat.device)
            with torch.cuda.stream(rep.stream):
                backward(lb)
                ops.join_wgrad(self.flat.device)
            main.wait_stream(rep.stream)
        else:
            backward(lb)
        self.opt.step(partner=rep.flat)
        self.flat.zero_grad()
        rep.flat.zero_grad()
        loss_acc += la.detach() + lb.detach()

    def step(self, b: PackedBatch, loss_acc: torch.Tensor) -> None:
        """One optimizer step on one batch; the loss is accumulated on the device (no sync)."""
        if isinstance(b, MicroBatches):
            if self.micro is not None and len(b) == 2:
                return self._step_micro(b, loss_acc)
            raise ValueError("micro-batches need a LocalTrainer with a micro replica (2 parts)")
        self.model.train()
        logits = self.model(b)
        loss = ops.cross_entropy(logits, b.labels)
        if self.opt.overlap_active():
            # per-layer AdamW on a side stream, launched from the gradient hooks mid-backward
            self.opt.begin_overlapped()
            backward(loss)
            ops.join_wgrad(self.flat.device)
            self.opt.finish_overlapped()
        else:
            backward(loss)
            if self.flat.device.type == "cuda":
                ops.join_wgrad(self.flat.device)  # overlapped weight gradients -> optimizer
            self.opt.step()
        self.flat.zero_grad()
        loss_acc += loss.detach()

    def train_epoch(self, batches: Sequence[PackedBatch], lr_fn=None,
                    step_hook=None) -> Dict[str, torch.Tensor]:
        """``step_hook()`` runs after every optimizer step (async gossip: neighbours' updates
        that have arrived are applied between local steps)."""
        loss_acc = torch.zeros((), dtype=torch.float32, device=self.flat.device)
        for i, b in enumerate(batches):
            if lr_fn is not None:
                self.opt.lr = lr_fn(i)
            self.step(b, loss_acc)
            if step_hook is not None:
                step_hook()
        return {"loss_sum": loss_acc, "batches": len(batches),
                "tokens": sum(b.real_tokens for b in batches),
                "examples": sum(b.batch_size for b in batches)}

    @torch.no_grad()
    def evaluate_device(self, batches: Sequence[PackedBatch]) -> torch.Tensor:
        """[correct, count, loss_sum, batch_mean_sum] as a device fp64 tensor (no host sync)."""
        m = self.model
        m.eval()
        dev = self.flat.device
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        for b in batches:
            ops.xent_stats_(m(b), b.labels, acc)  # one kernel per batch on the GPU (K9)
        return acc

    def evaluate(self, batches: Sequence[PackedBatch]) -> EvalResult:
        a = self.evaluate_device(batches).cpu().tolist()
        return EvalResult(int(a[0]), int(a[1]), a[2], a[3])
