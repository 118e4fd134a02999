"""Local / global evaluation of a federation: the global draw, sharded and averaged scoring, the side-stream
overlapped evaluation, deferred local scores and the server's hold-out gate (mixed into
:class:`~bcfl.fl.federation.Federation`). Reference: ``evaluate_model`` / ``evaluate_global_model`` /
``test()`` (``src/Serverlesscase/serverless_IID_IMDB.py:172-187,235-246``, ``src/Servercase/server_IID_IMDB.py:121-135``)."""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..data.batching import ClientLoader
from ..data.partition import global_test_indices, majority_rate
from ..models import build_model
from ..parallel import dist as D
from ..parallel.flat import FlatParams
from ..parallel.gossip import MailboxGossip
from .trainer import EvalResult, LocalTrainer
from .fedutil import weighted_average
from .lanes import _share_frozen


# BCFL_EVAL_READ_SYNC=1: read evaluation results with .cpu() at resolve time (A/B baseline)
_SYNC_READS = bool(os.environ.get("BCFL_EVAL_READ_SYNC"))
# BCFL_EVAL_LOCAL_EARLY=1: issue a local evaluation right after its snapshot (A/B baseline)
_EARLY_LOCAL = bool(os.environ.get("BCFL_EVAL_LOCAL_EARLY"))


def _host_copy(t: torch.Tensor) -> torch.Tensor:
    """Queue a D2H copy of a small device result on the CURRENT stream into pinned host memory
    (record the completion event after it). ``t.cpu()`` at read time would synchronise the reading
    thread's current stream — the training stream — and drain every launch queued on it."""
    if _SYNC_READS:
        return t
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t, non_blocking=True)
    return h


class EvalMixin:
    def _cached_batches(self, key, build):
        """Evaluation batches are a pure function of the (per-round when resampling) draw: build
        and upload them once, keep them resident on the device (read-only afterwards)."""
        if not hasattr(self, "_batch_cache"):
            self._batch_cache = {}
        if key not in self._batch_cache:
            if len(self._batch_cache) > 4 * (self.cfg.num_clients + 1):
                self._batch_cache.clear()  # resampling draws: keep only recent rounds
            self._batch_cache[key] = build()
        return self._batch_cache[key]

    def _eval_batches(self, key, make_loader):
        """Cached evaluation batches of ``key``; a draw packed ahead on the prefetch thread
        (:meth:`_prefetch_eval`) is only uploaded here."""
        def build():
            fut = getattr(self, "_prefetched", {}).pop(key, None)
            if fut is not None:
                ld, staged = fut.result()
                return ld.upload(staged, self.device)
            return make_loader().device_batches(self.device)
        return self._cached_batches(key, build)

    def _draw_key(self, r: int) -> int:
        return r if self.cfg.resample_each_round else 0

    def _test_loader(self, c: int, r: int) -> ClientLoader:
        return ClientLoader(self.test_ds, self.partitions(r)[c].test, self.cfg.batch_size,
                            pad_multiple=self.pad_multiple)

    def test_batches(self, c: int, r: int):
        return self._eval_batches(("test", c, self._draw_key(r)), lambda: self._test_loader(c, r))

    def global_test_idx(self, r: int) -> np.ndarray:
        c = self.cfg
        return global_test_indices(len(self.test_ds), c.global_test_samples, c.seed,
                                   r if c.resample_each_round else None,
                                   self.test_ds.labels if c.global_test_stratified else None)

    def _sharded_eval(self) -> bool:
        c = self.cfg
        return c.mode == "serverless" and c.global_eval_models == "all" and not c.compat_chain

    def _global_eval_rows(self, r: int, c: Optional[int] = None) -> np.ndarray:
        """Rows of round r's global draw scored by client c's model (sharded evaluation: client c
        takes rows c, c + K, c + 2K, ... of the class-balanced draw) or by this rank (c None:
        the whole draw when collective-free, else a rank stride of it)."""
        idx = self.global_test_idx(r)
        if c is not None:
            return idx[c::self.cfg.num_clients]
        return idx if self.collective_free else idx[self.rt.rank::self.rt.world]

    def global_majority_rate(self, r: int) -> float:
        """Best constant-predictor accuracy on the rows this rank scored in round r (printed
        beside accuracy so a collapsed model cannot pass for a trained one)."""
        if self._sharded_eval():
            idx = np.concatenate([self._global_eval_rows(r, c) for c in self.local_clients])
        else:
            idx = self.global_test_idx(r)
        return majority_rate(self.test_ds.labels, idx)

    def _global_loader(self, r: int, c: Optional[int] = None) -> ClientLoader:
        return ClientLoader(self.test_ds, self._global_eval_rows(r, c),
                            max(self.cfg.global_eval_batch, 1), pad_multiple=self.pad_multiple)

    def _hosted_loader(self, r: int) -> ClientLoader:
        """One model on the union of the hosted clients' strides (identical hosted models)."""
        return ClientLoader(self.test_ds, np.sort(np.concatenate(
            [self._global_eval_rows(r, c) for c in self.local_clients])),
            max(self.cfg.global_eval_batch, 1), pad_multiple=self.pad_multiple)

    def global_test_batches(self, r: int, c: Optional[int] = None):
        if len(self._global_eval_rows(r, c)) == 0:
            return []
        return self._eval_batches(("global", self._draw_key(r), c), lambda: self._global_loader(r, c))

    def _global_eval_sets(self, r: int):
        """[(client, batches)] this rank scores for round r's global evaluation. Sharded
        (serverless default): every hosted client's mixed model on its stride of the draw, so the
        federation's models are all scored and the job evaluates the draw exactly once per round
        whatever the GPU count. Otherwise one model (client None = the model bound to
        ``self.flat``: the global model in server mode, the first hosted client in serverless)."""
        if self._sharded_eval():
            if len(self.local_clients) > 1 and self._hosted_models_identical():
                # every hosted client holds the same model: one model on the union of their
                # strides scores exactly the same rows with exactly the same predictions, in
                # fewer, larger forwards and with one snapshot instead of one per client
                c0 = self.local_clients[0]
                return [(c0, self._eval_batches(("global", self._draw_key(r), "hosted"),
                                                lambda: self._hosted_loader(r)))]
            return [(c, self.global_test_batches(r, c)) for c in self.local_clients]
        if self._average_eval():
            self._refresh_average()
            self._avg_round = r
            return [(-1, self.global_test_batches(r))]
        return [(None, self.global_test_batches(r))]

    def _hosted_models_identical(self) -> bool:
        """Round-complete delta gossip with every hosted client's round end fused: each model was
        set back to its round-start record and every complete round was applied to all of them
        with the same shared update, so they are bit-identical at the round end (the models of a
        federation whose rounds are all complete are the same model)."""
        g = self.gossip
        return (isinstance(g, MailboxGossip) and g.exchange == "delta" and g.apply_mode == "complete"
                and g._fused == set(self.local_clients) and not g.suppressed and not g.tamper
                and (self._gossip_filter or (self.filter is None and not self.cfg.inject_byzantine))
                and self.cfg.topology == "full" and self.cfg.mixing == "average")

    def _average_eval(self) -> bool:
        c = self.cfg
        return (c.mode == "serverless" and c.global_eval_models == "average" and self.multi
                and not c.compat_chain)

    @torch.no_grad()
    def _refresh_average(self) -> None:
        """Reference-faithful global model (``serverless_NonIID_IMDB.py:296-304``: ONE averaged
        ``global_model`` scored on the whole draw): the unweighted mean of this rank's hosted
        client models (every client on one GPU: all of them), cast to the compute dtype."""
        cs = self.local_clients
        if not hasattr(self, "_avg_master"):
            self._avg_master = torch.empty_like(self.flat.master)
            self._avg_param = torch.empty(self.flat.numel, dtype=self.flat.dtype, device=self.device)
        src = [self.client_master[c] for c in cs]
        self._avg_master.copy_(src[0])
        ops.gossip_mix_(self._avg_master, src[1:], 1.0 / len(src), [1.0 / len(src)] * (len(src) - 1),
                        self._avg_param if self._avg_param.dtype != torch.float32 else None)
        if self._avg_param.dtype == torch.float32:
            self._avg_param.copy_(self._avg_master)

    def _bind_client(self, c: Optional[int]) -> None:
        """Point ``self.flat`` (lane 0's replica) at client c's current state for evaluation
        (c = -1: the averaged model of ``global_eval_models='average'``)."""
        if c is None or not self.multi:
            return
        if c == -1:
            self.flat.rebind(self._avg_master, self._avg_param)
            return
        if self.lanes:
            self.flat.rebind(self.client_master[c], self.client_param[c])
        else:
            self.flat.load_master(self.client_master[c])

    def _client_param(self, c: Optional[int]) -> torch.Tensor:
        if c == -1:
            return self._avg_param
        if c is not None and self.lanes:
            return self.client_param[c]
        if c is not None and self.multi:
            raise RuntimeError("overlapped evaluation of a non-resident client")
        return self.flat.param

    def _note_global_counts(self, r: int, acc4) -> None:
        self._last_global_counts = (r, float(acc4[0]), float(acc4[1]))

    def federation_accuracy(self) -> Dict[str, float]:
        """Accuracy of the LAST evaluated round over the whole job (a collective in a
        collective-free run: every rank's [correct, rows] are gathered). With sharded evaluation
        this is the mean accuracy of all client models, each on its disjoint stride of the
        class-balanced draw."""
        last = getattr(self, "_last_global_counts", None)
        parts = [last] if not (self.collective_free and self.rt.distributed) else \
            D.all_gather_object(last)
        parts = [x for x in parts if x is not None]
        if not parts:
            return {}
        rounds = {x[0] for x in parts}
        correct = sum(x[1] for x in parts)
        rows = sum(x[2] for x in parts)
        return {"accuracy": correct / max(rows, 1.0), "rows": rows, "round": max(rounds),
                "ranks": len(parts), "rounds_agree": len(rounds) == 1}

    # ---------------- overlapped global evaluation ----------------------------------------------
    def _build_eval_overlap(self, vocab: int, mdtype: torch.dtype):
        """Global evaluation off the critical path: round r's evaluated model is snapshotted into
        an eval replica (one D2D copy of the bf16 parameters) and scored on a side stream, so the
        forward passes over the global draw run concurrently with round r+1's training (with one
        client per GPU — the 8-GPU layout — a training step leaves most CUs idle between
        kernels). The evaluated model, rows and kernels are exactly those of the inline path;
        only the host read is deferred (``_resolve_eval``). In collective mode (server FedAvg
        over RCCL, lock-step gossip) the statistics are all-reduced at that deferred read, which
        every rank reaches at the same point of its program."""
        cfg = self.cfg
        self._eval_pending = None
        self.eval_model = self.eval_flat = self.eval_trainer = self.eval_stream = None
        on = cfg.overlap_global_eval
        if on is None:
            big = self.flat.numel > 1_000_000_000
            on = self.is_cuda and not big and not cfg.deterministic and not cfg.compat_chain
        if not (on and cfg.eval_global and self.is_cuda):
            return
        self.eval_model = build_model(cfg.model, self.num_labels, device=self.device, dtype=mdtype,
                                      dropout=cfg.dropout, vocab_size=vocab, seed=cfg.seed,
                                      lora_rank=cfg.lora_rank, lora_alpha=cfg.lora_alpha)
        _share_frozen(self.eval_model, self.model)
        self.eval_flat = FlatParams.from_model(self.eval_model, self.device, mdtype)
        self.eval_trainer = LocalTrainer(self.eval_model, self.eval_flat, None)
        self.eval_stream = torch.cuda.Stream(device=self.device)

    def _launch_eval_global(self, r: int) -> None:
        """Snapshot the model(s) the inline path would score and queue their evaluation."""
        self._resolve_eval()
        with self.timer.phase("eval_global"):
            sets = self._global_eval_sets(r)   # first use uploads on the current stream
            main = torch.cuda.current_stream(self.device)
            es = self.eval_stream
            if not hasattr(self, "_eval_snaps"):
                self._eval_snaps = {}
            # the snapshots are taken on the TRAINING stream: later writers of the sources (next
            # round's optimizer / mixing) are ordered after them by stream order, and the training
            # stream never waits for the side stream (a copy queued there would wait behind the
            # local evaluation already running on it). The previous global evaluation, the only
            # reader of these buffers, was resolved (synchronised) above.
            snaps = []
            for c, _ in sets:
                if len(sets) == 1:
                    snap = self.eval_flat.param
                else:
                    snap = self._eval_snaps.get(c)
                    if snap is None:
                        snap = self._eval_snaps[c] = torch.empty_like(self.eval_flat.param)
                snap.copy_(self._client_param(c))
                snaps.append(snap)
            es.wait_stream(main)               # the snapshots and the batches are ready
            with torch.cuda.stream(es):
                t_beg = torch.cuda.Event(enable_timing=True)
                t_beg.record(es)
                acc = torch.zeros(4, dtype=torch.float64, device=self.device)
                for (c, gb), snap in zip(sets, snaps):
                    if gb:
                        self.eval_flat.rebind(self.eval_flat.master, snap)
                        acc += self._eval_forward(snap, gb)
                # collective-free: the counts cross to pinned host memory on the side stream, so
                # the host read never synchronises the training stream (acc.cpu() would: it drains
                # the round queued on the reading thread's current stream first)
                self._eval_host = _host_copy(acc) if self.collective_free and not _SYNC_READS else None
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(es)
            self._eval_pending = (r, acc, sets, ev, t_beg)

    def _eval_forward(self, snap: torch.Tensor, batches) -> torch.Tensor:
        """The side stream's evaluation of the replica bound to ``snap`` on ``batches`` (cached,
        fixed device batches): eager the first time, then captured once into a hipGraph per
        (snapshot buffer, batch set) and replayed. A BERT-base forward over a few batches is ~200
        launches, ~2.2 ms of host issue per evaluation, which with one client per GPU the host
        spent while the training stream had nothing queued; a replay is one launch. The graph
        reads the same snapshot buffer and batches every round (both kept alive with it) and
        runs exactly the eager kernels. Opt-in (``BCFL_EVAL_GRAPHS=1``): once the round-start
        read stopped waiting for the evaluation, replays and eager issue measured the same
        (one-client layout, 3 interleaved reps each, ``profiles/host_issue_r6.json``)."""
        if os.environ.get("BCFL_EVAL_GRAPHS", "0") != "1" or not batches:
            return self.eval_trainer.evaluate_device(batches)
        if not hasattr(self, "_eval_graphs"):
            self._eval_graphs, self._eval_seen = {}, set()
        key = (snap.data_ptr(), id(batches))
        if key in self._eval_graphs and self._eval_graphs[key] is None:
            return self.eval_trainer.evaluate_device(batches)
        ent = self._eval_graphs.get(key)
        if ent is None:
            if key not in self._eval_seen:   # first use eager: allocator and kernels warm
                self._eval_seen.add(key)
                return self.eval_trainer.evaluate_device(batches)
            g = torch.cuda.CUDAGraph()
            try:
                # thread-local capture: the checkpoint writer thread may copy concurrently
                with torch.cuda.graph(g, stream=torch.cuda.current_stream(self.device),
                                      capture_error_mode="thread_local"):
                    out = self.eval_trainer.evaluate_device(batches)
            except RuntimeError as e:   # a model whose forward cannot be captured stays eager
                import warnings
                warnings.warn(f"evaluation forward not capturable ({e}); issuing it eagerly")
                self._eval_graphs[key] = None
                return self.eval_trainer.evaluate_device(batches)
            ent = self._eval_graphs[key] = (g, out, batches, snap)
        ent[0].replay()
        return ent[1]

    def _resolve_eval(self) -> None:
        """Host-read a queued global evaluation and file it under its round."""
        p, self._eval_pending = self._eval_pending, None
        if p is None:
            return
        r, acc, _sets, ev, t_beg = p
        host, self._eval_host = getattr(self, "_eval_host", None), None
        ev.synchronize()
        self.timer.add_hidden("eval_global", t_beg.elapsed_time(ev) / 1000.0)
        if not self.collective_free:
            D.all_reduce_(acc)
        a = host.tolist() if host is not None else acc.cpu().tolist()
        ge = EvalResult(int(a[0]), int(a[1]), a[2], a[3])
        self._note_global_counts(r, a)
        self.global_accuracies.append(ge.accuracy)
        self.global_accuracy_rounds.append(int(r))
        if self.verbose and self.cfg.reference_prints:
            print(f"Global Model Accuracy: {ge.accuracy * 100:.2f}%", flush=True)
        upd = {"global_acc": ge.accuracy, "global_majority_rate": self.global_majority_rate(r),
               "global_eval_rows": int(ge.count), "global_loss": ge.loss}
        for rec in reversed(self.history):
            if rec.get("round") == r:
                rec.update(upd)
                break
        self.metrics.write({"round": r, "deferred_global_eval": True, **upd})

    def _global_eval_due(self, r: int) -> bool:
        """Score the global draw this round? Every ``eval_global_every``-th round and always the
        last one (an 8B model's 1000-row evaluation costs about a third of its round)."""
        cfg = self.cfg
        if not cfg.eval_global:
            return False
        k = max(1, int(cfg.eval_global_every))
        return k == 1 or (r + 1) % k == 0 or r >= cfg.num_rounds - 1

    def _eval_global(self, r: int) -> EvalResult:
        with self.timer.phase("eval_global"):
            acc = torch.zeros(4, dtype=torch.float64, device=self.device)
            sets = self._global_eval_sets(r)
            for c, gb in sets:
                if gb:
                    self._bind_client(c)
                    acc += self.trainer.evaluate_device(gb)
            if len(sets) > 1 or (sets and sets[0][0] == -1):
                self._bind_client(self.local_clients[0])  # self.flat shows the first client again
            if not self.collective_free:
                D.all_reduce_(acc)
            a = acc.cpu().tolist()
        self._note_global_counts(r, a)
        return EvalResult(int(a[0]), int(a[1]), a[2], a[3])

    def _local_metrics(self, local_eval: Dict[int, torch.Tensor]) -> list:
        """Device [correct, count, loss_sum, batch_mean_sum] per client -> the reference's
        per-client metrics (gathered across ranks when not collective-free), printed like it."""
        cfg = self.cfg
        loc = []
        for c, t in local_eval.items():
            a = t.cpu().tolist()
            e = EvalResult(int(a[0]), int(a[1]), a[2], a[3])
            loc.append((c, e.count, {"accuracy": e.accuracy, "loss": e.ref_loss if cfg.compat_bad_test_loss else e.loss}))
        client_metrics = self._gather_metrics(loc) if cfg.eval_local else []
        if self.verbose and cfg.reference_prints:
            for c, _, m in sorted(client_metrics):
                print("local_accuracy" + " :" + str(m["accuracy"]), flush=True)
        return client_metrics

    def _file_local_eval(self, r: int, local_eval: Dict[int, torch.Tensor]) -> None:
        """Deferred host read of round r's local scores (collective-free single-process runs)."""
        cm = self._local_metrics(local_eval)
        for c, n_, m in cm:
            self.metrics.write({"round": r, "client": c, "local_acc": m.get("accuracy"),
                                "local_loss": m.get("loss"), "examples": n_})
        agg = weighted_average([(n_, m) for _, n_, m in cm]) if cm else {}
        self._patch_history(r, distributed_acc=agg.get("accuracy"),
                            distributed_loss=agg.get("loss"))

    # ---- local evaluation off the critical path (one client trained at a time) ----------------
    def _defer_local_eval(self) -> bool:
        """A rank that trains its clients one at a time (the 8-GPU layout: one client per GPU)
        scores the trained model on its local test rows on the eval side stream, from a snapshot,
        while gossip and the next round run (collective-free federations only: the metrics are
        filed when the host reads them, the next round)."""
        # single-process runs only: with several processes time-slicing one GPU (the multi-rank
        # rehearsal) the extra side-stream work per rank slowed rounds and stretched the ranks'
        # lead waits
        return (self.eval_stream is not None and self.collective_free and not self.lanes
                and self.cfg.eval_local and not self.cfg.compat_chain
                and not self.rt.distributed)

    def _launch_eval_local(self, c: int, r: int) -> None:
        """Snapshot client c's trained model on the training stream; its forward passes are
        issued on the side stream by :meth:`_issue_eval_local` after the round's exchange, so the
        host queues the round-end work of the training stream (commitment, exchange, mixing)
        first: with one client per GPU the host is barely ahead of the device at the end of
        training, and issuing ~200 evaluation kernels there left the training stream idle."""
        main = torch.cuda.current_stream(self.device)
        if not hasattr(self, "_local_snaps"):
            self._local_snaps = [torch.empty_like(self.flat.param) for _ in range(2)]
            self._local_done: List[Optional[torch.cuda.Event]] = [None, None]
            self._local_pending: List[tuple] = []
            self._local_queued: List[tuple] = []
            self._local_k = 0
        i = self._local_k % 2
        self._local_k += 1
        if any(q[5] == i for q in self._local_queued):
            self._issue_eval_local()               # its snapshot slot is about to be reused
        if self._local_done[i] is not None:
            main.wait_event(self._local_done[i])   # the evaluation that last read this snapshot
        snap = self._local_snaps[i]
        snap.copy_(self.flat.param)                # the trained model, before the mix
        batches = self.test_batches(c, r)          # uploaded on the training stream
        ready = torch.cuda.Event()
        ready.record(main)
        self._local_queued.append((r, c, snap, batches, ready, i))
        if _EARLY_LOCAL:
            self._issue_eval_local()

    def _issue_eval_local(self) -> None:
        """Queue the forward passes of the snapshotted local evaluations on the side stream."""
        q = getattr(self, "_local_queued", None)
        if not q:
            return
        self._local_queued = []
        es = self.eval_stream
        own = self.eval_flat.param
        for r, c, snap, batches, ready, i in q:
            es.wait_event(ready)
            with torch.cuda.stream(es):
                self.eval_flat.rebind(self.eval_flat.master, snap)
                stats = self._eval_forward(snap, batches)
                host = _host_copy(stats)
                ev = torch.cuda.Event()
                ev.record(es)
            self._local_done[i] = ev
            # the batches stay referenced until the statistics are read (their memory belongs to
            # the training stream's pool)
            self._local_pending.append((r, c, host, ev, batches))
        # the queued kernels hold the snapshots' pointers; the replica's own buffer is what the
        # global evaluation copies into (no later reader of a snapshot but its evaluation)
        self.eval_flat.rebind(self.eval_flat.master, own)

    def _resolve_eval_local(self, block: bool = True) -> None:
        """File the deferred local scores. ``block=False`` (the round start) files only those
        whose evaluation has finished: the last round's is usually still running on the side
        stream, and waiting for it there left the training stream idle ~5 ms per round."""
        self._issue_eval_local()
        pend = getattr(self, "_local_pending", None)
        if not pend:
            return
        k = 0
        while k < len(pend) and (block or pend[k][3].query()):
            k += 1
        pend, self._local_pending = pend[:k], pend[k:]
        by_round: Dict[int, list] = {}
        for r, c, host, ev, _b in pend:
            ev.synchronize()
            a = (host if host.device.type == "cpu" else host.cpu()).tolist()
            e = EvalResult(int(a[0]), int(a[1]), a[2], a[3])
            m = {"accuracy": e.accuracy, "loss": e.ref_loss if self.cfg.compat_bad_test_loss else e.loss}
            by_round.setdefault(r, []).append((c, e.count, m))
            if self.verbose and self.cfg.reference_prints:
                print("local_accuracy" + " :" + str(m["accuracy"]), flush=True)
            self.metrics.write({"round": r, "client": c, "local_acc": m.get("accuracy"),
                                "local_loss": m.get("loss"), "examples": e.count,
                                "deferred_local_eval": True})
        for r, cm in by_round.items():
            agg = weighted_average([(n_, m) for _, n_, m in cm])
            for rec in reversed(self.history):
                if rec.get("round") == r:
                    rec["distributed_acc"] = agg.get("accuracy")
                    break

    @torch.no_grad()
    def _score_model(self, master: torch.Tensor, r: int, ds=None, idx=None, key=None,
                     reduce: bool = False) -> float:
        """Accuracy of an fp32 model on ``idx`` rows of ``ds`` (default: round r's whole global
        draw of the test split), inline with a host read. ``reduce``: the rows are this rank's
        stride and the counts are all-reduced (collective mode)."""
        if not hasattr(self, "_score_param"):
            self._score_param = torch.empty(self.flat.numel, dtype=self.flat.dtype, device=self.device)
        ops.cast_copy_(self._score_param, master)
        keep = (self.flat.master, self.flat.param)
        self.flat.rebind(master, self._score_param)
        ds = self.test_ds if ds is None else ds
        if idx is None:
            idx, key = self.global_test_idx(r), ("score", self._draw_key(r))
        try:
            gb = self._cached_batches(key, lambda: ClientLoader(
                ds, idx, max(self.cfg.global_eval_batch, 1),
                pad_multiple=self.pad_multiple).device_batches(self.device)) if len(idx) else []
            a = (self.trainer.evaluate_device(gb) if gb else
                 torch.zeros(4, dtype=torch.float64, device=self.device))
            if reduce:
                a = a.double()
                D.all_reduce_(a)
            a = a.cpu().tolist()
        finally:
            self.flat.rebind(*keep)
        return a[0] / max(a[1], 1.0)

    @torch.no_grad()
    def _score_async(self, master: torch.Tensor, r: int):
        """Accuracy of an fp32 model on round r's whole global draw, queued on the evaluation side
        stream. The bf16 snapshot is taken on the TRAINING stream (one cast pass; ``master`` may be
        overwritten right after it), so the training stream never waits behind the round's
        global evaluation already queued on the side stream. Returns a function that waits for
        the result — called by the checkpoint writer thread, never by the training loop. Without
        a side stream (CPU) the model is scored inline."""
        if self.eval_stream is None:
            acc = self._score_model(master, r)
            return lambda: acc
        main = torch.cuda.current_stream(self.device)
        es = self.eval_stream
        idx = self.global_test_idx(r)
        gb = self._cached_batches(("score", self._draw_key(r)), lambda: ClientLoader(
            self.test_ds, idx, max(self.cfg.global_eval_batch, 1),
            pad_multiple=self.pad_multiple).device_batches(self.device))
        if not hasattr(self, "_score_snap"):
            self._score_snap = torch.empty(self.flat.numel, dtype=self.flat.dtype, device=self.device)
            self._score_done = None
        if self._score_done is not None:
            main.wait_event(self._score_done)      # the previous save round's scoring read it
        ops.cast_copy_(self._score_snap, master)
        es.wait_stream(main)                       # the snapshot and the batches are ready
        own = self.eval_flat.param
        with torch.cuda.stream(es):
            self.eval_flat.rebind(self.eval_flat.master, self._score_snap)
            stats = self.eval_trainer.evaluate_device(gb)
            done = torch.cuda.Event()
            done.record(es)
        self.eval_flat.rebind(self.eval_flat.master, own)
        self._score_done = done

        def result(stats=stats, done=done, gb=gb):
            done.synchronize()
            a = stats.cpu().tolist()
            return a[0] / max(a[1], 1.0)
        return result

    def _holdout_rows(self) -> np.ndarray:
        """The server's validation slice: ``server_holdout`` train-split rows that no client
        trains on (round 0's partition), drawn once with the run's seed; in collective mode each
        rank scores its stride of it."""
        if not hasattr(self, "_holdout_idx"):
            used = np.zeros(len(self.train_ds), dtype=bool)
            for sp in self.partitions(0):
                used[np.asarray(sp.train, dtype=np.int64)] = True
            free = np.flatnonzero(~used)
            rng = np.random.default_rng(self.cfg.seed + 7919)
            k = min(int(self.cfg.server_holdout), len(free))
            self._holdout_idx = np.sort(rng.choice(free, size=k, replace=False))
        idx = self._holdout_idx
        if self.rt.distributed and not self.collective_free:
            return idx[self.rt.rank::self.rt.world]
        return idx

    def _holdout_gate(self, r: int, new: torch.Tensor) -> dict:
        """Server hold-out selection (``server_holdout``): score the aggregated model on the
        validation slice and adopt it unless it falls more than ``server_holdout_tol`` below the
        best adopted score (``server_holdout_patience`` > 0: at most that many rejections in a
        row; 0: model selection — the served global model never drops more than the tolerance
        below its best). Every rank reaches the same decision (all-reduced counts, or identical
        local scores)."""
        cfg = self.cfg
        acc = self._score_model(new, r, ds=self.train_ds, idx=self._holdout_rows(),
                                key=("holdout",),
                                reduce=self.rt.distributed and not self.collective_free)
        best = getattr(self, "_holdout_best", -1.0)
        streak = getattr(self, "_holdout_streak", 0)
        pat = int(cfg.server_holdout_patience)
        gated = best >= float(cfg.server_holdout_min)
        adopt = (not gated or acc >= best - float(cfg.server_holdout_tol)
                 or (pat > 0 and streak >= pat))
        if adopt:
            # ungated (before the best reaches server_holdout_min) the best follows the adopted
            # models; gated it only rises
            self._holdout_best = max(best, acc) if gated else acc
            self._holdout_streak = 0
        else:
            self._holdout_streak = streak + 1
        return {"holdout_acc": acc, "holdout_adopted": bool(adopt), "holdout_best": max(best, acc if adopt else best)}
