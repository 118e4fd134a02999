"""Client lanes: concurrent client training on one GPU, one model replica and HIP stream per lane (split out of
:mod:`bcfl.fl.federation`; mixed into :class:`~bcfl.fl.federation.Federation`)."""
from __future__ import annotations

import contextlib
import json
import time
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional

import torch

from .. import ops
from ..models import build_model
from ..parallel.flat import FlatAdamW, FlatParams
from .trainer import LocalTrainer, MicroReplica


def _share_frozen(dst: torch.nn.Module, src: torch.nn.Module) -> None:
    """Point ``dst``'s frozen parameters (and buffers) at ``src``'s tensors: every lane of a
    LoRA federation reads ONE copy of the 16 GB Llama-3-8B base instead of one per lane."""
    for (_, md), (_, ms) in zip(dst.named_modules(), src.named_modules()):
        for name, p in list(ms._parameters.items()):
            if p is not None and not p.requires_grad:
                md._parameters[name] = p
        for name, b in list(ms._buffers.items()):
            if b is not None:
                md._buffers[name] = b
    if torch.cuda.is_available():
        torch.cuda.empty_cache()


@dataclass
class ClientLane:
    """One concurrent training lane: a model replica with its own flat buffers / optimizer and its
    own HIP stream. Lanes train different clients at the same time, so the small per-client GEMMs,
    attention and normalisation kernels of several clients share the 256 CUs instead of each
    leaving most of the chip idle in its tail (MI355X has 4 hardware queues per process)."""
    index: int
    model: torch.nn.Module
    flat: FlatParams
    opt: FlatAdamW
    trainer: LocalTrainer
    stream: Optional["torch.cuda.Stream"] = None
    clients: List[int] = field(default_factory=list)


class LanesMixin:
    def _build_lanes(self, vocab: int, mdtype: torch.dtype) -> List[ClientLane]:
        cfg = self.cfg
        if not (self.multi and not cfg.compat_chain):
            return []
        if cfg.deterministic:
            n = 1  # concurrent lanes reorder library reductions (timing-dependent, ~1e-7)
        elif cfg.micro_batches == 2:
            n = 1  # concurrency comes from the two micro-batch streams of the one lane
        elif cfg.client_lanes:
            n = cfg.client_lanes
        elif not self.is_cuda:
            n = 1
        else:
            # activation memory per lane grows with the model: an 8B-parameter client step holds
            # ~45 GB of saved activations at 11k tokens, so big models get 2 lanes (288 GB HBM;
            # config 5: 1 / 2 / 3 / 4 lanes 18.1 / 16.6 / 19.2 / 21.8 s/round). BERT-size models:
            # serverless 6 (8 clients: 6 lanes beat 8 in 4 / 4 interleaved reps, 0.548 vs 0.560
            # s/round; the box runs 4 hardware queues per process), server 8 (config 2, 4 steps per
            # client: 8 lanes beat 6, 0.338-0.345 vs 0.374-0.380; profiles/lanes_count_ab_r3.json)
            # serverless with more than 8 hosted clients: 10 lanes (two waves of 10 at 20 clients,
            # one at 10: 10 clients 0.400 vs 0.426 s/round with 6, 20 clients 0.734 vs 0.751,
            # server 0.399 / 0.748; profiles/worker_grid_r5_lanes.json)
            big = sum(p.numel() for p in self.model.parameters()) > 1_000_000_000
            hosted = len(self.local_clients)
            n = min(2 if big else (8 if cfg.mode == "server" else (6 if hosted <= 8 else 10)), hosted)
        n = max(1, min(n, len(self.local_clients)))
        lanes = []
        for i in range(n):
            if i == 0:
                model, flat, opt, tr = self.model, self.flat, self.opt, self.trainer
            else:
                model = build_model(cfg.model, self.num_labels, device=self.device, dtype=mdtype,
                                    dropout=cfg.dropout, vocab_size=vocab, seed=cfg.seed,
                                    lora_rank=cfg.lora_rank, lora_alpha=cfg.lora_alpha)
                _share_frozen(model, self.model)
                flat = FlatParams.from_model(model, self.device, mdtype)
                flat.load_master(self.flat.master)
                opt = FlatAdamW(flat, cfg.lr, cfg.adam_betas, cfg.adam_eps, cfg.weight_decay,
                                cfg.adam_mode, cfg.max_grad_norm)
                tr = LocalTrainer(model, flat, opt)
            stream = torch.cuda.Stream(device=self.device) if self.is_cuda else None
            lanes.append(ClientLane(i, model, flat, opt, tr, stream,
                                    list(self.local_clients[i::n])))
        return lanes

    def _build_micro(self, vocab: int, mdtype: torch.dtype):
        """Micro-batch replica for ranks that train one client at a time (e.g. 8 clients on 8
        GPUs), whose step's kernels otherwise run one after another on one stream (13.9 ms/step
        alone vs 9.3 ms/step per client with concurrent streams,
        profiles/graph_capture_probe.json). Off by default: for BERT-base the two half-batch
        passes double the host-side launch work (~7 -> ~17 ms/step) and the step becomes
        host-bound (1-client round 0.157 -> 0.178 s, profiles/micro_batches_1client.json); it
        pays when a step's device time dwarfs its launch cost."""
        cfg = self.cfg
        self.micro_split = 1
        n = cfg.micro_batches
        if n == 0:
            n = 1
        if n <= 1:
            return
        if n != 2:
            raise ValueError("micro_batches must be 0 (auto), 1 or 2")
        model = build_model(cfg.model, self.num_labels, device=self.device, dtype=mdtype,
                            dropout=cfg.dropout, vocab_size=vocab, seed=cfg.seed,
                            lora_rank=cfg.lora_rank, lora_alpha=cfg.lora_alpha)
        _share_frozen(model, self.model)
        flat = FlatParams.from_model(model, self.device, mdtype)
        flat.rebind(self.flat.master, self.flat.param)
        stream = torch.cuda.Stream(device=self.device) if self.is_cuda else None
        self.trainer.micro = MicroReplica(model, flat, stream)
        self.micro_split = 2

    def _on(self, lane: ClientLane):
        return torch.cuda.stream(lane.stream) if lane.stream is not None else contextlib.nullcontext()

    def _mark_start(self, c: int, master: torch.Tensor) -> None:
        self._phase[c] = "training"
        g = getattr(self, "gossip", None)
        if g is not None and hasattr(g, "mark_start"):
            g.mark_start(c, master)

    def _mid_round_targets(self, c: int) -> List[tuple]:
        """Buffers that follow a hosted client when a neighbour's snapshot is applied mid-round:
        (model space) the drift correction's round-start copy while the client trains, and (aux
        space) its correction d_c = c_hat - c_c, into which the neighbour's NEW control variate
        enters at once (the AdamW steps that follow already use it)."""
        out = []
        if self.drift.exchange:
            if self._phase.get(c) == "training" and self.drift.start_of is None:
                out.append((self.drift.cv[c], "model"))
            if self.drift.ready.get(c):
                out.append((self.drift.buf[c], "aux"))
        return out

    @contextlib.contextmanager
    def _client_rng(self, c: int):
        g = ops.rng.global_rng()
        g.load_state(self.client_rng[c])
        try:
            yield
        finally:
            self.client_rng[c] = g.state()

    def _lane_worker(self, lane: ClientLane, r: int, need_prev: bool, out: dict) -> Iterator[None]:
        """Generator: trains the lane's clients one after another, yielding after every optimizer
        step so the round driver can interleave the lanes' launches (streams run concurrently)."""
        cfg = self.cfg
        for c in lane.clients:
            with self._on(lane):
                lane.flat.rebind(self.client_master[c], self.client_param[c])
                if self.keep_opt and c in self.client_opt:
                    lane.opt.load_state_dict(self.client_opt[c])
                else:
                    lane.opt.reset()
                self.drift.attach(lane.opt, c, lane.flat.master, round_idx=r)
                self._mark_start(c, lane.flat.master)
                prev = lane.flat.master.detach().clone() if need_prev else None
                loss_acc = torch.zeros((), dtype=torch.float32, device=self.device)
            st = {"batches": 0, "tokens": 0, "examples": 0}
            for e in range(cfg.local_epochs):
                with self._on(lane):
                    batches = self.train_batches(c, r, e)
                for b in batches:
                    lane.opt.lr = self.lr_at(r, st["batches"])
                    with self._on(lane), self._client_rng(c):
                        lane.trainer.step(b, loss_acc)
                    st["batches"] += 1
                    st["tokens"] += b.real_tokens
                    st["examples"] += b.batch_size
                    if cfg.progress and st["batches"] % 10 == 0:
                        self.log(f"[round {r}] client {c}: step {st['batches']} issued "
                                 f"(T={b.num_tokens}, HBM {torch.cuda.memory_allocated() / 2**30:.1f} GiB)"
                                 if self.is_cuda else f"[round {r}] client {c}: step {st['batches']}")
                    yield
            st["loss_t"] = loss_acc
            self.tokens_trained += st["tokens"]
            if cfg.progress:
                self.log(f"[round {r}] client {c} (lane {lane.index}): {st['batches']} steps issued")
            if c in cfg.inject_slow:
                time.sleep(cfg.inject_slow[c] / 1000.0)
            with self._on(lane):
                if prev is not None:
                    self._clip_update(self._update_ref(c, prev), lane.flat)
                self.drift.after_train(c, lane.flat.master, self.lr_sum(r, st["batches"]))
                self._phase[c] = "trained"
                self.drift.detach(lane.opt)
                if prev is not None:
                    ref = self._update_ref(c, prev)
                    self._inject_byzantine(c, ref, lane.flat)
                    if self.filter is not None and not self._gossip_filter:
                        out["sk"][c], out["nr"][c] = self._update_stats(ref, lane.flat)
                out["losses"][c] = st
                if cfg.eval_local:
                    out["local_eval"][c] = lane.trainer.evaluate_device(self.test_batches(c, r))
                out["roots"][c] = (ops.merkle_root_deferred(lane.flat.master)
                                   if self.ledger is not None and not self._gossip_roots else None)
                if self.keep_opt:
                    self.client_opt[c] = {k: (v.clone() if torch.is_tensor(v) else v)
                                          for k, v in lane.opt.state_dict().items()}
            yield

    def _train_lanes(self, r: int, need_prev: bool) -> dict:
        """All hosted clients of this rank, trained concurrently on the client lanes."""
        out = {"sk": {}, "nr": {}, "losses": {}, "local_eval": {}, "roots": {}}
        main = torch.cuda.current_stream(self.device) if self.is_cuda else None
        for ln in self.lanes:
            if ln.stream is not None:
                ln.stream.wait_stream(main)  # last round's mixing / checkpoint reads are ordered
        with self.timer.phase("train"):
            gens = [self._lane_worker(ln, r, need_prev, out) for ln in self.lanes]
            while gens:
                for g in list(gens):
                    try:
                        next(g)
                    except StopIteration:
                        gens.remove(g)
                self._gossip_poll()
            # the join is part of the phase: its device end event then covers every lane
            for ln in self.lanes:
                if ln.stream is not None:
                    main.wait_stream(ln.stream)
        return out

    def _server_lane_worker(self, lane: ClientLane, r: int, G: torch.Tensor, w: Dict[int, float],
                            keep: bool, out: dict) -> Iterator[None]:
        """Server round on a lane: each of the lane's clients starts from the global model G,
        trains its local epoch(s) and adds w_c * x_c into the lane's partial FedAvg sum (or, when
        the anomaly filter needs every update, keeps a copy). Yields after every optimizer step."""
        cfg = self.cfg
        acc = out["acc"][lane.index]
        for c in lane.clients:
            with self._on(lane):
                lane.flat.load_master(G)
                if self.keep_opt and c in self.client_opt:
                    lane.opt.load_state_dict(self.client_opt[c])
                else:
                    lane.opt.reset()
                self.drift.attach(lane.opt, c, lane.flat.master)
                loss_acc = torch.zeros((), dtype=torch.float32, device=self.device)
            st = {"batches": 0, "tokens": 0, "examples": 0}
            for e in range(cfg.local_epochs):
                with self._on(lane):
                    batches = self.train_batches(c, r, e)
                for b in batches:
                    lane.opt.lr = self.lr_at(r, st["batches"])
                    with self._on(lane), self._client_rng(c):
                        lane.trainer.step(b, loss_acc)
                    st["batches"] += 1
                    st["tokens"] += b.real_tokens
                    st["examples"] += b.batch_size
                    yield
            st["loss_t"] = loss_acc
            self.tokens_trained += st["tokens"]
            if c in cfg.inject_slow:
                time.sleep(cfg.inject_slow[c] / 1000.0)
            with self._on(lane):
                self._clip_update(G, lane.flat)
                self.drift.after_train(c, lane.flat.master, self.lr_sum(r, st["batches"]))
                self.drift.detach(lane.opt)
                self._inject_byzantine(c, G, lane.flat)
                if self.filter is not None:
                    out["sk"][c], out["nr"][c] = self._update_stats(G, lane.flat)
                out["losses"][c] = st
                out["roots"][c] = (ops.merkle_root_deferred(lane.flat.master)
                                   if self.ledger is not None else None)
                if keep:
                    out["trained"][c] = lane.flat.master.detach().clone()
                else:
                    ops.weighted_accumulate_(acc, lane.flat.master, float(w[c]))
                if self.keep_opt:
                    self.client_opt[c] = {k: (v.clone() if torch.is_tensor(v) else v)
                                          for k, v in lane.opt.state_dict().items()}
            yield

    def _server_train_lanes(self, r: int, G: torch.Tensor, w: Dict[int, float], keep: bool) -> dict:
        """All hosted clients of a server round, trained concurrently on the client lanes. The
        FedAvg sum is accumulated per lane (fp32) and the lane partials are added in lane order
        (deterministic for a given lane count)."""
        if not hasattr(self, "_lane_acc") or len(self._lane_acc) != len(self.lanes):
            self._lane_acc = [torch.zeros_like(self.flat.master) for _ in self.lanes]
        out = {"sk": {}, "nr": {}, "losses": {}, "roots": {}, "trained": {}, "acc": self._lane_acc}
        main = torch.cuda.current_stream(self.device) if self.is_cuda else None
        for a in self._lane_acc:
            a.zero_()
        for ln in self.lanes:
            if ln.stream is not None:
                ln.stream.wait_stream(main)
        with self.timer.phase("train"):
            gens = [self._server_lane_worker(ln, r, G, w, keep, out) for ln in self.lanes]
            while gens:
                for g in list(gens):
                    try:
                        next(g)
                    except StopIteration:
                        gens.remove(g)
            for ln in self.lanes:
                if ln.stream is not None:
                    main.wait_stream(ln.stream)
        if not keep:
            for a in self._lane_acc:
                ops.weighted_accumulate_(self.acc, a, 1.0)
        return out

    def _server_eval_local(self, r: int, G: torch.Tensor) -> Dict[int, torch.Tensor]:
        """Flower's evaluate_round: every hosted client scores the new global model G on its own
        test split. With client lanes the clients' evaluations run concurrently, each lane's
        replica holding G (lane 0's flat buffer already does); otherwise one after another.
        Device tensors [correct, count, loss_sum, batch_mean_sum] per client, no host sync."""
        if len(self.lanes) <= 1:
            return {c: self.trainer.evaluate_device(self.test_batches(c, r))
                    for c in self.local_clients}
        main = torch.cuda.current_stream(self.device) if self.is_cuda else None
        res: Dict[int, torch.Tensor] = {}
        for ln in self.lanes:
            if ln.stream is not None:
                ln.stream.wait_stream(main)  # G is final on the main stream
            with self._on(ln):
                if ln.flat is not self.flat:
                    ln.flat.load_master(G)   # the next round's lane worker reloads G anyway
                for c in ln.clients:
                    res[c] = ln.trainer.evaluate_device(self.test_batches(c, r))
        for ln in self.lanes:
            if ln.stream is not None:
                main.wait_stream(ln.stream)
        return res
