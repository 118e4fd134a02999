"""The federation runner: server FedAvg and serverless (async) P2P gossip on one client per GPU.

Reference call stacks:

* server (§3.1): Flower ``start_simulation`` with ``FedAvg(fraction_fit=1, fraction_evaluate=1,
  evaluate_metrics_aggregation_fn=weighted_average)`` (``src/Servercase/server_IID_IMDB.py:199-218``)
  -> here :meth:`Federation.server_round`: every rank trains its client(s) from the global model,
  the weighted sum Σ n_k w_k / Σ n is ONE RCCL all-reduce of the fp32 flat buffer, client-side
  evaluation of the new global model is aggregated with ``weighted_average``.
* serverless (§3.2): the sequential chain + host mean of ``serverless_*.py:284-318``
  -> :meth:`Federation.serverless_round`: clients train concurrently (one per GPU), exchange over
  RCCL send/recv (:class:`bcfl.parallel.gossip.GossipEngine`), async by default, and mix.
  ``compat_chain=True`` reproduces the reference chain exactly (single process).

Around both: partitioning (IID / reference contiguous / label shards / Dirichlet), update anomaly
filtering, the hash-chained ledger, async HF-layout checkpoints, metrics JSONL and the reference's
console lines.

Module layout (round 6: one concern per module, all behind this :class:`Federation`):

* this file — construction (data, model, lanes, gossip engine, trust layer, IO), data / learning-
  rate helpers, the batch prefetcher and the round driver (``run_round`` / ``run`` / ``finish``);
* :mod:`.lanes` — concurrent client lanes (one replica + HIP stream each), serverless and server;
* :mod:`.server` — the FedAvg round; :mod:`.serverless` — the gossip round, the asynchronous
  protocol's waits and polls, deferred host reads, the reference chain;
* :mod:`.evaluation` — local / global / overlapped evaluation and the server hold-out gate;
* :mod:`.ledgering` — update statistics, collective anomaly filter, fault injection, ledger;
* :mod:`.checkpointing` — the federation's global model, async checkpoints and resume.
"""
from __future__ import annotations

import json
import math
import os
import time
import warnings
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..ckpt import AsyncCheckpointer, dir_size_gb, mirror_dir
from ..config import FLConfig
from ..data.batching import ClientLoader
from ..data.partition import partition_clients
from ..data.registry import get_dataset, load_split
from ..models import build_model, model_config, special_tokens
from ..parallel import dist as D
from ..parallel.flat import FlatAdamW, FlatParams
from ..parallel.gossip import GossipEngine, MailboxGossip
from ..parallel.mailbox import MailboxUnavailable
from ..parallel.topology import clients_of_rank, mixing_matrix, neighbours
from ..trust.anomaly import UpdateAnomalyFilter, Verdicts
from ..trust.ledger import Ledger
from ..utils import streamcheck
from ..utils.obs import MetricsWriter, PhaseTimer, Telemetry
from .drift import DriftCorrection, resolve_mode as resolve_drift
from .outer import OuterOptimizer
from .trainer import EvalResult, LocalTrainer
from .checkpointing import CheckpointMixin
from .evaluation import EvalMixin
from .fedutil import DATA_SEED, _cseed, weighted_average  # noqa: F401  (re-exported)
from .lanes import ClientLane, LanesMixin, _share_frozen  # noqa: F401
from .ledgering import TrustMixin
from .server import ServerRoundMixin
from .serverless import ServerlessRoundMixin


class Federation(LanesMixin, EvalMixin, TrustMixin, ServerRoundMixin,
                 ServerlessRoundMixin, CheckpointMixin):
    def __init__(self, cfg: FLConfig, verbose: bool = True):
        self.cfg = cfg
        self.rt = D.init_runtime(cfg.device, cfg.backend)
        self.device = self.rt.device
        self.is_cuda = self.device.type == "cuda"
        self.verbose = verbose and self.rt.is_main
        self.dtype = torch.bfloat16 if (self.is_cuda and cfg.dtype == "bf16") else torch.float32
        if self.is_cuda and cfg.dtype == "fp32" and not cfg.model.startswith("llama"):
            raise ValueError("dtype='fp32' on the GPU: the bcfl MFMA kernels (attention, wgrad, "
                             "fused LayerNorm) compute in bf16 with fp32 accumulation and fp32 "
                             "master weights; use dtype='bf16' (fp32 runs on device='cpu')")
        if cfg.deterministic:
            torch.use_deterministic_algorithms(True, warn_only=True)
        self.stream_races: Optional[List[str]] = None
        if self.is_cuda and streamcheck.requested():
            streamcheck.enable()   # BCFL_DEBUG_STREAMS=1: happens-before checks on every stream
        self.telemetry = Telemetry()
        # ---------------- data --------------------------------------------------------------
        self.spec = get_dataset(cfg.dataset)
        cls_id, sep_id, vocab = special_tokens(cfg.model)
        vocab = cfg.vocab_size or vocab
        _, mcfg = model_config(cfg.model)
        self.max_len = min(cfg.max_seq_len, getattr(mcfg, "max_position_embeddings", cfg.max_seq_len))
        self.train_ds = load_split(cfg.dataset, "train", vocab, self.max_len, DATA_SEED, cls_id,
                                   sep_id, cfg.synthetic_signal)
        self.test_ds = load_split(cfg.dataset, "test", vocab, self.max_len, DATA_SEED, cls_id,
                                  sep_id, cfg.synthetic_signal)
        self.num_labels = cfg.num_labels or self.spec.num_classes
        self._parts: Dict[int, list] = {}
        # ---------------- model + flat buffers ------------------------------------------------
        mdtype = self.dtype if not cfg.model.startswith("llama") else (
            torch.bfloat16 if self.is_cuda else torch.float32)
        self.model = build_model(cfg.model, self.num_labels, device=self.device, dtype=mdtype,
                                 dropout=cfg.dropout, vocab_size=vocab, seed=cfg.seed,
                                 lora_rank=cfg.lora_rank, lora_alpha=cfg.lora_alpha)
        self.flat = FlatParams.from_model(self.model, self.device, mdtype)
        if self.rt.distributed:
            D.broadcast_(self.flat.master, 0)
            self.flat.sync_param_from_master()
        self.opt = FlatAdamW(self.flat, cfg.lr, cfg.adam_betas, cfg.adam_eps, cfg.weight_decay,
                             cfg.adam_mode, cfg.max_grad_norm)
        self.trainer = LocalTrainer(self.model, self.flat, self.opt)
        # ---------------- clients ---------------------------------------------------------------
        n = cfg.num_clients
        self.local_clients = clients_of_rank(self.rt.rank, self.rt.world, n)
        self.multi = len(self.local_clients) > 1
        if cfg.compat_chain and self.rt.world > 1:
            raise ValueError("compat_chain reproduces the reference's single-process chain; world must be 1")
        self.client_rng = {c: {"seed": _cseed(cfg.seed, c), "counter": 0} for c in self.local_clients}
        self._phase: Dict[int, str] = {}   # hosted client -> "training" / "trained" this round
        self.client_opt: Dict[int, dict] = {}
        self.client_master: Dict[int, torch.Tensor] = {}
        if cfg.mode == "serverless" and self.multi and not cfg.compat_chain:
            for c in self.local_clients:
                self.client_master[c] = self.flat.master.detach().clone()
        self.lanes = self._build_lanes(vocab, mdtype)
        self._build_micro(vocab, mdtype)
        # lanes train every hosted client IN PLACE on its own resident buffers (FlatParams.rebind):
        # no per-client master copies in / out of a lane replica
        self.client_param: Dict[int, torch.Tensor] = {}
        if self.lanes and cfg.mode == "serverless":
            for c in self.local_clients:
                self.client_param[c] = torch.empty(self.flat.numel, dtype=self.flat.dtype,
                                                   device=self.device)
                ops.cast_copy_(self.client_param[c], self.client_master[c])
        self.drift = DriftCorrection(resolve_drift(cfg.drift_correction, cfg.partition),
                                     cfg.drift_correction_scale,
                                     self.local_clients, self.flat.numel, self.device)
        # round-level outer optimizer (FedAvgM / outer Nesterov; default lr 1, momentum 0 = the
        # reference's plain average): server mode keys the global model as -1
        self.outer = OuterOptimizer(cfg.outer_lr, cfg.outer_momentum, cfg.outer_nesterov,
                                    [-1] if cfg.mode == "server" else self.local_clients,
                                    self.flat.numel, self.device)
        # auto: on when one client trains at a time — except on a CU-masked device (multi-rank
        # rehearsals on slices of one GPU): the side-stream weight gradients, sized for 256 CUs,
        # then crowd the slice's 32 CUs (8-rank rehearsal: 3.6-4.1 s/round with, 2.2 s without)
        ov = cfg.overlap_wgrad if cfg.overlap_wgrad is not None else (
            len(self.lanes) <= 1 and not os.environ.get("HSA_CU_MASK"))
        if cfg.deterministic:
            ov = False  # the overlapped path's gradients are not bitwise reproducible
        ops.set_wgrad_overlap(bool(ov and self.is_cuda))
        # off by default: measured slower on the one-client round (0.0946 vs 0.0928 s/round,
        # profiles/bench_r4_1client_*.json) — the side-stream AdamW competes with the backward
        # GEMMs for HBM and the hooks add host work on the autograd thread
        oo = bool(cfg.overlap_optimizer) and cfg.max_grad_norm <= 0 and not cfg.deterministic
        if oo and self.is_cuda and len(self.lanes) <= 1 and self.micro_split == 1:
            self.opt.enable_overlap()
        if self.is_cuda and ops.native_available():
            # persistent GEMM grids (one workgroup per CU walking the tiles) pay with concurrent
            # client lanes (8-lane round 0.5635 -> 0.5604 s, profiles/g8_persistent_r3.json) and
            # cost a rank that trains one client with side-stream weight gradients, whose 64-slot
            # weight-gradient grid they crowd out (0.0975 vs 0.1021 s/round, 3 interleaved reps,
            # profiles/g8_persistent_1client_r3.json); BCFL_G8_PERSIST=0/1 overrides
            ops.native().set_g8_persistent(not bool(ov))
            # concurrent client lanes share the chip: 256-row GEMM tiles (best per FLOP) instead of
            # the lone-launch wave fit (8-lane bench -2.5 %, profiles/bench_r5_gemm_ab.json)
            big = self.flat.numel > 1_000_000_000
            ops.native().set_g8_block_rows(256 if len(self.lanes) > 1 and not big else 0)
            # one lane: the side-stream weight gradient may take 96 tile slots (64 with lanes)
            ops.native().set_wgrad_slots(cfg.wgrad_slots or (96 if len(self.lanes) <= 1 else 64))
        self.global_master: Optional[torch.Tensor] = None
        if cfg.mode == "server":
            self.global_master = self.flat.master.detach().clone()
            self.acc = torch.zeros_like(self.flat.master)
        # ---------------- gossip -------------------------------------------------------------------
        if cfg.gossip_transport not in ("auto", "mailbox", "rccl", "loopback"):
            raise ValueError(f"unknown gossip_transport {cfg.gossip_transport!r}")
        if cfg.global_eval_models == "average" and cfg.mode == "serverless" and self.rt.distributed:
            # the reference's averaged global_model needs every client model; a rank only holds
            # its own (averaging its partial set and all-reducing the scores would report the
            # mean accuracy of partial averages, not the federation average's — ADVICE r4)
            raise ValueError("global_eval_models='average' scores the mean of ALL client models "
                             "and needs world 1; with several ranks use 'all' (every client model "
                             "on its stride of the draw) or 'client0'")
        if cfg.gossip_transport == "loopback" and (self.rt.distributed or not cfg.async_gossip):
            raise ValueError("gossip_transport='loopback' runs the asynchronous multi-rank protocol "
                             "inside ONE process (world 1, async_gossip=True)")
        # drift correction across ranks: async mailbox gossip exchanges the clients' control
        # variates with their models (stale-exact SCAFFOLD, fl/drift.py) and never waits;
        # FLConfig.drift_same_round_mix instead waits for every neighbour's round-r snapshot
        self.same_round_mix = bool(cfg.mode == "serverless" and cfg.async_gossip
                                   and cfg.drift_same_round_mix and self.drift.enabled
                                   and self.rt.distributed)
        self.transport = cfg.gossip_transport
        if self.transport == "auto":
            # deterministic: the lock-step engine mixes exactly the previous round's states
            self.transport = "mailbox" if (cfg.async_gossip and not cfg.deterministic) else "rccl"
        loopback = self.transport == "loopback"
        # several ranks, or one process whose hosted clients are virtual ranks: the mixes are
        # stale, so the asynchronous protocol's exchanges apply
        multi_rank = self.rt.distributed or loopback
        cv_exchange = (cfg.mode == "serverless" and not cfg.compat_chain and self.drift.enabled
                       and self.transport in ("mailbox", "loopback")
                       and (cfg.drift_exchange == "on" or (
                           cfg.drift_exchange == "auto" and multi_rank
                           and cfg.async_gossip and not self.same_round_mix)))
        # A mailbox federation never waits on a peer: the per-round path is collective-free
        # (metrics, evaluation and ledger are rank-local) so a slow or exited rank cannot stall
        # the others. The update anomaly filter needs a global view and keeps its collectives.
        self.collective_free = (cfg.mode == "serverless" and self.transport in ("mailbox", "loopback")
                                and cfg.anomaly_filter == "none" and not cfg.compat_chain)
        # server FedAvg over mailboxes (liveness: a dead rank is left out, weights re-normalised)
        self.server_mbox = None
        if cfg.mode == "server" and cfg.server_transport in ("mailbox", "mailbox_rs"):
            self.collective_free = True
            if self.rt.distributed:
                from ..parallel.fedavg import MailboxFedAvg, MailboxReduceScatterFedAvg
                cls = MailboxReduceScatterFedAvg if cfg.server_transport == "mailbox_rs" else MailboxFedAvg
                self.server_mbox = cls(self.flat.numel, self.device, cfg.server_timeout_s,
                                       cfg.verify_updates)
        self.excluded: List[int] = []
        self.skipped_epochs = 0            # mailbox FedAvg: aggregation epochs this rank missed
        self.final_check: Optional[dict] = None
        self._lead_gone: Dict[int, int] = {}   # bounded staleness: neighbours given up on
        self._round_now: Optional[int] = None  # serverless round being trained (drift tagging)
        self.gossip: Optional[GossipEngine] = None
        self.filter = UpdateAnomalyFilter(cfg.anomaly_filter, cfg.anomaly_k,
                                          cfg.anomaly_modz_threshold) if cfg.anomaly_filter != "none" else None
        self._gossip_filter = False   # the filter runs inside the round-complete gossip (async)
        if cfg.mode == "serverless" and not cfg.compat_chain:
            if cfg.topology_probe and self.rt.distributed:
                from ..trust.probe import probe_and_filter
                self.excluded = probe_and_filter(self.flat.param, n)
            self.nbrs = neighbours(cfg.topology, n, self.excluded)
            states = ({c: self.client_master[c] for c in self.local_clients} if self.multi
                      else {self.local_clients[0]: self.flat.master})
            if self.transport in ("mailbox", "loopback"):
                aux = self.drift.use_exchange() if cv_exchange else None
                exch = cfg.gossip_exchange
                if exch == "auto":
                    # delta exchange where snapshots can be stale: several ranks, async, and a
                    # complete neighbour graph (applying every update once needs everyone's)
                    exch = ("delta" if (multi_rank and cfg.async_gossip
                                        and not self.same_round_mix
                                        and cfg.topology in ("full", "pagerank")) else "state")
                if exch == "delta" and cfg.topology == "ring":
                    raise ValueError("gossip_exchange='delta' applies each client's updates once "
                                     "and needs a complete topology (full / pagerank), not ring")
                try:
                    self.gossip = MailboxGossip(n, states, self.nbrs,
                                                "fp32" if cfg.wire_dtype == "fp32" else "bf16",
                                                sync=not cfg.async_gossip or self.same_round_mix,
                                                # same-round mix: a peer whose round-r post has not
                                                # landed within 10 s is declared dead for the mix
                                                # (its later posts bring it back), not waited on
                                                sync_timeout_s=10.0 if self.same_round_mix else 60.0,
                                                liveness_timeout=cfg.liveness_timeout,
                                                # in-process posts cross no link: nothing to verify
                                                verify=cfg.verify_updates and not loopback, aux=aux,
                                                aux_sink=self.drift if aux else None,
                                                exchange=exch,
                                                apply=cfg.gossip_apply if exch == "delta" else "arrival",
                                                virtual=loopback,
                                                lag_steps=tuple(cfg.loopback_lag_steps),
                                                source_lag=cfg.loopback_source_lag,
                                                seed=cfg.seed)
                    self.drift.stale_compensation = cfg.drift_stale_compensation
                    self.gossip.stale_decay = float(cfg.gossip_stale_decay)
                    self.gossip.apply_scale = float(cfg.gossip_apply_scale)
                    # the run's last round waits (bounded) for every live peer's last post
                    self.gossip.final_round = cfg.num_rounds - 1
                    self.gossip.final_timeout_s = float(cfg.gossip_lead_timeout_s)
                    if cfg.gossip_self_delay == "on" and self.gossip.exchange == "delta":
                        self.gossip.enable_self_delay()
                except MailboxUnavailable as e:
                    # every rank sees the same outcome (agreed collectively in the transport):
                    # fall back together to the lock-step RCCL engine
                    warnings.warn(f"hipIpc mailboxes unavailable ({e}); gossip falls back to "
                                  "RCCL send/recv (lock-step)", RuntimeWarning)
                    self.transport = "rccl"
                    self.collective_free = False
                    self.drift.drop_exchange()
            if self.transport not in ("mailbox", "loopback"):
                wire = cfg.wire_dtype if cfg.wire_dtype != "bf16" else "bf16_delta"
                if cfg.wire_dtype == "bf16_raw":
                    wire = "bf16"
                # the lock-step engine mixes stale-by-one states when async; drift correction
                # across ranks needs exactly mixed rounds there (the mix-derived c' = (x - x')/L)
                rccl_async = cfg.async_gossip and not (self.drift.enabled and self.rt.distributed)
                self.same_round_mix = bool(cfg.async_gossip and not rccl_async)
                self.gossip = GossipEngine(n, states, self.nbrs, wire, rccl_async,
                                           liveness_timeout=cfg.liveness_timeout,
                                           verify=cfg.verify_updates)
            if isinstance(self.gossip, MailboxGossip):
                if self.gossip.exchange == "delta" and self.drift.exchange:
                    # the gossip's round-start records double as the drift correction's x_c
                    self.drift.start_of = self.gossip.start
                # apply on arrival: neighbours' updates enter between local steps (delta exchange).
                # Not with the update anomaly filter or Byzantine injection: a mid-round
                # application would fold a neighbour's update into the model before this round's
                # verdict on it exists (the round-end mix applies verdicted weights only)
                self.gossip.W_mid = mixing_matrix(self.nbrs, cfg.mixing)
                if (self.filter is not None and self.gossip.exchange == "delta"
                        and self.gossip.apply_mode == "complete"):
                    # asynchronous trust: every complete round is judged by each receiver before
                    # it is applied (no collective, no previous-round verdicts)
                    self.gossip.enable_filter(self.filter, cfg.sketch_dim, cfg.filter_redistribute)
                    self._gossip_filter = True
                    self.collective_free = True
                if (self.gossip.apply_mode == "complete" and self.drift.exchange
                        and cfg.drift_correction_lag > 0):
                    self.drift.corr_lag = int(cfg.drift_correction_lag)
                if self.gossip.apply_mode == "complete" and self.drift.exchange:
                    self.drift.defer_cv = True   # formed in the gossip's fused round-end pass
                # (with the filter inside the round-complete application, verdicts exist before
                # any application, so mid-round application stays on)
                self.gossip.apply_on_arrival &= bool(cfg.gossip_apply_on_arrival and (
                    self._gossip_filter or (cfg.anomaly_filter == "none"
                                            and not cfg.inject_byzantine)))
                self.gossip._also = self._mid_round_targets
            self.gossip.suppressed = set(cfg.inject_drop) & set(self.local_clients)
            self.gossip.tamper = set(cfg.inject_tamper) & set(self.local_clients)
            self.gossip.seed_replicas(self.flat.master)
        # the clients' AdamW moments persist across rounds when asked for (keep_optimizer_state,
        # or async_keep_optimizer_state under asynchronous delta exchange: CPU tiny-bert, 8 ranks,
        # lr 5e-4 learns only with kept moments, 0.50 -> 0.995; MI355X BERT-base at the bench
        # config the other way round, so it is off by default)
        self.keep_opt = bool(cfg.keep_optimizer_state or (
            cfg.async_keep_optimizer_state and isinstance(self.gossip, MailboxGossip)
            and self.gossip.exchange == "delta"))
        self._single_opt = not self.multi   # one client, one optimizer: keep it in place
        self._opt_owner: Optional[int] = None
        # ---------------- trust ---------------------------------------------------------------------
        self.prev_verdicts = Verdicts()
        out = cfg.out_dir
        self.ledger = Ledger(genesis={"model": cfg.model, "mode": cfg.mode, "clients": n,
                                      "dataset": cfg.dataset, "partition": cfg.partition},
                             path=self._ledger_path() if cfg.ledger else None,
                             truncate=not cfg.resume,
                             ts=0.0) if cfg.ledger else None
        # ---------------- io ---------------------------------------------------------------------------
        self.metrics = MetricsWriter(os.path.join(out, "metrics.jsonl"),
                                     cfg.metrics_jsonl and self.rt.is_main, append=bool(cfg.resume))
        self.ckpt = AsyncCheckpointer(self.model, self.flat, cfg.async_ckpt) if (
            cfg.save_every > 0 and (self.rt.is_main or cfg.save_clients)) else None
        self.timer = PhaseTimer(sync_device=cfg.profile)
        self.timer.on_resolve = lambda rec: self.metrics.write(
            {"round": rec.get("round"), "device_phases": True,
             **{k: v for k, v in rec.items() if k.startswith("dev_t_")}})
        self._build_eval_overlap(vocab, mdtype)
        self.global_accuracies: List[float] = []
        # the round of every entry of global_accuracies (eval_global_every > 1 scores only some)
        self.global_accuracy_rounds: List[int] = []
        self.history: List[dict] = []
        self.start_round = 0
        self.ledger_audit: Optional[Dict[str, int]] = None
        self.tokens_trained = 0
        self.provenance_rows = 0
        if cfg.resume:
            self._resume(cfg.resume)


    # ================================ helpers ==================================================
    def log(self, *a):
        if self.verbose:
            print(*a, flush=True)

    def partitions(self, r: int):
        key = r if self.cfg.resample_each_round else 0
        parts = self._parts.get(key)
        if parts is None:
            c = self.cfg
            parts = partition_clients(c.partition, self.spec, self.train_ds.labels,
                                      self.test_ds.labels, c.num_clients, c.train_samples,
                                      c.test_samples, c.seed, key, c.dirichlet_alpha)
            # keep the newest two draws: the batch prefetcher packs round r + 1 while round r
            # still reads its own (a new dict, so a concurrent reader never sees a half update)
            keep = {k: v for k, v in self._parts.items() if k == key - 1}
            keep[key] = parts
            self._parts = keep
        return parts

    @property
    def steps_per_round(self) -> int:
        c = self.cfg
        return c.local_epochs * -(-min(c.train_samples, len(self.train_ds)) // c.batch_size)

    def lr_at(self, r: int, i: int) -> float:
        """Learning rate of local step ``i`` of round ``r``. Every client follows the same
        schedule over the run's global local-step index g = r * steps_per_round + i (linear
        warm-up, then constant / linear / cosine decay to ``lr_min_ratio * lr``)."""
        c = self.cfg
        if c.lr_schedule == "constant" and c.lr_warmup_steps <= 0:
            return c.lr
        g = r * self.steps_per_round + i
        if g < c.lr_warmup_steps:
            return c.lr * (g + 1) / c.lr_warmup_steps
        if c.lr_schedule == "constant":
            return c.lr
        total = max(c.num_rounds * self.steps_per_round - c.lr_warmup_steps, 1)
        t = min(max((g - c.lr_warmup_steps) / total, 0.0), 1.0)
        lo = c.lr * c.lr_min_ratio
        if c.lr_schedule == "linear":
            return lo + (c.lr - lo) * (1.0 - t)
        if c.lr_schedule == "cosine":
            return lo + (c.lr - lo) * 0.5 * (1.0 + math.cos(math.pi * t))
        raise KeyError(f"unknown lr_schedule {c.lr_schedule!r}")

    def lr_sum(self, r: int, steps: int) -> float:
        """Sum of the learning rates of round r's first ``steps`` local steps (drift correction)."""
        return float(sum(self.lr_at(r, i) for i in range(steps)))

    def client_examples(self, c: int, r: int) -> int:
        return int(len(self.partitions(r)[c].train))

    def fedavg_weight_counts(self, r: int) -> np.ndarray:
        n = self.cfg.num_clients
        if self.cfg.fedavg_weighting == "uniform":
            return np.ones(n)
        ex = np.array([self.client_examples(c, r) for c in range(n)], dtype=np.float64)
        if self.cfg.fedavg_weighting == "batches":  # Flower quirk: len(trainloader) (C10)
            return np.ceil(ex / self.cfg.batch_size)
        return ex

    @property
    def pad_multiple(self) -> int:
        # GPU: bucket T to a multiple of 256 (stable GEMM shapes); CPU: exact shapes
        return 256 if self.is_cuda else 0

    def _train_loader(self, c: int, r: int) -> ClientLoader:
        sp = self.partitions(r)[c]
        return ClientLoader(self.train_ds, sp.train, self.cfg.batch_size, shuffle=True,
                            seed=_cseed(self.cfg.seed, c), pad_multiple=self.pad_multiple,
                            split=self.micro_split, presort=self.is_cuda)

    def _stage_train(self, c: int, r: int, epoch: int):
        ld = self._train_loader(c, r)
        return ld, ld.stage(r * self.cfg.local_epochs + epoch, pin=self.is_cuda)

    def train_batches(self, c: int, r: int, epoch: int):
        fut = getattr(self, "_prefetched", {}).pop((c, r, epoch), None)
        ld, staged = fut.result() if fut is not None else self._stage_train(c, r, epoch)
        return ld.upload(staged, self.device)

    def _prefetch_train(self, r: int) -> None:
        """Pack round r's training batches for every hosted client on a host thread (GPU runs).
        Called at the start of round r - 1: the packing (numpy + one pinned buffer per client and
        epoch) overlaps that round's training instead of delaying round r's first launches — with
        one client per GPU the device otherwise idles for the packing at every round start. The
        batches are a pure function of (client, round, epoch), so prefetched and inline batches are
        identical."""
        cfg = self.cfg
        # auto: on with up to 4 lanes, and whenever every round draws fresh rows (the reference's
        # IID serverless scripts): then the round's training, local-test and global batches are
        # all new, and packing them inline idled the GPU at every round start
        on = cfg.prefetch_batches if cfg.prefetch_batches is not None else (
            len(self.lanes) <= 4 or cfg.resample_each_round)
        if not (self.is_cuda and on) or r >= cfg.num_rounds:
            return
        if not hasattr(self, "_prefetched"):
            import concurrent.futures as cf
            self._prefetched: Dict[tuple, object] = {}
            self._prefetch_pool = cf.ThreadPoolExecutor(1, thread_name_prefix="bcfl-prefetch")
        for k in [k for k in self._prefetched if isinstance(k[1], int) and k[0] in ("test", "global")
                  and (k[2] if k[0] == "test" else k[1]) < r - 1]:
            self._prefetched.pop(k)   # evaluation draws of rounds that are over
        for k in [k for k in self._prefetched if isinstance(k[0], int) and k[1] < r - 1]:
            self._prefetched.pop(k)   # rounds that never trained these clients (resume, sampling)
        for c in self.local_clients:
            for e in range(cfg.local_epochs):
                if (c, r, e) not in self._prefetched:
                    self._prefetched[(c, r, e)] = self._prefetch_pool.submit(self._stage_train, c, r, e)
        if cfg.resample_each_round:
            self._prefetch_eval(r)

    def _prefetch_eval(self, r: int) -> None:
        """Round r's evaluation draws (a fresh sample every round): the local test batches of the
        hosted clients and this rank's global-draw batches, packed on the prefetch thread."""
        cfg, dk = self.cfg, self._draw_key(r)
        jobs = []
        if cfg.eval_local:
            jobs += [(("test", c, dk), (lambda c=c: self._test_loader(c, r))) for c in self.local_clients]
        if self._global_eval_due(r):
            if self._sharded_eval():
                if len(self.local_clients) > 1 and self._hosted_models_identical():
                    jobs.append((("global", dk, "hosted"), lambda: self._hosted_loader(r)))
                else:
                    jobs += [(("global", dk, c), (lambda c=c: self._global_loader(r, c)))
                             for c in self.local_clients]
            elif not self._average_eval():
                jobs.append((("global", dk, None), lambda: self._global_loader(r, None)))
        for key, mk in jobs:
            if key not in self._prefetched and key not in getattr(self, "_batch_cache", {}):
                self._prefetched[key] = self._prefetch_pool.submit(
                    lambda mk=mk: (lambda ld: (ld, ld.stage(pin=True)))(mk()))


    def run_round(self, r: int) -> dict:
        self._log_provenance(r)
        self.timer.begin_round()
        t0 = time.perf_counter()
        self._prefetch_train(r + 1)   # packed on the host thread while round r trains
        res = self.server_round(r) if self.cfg.mode == "server" else self.serverless_round(r)
        ge: Optional[EvalResult] = res.get("global")
        gacc = ge.accuracy if ge is not None else None
        if gacc is not None:
            self.global_accuracies.append(gacc)
            self.global_accuracy_rounds.append(int(r))
        self._maybe_save(r)
        t_round = time.perf_counter() - t0
        if gacc is not None and self.verbose and self.cfg.reference_prints:
            print(f"Global Model Accuracy: {gacc * 100:.2f}%", flush=True)
        rec = {"round": r, "mode": self.cfg.mode, "t_round": t_round, "global_acc": gacc,
               "global_majority_rate": self.global_majority_rate(r) if gacc is not None else None,
               "global_eval_rows": int(ge.count) if ge is not None else 0,
               "global_loss": ge.loss if ge is not None else None,
               "distributed_acc": res.get("distributed_accuracy"), "train_loss": res.get("train_loss"),
               "rejected": res.get("rejected"), "bytes_sent": res.get("bytes_sent"),
               "dead_peers": res.get("dead_peers", []),
               **{k: res[k] for k in ("mixed", "stale_rounds", "stale_max", "wait_s", "lead_wait_s", "torn",
                                      "rejected_msgs", "absent_ranks", "live_weight",
                                      "view_mismatch", "rejoined_ranks", "epochs_skipped",
                                      "final_wait_s", "verdict_rounds", "holdout_acc",
                                      "holdout_adopted", "holdout_best",
                                      "applied_round", "post_lag_rounds") if k in res},
               "ledger_height": len(self.ledger) if self.ledger else 0,
               "tokens_trained": self.tokens_trained, **self.timer.snapshot()}
        if self.is_cuda:
            rec["hbm_peak_gb"] = torch.cuda.max_memory_allocated(self.device) / 1024 ** 3
        for c, n_, m in res.get("client_metrics", []):
            self.metrics.write({"round": r, "client": c, "local_acc": m.get("accuracy"),
                                "local_loss": m.get("loss"), "examples": n_})
        self.history.append(rec)
        self.timer.end_round(rec)  # device phase times land in rec once their events complete
        self.metrics.write({k: v for k, v in rec.items() if not k.startswith("dev_t_")})
        if self.cfg.progress:
            self.log(f"[round {r}] {t_round:.2f} s  global_acc={gacc}  train_loss={rec['train_loss']}")
        return rec


    def run(self, rounds: Optional[int] = None) -> List[dict]:
        cfg = self.cfg
        end = cfg.num_rounds if rounds is None else self.start_round + rounds
        r = self.start_round
        while r < end:
            self.run_round(r)
            r = self.next_round(r)
        self.finish()
        return self.history

    def drain(self):
        """Complete all in-flight communication (async gossip), evaluation and I/O."""
        self._resolve_eval()
        self._run_deferred()
        self._resolve_eval_local()
        if self.gossip is not None:
            self.gossip.drain()
        if self.server_mbox is not None:
            self.server_mbox.drain()
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self.timer.resolve(block=True)


    def finish(self, audit: bool = True):
        """Drain communication and I/O, verify the ledger (collective-free runs: cross-rank audit,
        a collective — pass ``audit=False`` when some rank has exited)."""
        self.drain()
        if hasattr(self, "_prefetch_pool"):
            self._prefetch_pool.shutdown(wait=True, cancel_futures=True)
            self._prefetched.clear()
        if self.ckpt is not None:
            self.ckpt.close()
            if self.rt.is_main and self.cfg.compat_save_path and self.ckpt.last_dir:
                mirror_dir(self.ckpt.last_dir, self.cfg.compat_save_path)
        if self.ledger is not None:
            bad = self.ledger.verify()
            if bad != -1:
                raise RuntimeError(f"ledger verification failed at height {bad}")
            if self.collective_free and self.rt.distributed and audit:
                self.ledger_audit = self.audit_ledgers()
                if self.ledger_audit["mismatched"]:
                    raise RuntimeError(f"ledger audit: {self.ledger_audit['mismatched']} accepted "
                                       "updates do not match their sender's commitment")
        if self.server_mbox is not None and self.rt.distributed and audit:
            self.final_check = self._final_model_check()
        if streamcheck.enabled():
            self.stream_races = streamcheck.report(streamcheck.disable())
            if self.stream_races and os.environ.get("BCFL_DEBUG_STREAMS") == "strict":
                raise RuntimeError(f"{len(self.stream_races)} unordered cross-stream access(es): "
                                   + self.stream_races[0])
        tel = self.telemetry.finish()
        if self.verbose and self.cfg.reference_prints:
            gdir = os.path.join(self.cfg.out_dir, "global")
            size = dir_size_gb(gdir) if os.path.isdir(gdir) else None
            Telemetry.print_reference_lines(tel, self.global_accuracies, size)
            if self.cfg.log_provenance:
                print(f"trained_data / tested_data: {self.provenance_rows} sampled train rows logged to "
                      f"{os.path.join(self.cfg.out_dir, 'provenance.jsonl')}", flush=True)
        self.metrics.write({"final": True, **tel, "global_accuracies": self.global_accuracies,
                            "global_accuracy_rounds": self.global_accuracy_rounds})
        self.metrics.close()
        return tel


