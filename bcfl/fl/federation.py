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
"""
from __future__ import annotations

import contextlib
import json
import math
import os
import time
import warnings
import zlib
from dataclasses import dataclass, field
from typing import Dict, Iterator, List, Optional

import numpy as np
import torch

from .. import ops
from ..ckpt import AsyncCheckpointer, dir_size_gb, mirror_dir, load_into
from ..config import FLConfig
from ..data.batching import ClientLoader
from ..data.partition import global_test_indices, majority_rate, partition_clients
from ..data.registry import get_dataset, load_split
from ..models import build_model, model_config, special_tokens
from ..parallel import dist as D
from ..parallel.flat import FlatAdamW, FlatParams
from ..parallel.gossip import GossipEngine, MailboxGossip
from ..parallel.mailbox import MailboxUnavailable
from ..parallel.topology import clients_of_rank, mixing_matrix, neighbours
from ..trust.anomaly import UpdateAnomalyFilter, Verdicts
from ..trust.ledger import Ledger
from ..utils.obs import MetricsWriter, PhaseTimer, Telemetry
from .drift import DriftCorrection, resolve_mode as resolve_drift
from .outer import OuterOptimizer
from .trainer import EvalResult, LocalTrainer, MicroReplica

DATA_SEED = 1234


def _cseed(seed: int, c: int) -> int:
    return zlib.crc32(f"{seed}:{c}".encode()) & 0x7FFFFFFF


def weighted_average(metrics):
    """Reference metric aggregation (``server_IID_IMDB.py:199-203``): Σ n_k·m_k / Σ n_k."""
    ex = sum(n for n, _ in metrics)
    out = {}
    for key in ("accuracy", "loss"):
        vals = [n * m[key] for n, m in metrics if key in m]
        if vals:
            out[key] = sum(vals) / max(ex, 1)
    return out


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


class Federation:
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
                if (self.gossip.apply_mode == "complete" and self.drift.exchange
                        and cfg.drift_correction_lag > 0):
                    self.drift.corr_lag = int(cfg.drift_correction_lag)
                if self.gossip.apply_mode == "complete" and self.drift.exchange:
                    self.drift.defer_cv = True   # formed in the gossip's fused round-end pass
                self.gossip.apply_on_arrival &= bool(cfg.gossip_apply_on_arrival
                                                     and cfg.anomaly_filter == "none"
                                                     and not cfg.inject_byzantine)
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
        self.filter = UpdateAnomalyFilter(cfg.anomaly_filter, cfg.anomaly_k,
                                          cfg.anomaly_modz_threshold) if cfg.anomaly_filter != "none" else None
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
        self.history: List[dict] = []
        self.start_round = 0
        self.ledger_audit: Optional[Dict[str, int]] = None
        self.tokens_trained = 0
        self.provenance_rows = 0
        if cfg.resume:
            self._resume(cfg.resume)

    def _ledger_path(self) -> Optional[str]:
        """Collective mode: one canonical chain, written by rank 0. Collective-free (mailbox)
        mode: every rank keeps its own chain (rank 0 -> ledger.jsonl, rank k -> ledger.rank{k}.jsonl)."""
        if self.rt.is_main:
            return os.path.join(self.cfg.out_dir, "ledger.jsonl")
        if self.collective_free:
            return os.path.join(self.cfg.out_dir, f"ledger.rank{self.rt.rank}.jsonl")
        return None

    # ================================ lanes ====================================================
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

    def _gossip_poll(self) -> None:
        """Between local steps: let arrived neighbour updates in (non-blocking)."""
        g = self.gossip
        if not isinstance(g, MailboxGossip) or not g.apply_on_arrival:
            return
        if self.lanes:
            streams = {c: ln.stream for ln in self.lanes for c in ln.clients}
            g.poll(streams, self.client_param, self._mid_round_targets)
        else:
            g.poll(None, {self.local_clients[0]: self.flat.param}, self._mid_round_targets)

    def _bound_lead(self, r: int) -> float:
        """Bounded staleness (SSP) for the asynchronous mailbox gossip, ``gossip_max_lead`` = s > 0:
        round r does not start while a live neighbour's newest applied update is more than s
        rounds behind this rank's own last one (round r - 1); arriving updates are applied while
        waiting. Ranks of equal speed never wait (a neighbour is at most ~1 round behind); ranks
        that share a GPU, or a persistently slower one, are held within s rounds of each other —
        without it 8 ranks time-sliced on one GPU drift 4-6 rounds apart and the fast ones train
        mostly on their own label shard. The bound has its own liveness (the round-based
        ``liveness_timeout`` would already have retired exactly the neighbours it must wait for):
        a neighbour still behind after ``gossip_lead_timeout_s`` is skipped until it posts again.
        Returns the seconds waited."""
        s, g = int(self.cfg.gossip_max_lead), self.gossip
        if s <= 0 or r == 0 or not isinstance(g, MailboxGossip) or not g.async_gossip:
            return 0.0
        posted = {}   # without apply-on-arrival: the newest round a neighbour has POSTED
        gone = self._lead_gone

        def seen(j):
            return max(g.replica_round[j], posted.get(j, -1), g.seen_round.get(j, -1))

        def lag():
            for j in [j for j in gone if seen(j) > gone[j]]:
                del gone[j]   # posted again: bounded again
            return [j for j in g.remote_needed if j not in gone and seen(j) < r - 1 - s]
        if not lag():
            return 0.0
        t0 = time.perf_counter()
        while True:
            late = lag()
            if not late:
                break
            if time.perf_counter() - t0 > float(self.cfg.gossip_lead_timeout_s):
                gone.update({j: seen(j) for j in late})
                break
            if g.apply_on_arrival:
                self._gossip_poll()
            else:
                for j, h in g.transport.headers(late).items():
                    nw = g.transport.newest(h)
                    if nw is not None:
                        posted[j] = nw[1].round
            # every poll queues header reads on the GPU: a few hundred per second, not thousands
            time.sleep(0.003)
        return time.perf_counter() - t0

    def _await_corrections(self, r: int) -> float:
        """Round-tagged drift correction (``drift_correction_lag``): round r applies the
        corrections of complete round r - lag on every client alike, so that round must have been
        applied here before round r starts. With bounded staleness every live source has posted
        it by now (equal-speed ranks finished it about a round ago), so this is at most one fetch;
        a source that is gone stops holding it back after ``gossip_lead_timeout_s`` (its round
        then completes without it, and a missing correction falls back to the newest older one).
        Returns the seconds waited."""
        g = self.gossip
        need = self.drift.correction_round_needed(r)
        if need is None or not isinstance(g, MailboxGossip) or g.applied_T >= need:
            return 0.0
        if int(self.cfg.gossip_max_lead) <= 0 and self.rt.distributed:
            # unbounded staleness was asked for: never wait; a client whose round r - lag has not
            # completed applies the newest older correction it holds (drift.lag_miss counts it)
            return 0.0
        t0 = time.perf_counter()
        while g.applied_T < need and time.perf_counter() - t0 < float(self.cfg.gossip_lead_timeout_s):
            self._gossip_poll()   # in-process virtual ranks: every poll is one tick of the clock
            if not g.virtual:
                time.sleep(0.002)
        return time.perf_counter() - t0

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
                    if self.filter is not None:
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
        on = cfg.prefetch_batches if cfg.prefetch_batches is not None else len(self.lanes) <= 4
        if not (self.is_cuda and on) or r >= cfg.num_rounds:
            return
        if not hasattr(self, "_prefetched"):
            import concurrent.futures as cf
            self._prefetched: Dict[tuple, object] = {}
            self._prefetch_pool = cf.ThreadPoolExecutor(1, thread_name_prefix="bcfl-prefetch")
        for k in [k for k in self._prefetched if k[1] < r - 1]:
            self._prefetched.pop(k)   # rounds that never trained these clients (resume, sampling)
        for c in self.local_clients:
            for e in range(cfg.local_epochs):
                if (c, r, e) not in self._prefetched:
                    self._prefetched[(c, r, e)] = self._prefetch_pool.submit(self._stage_train, c, r, e)

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

    def _draw_key(self, r: int) -> int:
        return r if self.cfg.resample_each_round else 0

    def test_batches(self, c: int, r: int):
        sp = self.partitions(r)[c]
        return self._cached_batches(
            ("test", c, self._draw_key(r)),
            lambda: ClientLoader(self.test_ds, sp.test, self.cfg.batch_size,
                                 pad_multiple=self.pad_multiple).device_batches(self.device))

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

    def global_test_batches(self, r: int, c: Optional[int] = None):
        mine = self._global_eval_rows(r, c)
        if len(mine) == 0:
            return []
        return self._cached_batches(
            ("global", self._draw_key(r), c),
            lambda: ClientLoader(self.test_ds, mine, max(self.cfg.global_eval_batch, 1),
                                 pad_multiple=self.pad_multiple).device_batches(self.device))

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
                return [(c0, self._cached_batches(
                    ("global", self._draw_key(r), "hosted"),
                    lambda: ClientLoader(
                        self.test_ds, np.sort(np.concatenate(
                            [self._global_eval_rows(r, c) for c in self.local_clients])),
                        max(self.cfg.global_eval_batch, 1),
                        pad_multiple=self.pad_multiple).device_batches(self.device)))]
            return [(c, self.global_test_batches(r, c)) for c in self.local_clients]
        if self._average_eval():
            self._refresh_average()
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
                and self.filter is None and not self.cfg.inject_byzantine
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

    def _activate(self, c: int, master: Optional[torch.Tensor] = None):
        if master is not None:
            self.flat.load_master(master)
        elif self.multi and c in self.client_master:
            self.flat.load_master(self.client_master[c])
        if self.keep_opt and c in self.client_opt:
            self.opt.load_state_dict(self.client_opt.pop(c) if self._single_opt else self.client_opt[c])
            self._opt_owner = c
        elif not (self.keep_opt and self._single_opt and self._opt_owner == c):
            self.opt.reset()
            self._opt_owner = c
        self.drift.attach(self.opt, c, self.flat.master, round_idx=self._round_now)
        self._mark_start(c, self.flat.master)
        ops.rng.global_rng().load_state(self.client_rng[c])

    def _deactivate(self, c: int):
        if self.multi and c in self.client_master:
            self.client_master[c].copy_(self.flat.master)
        if self.keep_opt and not self._single_opt:
            self.client_opt[c] = {k: (v.clone() if torch.is_tensor(v) else v)
                                  for k, v in self.opt.state_dict().items()}
        self.client_rng[c] = ops.rng.global_rng().state()

    def _train_client(self, c: int, r: int) -> Dict[str, float]:
        out = {"loss_sum": 0.0, "batches": 0, "tokens": 0, "examples": 0}
        loss_t = None
        for e in range(self.cfg.local_epochs):
            with self.timer.phase("data"):
                batches = self.train_batches(c, r, e)
            with self.timer.phase("train"):
                res = self.trainer.train_epoch(
                    batches, lr_fn=lambda i, e=e: self.lr_at(r, e * len(batches) + i),
                    step_hook=self._gossip_poll if self.cfg.mode == "serverless" else None)
            loss_t = res["loss_sum"] if loss_t is None else loss_t + res["loss_sum"]
            for k in ("batches", "tokens", "examples"):
                out[k] += res[k]
        out["loss_t"] = loss_t
        self.tokens_trained += out["tokens"]
        if c in self.cfg.inject_slow:
            time.sleep(self.cfg.inject_slow[c] / 1000.0)
        return out

    def _update_ref(self, c: int, prev: torch.Tensor) -> torch.Tensor:
        """What client c's own update of the round is measured from: the round-start copy, or —
        delta-exchange gossip — the gossip's round-start record, which also carries every
        neighbour update applied to the model during the round (so sketches, norms and injected
        scaling see this client's own progress only)."""
        g = self.gossip
        if isinstance(g, MailboxGossip) and g.exchange == "delta" and c in g._started:
            return g.start[c]
        return prev

    @torch.no_grad()
    def _inject_byzantine(self, c: int, ref: torch.Tensor, flat: Optional[FlatParams] = None):
        s = self.cfg.inject_byzantine.get(c)
        if s is None:
            return
        flat = flat or self.flat
        m = flat.master
        m.sub_(ref).mul_(s).add_(ref)
        flat.sync_param_from_master()

    @torch.no_grad()
    def _clip_update(self, ref: torch.Tensor, flat: Optional[FlatParams] = None) -> None:
        """Per-round trust region (``update_clip_ratio``): scale the round's update x - ref down
        to at most ratio * ||ref|| (device-side scalar, no host read). Early in training from
        random init a client's Adam-normalised round update can be large enough to throw a model
        that has just found the signal back onto the plateau."""
        rho = float(self.cfg.update_clip_ratio)
        if rho <= 0:
            return
        flat = flat or self.flat
        m = flat.master
        m.sub_(ref)
        scale = torch.clamp(rho * ref.norm() / (m.norm() + 1e-12), max=1.0)
        m.mul_(scale).add_(ref)
        flat.sync_param_from_master()

    @torch.no_grad()
    def _update_stats(self, ref: torch.Tensor, flat: Optional[FlatParams] = None):
        d = (flat or self.flat).master - ref
        return ops.block_sketch(d, self.cfg.sketch_dim).float(), d.norm().float()

    def _verdicts(self, sk_local: Dict[int, torch.Tensor], nrm_local: Dict[int, torch.Tensor]) -> Verdicts:
        if self.filter is None:
            return Verdicts()
        n = self.cfg.num_clients
        dim = self.cfg.sketch_dim
        mine = torch.zeros(n, dim + 1, dtype=torch.float32, device=self.device)
        for c in sk_local:
            mine[c, :dim] = sk_local[c]
            mine[c, dim] = nrm_local[c]
        D.all_reduce_(mine)  # each client row is written by exactly one rank
        a = mine.cpu().numpy()
        return self.filter(a[:, :dim], a[:, dim])

    def _merkle(self) -> str:
        return ops.merkle_root_sha256(self.flat.master).hex()

    def _ledger_round(self, r: int, recs: List[dict], extra: Optional[dict] = None):
        """Append this round's blocks. Collective mode: every rank appends the all-gathered
        records in one canonical order and the tips are compared across ranks every round
        (``consensus_check``; divergence aborts). Collective-free (mailbox) mode: each rank
        chains what it published and verified; chains are cross-audited in :meth:`finish`."""
        if self.ledger is None:
            return
        with self.timer.phase("ledger"):
            allrecs = recs if self.collective_free else [x for part in D.all_gather_object(recs)
                                                         for x in part]
            allrecs = sorted(allrecs, key=lambda x: (x["client"], x.get("kind", "update"),
                                                     x.get("metrics", {}).get("receiver_rank", -1)))
            for x in allrecs:
                root = x["root"]
                if not isinstance(root, str):   # a device root tensor (or raw digest bytes)
                    root = ops.root_bytes(root).hex()
                self.ledger.append(r, x["client"], x.get("kind", "update"), root, x["verdict"],
                                   x.get("metrics", {}), ts=x["ts"])
            if extra is not None:
                kind, root = extra.pop("kind", "round"), extra.pop("root", "")
                if not self.collective_free and self.rt.distributed:
                    # round-summary fields can be rank-local (async staleness, liveness view):
                    # every rank must append the SAME block, so record all ranks' views
                    views = D.all_gather_object(extra)
                    extra = views[0] if all(v == views[0] for v in views) else {"per_rank": views}
                self.ledger.append(r, -1, kind, root, "accept", extra, ts=float(r + 1))
            self.ledger.flush()
            if not self.collective_free and self.rt.distributed and not self.ledger.consensus_check():
                raise RuntimeError(f"ledger tips diverged across ranks at round {r}")

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
            es.wait_stream(main)               # the mixed model(s) and the batches are ready
            if not hasattr(self, "_eval_snaps"):
                self._eval_snaps = {}
            with torch.cuda.stream(es):
                t_beg = torch.cuda.Event(enable_timing=True)
                t_beg.record(es)
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
                copied = torch.cuda.Event()
                copied.record(es)
                # later writers of the sources (next round's optimizer / mixing, issued on main
                # or on lane streams that wait on main) are ordered after the snapshot copies
                # only; the forward passes overlap them
                main.wait_event(copied)
                acc = torch.zeros(4, dtype=torch.float64, device=self.device)
                for (c, gb), snap in zip(sets, snaps):
                    if gb:
                        self.eval_flat.rebind(self.eval_flat.master, snap)
                        acc += self.eval_trainer.evaluate_device(gb)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(es)
            self._eval_pending = (r, acc, sets, ev, t_beg)

    def _resolve_eval(self) -> None:
        """Host-read a queued global evaluation and file it under its round."""
        p, self._eval_pending = self._eval_pending, None
        if p is None:
            return
        r, acc, _sets, ev, t_beg = p
        ev.synchronize()
        self.timer.add_hidden("eval_global", t_beg.elapsed_time(ev) / 1000.0)
        if not self.collective_free:
            D.all_reduce_(acc)
        a = acc.cpu().tolist()
        ge = EvalResult(int(a[0]), int(a[1]), a[2], a[3])
        self._note_global_counts(r, a)
        self.global_accuracies.append(ge.accuracy)
        if self.verbose and self.cfg.reference_prints:
            print(f"Global Model Accuracy: {ge.accuracy * 100:.2f}%", flush=True)
        upd = {"global_acc": ge.accuracy, "global_majority_rate": self.global_majority_rate(r),
               "global_eval_rows": int(ge.count), "global_loss": ge.loss}
        for rec in reversed(self.history):
            if rec.get("round") == r:
                rec.update(upd)
                break
        self.metrics.write({"round": r, "deferred_global_eval": True, **upd})

    def _diag(self, r: int) -> None:
        """``BCFL_DIAG=1``: one stderr line per round and rank on the asynchronous protocol's
        state — the newest complete round applied, the classifier bias of this rank's first
        client (a label-sharded federation stuck on the plateau predicts from it), the norms of
        the client's drift correction and of its own update of the round (host reads: debugging
        only)."""
        import sys
        g, c = self.gossip, self.local_clients[0]
        m = self.client_master[c] if self.multi else self.flat.master
        bias = []
        for name, (o, n, _s) in zip(self.flat.names, self.flat.slots):
            if name.endswith("classifier_bias") or name.endswith("classifier.bias"):
                bias = [round(x, 4) for x in m[o:o + n].tolist()]
        corr = float(self.drift.buf[c].norm()) if self.drift.enabled else 0.0
        cum = float(g.cum[c].norm()) if getattr(g, "exchange", "") == "delta" else 0.0
        print(f"[diag] rank {self.rt.rank} round {r} applied_T {getattr(g, 'applied_T', None)} "
              f"bias {bias} corr {corr:.4g} cum {cum:.4g}", file=sys.stderr, flush=True)

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

    # ================================ rounds ====================================================
    def server_round(self, r: int) -> dict:
        cfg = self.cfg
        G = self.global_master
        counts = self.fedavg_weight_counts(r)
        recs, sk, nr, trained, losses = [], {}, {}, {}, {}
        need_copy = self.filter is not None and self.multi
        self.acc.zero_()
        w_all = counts / counts.sum()
        if self.lanes:
            if self.verbose and cfg.reference_prints:
                print("Training Started...", flush=True)
            o = self._server_train_lanes(r, G, {c: float(w_all[c]) for c in self.local_clients},
                                         keep=self.filter is not None)
            if self.verbose and cfg.reference_prints:
                print("Training Finished.", flush=True)
            sk, nr, losses, trained = o["sk"], o["nr"], o["losses"], o["trained"]
            for c in self.local_clients:
                root = ops.root_bytes(o["roots"][c]).hex() if o["roots"][c] is not None else ""
                recs.append({"client": c, "root": root, "ts": float(r) + 0.001 * (c + 1),
                             "verdict": "accept", "metrics": {"examples": losses[c]["examples"]}})
        for c in ([] if self.lanes else self.local_clients):
            self._activate(c, master=G)
            if self.verbose and cfg.reference_prints:
                print("Training Started...", flush=True)
            st = self._train_client(c, r)
            self._clip_update(G)
            self.drift.after_train(c, self.flat.master, self.lr_sum(r, st["batches"]))
            self.drift.detach(self.opt)
            self._inject_byzantine(c, G)
            if self.verbose and cfg.reference_prints:
                print("Training Finished.", flush=True)
            losses[c] = st
            if self.filter is not None:
                with self.timer.phase("anomaly"):
                    sk[c], nr[c] = self._update_stats(G)
            root = self._merkle() if self.ledger is not None else ""
            recs.append({"client": c, "root": root, "ts": float(r) + 0.001 * (c + 1),
                         "verdict": "accept", "metrics": {"examples": st["examples"]}})
            if need_copy:
                trained[c] = self.flat.master.detach().clone()
            elif self.filter is None:
                ops.weighted_accumulate_(self.acc, self.flat.master, float(w_all[c]))
            else:
                trained[c] = self.flat.master
            self._deactivate(c)
        with self.timer.phase("anomaly"):
            v = self._verdicts(sk, nr)
        if self.filter is not None:
            mask = np.array([0.0 if c in v.rejected else 1.0 for c in range(cfg.num_clients)])
            w = counts * mask
            w = w / max(w.sum(), 1e-30)
            for c in self.local_clients:
                ops.weighted_accumulate_(self.acc, trained[c], float(w[c]))
            for x in recs:
                x["verdict"] = v.verdict(x["client"])
        absent = []
        with self.timer.phase("comm"):
            if self.server_mbox is not None:
                wloc = float(sum(w_all[c] for c in self.local_clients))
                g_new, minfo = self.server_mbox.reduce(r, self.acc, wloc)
                self.acc.copy_(g_new)
                wire_bytes = minfo["bytes_sent"]
                absent = minfo["absent_ranks"]
                # ledger: this rank's post is an update block and every verified receive a verify
                # block, both keyed by the sending rank's id -(rank + 1) and the post's version,
                # so audit_ledgers() matches every accepted receive against its commitment
                for g in self.server_mbox.take_records():
                    if g["kind"] == "update":
                        rt_ = g.get("root_t")
                        recs.append({"client": g["client"], "kind": "update",
                                     "root": "" if rt_ is None else ops.root_bytes(rt_).hex(),
                                     "verdict": "accept", "ts": float(r) + 0.4,
                                     "metrics": {"sender_rank": self.rt.rank,
                                                 "version": g["version"]}})
                    elif g["kind"] == "recv":
                        recs.append({"client": g["client"], "kind": "verify", "root": g["root"],
                                     "verdict": "accept" if g["ok"] else "reject",
                                     "ts": float(r) + 0.5,
                                     "metrics": {"sender_rank": -g["client"] - 1,
                                                 "receiver_rank": self.rt.rank,
                                                 "version": g["version"], "src_round": g["src_round"]}})
                self._server_live = minfo
            elif cfg.server_wire_dtype == "bf16" and self.rt.distributed:
                # delta coding: each rank reduces sum_{k local} w_k (x_k - G), bf16 on the wire
                wloc = float(sum(w[c] for c in self.local_clients)) if self.filter is not None \
                    else float(sum(w_all[c] for c in self.local_clients))
                ops.axpby_(self.acc, G, -wloc, 1.0)
                wire_bytes = D.all_reduce_bf16_(self.acc)
                ops.axpby_(self.acc, G, 1.0, 1.0)
            else:
                D.all_reduce_(self.acc)
                wire_bytes = self.acc.numel() * 4 * 2 * max(self.rt.world - 1, 0) // max(self.rt.world, 1)
        for c in self.local_clients:   # SCAFFOLD's c' from the plain FedAvg result
            self.drift.after_mix(c, self.acc)
        self.outer.step(-1, self.acc, prev=G)   # FedAvgM / outer Nesterov (off by default)
        G.copy_(self.acc)
        self.flat.load_master(G)
        # Flower evaluate_round: every client evaluates the new global model on its test split
        client_metrics = []
        if cfg.eval_local:
            with self.timer.phase("eval_local"):
                dev_res = self._server_eval_local(r, G)
                loc = []
                for c, t in dev_res.items():
                    a = t.cpu().tolist()
                    e = EvalResult(int(a[0]), int(a[1]), a[2], a[3])
                    loc.append((c, e.count, {"accuracy": e.accuracy, "loss": e.ref_loss if cfg.compat_bad_test_loss else e.loss}))
                client_metrics = self._gather_metrics(loc)
        agg = weighted_average([(n_, m) for _, n_, m in client_metrics]) if client_metrics else {}
        ge = None
        if self._global_eval_due(r):
            if self.eval_stream is not None:
                self._launch_eval_global(r)   # the global model, scored beside round r + 1
            else:
                ge = self._eval_global(r)
        train_loss = self._reduce_train_loss(losses)
        extra = {"kind": "global", "root": self._merkle() if self.ledger else "",
                 "rejected": sorted(v.rejected)}
        if self.server_mbox is not None:
            sk = int(self._server_live.get("epochs_skipped", 0))
            extra.update(absent_ranks=absent, live_weight=self._server_live["live_weight"],
                         rejoined_ranks=self._server_live["rejoined_ranks"],
                         view_mismatch=self._server_live["view_mismatch"],
                         epoch=int(self._server_live.get("epoch", r + 1)), epochs_skipped=sk,
                         **({"absent_owners": self._server_live["absent_owners"]}
                            if "absent_owners" in self._server_live else {}))
            if sk:
                # this rank joined a later aggregation epoch (started late / excluded as slow):
                # the skipped epochs were aggregated WITHOUT it and are not trained rounds here
                self.skipped_epochs += sk
                warnings.warn(f"round {r}: this rank joined aggregation epoch "
                              f"{self._server_live.get('epoch')} and skipped {sk} epoch(s) the "
                              "federation aggregated without it", RuntimeWarning)
            if self._server_live["view_mismatch"]:
                warnings.warn(f"round {r}: rank(s) {self._server_live['view_mismatch']} aggregated "
                              "a different live-rank set last round than this rank (a timed-out "
                              "but live peer): the global models differed for that round",
                              RuntimeWarning)
        self._ledger_round(r, recs, extra)
        out = {"distributed_accuracy": agg.get("accuracy"), "distributed_loss": agg.get("loss"),
               "global": ge, "train_loss": train_loss, "rejected": sorted(v.rejected),
               "client_metrics": client_metrics, "bytes_sent": float(wire_bytes)}
        if self.server_mbox is not None:
            out.update(absent_ranks=absent, live_weight=self._server_live["live_weight"],
                       dead_peers=sorted(self.server_mbox.dead),
                       epochs_skipped=int(self._server_live.get("epochs_skipped", 0)),
                       view_mismatch=self._server_live["view_mismatch"],
                       rejoined_ranks=self._server_live["rejoined_ranks"])
        return out

    @property
    def _gossip_roots(self) -> bool:
        """The gossip engine hashes every published payload (its ledger commitment), so the
        update blocks use those roots and the trainer does not hash the master a second time."""
        return isinstance(getattr(self, "gossip", None), MailboxGossip) and self.gossip.verify

    def _gossip_records(self, r: int, recs: List[dict]) -> List[dict]:
        """Ledger records from the last exchange: published payload roots replace the update
        roots; every verified receive becomes a ``verify`` block (verdict accept / reject)."""
        out = []
        by_client = {x["client"]: x for x in recs}
        take = getattr(self.gossip, "take_records", None)
        for g in (take() if take is not None else []):
            if g["kind"] == "update":
                if g.get("root_t") is not None and g["client"] in by_client and self._gossip_roots:
                    # a device tensor stays one until the block is appended (_ledger_round):
                    # reading it here would wait for the publish hash
                    by_client[g["client"]]["root"] = g["root_t"]
                if g["client"] in by_client:
                    by_client[g["client"]].setdefault("metrics", {})["version"] = g["version"]
            elif g["kind"] == "recv":
                out.append({"client": g["client"], "kind": "verify", "root": g["root"],
                            "verdict": "accept" if g["ok"] else "reject",
                            "ts": float(r) + 0.5 + 0.001 * (g["client"] + 1),
                            "metrics": {"receiver_rank": self.rt.rank, "version": g["version"],
                                        "src_round": g["src_round"],
                                        **({} if g["ok"] else {"reason": "merkle root mismatch"})}})
        return out

    def _gather_metrics(self, loc: list) -> list:
        if self.collective_free:
            return list(loc)
        return [x for part in D.all_gather_object(loc) for x in part]

    def _reduce_train_loss(self, losses: Dict[int, dict]) -> float:
        if not losses:
            return 0.0
        t = torch.zeros(2, dtype=torch.float64, device=self.device)
        for st in losses.values():
            if st["loss_t"] is not None:
                t[0] += st["loss_t"].double()
            t[1] += st["batches"]
        if not self.collective_free:
            D.all_reduce_(t)
        a = t.cpu().tolist()
        return a[0] / max(a[1], 1)

    def serverless_round(self, r: int) -> dict:
        cfg = self.cfg
        if cfg.compat_chain:
            return self._chain_round(r)
        recs, sk, nr, losses, local_eval = [], {}, {}, {}, {}
        need_prev = (self.filter is not None or bool(cfg.inject_byzantine)
                     or cfg.update_clip_ratio > 0)
        self._run_deferred(block=False)  # earlier rounds' host reads whose kernels have finished
        self._resolve_eval_local()      # last round's deferred local scores (long finished)
        lead_wait = self._bound_lead(r)
        self._round_now = r
        corr_wait = self._await_corrections(r)
        if self.outer.enabled:
            for c in self.local_clients:
                self.outer.begin(c, self.client_master[c] if self.multi else self.flat.master)
        if self.lanes:
            o = self._train_lanes(r, need_prev)
            sk, nr, losses, local_eval = o["sk"], o["nr"], o["losses"], o["local_eval"]
            for c in self.local_clients:
                root = ops.root_bytes(o["roots"][c]).hex() if o["roots"][c] is not None else ""
                recs.append({"client": c, "root": root, "ts": float(r) + 0.001 * (c + 1),
                             "verdict": "accept", "metrics": {"examples": losses[c]["examples"]}})
        for c in ([] if self.lanes else self.local_clients):
            self._activate(c)
            prev = self.flat.master.detach().clone() if need_prev else None
            st = self._train_client(c, r)
            if prev is not None:
                self._clip_update(self._update_ref(c, prev))
            self.drift.after_train(c, self.flat.master, self.lr_sum(r, st["batches"]))
            self._phase[c] = "trained"
            self.drift.detach(self.opt)
            if prev is not None:
                ref = self._update_ref(c, prev)
                self._inject_byzantine(c, ref)
                if self.filter is not None:
                    with self.timer.phase("anomaly"):
                        sk[c], nr[c] = self._update_stats(ref)
            losses[c] = st
            if cfg.eval_local:
                with self.timer.phase("eval_local"):
                    if self._defer_local_eval():
                        self._launch_eval_local(c, r)
                    else:
                        local_eval[c] = self.trainer.evaluate_device(self.test_batches(c, r))
            root = self._merkle() if self.ledger is not None and not self._gossip_roots else ""
            recs.append({"client": c, "root": root, "ts": float(r) + 0.001 * (c + 1),
                         "verdict": "accept", "metrics": {"examples": st["examples"]}})
            self._deactivate(c)
        with self.timer.phase("anomaly"):
            v = self._verdicts(sk, nr)
        for x in recs:
            x["verdict"] = v.verdict(x["client"])
        # async mixes states published last round -> apply last round's verdicts to them
        use_v = self.prev_verdicts if (cfg.async_gossip and not self.same_round_mix) else v
        W = mixing_matrix(self.nbrs, cfg.mixing, use_v.rejected)
        if isinstance(self.gossip, MailboxGossip):
            self.gossip.W_mid = W
        with self.timer.phase("comm"):
            pout = (self.client_param if self.lanes else
                    None if self.multi else {self.local_clients[0]: self.flat.param})
            info = self.gossip.end_of_round(r, W, pout,
                                            steps={c: losses[c]["batches"] for c in losses})
        recs += self._gossip_records(r, recs)
        if os.environ.get("BCFL_DIAG") and isinstance(self.gossip, MailboxGossip):
            self._diag(r)
        self.prev_verdicts = v
        for c in self.local_clients:
            self.drift.after_mix(c, self.client_master[c] if self.multi else self.flat.master)
        if self.outer.enabled:
            for c in self.local_clients:
                if self.multi:
                    self.outer.step(c, self.client_master[c], self.client_param.get(c))
                else:
                    self.outer.step(c, self.flat.master, self.flat.param
                                    if self.flat.param is not self.flat.master else None)
        if self.multi:  # evaluate this rank's first client's mixed model
            c0 = self.local_clients[0]
            if self.lanes:
                self.flat.rebind(self.client_master[c0], self.client_param[c0])
            else:
                self.flat.load_master(self.client_master[c0])
        ge = None
        if self._global_eval_due(r):
            if self.eval_stream is not None:
                self._launch_eval_global(r)   # filed under round r by _resolve_eval
            else:
                ge = self._eval_global(r)
        host_deferred = self.collective_free and self.is_cuda and not self.rt.distributed
        client_metrics = []
        if host_deferred and local_eval:
            # the lanes' local scores are read at the next round's start with the other deferred
            # host reads (a read here would idle the GPU from the round's last kernel until the
            # next round's first launch)
            self._defer(lambda r=r, le=dict(local_eval): self._file_local_eval(r, le))
        else:
            client_metrics = self._local_metrics(local_eval)
        ledger_extra = {"kind": "mix", "rejected": sorted(v.rejected),
                        "stale_rounds": info.get("stale_rounds", 0.0),
                        "dead_peers": sorted(self.gossip.dead)}
        if self.collective_free and self.is_cuda and not self.rt.distributed:
            # nothing of this round is read back on the host now (the loss sum and the ledger's
            # Merkle roots wait for the round's last kernels): the next round's work is queued
            # while this round's tail still runs, and the reads happen at its start. Multi-rank
            # runs keep the round-end read: it paces the host to its GPU, so the bounded-lead
            # check compares rounds the device has actually finished (deferred, 8 ranks sharing
            # one GPU spent ~0.8 s per round in lead waits and ran 3x slower)
            train_loss = None
            self._defer(lambda r=r, losses=losses: self._patch_history(
                r, train_loss=self._reduce_train_loss(losses)))
            self._defer(lambda r=r, recs=recs, ex=ledger_extra: self._ledger_round(r, recs, ex))
        else:
            train_loss = self._reduce_train_loss(losses)
            self._ledger_round(r, recs, ledger_extra)
        agg = weighted_average([(n_, m) for _, n_, m in client_metrics]) if client_metrics else {}
        return {"distributed_accuracy": agg.get("accuracy"), "distributed_loss": agg.get("loss"),
                "global": ge, "train_loss": train_loss, "rejected": sorted(v.rejected),
                "client_metrics": client_metrics, "bytes_sent": info.get("bytes_sent", 0.0),
                "mixed": info.get("mixed", 0.0), "stale_rounds": info.get("stale_rounds", 0.0),
                "stale_max": info.get("stale_max", 0.0),
                "wait_s": info.get("wait_s", 0.0) + lead_wait + corr_wait, "lead_wait_s": lead_wait,
                "corr_wait_s": corr_wait,
                "final_wait_s": info.get("final_wait_s", 0.0),
                "dead_peers": sorted(self.gossip.dead), "torn": info.get("torn", 0.0),
                "rejected_msgs": info.get("rejected_msgs", 0.0)}

    # ---- host reads deferred to the next round --------------------------------------------------
    def _defer(self, fn) -> None:
        """Queue a host read of this round's device results. It runs once the work queued so far
        has finished on the device (an event recorded now), so a read never stalls the host in
        front of the next round's launches: at the next round start the round's tail is usually
        still running, and the read waits one more round instead of idling the GPU."""
        if not hasattr(self, "_deferred"):
            self._deferred = []
        ev = None
        if self.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self._deferred.append((fn, ev))

    def _run_deferred(self, block: bool = True) -> None:
        """Run the queued host reads in order; ``block=False`` stops at the first one whose
        device work has not finished yet (it stays queued)."""
        q = getattr(self, "_deferred", [])
        while q:
            fn, ev = q[0]
            if not block and ev is not None and not ev.query():
                break
            q.pop(0)
            fn()

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

    def _patch_history(self, r: int, **kw) -> None:
        for rec in reversed(self.history):
            if rec.get("round") == r:
                rec.update(kw)
                break
        self.metrics.write({"round": r, "deferred": True, **kw})

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
        main = torch.cuda.current_stream(self.device)
        if not hasattr(self, "_local_snaps"):
            self._local_snaps = [torch.empty_like(self.flat.param) for _ in range(2)]
            self._local_done: List[Optional[torch.cuda.Event]] = [None, None]
            self._local_pending: List[tuple] = []
            self._local_k = 0
        i = self._local_k % 2
        self._local_k += 1
        if self._local_done[i] is not None:
            main.wait_event(self._local_done[i])   # the evaluation that last read this snapshot
        snap = self._local_snaps[i]
        snap.copy_(self.flat.param)                # the trained model, before the mix
        batches = self.test_batches(c, r)          # uploaded on the training stream
        es = self.eval_stream
        es.wait_stream(main)
        own = self.eval_flat.param
        with torch.cuda.stream(es):
            self.eval_flat.rebind(self.eval_flat.master, snap)
            stats = self.eval_trainer.evaluate_device(batches)
            ev = torch.cuda.Event()
            ev.record(es)
        # the queued kernels hold the snapshot's pointers; the replica's own buffer is what the
        # global evaluation copies into (no later reader of the snapshot but this evaluation)
        self.eval_flat.rebind(self.eval_flat.master, own)
        self._local_done[i] = ev
        # the batches stay referenced until the statistics are read (their memory belongs to
        # the training stream's pool)
        self._local_pending.append((r, c, stats, ev, batches))

    def _resolve_eval_local(self) -> None:
        pend = getattr(self, "_local_pending", None)
        if not pend:
            return
        self._local_pending = []
        by_round: Dict[int, list] = {}
        for r, c, stats, ev, _b in pend:
            ev.synchronize()
            a = stats.cpu().tolist()
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

    def _chain_round(self, r: int) -> dict:
        """Reference C14 exactly: clients train one after another on ONE shared model; the
        round ends with the unweighted mean of the K snapshots."""
        snaps = torch.zeros_like(self.flat.master)
        client_metrics, losses = [], {}
        for c in self.local_clients:
            self.opt.reset()
            ops.rng.global_rng().load_state(self.client_rng[c])
            losses[c] = self._train_client(c, r)
            self.client_rng[c] = ops.rng.global_rng().state()
            ops.weighted_accumulate_(snaps, self.flat.master, 1.0 / len(self.local_clients))
            e = self.trainer.evaluate(self.test_batches(c, r))
            client_metrics.append((c, e.count, {"accuracy": e.accuracy, "loss": e.ref_loss}))
            if self.verbose and self.cfg.reference_prints:
                print("local_accuracy" + " :" + str(e.accuracy), flush=True)
        self.flat.load_master(snaps)
        ge = self._eval_global(r)
        return {"distributed_accuracy": weighted_average([(n, m) for _, n, m in client_metrics]).get("accuracy"),
                "global": ge, "train_loss": self._reduce_train_loss(losses), "rejected": [],
                "client_metrics": client_metrics, "bytes_sent": 0.0}

    # ================================ driver ====================================================
    def _log_provenance(self, r: int):
        """Reference C18 (``serverless_IID_IMDB.py:251-260,298-301``): every client's sampled
        train / test row indices, one JSONL record per (round, client) — written when the draw
        changes (every round with ``resample_each_round``, else round 0). Partitions are a pure
        function of the config, so the main rank writes all clients."""
        if not (self.cfg.log_provenance and self.rt.is_main):
            return
        if r != self.start_round and not self.cfg.resample_each_round:
            return
        path = os.path.join(self.cfg.out_dir, "provenance.jsonl")
        os.makedirs(self.cfg.out_dir, exist_ok=True)
        mode = "a" if (r != self.start_round or self.cfg.resume) else "w"
        with open(path, mode) as fh:
            for c, sp in enumerate(self.partitions(r)):
                fh.write(json.dumps({"round": r, "client": c, "trained_data": [int(i) for i in sp.train],
                                     "tested_data": [int(i) for i in sp.test]}) + "\n")
        self.provenance_rows += sum(len(sp.train) for sp in self.partitions(r))

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
                                      "final_wait_s",
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

    def _maybe_save(self, r: int):
        """Reference C16 (``save_pretrained`` every round, ``serverless_NonIID_IMDB.py:305``):
        ``<out>/global`` (rank 0), ``<out>/client_{k}`` for EVERY hosted client with
        ``save_clients``, and with ``save_resume_state`` the per-rank state a resumed run needs to
        continue bit-identically (``<out>/resume/rank{r}.pt``)."""
        cfg = self.cfg
        if cfg.save_every <= 0 or (r + 1) % cfg.save_every:
            return
        pend = self._eval_pending
        if pend is not None and pend[0] == r and not self.collective_free and self.rt.distributed:
            # multi-rank collective mode: the saved accuracy is the job's (all-reduced), so
            # resolve here — on EVERY rank, including those that write nothing (self.ckpt None):
            # the resolve is a collective, and a rank skipping it would pair its next all-reduce
            # with the others' FedAvg all-reduce
            self._resolve_eval()
        if self.ckpt is None:
            return
        if cfg.save_resume_state:
            self._run_deferred()   # the resume state must carry this round's ledger tip
        if self.ckpt.busy():
            if cfg.save_resume_state:
                # resumable runs never skip: every rank's files of a save belong to ONE round
                # (independent skips would let global/, client_*/ and resume/rank*.pt disagree)
                self.ckpt.wait()
            else:
                self.ckpt.skipped += 1   # skip BEFORE building any state (no wasted D2H copies)
                return
        with self.timer.phase("ckpt"):
            accs = list(self.global_accuracies)
            state = {"round": r, "rng": ops.rng.global_rng().state(),
                     "ledger_tip": self.ledger.tip if self.ledger else None,
                     "ledger_height": len(self.ledger) if self.ledger else 0,
                     "global_accuracies": accs, "config": cfg.to_dict()}
            pend = self._eval_pending
            if pend is not None and pend[0] == r:
                # round r's overlapped evaluation is still running: the writer thread waits for
                # its event and files the accuracy (no stall of the training stream here)
                _r, acc_t, _sets, ev_t, _t0 = pend

                def _fin(accs=accs, acc_t=acc_t, ev_t=ev_t):
                    ev_t.synchronize()
                    a = acc_t.cpu().tolist()
                    return {"global_accuracies": accs + [a[0] / max(a[1], 1.0)]}
                state["_finalize"] = _fin
            jobs = []
            if self.rt.is_main:
                src = self.global_master if cfg.mode == "server" else self.flat.master
                jobs.append(([os.path.join(cfg.out_dir, "global")], src))
            if cfg.save_clients:
                for c in self.local_clients:
                    src = self.client_master.get(c, self.flat.master)
                    jobs.append(([os.path.join(cfg.out_dir, f"client_{c}")], src))
            extra = None
            if cfg.save_resume_state:
                extra = {os.path.join(cfg.out_dir, "resume", f"rank{self.rt.rank}.pt"):
                         self.resume_state(r)}
            if jobs or extra:
                self.ckpt.save([], metadata={"round": str(r)},
                               state=state if self.rt.is_main else None, jobs=jobs,
                               extra_files=extra)

    def _opt_states(self) -> Dict[int, dict]:
        """Kept optimizer states per client (a one-client rank keeps its live optimizer)."""
        st = dict(self.client_opt)
        if self.keep_opt and self._single_opt and self._opt_owner is not None:
            st[self._opt_owner] = self.opt.state_dict()
        return st

    def resume_state(self, r: int) -> dict:
        """Per-rank training state (tensors on the host; loadable with ``weights_only=True``)."""
        cpu = lambda t: t.detach().cpu().clone()  # noqa: E731
        st = {"round": int(r), "rank": self.rt.rank, "world": self.rt.world,
              "rng": ops.rng.global_rng().state(),
              "client_rng": {int(c): dict(v) for c, v in self.client_rng.items()},
              "client_master": {int(c): cpu(t) for c, t in self.client_master.items()},
              "master": cpu(self.flat.master),
              "client_opt": {int(c): {"m": cpu(o["m"]), "v": cpu(o["v"]), "step": int(o["step"])}
                             for c, o in self._opt_states().items()},
              "prev_rejected": sorted(self.prev_verdicts.rejected),
              "drift": self.drift.state_dict(),
              "outer": self.outer.state_dict(),
              "tokens_trained": int(self.tokens_trained),
              "ledger_tip": self.ledger.tip if self.ledger else None,
              "ledger_height": len(self.ledger) if self.ledger else 0}
        if self.global_master is not None:
            st["global_master"] = cpu(self.global_master)
        if self.gossip is not None and hasattr(self.gossip, "state_dict"):
            st["gossip"] = self.gossip.state_dict()
        return st

    def next_round(self, r: int) -> int:
        """Round to run after round r: r + 1, except when the mailbox FedAvg joined a later
        aggregation epoch (this rank started late or was excluded as slow, fedavg.py): the rank
        then continues at the federation's round instead of replaying the ones it missed."""
        if self.server_mbox is not None:
            return max(r + 1, self.server_mbox.epoch)
        return r + 1

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

    def audit_ledgers(self) -> Dict[str, int]:
        """Cross-rank audit of the per-rank chains of a collective-free federation: every update
        a rank ACCEPTED must carry exactly the Merkle root its sender committed for that version."""
        mine = self.ledger.blocks()
        chains = D.all_gather_object(mine)
        committed = {}
        for ch in chains:
            for b in ch:
                if b["kind"] == "update":
                    v = json.loads(b["payload"] or "{}").get("version")
                    if v is not None:
                        committed[(b["client"], v)] = b["update_root"]
        checked = mismatched = rejected = 0
        for ch in chains:
            for b in ch:
                if b["kind"] != "verify":
                    continue
                if b["verdict"] != "accept":
                    rejected += 1
                    continue
                key = (b["client"], json.loads(b["payload"] or "{}").get("version"))
                if key in committed:
                    checked += 1
                    mismatched += int(committed[key] != b["update_root"])
        return {"checked": checked, "mismatched": mismatched, "rejected": rejected}

    def _final_model_check(self) -> dict:
        """Mailbox FedAvg: every rank's FINAL global model root, gathered (a collective, run once
        at the end). Ranks that aggregated different live sets in the last round(s) — a slow rank
        timed out by a fast one that then finished — end on different models; that split is
        recorded in every rank's ledger and warned about, never silent."""
        root = ops.merkle_root_sha256(self.global_master).hex()
        allr = D.all_gather_object({"rank": self.rt.rank, "root": root,
                                    "rounds": len(self.history), "epoch": self.server_mbox.epoch,
                                    "skipped_epochs": self.skipped_epochs})
        roots = [x["root"] for x in allr]
        split = len(set(roots)) > 1
        info = {"split": split, "ranks": allr}
        if self.ledger is not None:
            self.ledger.append(len(self.history), -1, "final_check", root,
                               "reject" if split else "accept", info, ts=float(len(self.history) + 1))
            self.ledger.flush()
        if split:
            groups = {}
            for x in allr:
                groups.setdefault(x["root"][:16], []).append(x["rank"])
            warnings.warn(f"mailbox FedAvg ended SPLIT: the ranks hold {len(groups)} different "
                          f"final global models {sorted(groups.values())} (a live-set "
                          "disagreement in the last aggregation epoch)", RuntimeWarning)
        return info

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
        tel = self.telemetry.finish()
        if self.verbose and self.cfg.reference_prints:
            gdir = os.path.join(self.cfg.out_dir, "global")
            size = dir_size_gb(gdir) if os.path.isdir(gdir) else None
            Telemetry.print_reference_lines(tel, self.global_accuracies, size)
            if self.cfg.log_provenance:
                print(f"trained_data / tested_data: {self.provenance_rows} sampled train rows logged to "
                      f"{os.path.join(self.cfg.out_dir, 'provenance.jsonl')}", flush=True)
        self.metrics.write({"final": True, **tel, "global_accuracies": self.global_accuracies})
        self.metrics.close()
        return tel

    def _resume(self, path: str):
        st_path = os.path.join(path, "global", "state.json")
        if not os.path.exists(st_path):
            raise FileNotFoundError(st_path)
        with open(st_path) as fh:
            st = json.load(fh)
        load_into(self.model, self.flat, os.path.join(path, "global"))
        if self.global_master is not None:
            self.global_master.copy_(self.flat.master)
        for c in self.client_master:
            self.client_master[c].copy_(self.flat.master)
            if c in self.client_param:
                ops.cast_copy_(self.client_param[c], self.client_master[c])
        if self.gossip is not None:
            self.gossip.seed_replicas(self.flat.master)
        self.start_round = int(st["round"]) + 1
        self.global_accuracies = list(st.get("global_accuracies", []))
        rs = os.path.join(path, "resume", f"rank{self.rt.rank}.pt")
        rst = None
        if os.path.exists(rs):
            rst = torch.load(rs, weights_only=True, map_location="cpu")
            if int(rst["round"]) != int(st["round"]):
                raise RuntimeError(f"resume state {rs} is from round {rst['round']} but "
                                   f"global/state.json is from round {st['round']}: the "
                                   "checkpoint files belong to different rounds")
            self._load_resume_state(rst)
        # each rank continues ITS OWN chain: collective-free runs keep one chain per rank
        # (ledger.rank{k}.jsonl), collective runs one canonical chain (ledger.jsonl)
        mine = self._ledger_path()
        led = os.path.join(path, os.path.basename(mine) if mine else "ledger.jsonl")
        tip, height = st.get("ledger_tip"), st.get("ledger_height")
        if rst is not None and "ledger_tip" in rst:
            tip, height = rst.get("ledger_tip"), rst.get("ledger_height")
        if self.ledger is not None and os.path.exists(led):
            old = Ledger.load(led)
            if old.verify() != -1:
                raise RuntimeError("ledger in resume dir fails verification")
            if height and len(old) > int(height):
                old = old.truncated(int(height))  # blocks after the checkpoint
            if tip and old.tip != tip:
                raise RuntimeError(f"ledger tip of {led} does not match the checkpoint's ledger_tip")
            self.ledger = old
            self.ledger.path = self._ledger_path()  # continue the chain in this run's out_dir
            self.ledger.rewrite()

    @torch.no_grad()
    def _load_resume_state(self, st: dict):
        if int(st["world"]) != self.rt.world:
            raise ValueError(f"resume state is for world {st['world']}, this run has {self.rt.world}")
        ops.rng.global_rng().load_state(st["rng"])
        for c, v in st["client_rng"].items():
            self.client_rng[int(c)] = dict(v)
        for c, t in st["client_master"].items():
            self.client_master[int(c)].copy_(t)
            if int(c) in self.client_param:
                ops.cast_copy_(self.client_param[int(c)], self.client_master[int(c)])
        self.flat.load_master(st["master"].to(self.device))
        for c, o in st["client_opt"].items():
            self.client_opt[int(c)] = {"m": o["m"].to(self.device), "v": o["v"].to(self.device),
                                       "step": int(o["step"])}
        if self.global_master is not None and "global_master" in st:
            self.global_master.copy_(st["global_master"])
        self.prev_verdicts = Verdicts(rejected=set(int(x) for x in st.get("prev_rejected", [])))
        self.drift.load_state_dict(st.get("drift"))
        self.outer.load_state_dict(st.get("outer"))
        self.tokens_trained = int(st.get("tokens_trained", 0))
        if self.gossip is not None and "gossip" in st:
            self.gossip.load_state_dict(st["gossip"])
