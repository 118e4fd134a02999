"""Truly asynchronous serverless gossip over one-sided peer mailboxes (split out of
:mod:`bcfl.parallel.gossip`): publish / fetch / verify, application on arrival, state and
delta mixing; the round-complete application lives in :mod:`bcfl.parallel.gossip_complete`."""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from . import dist as D
from .topology import client_rank
from .gossip import GossipEngine, _nullctx, _portable_records
from .gossip_complete import CompleteApplyMixin


class MailboxGossip(CompleteApplyMixin):
    """Truly asynchronous serverless gossip over one-sided peer mailboxes
    (:mod:`bcfl.parallel.mailbox`): no matched receive, no round lock-step.

    Per round, for every hosted client c (not suppressed):

    1. **publish** — version += 1; encode x_c for the wire into send slot ``version % 2``
       (``fp32`` or ``bf16`` full snapshot: a lossy mailbox cannot carry an error-feedback delta
       chain, a receiver may skip versions), hash it on the GPU (SHA-256 Merkle root = the
       sender's ledger commitment), and **post** it to every destination rank's inbox on side
       streams — the copies run over xGMI under the next round's training.
    2. **fetch** — for every remote neighbour, take whatever complete snapshot is newest in its
       inbox (skip if none is newer than the one held); re-hash and compare with the committed
       root, keep it only if they match.
    3. **mix** — x_c <- W_cc x_c + sum_j W_cj view_j with the freshest verified view of each
       neighbour; a neighbour whose newest snapshot is older than ``liveness_timeout`` rounds
       (slow, stopped or exited) is treated as dead and its weight folds into c's self-weight.

    ``sync=True`` turns step 2 into a bounded wait: poll until every live neighbour has published
    round r (or ``sync_timeout_s`` passes and it is declared dead) — lock-step semantics without
    any matched transfer, for the sync-vs-async comparison.

    ``exchange="delta"`` (complete topologies, asynchronous FedAvg semantics): instead of its
    model state, every client publishes the CUMULATIVE sum of its own local updates,
    ``S_c = sum_r (y_c^r - x_c^r)``, and a receiver adds each neighbour's NEW progress
    ``S_j^new - S_j^applied`` exactly once: ``x_c <- y_c - (1 - W_cc) u_c + sum_j W_cj dS_j``.
    A stale snapshot then only delays a neighbour's update by a round — it never pulls the mix
    back to an old state, which is what state mixing with stale snapshots does (2 / 4 ranks on
    one MI355X stayed at the majority rate, profiles/multirank_async_r4.json). Under exact
    same-round mixing both forms give the reference's mean of the trained models. Lost, torn or
    rejected versions are harmless: the next good snapshot's difference covers them, and the
    bf16 rounding of ``S_j`` telescopes (only the newest snapshot's rounding is ever present).

    ``aux`` (optional, per hosted client, fp32, same size as the model): a second state published
    in the SAME payload (``[model | aux]``, one version, one header, one Merkle commitment) — the
    clients' SCAFFOLD control variates (:mod:`bcfl.fl.drift`, exchange mode). ``aux_sink`` (the
    drift correction) gets, per hosted client and BEFORE the model mix,
    ``begin(c, self_w, views, weights, age)`` with the neighbours' aux halves, the live mixing
    weights and the mix's staleness ``age = sum_j W_cj * (rounds the view of j is behind)``; it
    may return extra ``[(tensor, weight)]`` terms for client c's model mix (staleness
    compensation); ``end(c)`` runs after the mix.
    """

    def __init__(self, num_clients: int, states: Dict[int, torch.Tensor], nbrs: Dict[int, List[int]],
                 wire: str = "bf16", sync: bool = False, liveness_timeout: int = 2,
                 verify: bool = True, sync_timeout_s: float = 60.0, rank: Optional[int] = None,
                 world: Optional[int] = None, aux: Optional[Dict[int, torch.Tensor]] = None,
                 aux_sink=None, exchange: str = "state", apply: str = "arrival",
                 virtual: bool = False, lag_steps=(1, 1), seed: int = 0,
                 source_lag: Optional[Dict[int, int]] = None):
        from .mailbox import MailboxTransport
        rt = D.runtime()
        self.rank = rt.rank if rank is None else rank
        self.world = rt.world if world is None else world
        self.n = num_clients
        self.states = states
        self.local = sorted(states)
        self.nbrs = nbrs
        if wire in ("bf16_delta", "bf16"):
            wire = "bf16"
        if wire not in ("bf16", "fp32"):
            raise ValueError(f"mailbox gossip carries full snapshots: wire must be bf16 or fp32, got {wire!r}")
        self.wire = wire
        self.async_gossip = not sync
        self.sync_timeout_s = sync_timeout_s
        self.verify = verify
        any_state = next(iter(states.values()))
        self.numel, self.device = any_state.numel(), any_state.device
        self.aux = aux
        self.aux_sink = aux_sink
        if aux is not None and sorted(aux) != self.local:
            raise ValueError("aux states must cover exactly the hosted clients")
        self.msg_numel = self.numel * (2 if aux is not None else 1)
        self.wire_dtype = torch.float32 if wire == "fp32" else torch.bfloat16
        if apply not in ("arrival", "complete"):
            raise ValueError(f"apply must be 'arrival' or 'complete', got {apply!r}")
        if apply == "complete" and exchange != "delta":
            raise ValueError("round-complete application applies cumulative updates (exchange='delta')")
        self.apply_mode = apply
        # virtual ranks (in-process loopback transport): every hosted client is its own rank, so
        # every OTHER client is remote to it — updates arrive late, through the transport
        self.virtual = bool(virtual)
        complete = apply == "complete"
        if self.virtual:
            self.remote_needed = sorted({j for c in self.local for j in nbrs[c]}
                                        | (set(self.local) if complete else set()))
        else:
            self.remote_needed = sorted({j for c in self.local for j in nbrs[c]
                                         if client_rank(j, self.world) != self.rank})
        send_plan = []
        for c in self.local:
            dsts = sorted({client_rank(i, self.world) for i in range(self.n) if c in nbrs[i]}
                          - {self.rank})
            send_plan += [(c, r) for r in dsts]
        if self.virtual:
            from .loopback import LoopbackTransport
            self.transport = LoopbackTransport(self.msg_numel, self.wire_dtype, self.device,
                                               self.local, lag_steps, seed, source_lag)
        else:
            self.transport = MailboxTransport(self.msg_numel, self.wire_dtype, self.device,
                                              self.remote_needed, send_plan, self.rank, self.world)
        z = lambda: torch.zeros(self.msg_numel, dtype=self.wire_dtype, device=self.device)  # noqa: E731
        self.send_buf = {c: [z(), z()] for c in self.local}
        self.replica = {j: z() for j in self.remote_needed}
        self.stage = {j: z() for j in self.remote_needed}
        # round-complete application: every source's applied snapshot is held in a replica, the
        # hosted clients' own posts included (their send slots are read where they are)
        self.sources = sorted(set(self.remote_needed) | (set(self.local) if complete else set()))
        if complete:
            for c in self.local:
                if c not in self.replica:
                    self.replica[c] = z()
        self.apply_scale = 1.0   # delta exchange: fraction of the federation's mean update applied
        self.final_round: Optional[int] = None   # complete mode: this round closes synchronously
        self.final_timeout_s = 30.0
        self.applied_T = -1                                  # newest round applied everywhere
        self.seen_round = {j: -1 for j in self.sources}      # newest round each source posted
        self.slot_meta = {c: [(0, -1), (0, -1)] for c in self.local}   # (version, round) per slot
        self._last_round = -1
        self.liveness_timeout = liveness_timeout
        self.version = {c: 0 for c in self.local}
        self.steps = {c: 0 for c in self.local}
        self.applied = {j: 0 for j in self.sources}           # version held in replica[j]
        # newest version of each source that failed verification: never fetched (or ledgered)
        # again — a tampering neighbour costs one re-hash per version, not one per local step
        self.rejected_version = {j: 0 for j in self.sources}
        self.replica_round = {j: -1 for j in self.sources}
        self.suppressed: set = set()
        self.tamper: set = set()     # fault injection: corrupt these clients' payloads after hashing
        self.dead: set = set()
        self.torn = 0
        self.rejected_msgs = 0
        self.records: List[dict] = []  # ledger records of this round (published + verified)
        self._round_local = -1
        self.wait_s = 0.0              # host time spent waiting for peers (sync mode only)
        self.stale_decay = 0.0         # see _age_weighted
        if exchange not in ("state", "delta"):
            raise ValueError(f"exchange must be 'state' or 'delta', got {exchange!r}")
        self.exchange = exchange
        self._fresh: Dict[int, object] = {}
        if exchange == "delta":
            f32 = lambda: torch.zeros(self.numel, dtype=torch.float32, device=self.device)  # noqa: E731
            self.start = {c: f32() for c in self.local}   # round-start model, then u_c
            self.cum = {c: f32() for c in self.local}     # S_c, the published quantity
        # apply on arrival (delta exchange, async): mixing weights for mid-round application,
        # the in-flight non-blocking fetch, the events of the last applications (the next fetch
        # may overwrite the buffers they read only after them), hosted clients whose round began
        self.apply_on_arrival = exchange == "delta" and not sync
        self._also = None              # callback c -> extra buffers updated with mid-round deltas
        self.W_mid: Optional[np.ndarray] = None
        self._inflight = None
        self._apply_events: List = []
        self._started: set = set()
        self.applied_mid = 0
        self.pend: Optional[Dict[int, torch.Tensor]] = None   # see enable_self_delay
        self._fused: set = set()       # clients whose round end ran as one fused pass
        self._start_live: set = set()  # ... whose start record still equals the live model
        self.fuse_round_end = True     # False: the separate passes (tests compare the two)
        # round-complete mode: the update anomaly filter runs INSIDE the application — every
        # complete round's updates are judged by the receiver before any of them is applied
        # (enable_filter); a rejected source's round is skipped (its replica still advances, so
        # the update is never applied later) and the others' weights are re-normalised
        self.filter = None
        self.sketch_dim = 8192
        self.verdict_log: List[tuple] = []   # (round T, sorted rejected sources) per application
        self._rej: set = set()               # sources rejected in the newest application

    def enable_self_delay(self) -> None:
        """Delta exchange: this rank's OWN updates (every hosted client's u_c of round r) enter
        the hosted models one round late, at the round-(r + 1) mix — about when the remote
        neighbours' round-r updates, fetched and applied during round r + 1, have landed. Every
        model then holds (nearly) complete rounds of updates. Without it a model holds its own
        latest update a round before the others' of the same round: on label shards that is a
        tilt toward its own class that the same round's opposite-class updates have not yet
        cancelled, and on a weak early signal it decides the model's predictions."""
        if self.exchange != "delta":
            raise ValueError("self delay applies to the delta exchange")
        self.pend = {c: torch.zeros(self.numel, dtype=torch.float32, device=self.device)
                     for c in self.local}

    # ------------------------------------------------------------------------------------
    def seed_replicas(self, initial: torch.Tensor):
        """Every client starts from the identical initial model, so every replica (version 0)
        starts equal to it: a neighbour that never publishes is mixed as the initial model until
        the staleness bound retires it (delta exchange: version 0 = no progress, S = 0). Aux
        halves (control variates) start at zero."""
        n = self.numel
        for t in list(self.replica.values()) + [b for c in self.local for b in self.send_buf[c]]:
            if self.exchange == "delta":
                t[:n].zero_()
            else:
                ops.cast_copy_(t[:n], initial)
            if self.aux is not None:
                t[n:].zero_()
        if self.exchange == "delta":
            for c in self.local:
                self.cum[c].zero_()

    def mark_start(self, c: int, x: torch.Tensor) -> None:
        """Delta exchange: record hosted client c's round-start model (stream-ordered before its
        first optimizer step); its update u_c = y_c - x_c is formed at publish."""
        if self.exchange == "delta":
            if c in self._start_live:   # the fused round end left start == model, and every
                self._start_live.discard(c)   # application since went to both: nothing to copy
            else:
                self.start[c].copy_(x)
            self._started.add(c)

    # ---- apply on arrival ---------------------------------------------------------------------
    def _want(self, js) -> Dict[int, int]:
        """Fetch only versions newer than both the applied and the last rejected one."""
        return {j: max(self.applied[j], self.rejected_version[j]) for j in js}

    def _reject(self, j: int, version: int) -> None:
        self.rejected_msgs += 1
        self.rejected_version[j] = max(self.rejected_version[j], int(version))

    def _hash(self, t: torch.Tensor):
        return ops.merkle_root_deferred(t)

    @torch.no_grad()
    def poll(self, streams: Optional[Dict[int, object]] = None,
             param_out: Optional[Dict[int, torch.Tensor]] = None, also=None) -> int:
        """Asynchronous gossip overlapped with local training (delta exchange): NON-BLOCKING.
        Advances the in-flight fetch by one step (header read -> payload copy, seqlock re-read
        and receiver re-hash on the fetch stream -> host checks, each step only an event query);
        when its snapshots are complete and verified, every hosted client c gets each fresh
        neighbour's new progress ``W_cj (S_j^new - S_j^applied)`` added to its model (on c's own
        lane stream, after the fetch; ``param_out[c]`` refreshed in the same kernel), to its
        round-start record if its round has begun (u_c stays its own progress) and to the
        buffers ``also(c)`` returns; then the next fetch starts. Called between local steps, so
        a neighbour's update enters a round or more earlier than at the round's end mix.
        Returns the number of snapshots applied."""
        tr = self.transport
        if self.virtual:
            tr.tick()                 # one local step of every lane: the in-process clock
        if not (self.apply_on_arrival and self.sources) or self.W_mid is None:
            return 0
        if self.apply_mode == "complete":
            return self._poll_complete(streams, param_out)
        h = self._inflight
        if h is None:
            md = getattr(self, "_mix_done", None)   # the round-end mix read stage / replica too
            self._inflight = tr.fetch_begin(self._want(self.remote_needed), self.stage,
                                            after=self._apply_events + ([md] if md is not None else []))
            self._apply_events = []
            h = self._inflight
        res = tr.fetch_advance(h, self._hash if self.verify else None)
        if res is None:
            return 0
        self._inflight = None
        return self._apply_fetched(res, h, streams, param_out, also)

    @torch.no_grad()
    def _finish_inflight(self, param_out=None, also=None) -> int:
        """Complete an in-flight fetch (blocking) and apply it on the current stream."""
        h, self._inflight = self._inflight, None
        if h is None:
            return 0
        res = self.transport.fetch_wait(h, self._hash if self.verify else None)
        return self._apply_fetched(res, h, None, param_out, also)

    def _apply_fetched(self, res, h, streams, param_out, also) -> int:
        if not res:
            return 0
        self.torn = self.transport.torn
        good = {}
        for j, snap in res.items():
            if self.verify:
                got = h.roots.get(j)
                if got is None:   # CPU path: the fetch was synchronous, hash here
                    got = ops.root_bytes(ops.merkle_root_deferred(self.stage[j]))
                ok = got == snap.root
            else:
                ok = True
            self.records.append({"client": j, "kind": "recv", "version": snap.version,
                                 "root": snap.root.hex(), "ok": ok, "src_round": snap.round})
            if not ok:
                self._reject(j, snap.version)
                continue
            good[j] = snap
        if not good:
            return 0
        n, W = self.numel, self.W_mid
        cuda = self.transport.is_cuda
        for c in self.local:
            views, ws, aviews = [], [], []
            for j in good:
                if W[c, j] != 0.0 and self._remote(c, j):
                    views += [self.stage[j][:n], self.replica[j][:n]]
                    wj = float(W[c, j]) * self.apply_scale
                    ws += [wj, -wj]
                    if self.aux is not None:
                        aviews += [self.stage[j][n:], self.replica[j][n:]]
            if not views:
                continue
            st = (streams or {}).get(c) if cuda else None
            cur = st if st is not None else (torch.cuda.current_stream(self.device) if cuda else None)
            with (torch.cuda.stream(cur) if cuda else _nullctx()):
                if cuda and h.done_event is not None:
                    cur.wait_event(h.done_event)
                ops.gossip_mix_(self.states[c], views, 1.0, ws, (param_out or {}).get(c))
                if c in self._started:
                    ops.gossip_mix_(self.start[c], views, 1.0, ws)
                for t, half in (also(c) if also is not None else []):
                    if half == "aux" and aviews:
                        # aux-space target (drift d_c = c_hat - c_c): the neighbour's new control
                        # variate replaces its old one in c_hat right away
                        ops.gossip_mix_(t, aviews, 1.0, ws)
                    elif half == "model":
                        ops.gossip_mix_(t, views, 1.0, ws)
                if cuda:
                    ev = torch.cuda.Event()
                    ev.record(cur)
                    self._apply_events.append(ev)
        for j, snap in good.items():
            self.replica[j], self.stage[j] = self.stage[j], self.replica[j]
            self.applied[j] = snap.version
            self.replica_round[j] = snap.round
        self.applied_mid += len(good)
        return len(good)

    # ---- round-complete application (apply="complete") ---------------------------------------
    # Every model holds COMPLETE rounds of the federation's updates: the round-T posts of every
    # live source (this rank's own clients included) are applied together, once the last of them
    # has landed, and a client's own update leaves its live model at the round end until its
    # round is complete. With label shards each post pulls towards one class; a model that holds
    # some sources' round-r updates and not others' is tilted towards whichever classes arrived
    # first (8 ranks on CU slices: 0.73-0.95 final accuracy, multirank_cu_split_r4.json). Here
    # nothing ever waits: training continues on the last complete base while a round is in
    # flight, and with every post visible at the round end the result is exactly the synchronous
    # mean (FedAvg with the reference's unweighted average, serverless_NonIID_IMDB.py:296).

    def _remote(self, c: int, j: int) -> bool:
        """Does client c receive client j's updates through the transport (late)? Hosted
        neighbours are exact and same-round, except on virtual ranks (every client its own)."""
        return j != c if self.virtual else j not in self.states

    def _msg(self, j: int, c: Optional[int] = None) -> torch.Tensor:
        if j in self.states and not (self.virtual and c is not None and j != c):
            return self.send_buf[j][self.version[j] % 2]
        return self.replica[j]

    def view(self, j: int) -> torch.Tensor:
        """Newest verified model of client j (the model half of its message)."""
        return self._msg(j)[: self.numel]

    def aux_view(self, j: int, c: Optional[int] = None) -> torch.Tensor:
        """Newest verified aux state (control variate) of client j as receiver c holds it, same
        version as :meth:`view` (delta exchange: a snapshot fetched this round is still in the
        staging buffer)."""
        if j in self._fresh:
            return self.stage[j][self.numel:]
        return self._msg(j, c)[self.numel:]

    def publish(self, round_idx: int, steps: Optional[Dict[int, int]] = None,
                param_out: Optional[Dict[int, torch.Tensor]] = None):
        from .mailbox import Snapshot
        roots = {}
        self._fused = set()
        if self.exchange == "delta":
            defer = self.aux is not None and getattr(self.aux_sink, "defer_cv", False)
            for c in self.local:   # u_c = y_c - x_c (in place), S_c += u_c
                if self._fused_round_end(c):
                    continue
                terms = self.aux_sink.round_end_terms(c) if defer else None
                if terms is not None:   # the deferred control variate (x - y) / L - s d
                    d, sc, inv_l = terms
                    ops.gossip_mix_(self.aux[c], [self.start[c], self.states[c]], 0.0, [inv_l, -inv_l])
                    if d is not None:
                        ops.axpby_(self.aux[c], d, -sc, 1.0)
                ops.axpby_(self.start[c], self.states[c], 1.0, -1.0)
                ops.axpby_(self.cum[c], self.start[c], 1.0, 1.0)
            self._started = set()
        for c in self.local:
            if c in self.suppressed:
                continue
            self.version[c] += 1
            self.steps[c] += int((steps or {}).get(c, 0))
            slot = self.version[c] % 2
            if self.transport.is_cuda:
                self.transport.wait_slot_free(c, slot)
            buf = self.send_buf[c][slot]
            if self._fused_round_end(c):
                terms = self.aux_sink.round_end_terms(c) if self.aux is not None else None
                d, sc, inv_l = terms if terms is not None else (None, 0.0, 0.0)
                cv = self.aux[c] if self.aux is not None else None
                if cv is not None and terms is None:   # untrained client: its cv stands
                    ops.cast_copy_(buf[self.numel:], cv)
                    cv = None
                ops.delta_round_end_(self.states[c], self.start[c], self.cum[c],
                                     buf if cv is not None else buf[: self.numel],
                                     (param_out or {}).get(c), d, cv, inv_l, sc)
                self._fused.add(c)
                # model == start again: applications until the next round start go to both
                self._started.add(c)
                self._start_live.add(c)
            else:
                ops.cast_copy_(buf[: self.numel],
                               self.cum[c] if self.exchange == "delta" else self.states[c])
                if self.aux is not None:
                    ops.cast_copy_(buf[self.numel:], self.aux[c])
            self.slot_meta[c][slot] = (self.version[c], round_idx)
            roots[c] = ops.merkle_root_deferred(buf) if self.verify else None
            if c in self.tamper:  # in-flight corruption AFTER the commitment was computed
                buf.view(-1)[: min(64, buf.numel())].add_(1.0)
            snap = Snapshot(self.version[c], round_idx, self.steps[c], buf.numel() * buf.element_size(),
                            b"\0" * 32)
            rd = roots[c]
            if rd is not None and not torch.is_tensor(rd):
                snap.root = bytes(rd)
                rd = None
            self.transport.post(c, buf, snap, rd)
        for c, rd in roots.items():
            self.records.append({"client": c, "kind": "update", "version": self.version[c],
                                 "root_t": rd})

    @torch.no_grad()
    def collect(self, round_idx: int):
        """Fetch every newer complete snapshot (sync: wait for round ``round_idx``), verify its
        Merkle root against the sender's commitment, adopt the good ones."""
        import time as _time
        want = self._want(self.remote_needed)
        tr = self.transport
        fs = tr.fetch_stream  # GPU: the whole receive path runs on the transport's side stream
        after = getattr(self, "_mix_done", None)
        if fs is not None:
            for ev in self._apply_events:   # mid-round applications read stage / replica
                fs.wait_event(ev)
            self._apply_events = []
        got = tr.fetch(want, self.stage, after=after)
        if not self.async_gossip:
            t0 = _time.perf_counter()
            need = {j for j in self.remote_needed if j not in self.dead}
            have = {j for j, s in got.items() if s.round >= round_idx}
            if not hasattr(self, "scratch"):
                self.scratch = {j: torch.empty_like(self.stage[j]) for j in self.remote_needed}
            while need - have and _time.perf_counter() - t0 < self.sync_timeout_s:
                _time.sleep(0.0005)
                # re-fetch into scratch buffers: a torn re-fetch must not overwrite the complete
                # snapshot already staged for j (got[j] keeps describing stage[j])
                more = tr.fetch({j: max(self.applied[j], got[j].version if j in got else 0)
                                 for j in need - have}, self.scratch)
                for j in more:
                    self.stage[j], self.scratch[j] = self.scratch[j], self.stage[j]
                got.update(more)
                have |= {j for j, s in more.items() if s.round >= round_idx}
            self.wait_s += _time.perf_counter() - t0
        self.torn = tr.torn
        ok = {}
        if got and self.verify:
            # re-hash on the fetch stream: the root readback waits only for this stream
            with (torch.cuda.stream(fs) if fs is not None else _nullctx()):
                roots = {j: ops.merkle_root_deferred(self.stage[j]) for j in got}
                for j, rt in roots.items():
                    ok[j] = ops.root_bytes(rt) == got[j].root
        for j, snap in got.items():
            good = ok.get(j, True)
            self.records.append({"client": j, "kind": "recv", "version": snap.version,
                                 "root": snap.root.hex(), "ok": good, "src_round": snap.round})
            if not good:
                self._reject(j, snap.version)
                continue
            if self.exchange == "delta":
                self._fresh[j] = snap   # applied (S_new - S_applied) by the mix, then swapped
            else:
                self.replica[j], self.stage[j] = self.stage[j], self.replica[j]
            self.applied[j] = snap.version
            self.replica_round[j] = snap.round

    def _age_out(self, round_idx: int):
        for j in self.remote_needed:
            if round_idx - self.replica_round[j] > self.liveness_timeout:
                self.dead.add(j)
            else:
                self.dead.discard(j)
        for c in self.local:  # a suppressed (dead) local client stops being fresh too
            if c in self.suppressed and round_idx > self.liveness_timeout:
                self.dead.add(c)

    def live_matrix(self, W: np.ndarray) -> np.ndarray:
        return GossipEngine.live_matrix(self, W)

    @torch.no_grad()
    def mix_delta(self, W: np.ndarray, round_idx: int,
                  param_out: Optional[Dict[int, torch.Tensor]] = None,
                  extra: Optional[Dict[int, list]] = None):
        """x_c <- y_c - (1 - W_cc) u_c + sum_{j local} W_cj u_j
                   + sum_{j remote, new snapshot} a_j W_cj (S_j^new - S_j^applied)  (one kernel)

        ``a_j = 1 / (1 + stale_decay * max(0, tau_j - 1))`` with tau_j the rounds the snapshot is
        behind: the usual one-round async lag is applied in full, updates computed on a model
        several rounds old are damped (FedAsync-style staleness weighting)."""
        n = self.numel
        damp = {}
        for j, snap in self._fresh.items():
            tau = max(0, round_idx - snap.round)
            damp[j] = 1.0 / (1.0 + self.stale_decay * max(0, tau - 1))
        own = self.pend if self.pend is not None else self.start
        for c in self.local:
            a = self.apply_scale
            if self.pend is not None:   # y_c - u_c + W_cc u_c(previous round)
                views, ws = [self.start[c], self.pend[c]], [-1.0, a * float(W[c, c])]
            else:
                views, ws = [self.start[c]], [-(1.0 - a * float(W[c, c]))]
            for j in range(self.n):
                if j == c or W[c, j] == 0.0:
                    continue
                if not self._remote(c, j):
                    views.append(own[j])
                    ws.append(a * float(W[c, j]))
                elif j in self._fresh:
                    wj = a * float(W[c, j]) * damp[j]
                    views += [self.stage[j][:n], self.replica[j][:n]]
                    ws += [wj, -wj]
            for t, wt in ((extra or {}).get(c) or []):
                views.append(t)
                ws.append(float(wt))
            ops.gossip_mix_(self.states[c], views, 1.0, ws, (param_out or {}).get(c))
        for j in list(self._fresh):   # the new snapshot becomes the applied one
            self.replica[j], self.stage[j] = self.stage[j], self.replica[j]
        self._fresh = {}
        if self.pend is not None:     # this round's own updates wait for the next mix
            for c in self.local:      # (start[c] is re-recorded at the next round's start)
                self.pend[c], self.start[c] = self.start[c], self.pend[c]

    def _age_weighted(self, W: np.ndarray, round_idx: int) -> np.ndarray:
        """``stale_decay`` > 0: a neighbour view k rounds behind keeps W_cj / (1 + decay * k) of
        its weight (the rest moves to c's self-weight), so a far-behind snapshot pulls the mix
        back less; 0 = plain mixing."""
        if self.stale_decay <= 0:
            return W
        W = W.copy()
        for c in self.local:
            for j in self.remote_needed:
                if W[c, j] == 0.0:
                    continue
                k = max(0, round_idx - self.replica_round[j])
                keep = W[c, j] / (1.0 + self.stale_decay * k)
                W[c, c] += W[c, j] - keep
                W[c, j] = keep
        return W

    _uniform_rows = GossipEngine._uniform_rows

    @torch.no_grad()
    def mix(self, W: np.ndarray, param_out: Optional[Dict[int, torch.Tensor]] = None,
            extra: Optional[Dict[int, tuple]] = None):
        return GossipEngine.mix(self, W, param_out, extra)

    def end_of_round(self, round_idx: int, W: np.ndarray,
                     param_out: Optional[Dict[int, torch.Tensor]] = None,
                     steps: Optional[Dict[int, int]] = None) -> Dict[str, float]:
        if self.apply_mode == "complete":
            return self._end_complete(round_idx, W, param_out, steps)
        b0, w0 = self.transport.bytes_posted, self.wait_s
        if self._inflight is not None:
            # the round's training is done: complete the mid-round fetch before publishing (its
            # applications must land in the clients' start records before u_c is formed)
            self._finish_inflight(param_out, self._also)
        self.publish(round_idx, steps)
        self.collect(round_idx)
        self._age_out(round_idx)
        fs = self.transport.fetch_stream
        if fs is not None:  # the mix reads what the fetch stream wrote
            torch.cuda.current_stream(self.device).wait_stream(fs)
        Wl = self.live_matrix(W)
        if self.exchange != "delta":
            Wl = self._age_weighted(Wl, round_idx)
        extra = {}
        if self.aux is not None and self.aux_sink is not None:
            for c in self.local:
                nb = [j for j in range(self.n) if j != c and Wl[c, j] != 0.0]
                age = sum(float(Wl[c, j]) * max(0, round_idx - self.replica_round[j])
                          for j in nb if self._remote(c, j))
                extra[c] = self.aux_sink.begin(c, float(Wl[c, c]), [self.aux_view(j, c) for j in nb],
                                               [float(Wl[c, j]) for j in nb], age)
        if self.exchange == "delta":
            # updates are applied once with the topology's weights (a silent neighbour simply
            # contributes no new progress); the live weights above form c_hat
            self.mix_delta(W, round_idx, param_out, extra)
        else:
            self.mix(Wl, param_out, extra)
        if self.aux is not None and self.aux_sink is not None:
            for c in self.local:
                self.aux_sink.end(c)
        if fs is not None:  # the next fetch may overwrite the buffers this mix read after this
            self._mix_done = torch.cuda.Event()
            self._mix_done.record(torch.cuda.current_stream(self.device))
        ages = [round_idx - self.replica_round[j] for j in self.remote_needed if j not in self.dead]
        return {"mixed": 1.0, "stale_rounds": float(np.mean(ages)) if ages else 0.0,
                "stale_max": float(max(ages)) if ages else 0.0,
                "wait_s": float(self.wait_s - w0),
                "bytes_sent": float(self.transport.bytes_posted - b0),
                "dead_peers": float(len(self.dead)), "torn": float(self.torn),
                "rejected_msgs": float(self.rejected_msgs)}

    def drain(self):
        if self._inflight is not None and self._inflight.done_event is not None:
            self._inflight.done_event.synchronize()   # no fetch left writing into stage[]
        self.transport.drain()

    def close(self):
        self.transport.close()

    def take_records(self) -> List[dict]:
        out, self.records = self.records, []
        if self.virtual:   # in-process receipts: nothing crossed a process, nothing to ledger
            out = [g for g in out if g["kind"] != "recv"]
        return out

    def state_dict(self) -> dict:
        """Published snapshots, verified replicas, versions and liveness. Inbox contents are NOT
        state: after a restart peers simply post again (a replica's version tells what is new)."""
        self.drain()
        self._inflight = None          # an unapplied mid-round fetch is simply fetched again
        t = lambda d: {int(k): v.detach().cpu().clone() for k, v in d.items()}  # noqa: E731
        st = {"cum": t(self.cum)} if self.exchange == "delta" else {}
        if self.pend is not None:
            st["pend"] = t(self.pend)
        return {**st,
                "send_buf": {int(c): [b.detach().cpu().clone() for b in v] for c, v in self.send_buf.items()},
                "replica": t(self.replica), "version": dict(self.version), "steps": dict(self.steps),
                "applied": dict(self.applied), "replica_round": dict(self.replica_round),
                "dead": sorted(self.dead), "rejected_msgs": self.rejected_msgs,
                "applied_T": int(self.applied_T), "last_round": int(self._last_round),
                "rejected_version": {int(k): int(v) for k, v in self.rejected_version.items()},
                "seen_round": {int(k): int(v) for k, v in self.seen_round.items()},
                "slot_meta": {int(c): [list(x) for x in m] for c, m in self.slot_meta.items()},
                "records": _portable_records(self.records),
                "redistribute": {int(r): {int(j): float(w) for j, w in m.items()}
                                 for r, m in getattr(self, "_redis", {}).items()}}

    def load_state_dict(self, st: dict):
        for c, bufs in st["send_buf"].items():
            for dst, src in zip(self.send_buf[int(c)], bufs):
                dst.copy_(src.to(dst.device))
        for j, v in st["replica"].items():
            self.replica[int(j)].copy_(v.to(self.replica[int(j)].device))
        if self.exchange == "delta" and "cum" in st:
            for c, v in st["cum"].items():
                self.cum[int(c)].copy_(v.to(self.device))
        if self.pend is not None and "pend" in st:
            for c, v in st["pend"].items():
                self.pend[int(c)].copy_(v.to(self.device))
        for name in ("version", "steps", "applied", "replica_round"):
            getattr(self, name).update({int(k): int(v) for k, v in st[name].items()})
        self.dead = set(int(x) for x in st["dead"])
        self.rejected_msgs = int(st["rejected_msgs"])
        self.records = list(st.get("records", []))
        self.applied_T = int(st.get("applied_T", -1))
        self.rejected_version.update({int(k): int(v) for k, v in st.get("rejected_version", {}).items()})
        self._last_round = int(st.get("last_round", -1))
        self.seen_round.update({int(k): int(v) for k, v in st.get("seen_round", {}).items()})
        for c, m in st.get("slot_meta", {}).items():
            self.slot_meta[int(c)] = [tuple(int(y) for y in x) for x in m]
        if st.get("redistribute"):
            self._redis = {int(r): {int(j): float(w) for j, w in m.items()}
                           for r, m in st["redistribute"].items()}
