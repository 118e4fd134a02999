"""Round-complete application of the delta-exchange gossip (mixed into
:class:`bcfl.parallel.mailbox_gossip.MailboxGossip`): every source's round-T update is applied
together once the round is complete, judged first by the update anomaly filter when one is
enabled, with the SCAFFOLD corrections formed from the same round."""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from .gossip import _nullctx


class CompleteApplyMixin:
    def enable_filter(self, filt, sketch_dim: int = 8192, redistribute: str = "similar") -> None:
        """Asynchronous update anomaly filtering (round-complete delta exchange): when round T is
        complete, the receiver measures every source's round-T update ``S_j^T - S_j^applied`` (a
        signed block sketch and its norm, one fused pass, ops.update_stats), runs ``filt``
        (PageRank over the sketches' cosine graph + modified Z over the norms,
        bcfl.trust.anomaly) over the COMPLETE round, and only then applies the round without the
        rejected sources. Every receiver judges the same payloads, so every rank reaches the same
        verdicts without any collective, and a rejected update never touches an honest model."""
        if self.exchange != "delta" or self.apply_mode != "complete":
            raise ValueError("in-gossip anomaly filtering needs the round-complete delta exchange")
        self.filter = filt
        self.sketch_dim = int(sketch_dim)
        self.redistribute = redistribute
        self._redis = {}

    def take_verdicts(self) -> List[tuple]:
        """(round, rejected sources) of every application since the last call."""
        out, self.verdict_log = self.verdict_log, []
        return out

    @torch.no_grad()
    def _judge(self, T: int, src: Dict[int, tuple]) -> set:
        """Verdicts on complete round T before it is applied (host read of the statistics)."""
        js = sorted(src)
        n = self.numel
        if len(js) < int(getattr(self.filter, "min_clients", 4)):
            self.verdict_log.append((T, []))
            return set()
        rows = []
        for j in js:
            sk, nr = ops.update_stats(src[j][0][:n], self.replica[j][:n], self.sketch_dim)
            rows.append(torch.cat([sk.float(), nr.float().reshape(1)]))
        a = torch.stack(rows).cpu().double().numpy()
        v = self.filter(a[:, :-1], a[:, -1])
        rej = {js[i] for i in v.rejected}
        # where a rejected source's share goes (_row): to the accepted sources its FIRST rejected
        # update pointed like (sketch cosine, clamped at 0) — on label shards its class-mates, so
        # the accepted updates stay class-balanced (re-normalising uniformly left 3 vs 4 clients
        # per class and a federation stuck at the majority rate); uniformly when nothing points
        # its way. The map is kept: later updates of a rejected client carry the drift
        # correction towards the other classes and no longer point at its class-mates. An
        # attacker can only move its own share among honest clients.
        if rej and self.redistribute == "similar":
            sk = a[:, :-1]
            nrm = np.linalg.norm(sk, axis=1)
            nrm[nrm == 0] = 1.0
            u = sk / nrm[:, None]
            for i in v.rejected:
                if js[i] in self._redis:
                    continue   # the map of the first round a source was rejected in is kept
                self._redis[js[i]] = {js[k]: max(0.0, float(u[i] @ u[k]))
                                      for k in range(len(js)) if js[k] not in rej}
        for i, j in enumerate(js):
            self.records.append({"client": j, "kind": "verdict", "round": int(T),
                                 "ok": j not in rej, "reason": v.reasons.get(i, ""),
                                 "norm": float(a[i, -1])})
        self.verdict_log.append((T, sorted(rej)))
        return rej

    def _row(self, c: int, js, rej: set, scaled: bool = True) -> tuple:
        """Client c's application weights over the sources ``js`` (those whose update or control
        variate is applied): W_cj re-normalised so that they carry client c's WHOLE row — the
        share of a rejected source, and of a source that is silent / dead / unverified, goes to
        the applied ones (FedAvg over the results that arrived, Flower accept_failures; a rejected
        client's own row re-averages the honest updates, mixing_matrix semantics) — times
        apply_scale. Without the re-normalisation a missing source acts as a zero update and, in
        the SCAFFOLD correction, as a zero control variate: the corrections then no longer sum to
        zero over the clients and on label shards the remainder is a class bias (tiny-bert, 8
        clients, one silent: the federation never left the majority rate)."""
        W = self.W_mid
        full = sum(float(W[c, j]) for j in self.sources)
        ws = [0.0 if j in rej else float(W[c, j]) for j in js]
        red = getattr(self, "_redis", {})
        for r in rej:
            sims = red.get(r)
            share = float(W[c, r])
            if share > 0 and sims:
                tot = sum(sims.get(j, 0.0) for j in js if j not in rej)
                if tot > 0:
                    ws = [w + (share * sims.get(j, 0.0) / tot if j not in rej else 0.0)
                          for w, j in zip(ws, js)]
        keep = sum(ws)
        f = full / keep if keep > 0 else 0.0
        a = (self.apply_scale if scaled else 1.0) * f
        return tuple(w * a for w in ws)

    def _complete_behind(self) -> bool:
        """Has every live source already posted a round newer than the one applied?"""
        seen = self.seen_round
        live = [j for j in self.sources if self._last_round - seen[j] <= self.liveness_timeout]
        return bool(live) and min(seen[j] for j in live) > self.applied_T

    def _gate(self, remote_rounds: Dict[int, int]) -> Optional[int]:
        """Newest round every live source has posted (``None``: not newer than the one applied).
        A source silent for more than ``liveness_timeout`` rounds stops holding rounds back."""
        seen = self.seen_round
        for j, rr in remote_rounds.items():
            if rr > seen.get(j, -1):
                seen[j] = rr
        if not self.virtual:
            for c in self.local:
                if c not in self.suppressed:
                    seen[c] = max(seen[c], max(r for _, r in self.slot_meta[c]))
        live = [j for j in self.sources if self._last_round - seen[j] <= self.liveness_timeout]
        if not live:
            return None
        # one complete round per application: every round's control variates then form that
        # round's corrections (round-tagged SCAFFOLD, fl/drift.py), also when a burst of posts
        # completes several rounds at once (the next poll applies the next one)
        T = min(min(seen[j] for j in live), self.applied_T + 1)
        return T if T > self.applied_T else None

    def _local_sources(self, T: int) -> Dict[int, tuple]:
        """Hosted clients as sources (not virtual): the send slot of each one's newest post of a
        round <= T (read in place)."""
        out = {}
        if self.virtual:
            return out
        from .mailbox import Snapshot
        for c in self.local:
            cand = [(s, v, r) for s, (v, r) in enumerate(self.slot_meta[c])
                    if v > self.applied[c] and r >= 0]
            if not cand:
                continue
            ok = [x for x in cand if x[2] <= T]
            s_, v, r = max(ok, key=lambda x: x[1]) if ok else min(cand, key=lambda x: x[1])
            out[c] = (self.send_buf[c][s_], Snapshot(v, r, 0, 0, b""))
        return out

    @torch.no_grad()
    def _poll_complete(self, streams, param_out) -> int:
        tr = self.transport
        h = self._inflight
        if h is None:
            md = getattr(self, "_mix_done", None)
            remote = [j for j in self.remote_needed]
            if not remote:   # every source hosted here: the gate decides without a fetch
                T = self._gate({})
                return 0 if T is None else self._apply_complete(T, {}, None, streams, param_out)
            self._inflight = tr.fetch_begin(self._want(remote), self.stage,
                                            after=self._apply_events + ([md] if md is not None else []),
                                            gate=self._gate)
            self._apply_events = []
            h = self._inflight
        res = tr.fetch_advance(h, self._hash if self.verify else None)
        if res is None:
            return 0
        self._inflight = None
        if h.gate_round is None:
            return 0
        return self._apply_complete(h.gate_round, res, h, streams, param_out)

    def _verified(self, res, h) -> Dict[int, object]:
        good = {}
        for j, snap in res.items():
            ok = True
            if self.verify:
                got = h.roots.get(j) if h is not None else None
                if got is None:
                    got = ops.root_bytes(ops.merkle_root_deferred(self.stage[j]))
                ok = got == snap.root
            self.records.append({"client": j, "kind": "recv", "version": snap.version,
                                 "root": snap.root.hex(), "ok": ok, "src_round": snap.round})
            if not ok:
                self._reject(j, snap.version)
                continue
            good[j] = snap
        return good

    def _scratch(self, name: str) -> torch.Tensor:
        t = getattr(self, name, None)
        if t is None:
            t = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            setattr(self, name, t)
        return t

    @torch.no_grad()
    def _apply_complete(self, T: int, res, h, streams, param_out) -> int:
        """Apply every source's progress up to round T to every hosted client: model (and its
        compute-dtype copy), round-start record when its round has begun, then the drift
        correction's control variates from the same round.

        Hosted clients with the same mixing row (every client on a complete graph with average
        mixing) share one update ``D = sum_j W_cj (S_j^T - S_j^applied)``: it is formed once (one
        pass over the sources' snapshots) and added to each client's model in one fused pass."""
        good = self._verified(res, h) if res else {}
        src = {j: (self.stage[j], snap) for j, snap in good.items()}
        src.update(self._local_sources(T))
        n, W = self.numel, self.W_mid
        cuda = self.transport.is_cuda
        main = torch.cuda.current_stream(self.device) if cuda else None
        if cuda and h is not None and h.done_event is not None:
            main.wait_event(h.done_event)
        self._rej = self._judge(T, src) if (self.filter is not None and src) else set()
        groups: Dict[tuple, List[int]] = {}
        for c in self.local:
            row = self._row(c, list(src), self._rej)
            if any(w != 0.0 for w in row):
                groups.setdefault(row, []).append(c)
        evs = []
        for row, cs in groups.items():
            views, ws = [], []
            for (j, (buf, _snap)), w in zip(src.items(), row):
                if w != 0.0:
                    views += [buf[:n], self.replica[j][:n]]
                    ws += [w, -w]
            shared = len(cs) > 1
            if shared:   # D once, on the current stream (after the fetch)
                D_ = self._scratch("_delta")
                ops.gossip_mix_(D_, views, 0.0, ws)
            ready = torch.cuda.Event() if cuda else None
            if cuda:
                ready.record(main)
            for c in cs:
                st = (streams or {}).get(c) if cuda else None
                cur = st if st is not None else main
                with (torch.cuda.stream(cur) if cuda else _nullctx()):
                    if cuda and cur is not main:
                        cur.wait_event(ready)
                    if shared:
                        ops.gossip_mix_(self.states[c], [D_], 1.0, [1.0], (param_out or {}).get(c))
                        if c in self._started:
                            ops.axpby_(self.start[c], D_, 1.0, 1.0)
                    else:
                        ops.gossip_mix_(self.states[c], views, 1.0, ws, (param_out or {}).get(c))
                        if c in self._started:
                            ops.gossip_mix_(self.start[c], views, 1.0, ws)
                    if cuda and cur is not main:
                        ev = torch.cuda.Event()
                        ev.record(cur)
                        evs.append(ev)
            if cuda:   # the shared D (and the old replicas) are free only after every reader
                for ev in evs:
                    main.wait_event(ev)
                evs = []
        # the applied snapshots become the replicas (remote: buffer swap; hosted: a copy)
        for j, (buf, snap) in src.items():
            if j in self.stage and buf is self.stage[j]:
                self.replica[j], self.stage[j] = self.stage[j], self.replica[j]
            else:
                self.replica[j].copy_(buf)
            self.applied[j] = snap.version
            self.replica_round[j] = snap.round
        self.applied_T = T
        self.applied_mid += len(src)
        self._refresh_aux(streams, main if cuda else None)
        if cuda:   # the next fetch may overwrite stage[] (the old replicas) only after all this
            ev = torch.cuda.Event()
            ev.record(main)
            self._apply_events.append(ev)
        return len(src)

    @torch.no_grad()
    def _refresh_aux(self, streams, main) -> None:
        """Drift correction from the applied round: d_c = sum_j W_cj c_j^T - c_c^T (the
        sources' control variates as held in the replicas); with a shared mixing row the
        federation's c_hat = sum_j W_cj c_j^T is formed once."""
        if self.aux is None or self.aux_sink is None:
            return
        n, W = self.numel, self.W_mid
        live = [j for j in self.sources if self.applied[j] > 0]
        rej = self._rej & set(live)
        groups: Dict[tuple, List[int]] = {}
        for c in self.local:
            # a source rejected in this round contributes no control variate either (a scaled
            # update carries a scaled one); its weight goes to the accepted sources
            row = self._row(c, live, rej, scaled=False)
            groups.setdefault(row, []).append(c)
        for row, cs in groups.items():
            views = [self.replica[j][n:] for j, w in zip(live, row) if w != 0.0]
            ws = [w for w in row if w != 0.0]
            shared = len(cs) > 1
            if shared:
                chat = self._scratch("_chat")
                ops.gossip_mix_(chat, views, 0.0, ws)
            done = torch.cuda.Event() if main is not None else None
            if done is not None:
                done.record(main)     # the replica copies (and c_hat)
            evs = []
            for c in cs:
                own = self.replica[c][n:] if c in self.replica and self.applied.get(c, 0) > 0 else None
                st = (streams or {}).get(c) if main is not None else None
                cur = st if st is not None else main
                with (torch.cuda.stream(cur) if main is not None else _nullctx()):
                    if done is not None and cur is not main:
                        cur.wait_event(done)
                    if shared:
                        vs, wv = [chat], [1.0]
                    else:
                        vs, wv = list(views), list(ws)
                    if own is not None:
                        vs.append(own)
                        wv.append(-1.0)
                    self.aux_sink.set_correction(c, vs, wv, self.applied_T)
                    if main is not None and cur is not main:
                        ev = torch.cuda.Event()
                        ev.record(cur)
                        evs.append(ev)
            if main is not None:   # c_hat is rewritten by the next group / application
                for ev in evs:
                    main.wait_event(ev)

    @torch.no_grad()
    def _collect_complete(self, param_out) -> Optional[int]:
        tr = self.transport
        md = getattr(self, "_mix_done", None)
        if not self.remote_needed:
            T = self._gate({})
            if T is not None:
                self._apply_complete(T, {}, None, None, param_out)
            return T
        h = tr.fetch_begin(self._want(self.remote_needed), self.stage,
                           after=self._apply_events + ([md] if md is not None else []),
                           gate=self._gate)
        self._apply_events = []
        res = tr.fetch_wait(h, self._hash if self.verify else None)
        if h.gate_round is not None:
            self._apply_complete(h.gate_round, res, h, None, param_out)
        return h.gate_round

    @torch.no_grad()
    def _end_complete(self, round_idx: int, W: np.ndarray, param_out, steps) -> Dict[str, float]:
        b0 = self.transport.bytes_posted
        if self._inflight is not None:   # a mid-round fetch: complete and apply it first
            h, self._inflight = self._inflight, None
            res = self.transport.fetch_wait(h, self._hash if self.verify else None)
            if h.gate_round is not None:
                self._apply_complete(h.gate_round, res, h, None, param_out)
        self.publish(round_idx, steps, param_out)   # start[c] <- u_c (own progress of the round)
        self._last_round = round_idx
        for c in self.local:             # own progress waits for its round to complete
            if c in self._fused:         # (already retracted by the fused round-end pass)
                continue
            ops.gossip_mix_(self.states[c], [self.start[c]], 1.0, [-1.0], (param_out or {}).get(c))
        tr = self.transport
        # apply every round that is complete by now (one per collect: each round's control
        # variates form that round's corrections), so a rank that fell behind catches up
        for _ in range(4):
            if self._collect_complete(param_out) is None or not self._complete_behind():
                break
        t0 = time.perf_counter()
        waited = 0.0
        if (self.final_round is not None and round_idx >= self.final_round
                and self.applied_T < round_idx):
            # the run's last round closes synchronously: wait (bounded) until every live
            # source's last post has landed, so the final models hold every trained update
            while self.applied_T < round_idx and time.perf_counter() - t0 < self.final_timeout_s:
                if self.virtual:
                    tr.tick(tr.lag[1] + 1)     # in-process: the in-flight posts land now
                if self._collect_complete(param_out) is None and not self.virtual:
                    time.sleep(0.002)
            waited = time.perf_counter() - t0
        self.torn = tr.torn
        # dead: silent for more than liveness_timeout rounds, or posting only versions that fail
        # verification (a tampering neighbour: nothing of it accepted for that long)
        self.dead = {j for j in self.sources
                     if j not in self.local and (
                         round_idx - self.seen_round[j] > self.liveness_timeout
                         or (self.rejected_version[j] > self.applied[j]
                             and round_idx - self.replica_round[j] > self.liveness_timeout))}
        if tr.is_cuda:
            self._mix_done = torch.cuda.Event()
            self._mix_done.record(torch.cuda.current_stream(self.device))
        lag = float(round_idx - self.applied_T)
        ages = [round_idx - self.seen_round[j] for j in self.remote_needed if j not in self.dead]
        return {"mixed": 1.0, "stale_rounds": lag, "stale_max": lag,
                "post_lag_rounds": float(np.mean(ages)) if ages else 0.0,
                "applied_round": float(self.applied_T), "wait_s": 0.0, "final_wait_s": waited,
                "bytes_sent": float(tr.bytes_posted - b0),
                "dead_peers": float(len(self.dead)), "torn": float(self.torn),
                "rejected_msgs": float(self.rejected_msgs)}

    @torch.no_grad()
    def _fused_round_end(self, c: int) -> bool:
        """Round-complete delta exchange: client c's round end runs as ONE pass
        (ops.delta_round_end_: u, S, wire image, new control variate, own-progress retraction)."""
        return (self.fuse_round_end and self.exchange == "delta" and self.apply_mode == "complete"
                and c not in self.suppressed and c not in self.tamper
                and (self.aux is None or getattr(self.aux_sink, "defer_cv", False)))
