"""The serverless round (reference C14, ``src/Serverlesscase/serverless_NonIID_IMDB.py:284-318``): one-client-at-a-time
and lane training, the asynchronous gossip's waits and polls, deferred host reads and the reference chain
(mixed into :class:`~bcfl.fl.federation.Federation`)."""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import torch

from .. import ops
from ..parallel.gossip import MailboxGossip
from ..parallel.topology import mixing_matrix, neighbours
from ..trust.anomaly import Verdicts
from .fedutil import weighted_average


class ServerlessRoundMixin:
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
            if g.apply_on_arrival:
                self._gossip_poll()   # in-process virtual ranks: every poll is one tick of the clock
            else:
                # no mid-round application (poll() is a no-op then): fetch and apply the next
                # complete round directly instead of spinning out the timeout
                if g.virtual:
                    g.transport.tick()
                g._collect_complete(self._param_out())
            if not g.virtual and g.applied_T < need:
                time.sleep(0.002)
        return time.perf_counter() - t0

    def _param_out(self) -> Optional[Dict[int, torch.Tensor]]:
        """Compute-dtype copies the gossip refreshes with every model it changes."""
        if self.lanes:
            return self.client_param
        return None if self.multi else {self.local_clients[0]: self.flat.param}

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

    def serverless_round(self, r: int) -> dict:
        cfg = self.cfg
        if cfg.compat_chain:
            return self._chain_round(r)
        recs, sk, nr, losses, local_eval = [], {}, {}, {}, {}
        need_prev = ((self.filter is not None and not self._gossip_filter)
                     or bool(cfg.inject_byzantine) or cfg.update_clip_ratio > 0)
        self._run_deferred(block=False)  # earlier rounds' host reads whose kernels have finished
        self._resolve_eval_local(block=False)   # deferred local scores that are ready
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
                if self.filter is not None and not self._gossip_filter:
                    with self.timer.phase("anomaly"):
                        sk[c], nr[c] = self._update_stats(ref)
            losses[c] = st
            if cfg.eval_local:
                with self.timer.phase("eval_local"):
                    if self._defer_local_eval():
                        self._launch_eval_local(c, r)
                    else:
                        local_eval[c] = self.trainer.evaluate_device(self.test_batches(c, r))
            root = ""
            if self.ledger is not None and not self._gossip_roots:
                # the deferred ledger (below) reads a device root when the round's tail is done;
                # a host read here would drain the GPU in front of the round's remaining launches
                root = (ops.merkle_root_deferred(self.flat.master) if self._host_deferred
                        else self._merkle())
            recs.append({"client": c, "root": root, "ts": float(r) + 0.001 * (c + 1),
                         "verdict": "accept", "metrics": {"examples": st["examples"]}})
            self._deactivate(c)
        if self._gossip_filter:
            v = Verdicts()   # judged per complete round inside the gossip (verdict blocks)
        else:
            with self.timer.phase("anomaly"):
                v = self._verdicts(sk, nr)
        for x in recs:
            x["verdict"] = v.verdict(x["client"])
        # async mixes states published last round -> apply last round's verdicts to them
        use_v = self.prev_verdicts if (cfg.async_gossip and not self.same_round_mix) else v
        W = mixing_matrix(self.nbrs, cfg.mixing, () if self._gossip_filter else use_v.rejected)
        if isinstance(self.gossip, MailboxGossip):
            self.gossip.W_mid = W
        with self.timer.phase("comm"):
            pout = self._param_out()
            info = self.gossip.end_of_round(r, W, pout,
                                            steps={c: losses[c]["batches"] for c in losses})
        if self.eval_stream is not None:
            self._issue_eval_local()   # the clients' local scores, behind the round-end launches
        recs += self._gossip_records(r, recs)
        verdict_rounds = []
        if self._gossip_filter:
            # the rounds applied during this round, each judged before it was applied
            verdict_rounds = self.gossip.take_verdicts()
            v = Verdicts(rejected={j for _, rj in verdict_rounds for j in rj})
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
        host_deferred = self._host_deferred
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
        if host_deferred:
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
                "rejected_msgs": info.get("rejected_msgs", 0.0),
                **({"verdict_rounds": [[int(t), list(rj)] for t, rj in verdict_rounds]}
                   if self._gossip_filter else {})}

    # ---- host reads deferred to the next round --------------------------------------------------
    @property
    def _host_deferred(self) -> bool:
        """One-process collective-free GPU runs read a round's results at the next round start."""
        return (self.collective_free and self.is_cuda and not self.rt.distributed
                and not os.environ.get("BCFL_ROUND_SYNC"))

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

    def _patch_history(self, r: int, **kw) -> None:
        for rec in reversed(self.history):
            if rec.get("round") == r:
                rec.update(kw)
                break
        self.metrics.write({"round": r, "deferred": True, **kw})

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
