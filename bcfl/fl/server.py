"""The server FedAvg round (reference C11 / C12: Flower ``FedAvg`` over ``start_simulation``,
``src/Servercase/server_IID_IMDB.py:199-218``), mixed into :class:`~bcfl.fl.federation.Federation`."""
from __future__ import annotations

import warnings
from typing import Dict

import numpy as np
import torch

from .. import ops
from ..parallel import dist as D
from .trainer import EvalResult
from .fedutil import weighted_average


class ServerRoundMixin:
    def server_round(self, r: int) -> dict:
        cfg = self.cfg
        G = self.global_master
        counts = self.fedavg_weight_counts(r)
        recs, sk, nr, trained, losses = [], {}, {}, {}, {}
        need_copy = self.filter is not None and self.multi
        self.acc.zero_()
        w_all = counts / counts.sum()
        # hold-out selection with kept client optimizer states: a round whose global model is not
        # adopted is undone completely, its clients' AdamW moments included (otherwise the moments
        # keep accumulating the rejected direction and the next round repeats it)
        opt_before = self._opt_snapshot() if (cfg.server_holdout > 0 and self.keep_opt) else None
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
        gate = self._holdout_gate(r, self.acc) if cfg.server_holdout > 0 else None
        if gate is None or gate["holdout_adopted"]:
            G.copy_(self.acc)
        elif opt_before is not None:
            self._opt_restore(opt_before)
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
                 "rejected": sorted(v.rejected), **(gate or {})}
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
               "client_metrics": client_metrics, "bytes_sent": float(wire_bytes),
               **(gate or {})}
        if self.server_mbox is not None:
            out.update(absent_ranks=absent, live_weight=self._server_live["live_weight"],
                       wait_s=float(self._server_live.get("wait_s", 0.0)),
                       dead_peers=sorted(self.server_mbox.dead),
                       epochs_skipped=int(self._server_live.get("epochs_skipped", 0)),
                       view_mismatch=self._server_live["view_mismatch"],
                       rejoined_ranks=self._server_live["rejoined_ranks"])
        return out

    def _opt_snapshot(self) -> dict:
        """The hosted clients' kept optimizer states before a round. Lanes and the multi-client
        path REPLACE ``client_opt[c]`` after training (fresh tensors), so references suffice; a
        rank with one client keeps its live optimizer in place, which is copied."""
        snap = {"client_opt": dict(self.client_opt)}
        if self._single_opt:
            snap["live"] = {k: (v.clone() if torch.is_tensor(v) else v)
                            for k, v in self.opt.state_dict().items()}
            snap["owner"] = self._opt_owner
        return snap

    def _opt_restore(self, snap: dict) -> None:
        self.client_opt = dict(snap["client_opt"])
        if "live" in snap:
            self.opt.load_state_dict(snap["live"])
            self._opt_owner = snap["owner"]

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

    def next_round(self, r: int) -> int:
        """Round to run after round r: r + 1, except when the mailbox FedAvg joined a later
        aggregation epoch (this rank started late or was excluded as slow, fedavg.py): the rank
        then continues at the federation's round instead of replaying the ones it missed."""
        if self.server_mbox is not None:
            return max(r + 1, self.server_mbox.epoch)
        return r + 1
