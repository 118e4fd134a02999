"""Checkpoints and resume (reference C16 / C18: ``save_pretrained`` every round, the sampled indices),
mixed into :class:`~bcfl.fl.federation.Federation`."""
from __future__ import annotations

import json
import os
from typing import Dict

import torch

from .. import ops
from ..ckpt import load_into
from ..parallel import dist as D
from ..parallel.gossip import MailboxGossip
from ..trust.anomaly import Verdicts
from ..trust.ledger import Ledger


class CheckpointMixin:
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

    @torch.no_grad()
    def _global_model(self, r: int = -1) -> tuple:
        """(fp32 flat buffer, scope) of the model saved as ``<out>/global`` — the federation's
        model, as the reference saves it (serverless: ``avg_params`` = the unweighted mean of the
        client models, ``serverless_NonIID_IMDB.py:296-297,305``).

        * server: the FedAvg global model;
        * one process: the exact mean of every client model (one mix pass);
        * several ranks in lock-step (collective) mode: the mean through ONE all-reduce of the
          ranks' partial sums (every rank calls this at every save round);
        * several collective-free ranks under round-complete delta gossip: every client model at
          a round end IS the federation mean through the newest complete round applied
          (x0 + the mean update of every complete round, own progress retracted), so this rank's
          mean of its hosted models is saved and that round is recorded;
        * other collective-free gossip (no rank holds every model and nothing may wait): the mean
          of this rank's hosted models, labelled as such."""
        cfg = self.cfg
        if cfg.mode == "server":
            return self.global_master, "server FedAvg global model"
        if cfg.compat_chain:
            return self.flat.master, "mean of the K chain snapshots (reference C14)"
        srcs = [self.client_master[c] for c in self.local_clients] if self.multi else [self.flat.master]
        n_all = cfg.num_clients
        if len(srcs) == 1 and not self.rt.distributed:
            return srcs[0], "the only client model"
        if self._average_eval() and getattr(self, "_avg_round", None) == r:
            # global_eval_models='average' already built (and scored) this round's mean
            return self._avg_master, f"mean of all {n_all} client models (the scored global model)"
        if not hasattr(self, "_save_avg"):
            self._save_avg = torch.empty_like(self.flat.master)
        avg = self._save_avg
        collective = self.rt.distributed and not self.collective_free
        w = 1.0 / (n_all if collective else len(srcs))
        avg.copy_(srcs[0])
        ops.gossip_mix_(avg, srcs[1:], w, [w] * (len(srcs) - 1))
        if collective:
            D.all_reduce_(avg)
            return avg, f"mean of all {n_all} client models (all-reduce)"
        if not self.rt.distributed:
            return avg, f"mean of all {n_all} client models"
        g = self.gossip
        if isinstance(g, MailboxGossip) and g.exchange == "delta" and g.apply_mode == "complete":
            return avg, (f"federation mean through complete round {g.applied_T} (every client model "
                         "holds it at a round end; round-complete delta gossip)")
        return avg, f"mean of rank {self.rt.rank}'s {len(srcs)} hosted client models"

    def _maybe_save(self, r: int):
        """Reference C16 (``save_pretrained`` every round, ``serverless_NonIID_IMDB.py:305``):
        ``<out>/global`` (rank 0: the federation's model, :meth:`_global_model`),
        ``<out>/client_{k}`` for EVERY hosted client with ``save_clients``, and with
        ``save_resume_state`` the per-rank state a resumed run needs to continue bit-identically
        (``<out>/resume/rank{r}.pt``)."""
        cfg = self.cfg
        if cfg.save_every <= 0 or (r + 1) % cfg.save_every:
            return
        gsrc = None
        if self.rt.distributed and not self.collective_free and cfg.mode == "serverless":
            # the lock-step mean is a collective: every rank, before any rank-local skip below
            gsrc = self._global_model(r)
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
            acc_rounds = list(self.global_accuracy_rounds)
            state = {"round": r, "rng": ops.rng.global_rng().state(),
                     "ledger_tip": self.ledger.tip if self.ledger else None,
                     "ledger_height": len(self.ledger) if self.ledger else 0,
                     "global_accuracies": accs, "global_accuracy_rounds": acc_rounds,
                     "config": cfg.to_dict()}
            fins = []   # fields the writer thread resolves once the device work has finished
            jobs = []
            scored = False
            if self.rt.is_main:
                src, scope = gsrc if gsrc is not None else self._global_model(r)
                state["global_model"] = scope
                if cfg.mode == "serverless" and self.multi and not self._hosted_models_identical() \
                        and not self._average_eval() and src is not self.flat.master:
                    # the saved mean is not a model the round's evaluation scored: score it too,
                    # on the evaluation side stream (the writer thread reads the result)
                    score = self._score_async(src, r)
                    fins.append(lambda score=score: {"global_model_accuracy": score()})
                    scored = True
                elif (self.global_accuracy_rounds and self.global_accuracy_rounds[-1] == r):
                    state["global_model_accuracy"] = self.global_accuracies[-1]
                    scored = True
                jobs.append(([os.path.join(cfg.out_dir, "global")], src))
            pend = self._eval_pending
            if pend is not None and pend[0] == r:
                # round r's overlapped evaluation is still running: the writer thread waits for
                # its event and files the accuracy (no stall of the training stream here)
                _r, acc_t, _sets, ev_t, _t0 = pend

                def _fin(accs=accs, acc_t=acc_t, ev_t=ev_t, rr=acc_rounds + [int(r)], scored=scored):
                    ev_t.synchronize()
                    a = acc_t.cpu().tolist()
                    out = {"global_accuracies": accs + [a[0] / max(a[1], 1.0)],
                           "global_accuracy_rounds": rr}
                    if not scored:
                        out["global_model_accuracy"] = a[0] / max(a[1], 1.0)
                    return out
                fins.insert(0, _fin)
            if fins:
                state["_finalize"] = lambda fins=fins: {k: v for f in fins for k, v in f().items()}
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
              "holdout": [float(getattr(self, "_holdout_best", -1.0)),
                          int(getattr(self, "_holdout_streak", 0))],
              "ledger_tip": self.ledger.tip if self.ledger else None,
              "ledger_height": len(self.ledger) if self.ledger else 0}
        if self.global_master is not None:
            st["global_master"] = cpu(self.global_master)
        if self.gossip is not None and hasattr(self.gossip, "state_dict"):
            st["gossip"] = self.gossip.state_dict()
        return st

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
        self.global_accuracy_rounds = [int(x) for x in st.get(
            "global_accuracy_rounds", range(len(self.global_accuracies)))]
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
        if "holdout" in st:
            self._holdout_best, self._holdout_streak = float(st["holdout"][0]), int(st["holdout"][1])
        if self.gossip is not None and "gossip" in st:
            self.gossip.load_state_dict(st["gossip"])
