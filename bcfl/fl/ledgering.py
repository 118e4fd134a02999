"""Trust hooks of a federation round: update statistics and the collective anomaly filter, fault injection,
per-round ledger blocks, the cross-rank ledger audit and the final-model check (mixed into
:class:`~bcfl.fl.federation.Federation`)."""
from __future__ import annotations

import json
import os
import time
import warnings
from typing import Dict, List, Optional

import torch

from .. import ops
from ..parallel import dist as D
from ..parallel.flat import FlatParams
from ..parallel.gossip import MailboxGossip
from ..trust.anomaly import Verdicts
from ..trust.ledger import Ledger


class TrustMixin:
    def _ledger_path(self) -> Optional[str]:
        """Collective mode: one canonical chain, written by rank 0. Collective-free (mailbox)
        mode: every rank keeps its own chain (rank 0 -> ledger.jsonl, rank k -> ledger.rank{k}.jsonl)."""
        if self.rt.is_main:
            return os.path.join(self.cfg.out_dir, "ledger.jsonl")
        if self.collective_free:
            return os.path.join(self.cfg.out_dir, f"ledger.rank{self.rt.rank}.jsonl")
        return None

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
            elif g["kind"] == "verdict":
                # the anomaly filter's verdict on a source's complete-round update, taken by this
                # receiver before the round was applied
                out.append({"client": g["client"], "kind": "verdict", "root": "",
                            "verdict": "accept" if g["ok"] else "reject:" + (g["reason"] or "filter"),
                            "ts": float(r) + 0.6 + 0.001 * (g["client"] + 1),
                            "metrics": {"receiver_rank": self.rt.rank, "src_round": g["round"],
                                        "update_norm": g["norm"]}})
            elif g["kind"] == "recv":
                out.append({"client": g["client"], "kind": "verify", "root": g["root"],
                            "verdict": "accept" if g["ok"] else "reject",
                            "ts": float(r) + 0.5 + 0.001 * (g["client"] + 1),
                            "metrics": {"receiver_rank": self.rt.rank, "version": g["version"],
                                        "src_round": g["src_round"],
                                        **({} if g["ok"] else {"reason": "merkle root mismatch"})}})
        return out

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
