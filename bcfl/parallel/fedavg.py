"""Server FedAvg that survives dead ranks: the weighted sum over one-sided mailboxes.

Reference: Flower's ``FedAvg`` (``src/Servercase/server_IID_IMDB.py:205-209``) runs with
``accept_failures=True`` by default — a client that fails a round is left out of that round's
aggregate and the weights are re-normalised over the results that arrived (SURVEY.md §5.3 item
3). An RCCL all-reduce cannot do that: one exited rank blocks every survivor in the collective
until the process group times out.

Here every rank is its own aggregator:

1. it adds its hosted clients' models into a partial sum ``S_r = sum_{c on r} w_c x_c`` (global
   example-count weights) and posts ``S_r`` with its weight ``W_r = sum_{c on r} w_c`` (in the
   header) and the payload's SHA-256 Merkle root into every peer's inbox (one-sided copies on
   side streams, :mod:`bcfl.parallel.mailbox`);
2. it waits — bounded by ``timeout_s`` — for round r's post of every rank it still counts as
   live, verifies each payload's root, and declares the ranks that did not post (or posted a
   payload that fails verification) absent;
3. the new global model is ``G = sum_{r live} S_r / sum_{r live} W_r`` summed in rank order, so
   every survivor that saw the same live set computes the bit-identical G.

Live-set agreement. Each rank decides on its own which peers missed the timeout, so two ranks can
disagree (A times out on a slow-but-alive B while B still receives A's post): that round A and B
compute different G. Two rules keep such a split from becoming permanent:

* every post carries the live-rank set its sender aggregated in the previous round (a bitmask in
  the header's aux word); a receiver compares it with its own and reports the ranks whose view
  differed (``view_mismatch``, recorded in the ledger's round block) — a split is never silent;
* a post's version is the aggregation EPOCH, not the local round: a rank that finds a peer's
  newest post ahead of its own next epoch (it started late, or was excluded as slow) posts into
  that epoch, joining the federation's current aggregate (its skipped epochs are reported);
* an absent rank is not waited on again, but it is not excluded for good either: its inbox is
  checked (without waiting) every round; if that round's post is there it rejoins at once, and if
  a NEWER post than the last one seen is there (alive but lagging) it is waited on again (bounded)
  from the next round, which lets it catch up. G only depends on the posted partial sums, so the
  first round all ranks see the same live set they compute the bit-identical G again.

With every rank live, G equals the all-reduce result (up to the fp32 summation order). Payloads
are fp32 (exact partial sums); inboxes cost 2 slots x model bytes per peer (7 x 0.87 GB for
BERT-base on an 8-GPU node — small against 288 GB of HBM).
"""
from __future__ import annotations

import struct
import time
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops
from . import dist as D
from .mailbox import MailboxTransport, Snapshot


def _f2i(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


def _i2f(i: int) -> float:
    return struct.unpack("<d", struct.pack("<q", int(i)))[0]


class MailboxFedAvg:
    def __init__(self, numel: int, device: torch.device, timeout_s: float = 120.0,
                 verify: bool = True, rank: Optional[int] = None, world: Optional[int] = None):
        rt = D.runtime()
        self.rank = rt.rank if rank is None else rank
        self.world = rt.world if world is None else world
        self.peers = [r for r in range(self.world) if r != self.rank]
        self.numel, self.device = numel, device
        self.timeout_s = float(timeout_s)
        self.verify = verify
        # mailbox "clients" are ranks here: rank r posts its partial sum as client id r
        self.transport = MailboxTransport(numel, torch.float32, device, listen=self.peers,
                                          send_plan=[(self.rank, p) for p in self.peers],
                                          rank=self.rank, world=self.world)
        z = lambda: torch.zeros(numel, dtype=torch.float32, device=device)  # noqa: E731
        self.send_buf = [z(), z()]
        self.stage = {p: z() for p in self.peers}
        self.dead: set = set()
        self.records: List[dict] = []
        self.bytes_posted = 0
        self.prev_live_mask = (1 << self.world) - 1   # the live set of the previous round
        self.last_seen: Dict[int, int] = {p: 0 for p in self.peers}   # newest version seen
        self.epoch = 0                                # version of this rank's last post
        self._sum_done = None                         # event: last reader of the stage buffers

    @staticmethod
    def _mask(ranks) -> int:
        m = 0
        for q in ranks:
            m |= 1 << int(q)
        return m

    def reduce(self, r: int, partial: torch.Tensor, w_local: float) -> Tuple[torch.Tensor, Dict]:
        """Round r: post ``partial`` (this rank's weighted sum, fp32 flat) with weight
        ``w_local``; return (G, info) with G the re-normalised sum over the live ranks."""
        tr = self.transport
        # aggregation epoch = the post's version: one past this rank's last, or — when a peer is
        # already further (this rank started late or was excluded as slow) — the peer's newest,
        # so a lagging rank joins the federation's current aggregate instead of waiting for
        # posts that were overwritten long ago
        ahead = [nw[1].version for nw in (tr.newest(h) for h in tr.headers(self.peers).values())
                 if nw is not None]
        v = max([self.epoch + 1] + ahead)
        skipped = v - self.epoch - 1
        self.epoch = v
        slot = v % 2
        if tr.is_cuda:
            tr.wait_slot_free(self.rank, slot)
        buf = self.send_buf[slot]
        buf.copy_(partial)
        root = ops.merkle_root_deferred(buf) if self.verify else None
        snap = Snapshot(v, r, _f2i(w_local), buf.numel() * 4, b"\0" * 32, self.prev_live_mask)
        rd = root
        if rd is not None and not torch.is_tensor(rd):
            snap.root, rd = bytes(rd), None
        b0 = tr.bytes_posted
        tr.post(self.rank, buf, snap, rd)
        self.records.append({"client": -(self.rank + 1), "kind": "update", "version": v,
                             "root_t": root})
        # ---- wait (bounded) for round r from every rank counted live; absent ranks are only
        # checked, never waited on, and rejoin when they post again ---------------------------
        need = [p for p in self.peers if p not in self.dead]
        got: Dict[int, Snapshot] = {}
        t0 = time.perf_counter()
        after = self._sum_done
        while True:
            left = [p for p in need if p not in got]
            if not left:
                break
            got.update(tr.fetch_exact({p: v for p in left}, self.stage, after=after))
            after = None
            if all(p in got for p in need) or time.perf_counter() - t0 > self.timeout_s:
                break
            time.sleep(0.0005)
        wait_s = time.perf_counter() - t0
        back = [p for p in self.peers if p in self.dead]
        lagging = []
        if back:
            got.update(tr.fetch_exact({p: v for p in back}, self.stage, after=after))
            hdr = tr.headers([p for p in back if p not in got])
            for p, h in hdr.items():
                nw = tr.newest(h)
                if nw is not None and nw[1].version > self.last_seen[p]:
                    lagging.append(p)        # alive: waited on (bounded) again next round
                    self.last_seen[p] = nw[1].version
        for p, sn in got.items():
            self.last_seen[p] = max(self.last_seen[p], sn.version)
        absent = sorted(p for p in self.peers if p not in got)
        ok = {}
        if got and self.verify:
            fs = tr.fetch_stream
            ctx = torch.cuda.stream(fs) if fs is not None else None
            if ctx is not None:
                ctx.__enter__()
            try:
                for p in got:
                    ok[p] = ops.root_bytes(ops.merkle_root_deferred(self.stage[p])) == got[p].root
            finally:
                if ctx is not None:
                    ctx.__exit__(None, None, None)
            if fs is not None:
                torch.cuda.current_stream(self.device).wait_stream(fs)
        for p, sn in got.items():
            good = ok.get(p, True)
            self.records.append({"client": -(p + 1), "kind": "recv", "version": sn.version,
                                 "root": sn.root.hex(), "ok": good, "src_round": sn.round})
            if not good:
                absent.append(p)
        absent = sorted(set(absent))
        rejoined = sorted(p for p in back if p not in absent)
        self.dead = set(absent) - set(lagging)
        # ---- live-set agreement: every peer's view of the previous round vs this rank's -------
        mismatch = sorted(p for p, sn in got.items() if p not in absent and r > 0
                          and sn.aux != self.prev_live_mask)
        # ---- G = sum_{live} S_r / sum_{live} W_r, in rank order -------------------------------
        live = sorted([self.rank] + [p for p in got if p not in absent])
        out = torch.zeros_like(partial)
        wsum = 0.0
        for q in live:
            src = partial if q == self.rank else self.stage[q]
            ops.axpby_(out, src, 1.0, 1.0)
            wsum += w_local if q == self.rank else _i2f(got[q].steps)
        if wsum > 0 and abs(wsum - 1.0) > 1e-12:
            ops.scale_(out, 1.0 / wsum)
        if tr.is_cuda:  # the next round's fetch may overwrite stage[] only after this sum
            self._sum_done = torch.cuda.Event()
            self._sum_done.record(torch.cuda.current_stream(self.device))
        self.prev_live_mask = self._mask(live)
        self.bytes_posted += tr.bytes_posted - b0
        return out, {"live_ranks": live, "absent_ranks": absent, "live_weight": wsum,
                     "rejoined_ranks": rejoined, "view_mismatch": mismatch, "wait_s": wait_s,
                     "epoch": v, "epochs_skipped": skipped,
                     "bytes_sent": float(tr.bytes_posted - b0)}

    def take_records(self) -> List[dict]:
        out, self.records = self.records, []
        return out

    def drain(self):
        self.transport.drain()

    def close(self):
        self.transport.close()


class MailboxReduceScatterFedAvg:
    """Server FedAvg as a one-shot reduce-scatter + all-gather over the one-sided mailboxes
    ("the engine issues a direct one-shot reduce-scatter with send/recv over all 7
    peers"). The flat buffer is cut into ``world`` contiguous shards; rank k OWNS shard k:

    1. every rank posts shard p of its partial sum ``S_r`` (with its weight ``W_r``) into rank p's
       reduce inbox — one 1/world-sized copy per peer, all concurrently on side streams, so each
       xGMI link carries 1/world of the model instead of a full copy (MailboxFedAvg posts the whole
       partial sum to every peer: (world - 1) x the bytes);
    2. the owner waits (bounded) for shard k of every rank counted live, sums them in rank order
       and normalises by the live weight: ``G_k = sum_live S_{r,k} / sum_live W_r``;
    3. the owner posts ``G_k`` (with its live-rank mask in the header's aux word) to every peer's
       gather inbox, and every rank assembles ``G`` from the owners' shards.

    Liveness: a rank that misses step 2's deadline is left out of that shard's sum (weights
    re-normalised, Flower accept_failures as in :class:`MailboxFedAvg`) and only checked — not
    waited on — afterwards until it posts again; an OWNER that misses step 3's deadline leaves its
    shard undefined for that round, and each rank keeps its own normalised partial ``S_{r,k} / W_r``
    there (``absent_owners`` in the round info; the final-model check of the federation reports a
    resulting split). With every rank live the result equals the all-reduce FedAvg up to the fp32
    summation order.
    """

    def __init__(self, numel: int, device: torch.device, timeout_s: float = 120.0,
                 verify: bool = True, rank: Optional[int] = None, world: Optional[int] = None):
        rt = D.runtime()
        self.rank = rt.rank if rank is None else rank
        self.world = rt.world if world is None else world
        self.peers = [r for r in range(self.world) if r != self.rank]
        self.numel, self.device = numel, device
        self.timeout_s = float(timeout_s)
        self.verify = verify
        W = self.world
        self.shard = -(-numel // W)
        self.shard = -(-self.shard // 64) * 64          # 256-byte aligned shards
        self.bounds = [(k * self.shard, min(numel, (k + 1) * self.shard)) for k in range(W)]
        plan = [(self.rank, p) for p in self.peers]
        # reduce inboxes: "client" id = sending rank; gather inboxes: "client" id = owner rank
        self.rs = MailboxTransport(self.shard, torch.float32, device, listen=self.peers,
                                   send_plan=plan, rank=self.rank, world=self.world)
        self.ag = MailboxTransport(self.shard, torch.float32, device, listen=self.peers,
                                   send_plan=plan, rank=self.rank, world=self.world)
        z = lambda: torch.zeros(self.shard * W, dtype=torch.float32, device=device)  # noqa: E731
        self.send_buf = [z(), z()]                      # padded partial sums (one per slot)
        zs = lambda: torch.zeros(self.shard, dtype=torch.float32, device=device)  # noqa: E731
        self.gsend = [zs(), zs()]
        self.stage_rs = {p: zs() for p in self.peers}
        self.stage_ag = {p: zs() for p in self.peers}
        self.dead: set = set()
        self.records: List[dict] = []
        self.bytes_posted = 0
        self.epoch = 0
        self.prev_live_mask = (1 << W) - 1
        self.last_seen: Dict[int, int] = {p: 0 for p in self.peers}   # newest version seen
        self._done = None

    def _key(self, v: int, phase: int, who: int) -> int:
        """Ledger key of one post: every (sender, key) names ONE payload — the reduce posts of a
        version differ per destination ``who``, the gather post is one (``who`` = -1)."""
        return (2 * v + phase) * (self.world + 1) + who + 1

    def _post(self, tr, buf: torch.Tensor, snap: Snapshot, dsts, key: int) -> None:
        root = ops.merkle_root_deferred(buf) if self.verify else None
        rd = root
        if rd is not None and not torch.is_tensor(rd):
            snap.root, rd = bytes(rd), None
        tr.post_to(self.rank, buf, snap, dsts, rd)
        self.records.append({"client": -(self.rank + 1), "kind": "update", "version": key,
                             "root_t": root})

    def _gather(self, tr, want: Dict[int, int], stage: Dict[int, torch.Tensor],
                need, key) -> Dict[int, Snapshot]:
        """Bounded wait for version want[p] of every peer in ``need``; others are only checked."""
        got: Dict[int, Snapshot] = {}
        t0 = time.perf_counter()
        after = self._done
        while True:
            left = [p for p in need if p not in got]
            if not left:
                break
            got.update(tr.fetch_exact({p: want[p] for p in left}, stage, after=after))
            after = None
            if all(p in got for p in need) or time.perf_counter() - t0 > self.timeout_s:
                break
            time.sleep(0.0005)
        rest = [p for p in want if p not in need]
        if rest:
            got.update(tr.fetch_exact({p: want[p] for p in rest}, stage))
        ok = {}
        if got and self.verify:
            fs = tr.fetch_stream
            ctx = torch.cuda.stream(fs) if fs is not None else None
            if ctx is not None:
                ctx.__enter__()
            try:
                for p in got:
                    ok[p] = ops.root_bytes(ops.merkle_root_deferred(stage[p])) == got[p].root
            finally:
                if ctx is not None:
                    ctx.__exit__(None, None, None)
            if fs is not None:
                torch.cuda.current_stream(self.device).wait_stream(fs)
        good = {}
        for p, sn in got.items():
            g = ok.get(p, True)
            self.records.append({"client": -(p + 1), "kind": "recv", "version": key(sn.version),
                                 "root": sn.root.hex(), "ok": g, "src_round": sn.round})
            if g:
                good[p] = sn
        return good

    def _newest_peer_version(self) -> int:
        """Newest aggregation epoch any peer has posted (reduce or gather inbox), 0 if none."""
        best = 0
        for tr in (self.rs, self.ag):
            for h in tr.headers(self.peers).values():
                nw = tr.newest(h)
                if nw is not None:
                    best = max(best, int(nw[1].version))
        return best

    def reduce(self, r: int, partial: torch.Tensor, w_local: float) -> Tuple[torch.Tensor, Dict]:
        W, k, n = self.world, self.rank, self.numel
        # aggregation epoch = the posts' version, with MailboxFedAvg's catch-up rule: a rank that
        # finds a peer already further (started late, or excluded as slow for several rounds)
        # posts into the federation's current epoch instead of fetching versions its peers have
        # long overwritten (it would otherwise wait out two timeouts every round and never rejoin)
        v = max(self.epoch + 1, self._newest_peer_version())
        skipped = v - self.epoch - 1
        self.epoch = v
        slot = v % 2
        b0 = self.rs.bytes_posted + self.ag.bytes_posted
        t_start = time.perf_counter()
        # ---- 1. reduce-scatter: shard p of the partial sum to its owner p ----------------------
        if self.rs.is_cuda:
            self.rs.wait_slot_free(self.rank, slot)
        buf = self.send_buf[slot]
        buf[:n].copy_(partial)
        for p in self.peers:
            a, b = p * self.shard, (p + 1) * self.shard
            self._post(self.rs, buf[a:b], Snapshot(v, r, _f2i(w_local), self.shard * 4, b"\0" * 32,
                                                   self.prev_live_mask), [p], self._key(v, 0, p))
        # ---- 2. the owner reduces its shard over the live ranks ------------------------------------
        need = [p for p in self.peers if p not in self.dead]
        got = self._gather(self.rs, {p: v for p in self.peers}, self.stage_rs, need,
                           lambda ver: self._key(ver, 0, k))
        absent = sorted(p for p in self.peers if p not in got)
        rejoined = sorted(p for p in self.peers if p in self.dead and p in got)
        # an absent rank whose newest post advanced is alive but lagging: it is waited on
        # (bounded) again next round, which lets it catch up to the federation's epoch
        lagging = []
        for p, h in self.rs.headers(absent).items():
            nw = self.rs.newest(h)
            if nw is not None and nw[1].version > self.last_seen[p]:
                lagging.append(p)
                self.last_seen[p] = int(nw[1].version)
        for p, sn in got.items():
            self.last_seen[p] = max(self.last_seen[p], int(sn.version))
        self.dead = set(absent) - set(lagging)
        live = sorted([k] + list(got))
        a0 = k * self.shard
        gk = self.gsend[slot]
        if self.ag.is_cuda:
            self.ag.wait_slot_free(self.rank, slot)
        gk.zero_()
        wsum = 0.0
        for q in live:
            src = buf[a0:a0 + self.shard] if q == k else self.stage_rs[q]
            ops.axpby_(gk, src, 1.0, 1.0)
            wsum += w_local if q == k else _i2f(got[q].steps)
        if wsum > 0 and abs(wsum - 1.0) > 1e-12:
            ops.scale_(gk, 1.0 / wsum)
        mask = MailboxFedAvg._mask(live)
        # ---- 3. all-gather: every owner's G shard to every rank ------------------------------------
        self._post(self.ag, gk, Snapshot(v, r, _f2i(wsum), self.shard * 4, b"\0" * 32, mask),
                   self.peers, self._key(v, 1, -1))
        # owners absent from this round's reduce (dead or lagging) are only checked, never
        # waited on: a dead owner would otherwise cost the full timeout every round
        owners = self._gather(self.ag, {p: v for p in self.peers}, self.stage_ag,
                              [p for p in self.peers if p not in absent],
                              lambda ver: self._key(ver, 1, -1))
        out = torch.empty_like(partial)
        absent_owners = []
        for q in range(W):
            a, b = self.bounds[q]
            if b <= a:
                continue
            if q == k:
                out[a:b].copy_(gk[:b - a])
            elif q in owners:
                out[a:b].copy_(self.stage_ag[q][:b - a])
            else:   # owner gone: this rank's own normalised partial for that shard
                absent_owners.append(q)
                out[a:b].copy_(partial[a:b])
                if w_local > 0:
                    ops.scale_(out[a:b], 1.0 / w_local)
        mismatch = sorted(q for q, sn in owners.items() if sn.aux != mask)
        if self.rs.is_cuda:
            self._done = torch.cuda.Event()
            self._done.record(torch.cuda.current_stream(self.device))
        self.prev_live_mask = mask
        sent = self.rs.bytes_posted + self.ag.bytes_posted - b0
        self.bytes_posted += sent
        return out, {"live_ranks": live, "absent_ranks": absent, "live_weight": wsum,
                     "rejoined_ranks": rejoined, "view_mismatch": mismatch,
                     "absent_owners": absent_owners, "wait_s": time.perf_counter() - t_start,
                     "epoch": v, "epochs_skipped": skipped, "bytes_sent": float(sent)}

    def take_records(self) -> List[dict]:
        out, self.records = self.records, []
        return out

    def drain(self):
        self.rs.drain()
        self.ag.drain()

    def close(self):
        self.rs.close()
        self.ag.close()
