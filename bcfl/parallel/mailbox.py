"""One-sided peer mailboxes: truly asynchronous P2P gossip.

The paper's claim is *asynchronous* peer-to-peer exchange — a node's information-passing time is
the max over destinations, not the sum (``README.md:10``; ``Medical_Transcriptions_All_graphs.ipynb:
979-980``). RCCL send/recv cannot give that: every send needs a matching receive, so one slow or
dead peer stalls its neighbours. Here nothing is ever matched:

* every rank owns an **inbox** per remote client it listens to: a header region (2 slots x 16
  int64 words) and a payload region (2 slots of the wire-encoded model);
* inboxes are exported ONCE (``hipIpcGetMemHandle``; on CPU a ``/dev/shm`` file) and the handles
  all-gathered at start-up; each sender maps the inboxes of its destinations;
* **post** (sender, side HIP stream): for version v into slot v % 2 — header.begin = v, payload
  copy over xGMI (``hipMemcpyAsync`` into the peer's memory), header body (round, steps, bytes,
  SHA-256 Merkle root of the payload) and, fenced after it, header.end = v;
* **fetch** (receiver, any time): read both slot headers, take the newest slot with
  begin == end, copy its payload into a local replica, re-read the header — if begin moved, the
  sender lapped the slot mid-copy and the snapshot is dropped (seqlock). A peer that is slow,
  stopped, or gone simply leaves the last good snapshot in place; the gossip layer ages it out
  (staleness bound) instead of waiting.

The header's Merkle root is the sender's ledger commitment: the receiver re-hashes the fetched
payload on its GPU and rejects a snapshot whose root does not match (tampering in flight).

Backends: ``HipIpcBackend`` (GPU tensors; uncached device memory, peer-mapped) and ``ShmBackend``
(CPU tensors in shared-memory files, the CPU-test analogue with the identical protocol).
"""
from __future__ import annotations

import os
import uuid
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import dist as D

HDR_WORDS = 16
W_BEGIN, W_ROUND, W_STEPS, W_BYTES, W_ROOT, W_END, W_AUX = 0, 1, 2, 3, 4, 8, 9
ALIGN = 4096


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def root_to_words(root: bytes) -> List[int]:
    """32-byte SHA-256 root -> 4 signed int64 header words."""
    return [int(x) for x in np.frombuffer(root, dtype="<i8")]


def words_to_root(words: Sequence[int]) -> bytes:
    return np.asarray(list(words), dtype="<i8").tobytes()


@dataclass
class Snapshot:
    version: int
    round: int
    steps: int
    nbytes: int
    root: bytes
    aux: int = 0      # one protocol word (server FedAvg: the sender's previous live-rank set)


def _snap(h: np.ndarray, s: int, v: int) -> Snapshot:
    return Snapshot(v, int(h[s, W_ROUND]), int(h[s, W_STEPS]), int(h[s, W_BYTES]),
                    words_to_root(h[s, W_ROOT:W_ROOT + 4]), int(h[s, W_AUX]))


# ----------------------------------------------------------------------------------------------
class ShmBackend:
    """CPU analogue: regions are files under /dev/shm mapped with ``torch.from_file(shared=True)``;
    a handle is the file path. Writes are plain stores (x86 keeps store order)."""

    def __init__(self, tag: str):
        self.tag = tag
        self.owned: List[str] = []
        self.root = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"

    def alloc(self, nbytes: int, kind: str) -> Tuple[torch.Tensor, object]:
        path = os.path.join(self.root, f"bcfl_mbox_{self.tag}_{uuid.uuid4().hex[:12]}_{kind}")
        with open(path, "wb") as fh:
            fh.truncate(nbytes)
        self.owned.append(path)
        return torch.from_file(path, shared=True, size=nbytes, dtype=torch.uint8), path

    def peer_ok(self, owner_device: int) -> bool:
        return True

    def open(self, handle, nbytes: int, owner_device: int = -1) -> torch.Tensor:
        return torch.from_file(handle, shared=True, size=nbytes, dtype=torch.uint8)

    def hdr_store(self, hdr: torch.Tensor, slot: int, words: Sequence[int], off: int,
                  end_word: int = -1, end_value: int = 0):
        row = hdr[slot]
        if words:
            row[off:off + len(words)] = torch.tensor(list(words), dtype=torch.int64)
        if end_word >= 0:
            row[end_word] = int(end_value)

    def release_names(self):
        for p in self.owned:
            try:
                os.remove(p)
            except FileNotFoundError:
                pass
        self.owned.clear()

    close = release_names


class HipIpcBackend:
    """GPU: dedicated uncached device allocations exported with hipIpcGetMemHandle, mapped by
    peers with hipIpcOpenMemHandle (xGMI peer access); header stores are a fenced kernel."""

    def __init__(self, device: torch.device):
        from .. import ops
        self.C = ops.native()
        self.device = device

    def alloc(self, nbytes: int, kind: str) -> Tuple[torch.Tensor, object]:
        t = self.C.mbox_alloc(int(nbytes), int(self.device.index), 3)
        return t, bytes(self.C.ipc_handle(t))

    def peer_ok(self, owner_device: int) -> bool:
        """Peer access from this rank's device to the inbox owner's (same device: always)."""
        return owner_device < 0 or bool(self.C.can_access_peer(int(self.device.index), int(owner_device)))

    def open(self, handle, nbytes: int, owner_device: int = -1) -> torch.Tensor:
        return self.C.ipc_open(handle, int(nbytes), int(self.device.index), int(owner_device))

    def hdr_store(self, hdr: torch.Tensor, slot: int, words: Sequence[int], off: int,
                  end_word: int = -1, end_value: int = 0):
        self.C.hdr_store(hdr.view(-1), int(slot), [int(w) for w in words], int(off), int(end_word),
                         int(end_value))

    def release_names(self):
        pass

    def close(self):
        pass


# ----------------------------------------------------------------------------------------------
class _Box:
    """Views of one inbox (local or a peer's mapped copy)."""

    def __init__(self, hdr_raw: torch.Tensor, pay_raw: torch.Tensor, numel: int, dtype: torch.dtype):
        self.hdr = hdr_raw[: 2 * HDR_WORDS * 8].view(torch.int64).view(2, HDR_WORDS)
        esz = torch.tensor([], dtype=dtype).element_size()
        ps = _align(numel * esz)
        self.slots = [pay_raw[k * ps:k * ps + numel * esz].view(dtype) for k in (0, 1)]
        self._keep = (hdr_raw, pay_raw)


class MailboxUnavailable(RuntimeError):
    """Raised on EVERY rank when any rank could not allocate, export or map its inboxes (the
    outcome is agreed collectively, so all ranks can fall back to the RCCL engine together)."""


class MailboxTransport:
    """Inboxes for ``listen`` (remote clients this rank reads) and mapped peer inboxes for
    ``send_plan`` ((local client, destination rank) pairs). Construction is collective (one
    all-gather of handles); everything after it is one-sided."""

    def __init__(self, numel: int, dtype: torch.dtype, device: torch.device, listen: Sequence[int],
                 send_plan: Sequence[Tuple[int, int]], rank: Optional[int] = None,
                 world: Optional[int] = None):
        rt = D.runtime()
        self.rank = rt.rank if rank is None else rank
        self.world = rt.world if world is None else world
        self.numel, self.dtype, self.device = numel, dtype, device
        self.is_cuda = device.type == "cuda"
        esz = torch.tensor([], dtype=dtype).element_size()
        self.payload_bytes = numel * esz
        self.hdr_bytes = ALIGN
        self.pay_bytes = 2 * _align(self.payload_bytes)
        self.backend = HipIpcBackend(device) if self.is_cuda else ShmBackend(f"r{self.rank}")
        self.inbox: Dict[int, _Box] = {}
        handles, err = {}, None
        try:
            for j in listen:
                h, hh = self.backend.alloc(self.hdr_bytes, f"h{j}")
                p, ph = self.backend.alloc(self.pay_bytes, f"p{j}")
                self.inbox[j] = _Box(h, p, numel, dtype)
                handles[j] = (hh, ph)
        except Exception as e:  # reported collectively below, never left half-joined
            err = f"rank {self.rank} inbox allocation / export: {e!r}"
        # start-up handle exchange (with each rank's allocation outcome and device)
        dev_idx = device.index if self.is_cuda else -1
        table = D.all_gather_object({"handles": handles, "err": err, "device": dev_idx})
        self.outbox: Dict[int, List[Tuple[int, _Box]]] = {}
        if err is None and not any(t["err"] for t in table):
            try:
                for c, dst in send_plan:
                    owner = int(table[dst].get("device", -1))
                    if not self.backend.peer_ok(owner):
                        # fail loudly and collectively: every rank falls back together
                        raise RuntimeError(f"no peer access from device {dev_idx} to device "
                                           f"{owner} (rank {dst}'s inbox): hipDeviceCanAccessPeer = 0")
                    hh, ph = table[dst]["handles"][c]
                    box = _Box(self.backend.open(hh, self.hdr_bytes, owner),
                               self.backend.open(ph, self.pay_bytes, owner), numel, dtype)
                    self.outbox.setdefault(c, []).append((dst, box))
            except Exception as e:
                err = f"rank {self.rank} peer mapping: {e!r}"
        errs = [e for e in D.all_gather_object(err) if e] + [t["err"] for t in table if t["err"]]
        if errs:
            self.outbox.clear()
            self.inbox.clear()
            self.backend.release_names()
            raise MailboxUnavailable("; ".join(sorted(set(errs))))
        self.streams = ({d: torch.cuda.Stream(device=device) for d in {d for _, d in send_plan}}
                        if self.is_cuda else {})
        # every peer has mapped its destinations: shared-memory names can go now (mappings stay
        # valid), so nothing is left in /dev/shm even if a rank dies without closing
        D.barrier()
        self.backend.release_names()
        self.posted: Dict[Tuple[int, int], List["torch.cuda.Event"]] = {}  # (client, slot)
        self.torn = 0
        self.bytes_posted = 0
        # measured peer-copy times (GPU): the payload copy of every post is bracketed by timing
        # events on its side stream — the information-passing time over xGMI, measured in the run
        self._timed: List[Tuple[int, "torch.cuda.Event", "torch.cuda.Event"]] = []
        self._post_ms: List[Tuple[int, float]] = []

    # ------------------------------------------------------------------ sender
    def wait_slot_free(self, c: int, slot: int):
        """Make the current stream wait until the earlier posts that READ client c's send buffer
        ``slot`` have finished (the caller is about to overwrite it)."""
        for ev in self.posted.pop((c, slot), []):
            torch.cuda.current_stream(self.device).wait_event(ev)

    def post_to(self, c: int, payload: torch.Tensor, snap: Snapshot, dsts: Sequence[int],
                root_dev: Optional[torch.Tensor] = None):
        """:meth:`post` restricted to the destination ranks ``dsts`` (information-passing
        measurements: one destination at a time vs all at once)."""
        keep = self.outbox.get(c, [])
        self.outbox[c] = [(d, b) for d, b in keep if d in set(dsts)]
        try:
            self.post(c, payload, snap, root_dev)
        finally:
            self.outbox[c] = keep

    def post(self, c: int, payload: torch.Tensor, snap: Snapshot,
             root_dev: Optional[torch.Tensor] = None):
        """Publish ``payload`` (wire-encoded, ``numel`` elements) as version ``snap.version`` of
        client c to every destination inbox. Returns immediately on GPU (side streams).

        ``root_dev``: the payload's Merkle root as a 32-byte device tensor, copied device-to-device
        into the header (no host round trip); otherwise ``snap.root`` (host bytes) is written."""
        slot = snap.version % 2
        body = [snap.round, snap.steps, snap.nbytes]
        if root_dev is None:
            body += root_to_words(snap.root)
        evs = []
        if self.is_cuda:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.device))
        for dst, box in self.outbox.get(c, []):
            if self.is_cuda:
                st = self.streams[dst]
                st.wait_event(ready)
                with torch.cuda.stream(st):
                    self.backend.hdr_store(box.hdr, slot, [snap.version], W_BEGIN)
                    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    t0.record(st)
                    box.slots[slot].copy_(payload, non_blocking=True)
                    t1.record(st)
                    self._timed.append((dst, t0, t1))
                    if root_dev is not None:
                        box.hdr[slot, W_ROOT:W_ROOT + 4].copy_(root_dev.view(torch.int64),
                                                               non_blocking=True)
                    self.backend.hdr_store(box.hdr, slot, [snap.aux], W_AUX)
                    self.backend.hdr_store(box.hdr, slot, body, W_ROUND, W_END, snap.version)
                    ev = torch.cuda.Event()
                    ev.record(st)
                    evs.append(ev)
            else:
                self.backend.hdr_store(box.hdr, slot, [snap.version], W_BEGIN)
                box.slots[slot].copy_(payload)
                if root_dev is not None:
                    box.hdr[slot, W_ROOT:W_ROOT + 4] = root_dev.view(torch.int64)
                self.backend.hdr_store(box.hdr, slot, [snap.aux], W_AUX)
                self.backend.hdr_store(box.hdr, slot, body, W_ROUND, W_END, snap.version)
            self.bytes_posted += self.payload_bytes
        if evs:
            # extend, not replace: per-destination posts of one version (post_to) each add the
            # events of their copies, and the slot is free only after all of them. Events that
            # have completed are dropped here, so a caller that never calls wait_slot_free (the
            # information-passing measurement) does not grow the list without bound
            keep = [e for e in self.posted.get((c, slot), []) if not e.query()]
            self.posted[(c, slot)] = keep + evs

    def _collect_timings(self):
        keep = []
        for dst, t0, t1 in self._timed:
            if t1.query():
                self._post_ms.append((dst, t0.elapsed_time(t1)))
            else:
                keep.append((dst, t0, t1))
        self._timed = keep
        del self._post_ms[:-512]  # recent posts only

    def post_stats(self) -> Optional[Dict[str, float]]:
        """Measured payload-copy time per post (ms) and the implied per-destination bandwidth
        (GB/s): the information-passing time of one model update to one peer."""
        self._collect_timings()
        if not self._post_ms:
            return None
        ms = np.array([m for _, m in self._post_ms])
        return {"posts": int(ms.size), "payload_mb": self.payload_bytes / 1e6,
                "ms_median": float(np.median(ms)), "ms_max": float(ms.max()),
                "gb_per_s_median": float(self.payload_bytes / np.median(ms) / 1e6),
                "destinations": int(len({d for d, _ in self._post_ms}))}

    def drain(self):
        self._collect_timings()
        for evs in self.posted.values():
            for ev in evs:
                ev.synchronize()
        self.posted.clear()

    # ------------------------------------------------------------------ receiver
    @property
    def fetch_stream(self):
        """Side stream of the receive path (GPU): header reads, payload copies and the
        receiver's verification hashing run here, so polling a mailbox never waits for (drains)
        the compute stream; the host waits only for this stream's small, already-issued work."""
        if not self.is_cuda:
            return None
        if getattr(self, "_fs", None) is None:
            self._fs = torch.cuda.Stream(device=self.device)
        return self._fs

    def headers(self, js: Sequence[int]) -> Dict[int, np.ndarray]:
        """Both slot headers of every inbox in ``js`` (one device->host read, on the fetch
        stream: the read waits for nothing queued on the compute stream)."""
        if not js:
            return {}
        if self.is_cuda:
            with torch.cuda.stream(self.fetch_stream):
                h = torch.stack([self.inbox[j].hdr for j in js]).cpu().numpy()
        else:
            h = torch.stack([self.inbox[j].hdr for j in js]).cpu().numpy()
        return {j: h[i] for i, j in enumerate(js)}

    @staticmethod
    def newest(h: np.ndarray) -> Optional[Tuple[int, Snapshot]]:
        best = None
        for s in (0, 1):
            v = int(h[s, W_BEGIN])
            if v > 0 and v == int(h[s, W_END]) and (best is None or v > best[1].version):
                best = (s, _snap(h, s, v))
        return best

    @staticmethod
    def pick(h: np.ndarray, want_v: int, max_round: Optional[int] = None
             ) -> Optional[Tuple[int, Snapshot]]:
        """Slot to fetch from one inbox's header pair: the newest complete version newer than
        ``want_v``; with ``max_round`` the newest such version posted in a round <= max_round (a
        round-gated receiver applies every source's round-T post together). A sender already
        two rounds past ``max_round`` has no such slot left: its oldest newer version is taken."""
        cands = []
        for s in (0, 1):
            v = int(h[s, W_BEGIN])
            if v > 0 and v == int(h[s, W_END]) and v > want_v:
                cands.append((s, _snap(h, s, v)))
        if not cands:
            return None
        if max_round is None:
            return max(cands, key=lambda x: x[1].version)
        ok = [x for x in cands if x[1].round <= max_round]
        return max(ok, key=lambda x: x[1].version) if ok else min(cands, key=lambda x: x[1].version)

    @classmethod
    def _select(cls, h: "AsyncFetch", first: Dict[int, np.ndarray]) -> Dict[int, Tuple[int, Snapshot]]:
        """Step 1 of every fetch: the round gate (if any) sees the newest complete round of every
        inbox and returns the round to fetch (``None``: nothing to fetch now), then one slot per
        inbox is picked."""
        T = None
        if h.gate is not None:
            nr = {}
            for j, hj in first.items():
                nw = cls.newest(hj)
                if nw is not None:
                    nr[j] = nw[1].round
            T = h.gate(nr)
            h.gate_round = T
            if T is None:
                return {}
        picked = {}
        for j, hj in first.items():
            nw = cls.pick(hj, h.want[j], T)
            if nw is not None:
                picked[j] = nw
        return picked

    def fetch(self, want: Dict[int, int], out: Dict[int, torch.Tensor],
              after: Optional["torch.cuda.Event"] = None, gate=None,
              handle: Optional["AsyncFetch"] = None) -> Dict[int, Snapshot]:
        """For every inbox j with a complete version newer than ``want[j]``, copy it into
        ``out[j]`` and return the validated snapshots; torn reads are dropped.

        ``gate(newest_rounds: {j: round}) -> Optional[int]``: round-gated fetch — the slot of
        round <= the returned round is taken (:meth:`pick`); ``None`` fetches nothing. The gate's
        decision is left in ``handle.gate_round`` when a handle is passed.

        GPU: everything runs on :attr:`fetch_stream`, first ordered after ``after`` (the event
        after which the ``out`` buffers are no longer read, e.g. the previous mix); a consumer on
        another stream must wait for it (``stream.wait_stream(transport.fetch_stream)``)."""
        js = list(want)
        fs = self.fetch_stream
        if fs is not None and after is not None:
            fs.wait_event(after)
        first = self.headers(js)
        hd = handle if handle is not None else AsyncFetch(want, out)
        hd.gate = gate
        picked = self._select(hd, first)
        for j, nw in picked.items():
            if fs is not None:
                with torch.cuda.stream(fs):
                    out[j].copy_(self.inbox[j].slots[nw[0]], non_blocking=True)
            else:
                out[j].copy_(self.inbox[j].slots[nw[0]])
        if not picked:
            return {}
        second = self.headers(list(picked))  # stream-ordered after the payload copies
        good = {}
        for j, (slot, snap) in picked.items():
            h = second[j]
            if int(h[slot, W_BEGIN]) == snap.version and int(h[slot, W_END]) == snap.version:
                good[j] = snap
            else:
                self.torn += 1
        if fs is not None:  # device-side dependency only: the caller's stream reads out[] later
            torch.cuda.current_stream(self.device).wait_stream(fs)
        return good

    def fetch_exact(self, want: Dict[int, int], out: Dict[int, torch.Tensor],
                    after: Optional["torch.cuda.Event"] = None) -> Dict[int, Snapshot]:
        """Like :meth:`fetch` but for EXACTLY version ``want[j]`` (a slot whose begin == end ==
        that version): round-synchronous protocols (server FedAvg over mailboxes) need round r's
        post even when the sender has already posted round r + 1 into its other slot.
        ``after``: as in :meth:`fetch` (the ``out`` buffers' last reader)."""
        js = list(want)
        fs = self.fetch_stream
        if fs is not None and after is not None:
            fs.wait_event(after)
        first = self.headers(js)
        picked: Dict[int, Tuple[int, Snapshot]] = {}
        for j in js:
            h = first[j]
            for slot in (0, 1):
                v = int(h[slot, W_BEGIN])
                if v == want[j] and v == int(h[slot, W_END]):
                    picked[j] = (slot, _snap(h, slot, v))
                    if fs is not None:
                        with torch.cuda.stream(fs):
                            out[j].copy_(self.inbox[j].slots[slot], non_blocking=True)
                    else:
                        out[j].copy_(self.inbox[j].slots[slot])
                    break
        if not picked:
            return {}
        second = self.headers(list(picked))
        good = {}
        for j, (slot, snap) in picked.items():
            h = second[j]
            if int(h[slot, W_BEGIN]) == snap.version and int(h[slot, W_END]) == snap.version:
                good[j] = snap
            else:
                self.torn += 1
        if fs is not None:
            torch.cuda.current_stream(self.device).wait_stream(fs)
        return good

    # ---------------------------------------------------------- non-blocking receive
    def fetch_begin(self, want: Dict[int, int], out: Dict[int, torch.Tensor],
                    after: Sequence["torch.cuda.Event"] = (), gate=None) -> "AsyncFetch":
        """Start a NON-BLOCKING fetch (GPU): the header read is queued on the fetch stream into
        pinned host memory and nothing waits; :meth:`fetch_advance` moves it on when its event
        has completed. ``after``: events after which the ``out`` buffers are free (their last
        readers); ``gate``: as in :meth:`fetch`. CPU: completes synchronously (the shared-memory
        copies are host copies)."""
        h = AsyncFetch(want, out)
        h.gate = gate
        if not self.is_cuda:
            h.result = self.fetch(want, out, gate=gate, handle=h)
            return h
        fs = self.fetch_stream
        for ev in after:
            fs.wait_event(ev)
        js = list(want)
        if not js:
            h.result = {}
            return h
        with torch.cuda.stream(fs):
            dev = torch.stack([self.inbox[j].hdr for j in js])
            h.hdr = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True)
            h.hdr.copy_(dev, non_blocking=True)
            h.ev = torch.cuda.Event()
            h.ev.record(fs)
        h.js = js
        return h

    def fetch_advance(self, h: "AsyncFetch", hash_fn=None) -> Optional[Dict[int, Snapshot]]:
        """Advance a non-blocking fetch by one step if its queued work has completed; returns
        the validated snapshots when done (``None`` while pending). Step 1: pick every inbox with
        a complete version newer than wanted, queue its payload copy, the seqlock re-read of its
        header and (``hash_fn``) the receiver's re-hash, all on the fetch stream. Step 2: drop
        torn copies; ``h.roots[j]`` holds the receiver-side root bytes."""
        if h.result is not None:
            return h.result
        if not h.ev.query():
            return None
        fs = self.fetch_stream
        if h.step == 1:
            hn = h.hdr.numpy()
            picked = self._select(h, {j: hn[i] for i, j in enumerate(h.js)})
            if not picked:
                h.result = {}
                return h.result
            pj = list(picked)
            with torch.cuda.stream(fs):
                for j in pj:
                    h.out[j].copy_(self.inbox[j].slots[picked[j][0]], non_blocking=True)
                dev = torch.stack([self.inbox[j].hdr for j in pj])
                h.hdr2 = torch.empty(dev.shape, dtype=dev.dtype, pin_memory=True)
                h.hdr2.copy_(dev, non_blocking=True)
                if hash_fn is not None:
                    rts = [hash_fn(h.out[j]) for j in pj]
                    h.root_host = torch.empty((len(pj), 32), dtype=torch.uint8, pin_memory=True)
                    h.root_host.copy_(torch.stack([r.view(torch.uint8).reshape(32) for r in rts]),
                                      non_blocking=True)
                h.ev = torch.cuda.Event()
                h.ev.record(fs)
            h.picked, h.pj, h.step = picked, pj, 2
            return None
        second = h.hdr2.numpy()
        good = {}
        for i, j in enumerate(h.pj):
            slot, snap = h.picked[j]
            if int(second[i][slot, W_BEGIN]) == snap.version and int(second[i][slot, W_END]) == snap.version:
                good[j] = snap
                if h.root_host is not None:
                    h.roots[j] = bytes(h.root_host[i].numpy().tobytes())
            else:
                self.torn += 1
        h.result = good
        return good

    def fetch_wait(self, h: "AsyncFetch", hash_fn=None) -> Dict[int, Snapshot]:
        """Drive a non-blocking fetch to completion (blocking on its events)."""
        while True:
            r = self.fetch_advance(h, hash_fn)
            if r is not None:
                return r
            h.ev.synchronize()

    def close(self):
        self.drain()
        self.outbox.clear()
        self.inbox.clear()
        self.backend.close()


class AsyncFetch:
    """Handle of a non-blocking mailbox fetch (:meth:`MailboxTransport.fetch_begin`)."""

    def __init__(self, want: Dict[int, int], out: Dict[int, torch.Tensor]):
        self.want, self.out = dict(want), out
        self.result: Optional[Dict[int, Snapshot]] = None
        self.step = 1
        self.ev = None
        self.js: List[int] = []
        self.hdr = self.hdr2 = self.root_host = None
        self.roots: Dict[int, bytes] = {}
        self.gate = None                  # round gate (MailboxTransport.fetch)
        self.gate_round: Optional[int] = None

    @property
    def done_event(self):
        """Event after the fetch's last queued device work (None on CPU / when nothing ran)."""
        return self.ev
