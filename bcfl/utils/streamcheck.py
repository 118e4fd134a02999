"""Happens-before race detector for HIP streams ("HIP event ordering asserts in
debug builds").

bcfl overlaps work on many streams: client lanes, side-stream weight gradients, the overlapped
global / local evaluation, the checkpoint copy stream, the mailbox post / fetch streams. Any buffer
that one stream writes and another reads (or writes) must be ordered by an event the consumer
waited on — otherwise the consumer may see the producer's old or half-written data, and the run
is only reproducible by luck. This module checks that ordering at run time.

Model: every stream carries a **vector clock** (stream -> count). An access on stream ``s`` is
stamped with ``s``'s own count; recording an event snapshots ``s``'s clock and advances it; a wait
joins the event's snapshot into the waiting stream's clock; a host synchronisation (event /
stream / device synchronize, a blocking D2H read) joins into the HOST clock, which every later
launch inherits (a kernel launched after the host saw an event complete runs after it). Two
accesses to overlapping bytes from different streams, at least one a write, RACE unless the later
one's stream clock covers the earlier one's stamp.

What is observed:

* every ATen op on CUDA tensors, through a ``TorchDispatchMode`` (the op schema says which
  arguments are written; fresh outputs count as writes, so a caching-allocator block reused on one
  stream while another stream still used it — the missing ``record_stream`` hazard — is caught);
* bcfl's own HIP kernels, through a proxy around the native module (:data:`NATIVE_WRITES` lists
  the arguments each kernel writes; everything else it is given is read);
* ``torch.cuda.Event.record / wait / synchronize / query``, ``Stream.wait_event / wait_stream /
  synchronize / query`` and ``torch.cuda.synchronize`` (patched while enabled).

Enable with ``BCFL_DEBUG_STREAMS=1`` (the federation turns it on at construction and reports in
``finish()``), or explicitly with :func:`enable` / :func:`disable`. The core (:class:`HBDetector`)
is pure Python over abstract stream ids and is unit-tested on the CPU.
"""
from __future__ import annotations

import os
import sys
import threading
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Tuple

# argument positions each native kernel WRITES (bcfl/csrc/bindings.cpp); other tensor arguments
# are reads, returned tensors are fresh writes
NATIVE_WRITES: Dict[str, Tuple[int, ...]] = {
    "xent_stats": (2,),
    "adamw": (0, 2, 3, 4),
    "adamw_mt": (0, 1, 2, 3),
    "mix": (0, 4),
    "axpby": (0,),
    "delta_round_end": (0, 2, 3, 4, 6),
    "cast_copy": (0,),
    "delta_encode": (1, 2),
    "linear_dgrad_acc": (2,),
    "linear_fwd_acc": (2,),
    "gemm8": (8,),
}


@dataclass
class Access:
    stream: int
    clock: int
    lo: int
    hi: int
    write: bool
    where: str


@dataclass
class Race:
    key: int
    first: Access
    second: Access

    def __str__(self) -> str:
        kind = ("write-write" if self.first.write and self.second.write else
                "write-read" if self.first.write else "read-write")
        return (f"{kind} race on bytes [{max(self.first.lo, self.second.lo):#x}, "
                f"{min(self.first.hi, self.second.hi):#x}): stream {self.first.stream} "
                f"({self.first.where}) then stream {self.second.stream} ({self.second.where}) "
                "with no event ordering them")


def _join(a: Dict[int, int], b: Dict[int, int]) -> None:
    for k, v in b.items():
        if a.get(k, 0) < v:
            a[k] = v


class HBDetector:
    """Vector-clock happens-before checker over abstract stream ids and byte ranges."""

    def __init__(self, keep_per_stream: int = 16, max_races: int = 64):
        self.vc: Dict[int, Dict[int, int]] = {}
        self.host: Dict[int, int] = {}
        self.events: Dict[int, Dict[int, int]] = {}
        self.acc: Dict[int, Dict[int, List[Access]]] = {}   # storage key -> stream -> accesses
        self.races: List[Race] = []
        self.keep = keep_per_stream
        self.max_races = max_races
        self.checked = 0
        self._seen_pairs = set()
        self._lock = threading.Lock()

    def _clock(self, s: int) -> Dict[int, int]:
        c = self.vc.get(s)
        if c is None:
            c = self.vc[s] = {s: 1}
        return c

    # ---- synchronisation ---------------------------------------------------------------
    def record(self, s: int, ev: int) -> None:
        with self._lock:
            c = self._clock(s)
            _join(c, self.host)
            self.events[ev] = dict(c)
            c[s] += 1

    def wait_event(self, s: int, ev: int) -> None:
        with self._lock:
            snap = self.events.get(ev)
            if snap is not None:      # an event never recorded is a no-op wait
                _join(self._clock(s), snap)

    def wait_stream(self, s: int, t: int) -> None:
        with self._lock:
            c = self._clock(t)
            _join(self._clock(s), c)
            c[t] += 1

    def host_event(self, ev: int) -> None:
        with self._lock:
            snap = self.events.get(ev)
            if snap is not None:
                _join(self.host, snap)

    def host_stream(self, s: int) -> None:
        with self._lock:
            c = self._clock(s)
            _join(self.host, c)
            c[s] += 1

    def host_all(self) -> None:
        with self._lock:
            for s, c in self.vc.items():
                _join(self.host, c)
                c[s] += 1

    # ---- accesses ----------------------------------------------------------------------
    def access(self, s: int, key: int, lo: int, hi: int, write: bool, where: str = "",
               fresh: bool = False) -> None:
        """Stream ``s`` reads (or writes) bytes [lo, hi) of storage ``key``. ``fresh``: a new
        allocation landing there — checked like a write against every other stream's use."""
        if hi <= lo:
            return
        with self._lock:
            c = self._clock(s)
            _join(c, self.host)
            me = Access(s, c[s], lo, hi, write or fresh, where)
            per = self.acc.setdefault(key, {})
            self.checked += 1
            for t, lst in per.items():
                if t == s:
                    continue
                seen = c.get(t, 0)
                for a in lst:
                    if a.hi <= lo or a.lo >= hi or not (a.write or me.write):
                        continue
                    if seen < a.clock:
                        self._report(key, a, me)
            lst = per.setdefault(s, [])
            if me.write:   # a write on s supersedes s's earlier accesses it covers
                lst[:] = [a for a in lst if not (a.lo >= lo and a.hi <= hi)]
            lst.append(me)
            if len(lst) > self.keep:
                del lst[: len(lst) - self.keep]

    def _report(self, key: int, a: Access, b: Access) -> None:
        sig = (a.where, b.where, a.stream, b.stream)
        if sig in self._seen_pairs or len(self.races) >= self.max_races:
            return
        self._seen_pairs.add(sig)
        self.races.append(Race(key, a, b))

    def forget(self, key: int) -> None:
        """Storage handed back with ``record_stream`` ordering: the allocator itself delays its
        reuse until the recorded streams are done, so a later allocation there is not a race."""
        with self._lock:
            self.acc.pop(key, None)


# ---------------------------------------------------------------------------------------------
# torch / HIP integration
# ---------------------------------------------------------------------------------------------
_STATE: Dict[str, object] = {}


def detector() -> Optional[HBDetector]:
    return _STATE.get("det")   # type: ignore[return-value]


def enabled() -> bool:
    return "det" in _STATE


def _where(op: str) -> str:
    """Op name + the innermost bcfl caller outside this module and the op wrappers."""
    f = sys._getframe(2)
    while f is not None:
        fn = f.f_code.co_filename
        if "/bcfl/" in fn and not fn.endswith(("streamcheck.py", "/ops/_native.py")):
            return f"{op} @ {fn.split('/bcfl/')[-1]}:{f.f_lineno}"
        f = f.f_back
    return op


def _sid(stream) -> int:
    return int(stream.cuda_stream)


def _span(t) -> Tuple[int, int, int]:
    """(storage key, lo, hi) of the bytes a tensor view can touch."""
    st = t.untyped_storage()
    base = st.data_ptr()
    if t.numel() == 0:
        return base, 0, 0
    es = t.element_size()
    lo = t.data_ptr()
    ext = 1 + sum((n - 1) * abs(s) for n, s in zip(t.shape, t.stride()) if n > 0)
    return base, lo, lo + ext * es


def _tensors(v) -> Iterable:
    import torch
    if isinstance(v, torch.Tensor):
        yield v
    elif isinstance(v, (list, tuple)):
        for x in v:
            if isinstance(x, torch.Tensor):
                yield x


def _note(t, write: bool, where: str, fresh: bool = False) -> None:
    if not getattr(t, "is_cuda", False):
        return
    import torch
    det = detector()
    key, lo, hi = _span(t)
    det.access(_sid(torch.cuda.current_stream(t.device)), key, lo, hi, write, where, fresh)


class _NativeProxy:
    """The native extension module with every kernel call reported to the detector."""

    def __init__(self, mod):
        self._mod = mod
        self._cache: Dict[str, object] = {}

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn):
            return fn
        w = self._cache.get(name)
        if w is None:
            writes = NATIVE_WRITES.get(name, ())

            def w(*args, _fn=fn, _name=name, _writes=writes, **kwargs):
                where = _where("native." + _name)
                for i, a in enumerate(args):
                    for t in _tensors(a):
                        _note(t, i in _writes, where)
                for a in kwargs.values():
                    for t in _tensors(a):
                        _note(t, False, where)
                out = _fn(*args, **kwargs)
                for t in _tensors(out):
                    _note(t, True, where, fresh=True)
                return out
            self._cache[name] = w
        return w


def _make_mode():
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode

    class _Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            out = func(*args, **kwargs)
            try:
                self._observe(func, args, kwargs, out)
            except Exception:   # the checker must never break the run it checks
                pass
            return out

        @staticmethod
        def _observe(func, args, kwargs, out):
            name = func.__name__
            if name.startswith("record_stream"):
                for t in _tensors(args[0] if args else None):
                    if t.is_cuda:
                        detector().forget(_span(t)[0])
                return
            schema = func._schema
            ins, outs = [], []
            any_cuda = False
            to_host = False
            for i, a in enumerate(schema.arguments):
                v = args[i] if i < len(args) else kwargs.get(a.name)
                w = a.alias_info is not None and a.alias_info.is_write
                for t in _tensors(v):
                    if t.is_cuda:
                        any_cuda = True
                        (outs if w else ins).append(t)
                    elif w:
                        to_host = True
            rets = list(_tensors(out))
            aliases = all(r.alias_info is not None for r in schema.returns) if schema.returns else False
            if aliases and not outs:
                return        # a view: no data is touched
            where = None
            for t in ins:
                where = where or _where("aten." + name)
                _note(t, False, where)
            for t in outs:
                where = where or _where("aten." + name)
                _note(t, True, where)
            in_ptrs = {x.untyped_storage().data_ptr() for x in ins + outs}
            for t in rets:
                if t.is_cuda and t.untyped_storage().data_ptr() not in in_ptrs:
                    where = where or _where("aten." + name)
                    _note(t, True, where, fresh=True)
                elif not t.is_cuda and any_cuda:
                    to_host = True
            if to_host and any_cuda and not kwargs.get("non_blocking", False):
                # a blocking device -> host read synchronises the current stream
                detector().host_stream(_sid(torch.cuda.current_stream()))

    return _Mode()


def enable() -> HBDetector:
    """Install the detector (dispatch mode + stream/event hooks + native proxy)."""
    import torch
    if enabled():
        return detector()   # type: ignore[return-value]
    det = HBDetector()
    _STATE["det"] = det
    C = torch.cuda
    orig = {
        "ev_record": C.Event.record, "ev_wait": C.Event.wait, "ev_sync": C.Event.synchronize,
        "ev_query": C.Event.query, "st_wait_event": C.Stream.wait_event,
        "st_wait_stream": C.Stream.wait_stream, "st_sync": C.Stream.synchronize,
        "st_query": C.Stream.query, "sync": C.synchronize,
    }
    _STATE["orig"] = orig

    def ev_record(self, stream=None):
        s = stream if stream is not None else C.current_stream()
        det.record(_sid(s), id(self))
        return orig["ev_record"](self, stream)

    def ev_wait(self, stream=None):
        s = stream if stream is not None else C.current_stream()
        det.wait_event(_sid(s), id(self))
        return orig["ev_wait"](self, stream)

    def ev_sync(self):
        r = orig["ev_sync"](self)
        det.host_event(id(self))
        return r

    def ev_query(self):
        r = orig["ev_query"](self)
        if r:
            det.host_event(id(self))
        return r

    def st_wait_event(self, event):
        det.wait_event(_sid(self), id(event))
        return orig["st_wait_event"](self, event)

    def st_wait_stream(self, stream):
        det.wait_stream(_sid(self), _sid(stream))
        # the original records a fresh event on `stream` and waits on it: call the raw methods
        ev = C.Event()
        orig["ev_record"](ev, stream)
        return orig["st_wait_event"](self, ev)

    def st_sync(self):
        r = orig["st_sync"](self)
        det.host_stream(_sid(self))
        return r

    def st_query(self):
        r = orig["st_query"](self)
        if r:
            det.host_stream(_sid(self))
        return r

    def sync(device=None):
        r = orig["sync"](device)
        det.host_all()
        return r

    C.Event.record, C.Event.wait, C.Event.synchronize, C.Event.query = ev_record, ev_wait, ev_sync, ev_query
    C.Stream.wait_event, C.Stream.wait_stream = st_wait_event, st_wait_stream
    C.Stream.synchronize, C.Stream.query = st_sync, st_query
    C.synchronize = sync
    mode = _make_mode()
    mode.__enter__()
    _STATE["mode"] = mode
    return det


def disable() -> Optional[HBDetector]:
    """Remove the hooks; returns the detector (its ``races``)."""
    import torch
    det = _STATE.pop("det", None)
    if det is None:
        return None
    mode = _STATE.pop("mode", None)
    if mode is not None:
        mode.__exit__(None, None, None)
    orig = _STATE.pop("orig")
    C = torch.cuda
    C.Event.record, C.Event.wait = orig["ev_record"], orig["ev_wait"]
    C.Event.synchronize, C.Event.query = orig["ev_sync"], orig["ev_query"]
    C.Stream.wait_event, C.Stream.wait_stream = orig["st_wait_event"], orig["st_wait_stream"]
    C.Stream.synchronize, C.Stream.query = orig["st_sync"], orig["st_query"]
    C.synchronize = orig["sync"]
    return det


def wrap_native(mod):
    """The native module as the ops layer should call it (a reporting proxy while enabled)."""
    if not enabled():
        return mod
    px = _STATE.get("proxy")
    if px is None or px._mod is not mod:
        px = _STATE["proxy"] = _NativeProxy(mod)
    return px


def requested() -> bool:
    return os.environ.get("BCFL_DEBUG_STREAMS", "") not in ("", "0")


def report(det: Optional[HBDetector] = None, stream=None) -> List[str]:
    det = det or detector()
    if det is None:
        return []
    lines = [str(r) for r in det.races]
    out = stream if stream is not None else sys.stderr
    print(f"[streamcheck] {det.checked} accesses checked, {len(lines)} race(s)", file=out, flush=True)
    for ln in lines:
        print("[streamcheck] " + ln, file=out, flush=True)
    return lines
