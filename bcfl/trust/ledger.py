"""Blockchain ledger of federated updates (BC-FL).

The reference names a blockchain layer but has no ledger code. Here every client
update becomes a block ``{height, prev_hash, ts, round, client, kind, update_root, verdict,
payload}`` whose SHA-256 hash commits to its predecessor; ``update_root`` is the SHA-256 Merkle root
of the client's flat parameter buffer, hashed on the GPU. All ranks append the same blocks in the
same order from all-gathered records, so their tips must match — :meth:`Ledger.consensus_check`
compares tips across ranks every round (a cheap agreement protocol over RCCL/gloo).

Backed by the native C++ chain (``bcfl._host.Ledger``) when built; a pure-Python chain with the
identical preimage/hash format otherwise.
"""
from __future__ import annotations

import hashlib
import json
import os
import time
from typing import Any, Dict, Iterable, List, Optional

try:
    from .. import _host as _H  # type: ignore
except Exception:  # pragma: no cover
    _H = None

ZERO = "0" * 64


def block_preimage(b: Dict[str, Any]) -> str:
    return "|".join([str(int(b["height"])), b["prev_hash"], f"{float(b['ts']):.6f}",
                     str(int(b["round"])), str(int(b["client"])), b["kind"], b["update_root"],
                     b["verdict"], b["payload"]])


def block_hash(b: Dict[str, Any]) -> str:
    return hashlib.sha256(block_preimage(b).encode()).hexdigest()


class _PyChain:
    def __init__(self, genesis_payload: str, ts: float):
        g = dict(height=0, prev_hash=ZERO, ts=ts, round=-1, client=-1, kind="genesis",
                 update_root="", verdict="", payload=genesis_payload)
        g["hash"] = block_hash(g)
        self.chain = [g]

    def append(self, round, client, kind, root, verdict, payload, ts):
        b = dict(height=len(self.chain), prev_hash=self.chain[-1]["hash"], ts=ts, round=round,
                 client=client, kind=kind, update_root=root, verdict=verdict, payload=payload)
        b["hash"] = block_hash(b)
        self.chain.append(b)
        return dict(b)

    def verify(self) -> int:
        for i, b in enumerate(self.chain):
            if b["height"] != i:
                return i
            if b["prev_hash"] != (ZERO if i == 0 else self.chain[i - 1]["hash"]):
                return i
            if block_hash(b) != b["hash"]:
                return i
        return -1

    def tip(self):
        return self.chain[-1]["hash"]

    def __len__(self):
        return len(self.chain)

    def block(self, i):
        return dict(self.chain[i])

    def set_field(self, i, k, v):
        self.chain[i][k] = v

    def push_raw(self, d):
        self.chain.append(dict(d))

    def clear(self):
        self.chain.clear()


class Ledger:
    def __init__(self, genesis: Optional[Dict[str, Any]] = None, path: Optional[str] = None,
                 native: Optional[bool] = None, ts: Optional[float] = None, truncate: bool = True):
        payload = json.dumps(genesis or {}, sort_keys=True, separators=(",", ":"))
        ts = time.time() if ts is None else ts
        use_native = (_H is not None) if native is None else (native and _H is not None)
        self._c = _H.Ledger(payload, ts) if use_native else _PyChain(payload, ts)
        self.native = use_native
        self.path = path
        self._flushed = 0
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            if truncate and os.path.exists(path):
                os.remove(path)

    # ------------------------------------------------------------------------------------
    def append(self, round_idx: int, client: int, kind: str, update_root: str = "",
               verdict: str = "accept", payload: Optional[Dict[str, Any]] = None,
               ts: Optional[float] = None) -> Dict[str, Any]:
        p = json.dumps(payload or {}, sort_keys=True, separators=(",", ":"))
        return self._c.append(int(round_idx), int(client), kind, update_root, verdict, p,
                              time.time() if ts is None else float(ts))

    def verify(self) -> int:
        """-1 if the chain is intact, else the first bad height."""
        return int(self._c.verify())

    @property
    def tip(self) -> str:
        return self._c.tip()

    def __len__(self) -> int:
        return len(self._c)

    def block(self, i: int) -> Dict[str, Any]:
        return self._c.block(i)

    def blocks(self) -> List[Dict[str, Any]]:
        return [self.block(i) for i in range(len(self))]

    def tamper(self, i: int, field: str, value: str):
        """Fault injection for tests: mutate a committed block in place."""
        self._c.set_field(i, field, value)

    def flush(self):
        if not self.path:
            return
        with open(self.path, "a") as fh:
            for i in range(self._flushed, len(self)):
                fh.write(json.dumps(self.block(i), sort_keys=True) + "\n")
        self._flushed = len(self)

    @classmethod
    def load(cls, path: str, native: Optional[bool] = None, verify: bool = True) -> "Ledger":
        """Load a JSONL chain. Rows are untrusted input: the chain is re-verified (heights,
        prev-hash links, block hashes) before it is returned; ``verify=False`` only for forensics."""
        with open(path) as fh:
            rows = [json.loads(l) for l in fh if l.strip()]
        led = cls(native=native, truncate=False)
        led._c.clear()
        for r in rows:
            led._c.push_raw(r)
        led.path, led._flushed = path, len(rows)
        if verify:
            bad = led.verify()
            if bad != -1:
                raise ValueError(f"ledger {path} fails verification at height {bad}")
        return led

    def truncated(self, height: int) -> "Ledger":
        """A copy holding blocks [0, height) (resume: drop blocks appended after a checkpoint)."""
        led = Ledger(native=self.native, truncate=False)
        led._c.clear()
        for i in range(min(height, len(self))):
            led._c.push_raw(self.block(i))
        return led

    def rewrite(self):
        """Rewrite the JSONL file from the in-memory chain."""
        if not self.path:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as fh:
            for i in range(len(self)):
                fh.write(json.dumps(self.block(i), sort_keys=True) + "\n")
        os.replace(tmp, self.path)
        self._flushed = len(self)

    def consensus_check(self) -> bool:
        """All ranks hold the same tip (ranks append identical blocks in identical order)."""
        from ..parallel import dist as D
        tips = D.all_gather_object(self.tip)
        return all(t == tips[0] for t in tips)
