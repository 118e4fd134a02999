"""Client-drift correction for Non-IID federations (SCAFFOLD control variates in update space).

Why: with label-sharded Non-IID data (reference ``serverless_NonIID_IMDB.py:59-60`` shards the
label-sorted IMDB split contiguously, so each client sees essentially one class) every local epoch
pulls a client towards predicting ITS label; averaging / gossip cancels those pulls and the
federation oscillates around the majority rate (profiles/accuracy_sweep_federated.json). SCAFFOLD
(Karimireddy et al., 2020) removes the per-client bias with control variates: client ``i`` steps
along ``g - c_i + c`` where ``c_i`` is its own average update direction and ``c`` the federation's.

MI355X-first formulation — no extra communication and one fused term in the optimizer:

* the correction lives in UPDATE space (what AdamW applies per unit of lr), so it composes with the
  adaptive optimizer: each step is ``p -= lr * (adam_update + s * d_i)``; ``d_i = c - c_i`` is a
  flat fp32 buffer read by the multi-tensor AdamW kernel in the same pass (``corr`` argument of
  ``adamw_mt_kernel``, elementwise.hip) — no extra launch per step;
* ``d_i`` is derived from states the round already has. With ``L = sum of the round's local lrs``,
  ``x`` the round-start model, ``y_i`` the client's trained model and ``x'`` its model after
  aggregation (FedAvg result / gossip mix), SCAFFOLD option II gives
  ``c_i' = (x - y_i) / L - d_i`` and ``c' = mean_j c_j' = (x - x') / L``, so
  ``d_i' = c' - c_i' = (y_i - x') / L + d_i``: two axpby passes per client per round
  (:meth:`after_train`, :meth:`after_mix`), nothing on the wire. With a damping scale ``s`` the
  steps applied ``s * d_i``, so the carried term is ``s * d_i`` (still exactly ``c' - c_i'``).
  Under gossip with a partial topology ``x'`` is the neighbourhood mean, i.e. the neighbourhood
  estimate of ``c``.

Measured (CPU, tiny-bert, 8 one-class clients, 16 rounds, /tmp-free test in tests/test_fl.py):
without correction the global accuracy peaks near 0.95 and collapses back to 0.5; with it both
server FedAvg and serverless gossip reach >= 0.99 and stay there.

**Asynchronous gossip (exchanged control variates).** ``c' = (x - x') / L`` is exact only when
``x'`` mixes models trained in the SAME round from the same start. An asynchronous multi-rank
federation mixes whatever neighbour snapshot is newest (stale by one or more rounds), and a stale
label-shard model carries its client's old per-class pull, so ``(x - x') / L`` no longer estimates
``c`` (2 ranks on one MI355X stayed at the majority rate, profiles/multirank_learning_r3.json).
With ``exchange=True`` every client instead keeps its own control variate explicitly and
PUBLISHES it with its model, in the same versioned, Merkle-committed mailbox payload
(``[model | c_i]``, so a model and its control variate always come from the same version):

* round start (``attach``): ``cv_i <- x_i`` (the start model, needed for ``c_i'``);
* after training (``after_train``): ``c_i' = (x_i - y_i) / L - s * d_i`` — SCAFFOLD option II,
  the client's mean update direction with the applied correction removed (``d_i`` is the
  correction frozen at the round start, ``attach``: a newer one received mid-round waits for the
  next round, so the removed term is exactly the applied one);
* after the exchange (``after_exchange``): ``d_i = sum_j W_ij c_j' - c_i'`` over the newest
  verified snapshots of the neighbours (whatever round they are from) — the stale-exact
  federation control variate, no waiting on any peer.

Under exact same-round mixing on a complete graph both formulations give the identical
``d_i' = (y_i - x') / L + s * d_i`` (``tests/test_fl.py::test_drift_exchange_matches_mix_derived``);
the exchange costs one extra bf16 copy of the parameters on the wire per post.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence

import torch

from .. import ops

MODES = ("none", "scaffold")
# partitions whose clients see skewed label distributions (bcfl/data/partition.py)
LABEL_SKEWED = ("label_shards", "ref_contiguous", "dirichlet")


def resolve_mode(mode: str, partition: str) -> str:
    """``auto``: SCAFFOLD where local optima disagree (label-skewed shards), off for IID splits,
    where the control variates only add noise (profiles/accuracy_curves_iid_mi355x.json)."""
    if mode == "auto":
        return "scaffold" if partition in LABEL_SKEWED else "none"
    return mode


class DriftCorrection:
    def __init__(self, mode: str, scale: float, clients: Iterable[int], numel: int, device):
        if mode not in MODES:
            raise ValueError(f"drift_correction must be one of {MODES}, got {mode!r}")
        self.mode, self.scale = mode, float(scale)
        self.enabled = mode != "none"
        self.clients = list(clients)
        self.numel, self.device = numel, device
        self.buf: Dict[int, torch.Tensor] = {}
        self.ready: Dict[int, bool] = {}
        self.lr_sum: Dict[int, float] = {}
        self.exchange = False
        self.stale_compensation = "none"
        self._pending: Dict[int, Optional[tuple]] = {}
        self.cv: Dict[int, torch.Tensor] = {}   # exchange mode: own control variate c_i
        # exchange mode: per-client buffers that already hold the round-start model (+ the
        # neighbours' updates applied on arrival) — the delta-exchange gossip's start records;
        # when set, cv does not keep its own copy (one model-sized copy per round and one
        # apply pass per arrival less)
        self.start_of: Optional[Dict[int, torch.Tensor]] = None
        # exchange mode: the correction a client's optimizer applies during a round is FROZEN at
        # the round start (a copy of buf), and exactly that one is removed from its new control
        # variate. buf keeps receiving the neighbours' newer control variates mid-round (complete
        # rounds applied between local steps), but they take effect at the next round: with a
        # correction that changes after a rank-dependent number of steps, c_i' = (x - y) / L -
        # s d_i no longer removes what was applied, every client's control variate carries its
        # own error, and on label shards that error is a per-class bias (8 ranks x 1 client on
        # one MI355X: 5 of 10 runs stayed on the majority plateau, profiles/async_protocol_r5_*)
        self.active: Dict[int, torch.Tensor] = {}
        self.used: Dict[int, bool] = {}
        self._used_t: Dict[int, Optional[torch.Tensor]] = {}
        # Round-tagged corrections (exchange mode with round-complete gossip): round r's steps
        # apply d^(r - corr_lag), the correction formed from the control variates of COMPLETE
        # round r - corr_lag, on every client of the federation alike. SCAFFOLD's corrections sum
        # to zero over the clients (sum_i (c_hat - c_i) = 0) only when every client applies
        # the same round's: a client that happens to hold the newest round (the last rank to
        # finish sees it complete at its round end) and one that does not would apply corrections
        # of different rounds, and on label shards the non-zero sum is a class bias that the
        # federation chases round after round (8 ranks x 1 client on 32-CU slices of one MI355X:
        # majority-rate plateau in 6 of 6 runs; in-process virtual ranks, where every client sees
        # a round complete at the same local step, never hit it). Two slots per client (rounds
        # r - 2 in use, r - 1 arriving); the federation makes sure round r - corr_lag has been
        # applied before round r starts (with bounded staleness it always has been posted).
        self.corr_lag: Optional[int] = None
        # round-complete gossip: the new control variate is formed by the gossip's fused round-end
        # pass (ops.delta_round_end_, from round_end_terms) instead of in after_train
        self.defer_cv = False
        self._pend_L: Dict[int, float] = {}
        self.ring: Dict[int, List[torch.Tensor]] = {}
        self.ring_round: Dict[int, List[int]] = {}
        self.lag_miss = 0
        if self.enabled:
            for c in self.clients:
                self.buf[c] = torch.zeros(numel, dtype=torch.float32, device=device)
                self.ready[c] = False

    def use_exchange(self) -> Dict[int, torch.Tensor]:
        """Switch to exchanged control variates (asynchronous gossip); returns the per-client
        ``c_i`` buffers the gossip engine publishes beside the models."""
        if not self.enabled:
            raise RuntimeError("use_exchange() without drift correction")
        self.exchange = True
        for c in self.clients:
            if c not in self.cv:
                self.cv[c] = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        return self.cv

    def drop_exchange(self) -> None:
        self.exchange = False
        self.cv = {}

    def attach(self, opt, c: int, start: Optional[torch.Tensor] = None,
               round_idx: Optional[int] = None) -> None:
        """Before client ``c``'s local steps: its optimizer applies ``d_c`` (round 0: nothing).
        Exchange mode: ``start`` (the round-start model) is kept for ``c_c'``; with round-tagged
        corrections (``corr_lag``) round ``round_idx`` applies d^(round_idx - corr_lag)."""
        if not self.enabled:
            return
        opt.corr_scale = self.scale
        if self.exchange and self.corr_lag is not None and round_idx is not None:
            self._attach_tagged(opt, c, round_idx)
        elif self.exchange and self.ready[c]:
            self.used[c] = True
            a = self.active.get(c)
            if a is None:
                a = self.active[c] = torch.empty_like(self.buf[c])
            a.copy_(self.buf[c])
            opt.corr = a
            self._used_t[c] = a
        else:
            self.used[c] = bool(self.ready[c])
            opt.corr = self.buf[c] if self.ready[c] else None
            self._used_t[c] = opt.corr
        if self.exchange and self.start_of is None:
            if start is None:
                raise ValueError("exchanged control variates need the round-start model")
            self.cv[c].copy_(start)

    def _attach_tagged(self, opt, c: int, r: int) -> None:
        target = r - int(self.corr_lag)
        rounds = self.ring_round.get(c, [])
        t = None
        if target >= 0 and target in rounds:
            t = self.ring[c][rounds.index(target)]     # never rewritten during this round
        elif target >= 0 and any(x >= 0 for x in rounds):
            # round `target` never arrived (a dead source's timeout): the nearest older one,
            # copied, since the slot it sits in may be rewritten while the round runs
            self.lag_miss += 1
            older = [x for x in rounds if 0 <= x <= target] or [max(rounds)]
            src = self.ring[c][rounds.index(max(older))]
            t = self.active.get(c)
            if t is None:
                t = self.active[c] = torch.empty_like(src)
            t.copy_(src)
        opt.corr = t
        self.used[c] = t is not None
        self._used_t[c] = t

    def round_end_terms(self, c: int):
        """Deferred control variate (``defer_cv``): ``(d, scale, 1 / L)`` for
        ``c_c' = (x - y) / L - scale * d`` with the correction the round's steps applied (None:
        none was); ``None`` when client c did not train this round (nothing to form)."""
        L = self._pend_L.pop(c, 0.0)
        if not (self.enabled and self.exchange and self.defer_cv) or L <= 0:
            return None
        used = self._used_t.get(c) if self.used.get(c) else None
        return used, self.scale, 1.0 / L

    def correction_round_needed(self, r: int) -> Optional[int]:
        """Round-tagged mode: the complete round whose corrections round ``r`` applies."""
        if not (self.enabled and self.exchange and self.corr_lag is not None):
            return None
        t = r - int(self.corr_lag)
        return t if t >= 0 else None

    @staticmethod
    def detach(opt) -> None:
        opt.corr = None

    @torch.no_grad()
    def after_train(self, c: int, trained: torch.Tensor, lr_sum: float) -> None:
        """Mix-derived: ``buf <- y_c / L + s * d_c``. Exchange: ``cv <- (x_c - y_c) / L - s * d_c``
        (stream-ordered after the client's last optimizer step)."""
        if not self.enabled or lr_sum <= 0:
            return
        self.lr_sum[c] = float(lr_sum)
        if self.exchange and self.defer_cv:
            self._pend_L[c] = float(lr_sum)   # formed at the round end (round_end_terms)
            return
        if self.exchange:
            if self.start_of is not None:   # cv = (x_c - y_c) / L in one pass
                ops.gossip_mix_(self.cv[c], [self.start_of[c], trained], 0.0,
                                [1.0 / lr_sum, -1.0 / lr_sum])
            else:
                ops.axpby_(self.cv[c], trained, -1.0 / lr_sum, 1.0 / lr_sum)
            used = self._used_t.get(c)
            if self.used.get(c) and used is not None:   # the correction the steps applied
                ops.axpby_(self.cv[c], used, -self.scale, 1.0)
            return
        ops.axpby_(self.buf[c], trained, 1.0 / lr_sum, self.scale if self.ready[c] else 0.0)

    @torch.no_grad()
    def after_mix(self, c: int, aggregated: torch.Tensor) -> None:
        """``d_c' = buf - x'_c / L`` once the client's post-aggregation model is known
        (mix-derived mode; exchange mode forms ``d_c`` in :meth:`after_exchange`)."""
        if not self.enabled or self.exchange or c not in self.lr_sum:
            return
        ops.axpby_(self.buf[c], aggregated, -1.0 / self.lr_sum.pop(c), 1.0)
        self.ready[c] = True

    @torch.no_grad()
    def begin(self, c: int, self_w: float, views: Sequence[torch.Tensor],
              weights: Sequence[float], age: float = 0.0):
        """Exchange mode, BEFORE the model mix: remembers the neighbours' published control
        variates ``views`` (any dtype) and live weights for :meth:`end`. With staleness
        compensation and a stale mix (``age`` = weighted rounds the neighbours' snapshots are
        behind) returns extra model-mix terms that advance the stale views to the present:

        * ``"own"``: + age * (y_c - x_c) = -age * L * (c_c' + s * d_c) — this client's own update
          of the round stands in for what each neighbour did since its snapshot;
        * ``"global"``: -age * L * c_hat (needs c_hat first, so it is formed here)."""
        if not (self.enabled and self.exchange) or c not in self.lr_sum:
            return None
        L = self.lr_sum.pop(c)
        self._pending[c] = (float(self_w), list(views), [float(w) for w in weights])
        mode = self.stale_compensation
        if not mode or mode == "none" or age <= 0 or not self.ready[c]:
            return None
        if mode == "own":
            d_used = self._used_t.get(c) if self.used.get(c) else None
            d_used = d_used if d_used is not None else self.buf[c]
            return [(self.cv[c], -L * float(age)), (d_used, -L * float(age) * self.scale)]
        if mode == "global":
            d = self.buf[c]
            d.copy_(self.cv[c])
            ops.gossip_mix_(d, list(views), float(self_w), [float(w) for w in weights])
            self._pending[c] = None          # buf already holds c_hat
            return [(d, -L * float(age))]
        raise ValueError(f"unknown drift_stale_compensation {mode!r}")

    @torch.no_grad()
    def end(self, c: int) -> None:
        """After the model mix: ``d_c = c_hat - c_c'`` with
        ``c_hat = self_w * c_c' + sum_j w_j c_j'`` (fp32 accumulate in the mix kernel)."""
        if c not in self._pending:
            return
        p = self._pending.pop(c)
        d = self.buf[c]
        if p is not None:
            self_w, views, weights = p
            d.copy_(self.cv[c])
            ops.gossip_mix_(d, views, self_w - 1.0, weights)
        else:
            ops.axpby_(d, self.cv[c], -1.0, 1.0)
        self.ready[c] = True

    @torch.no_grad()
    def set_correction(self, c: int, views: Sequence[torch.Tensor], weights: Sequence[float],
                       round_idx: Optional[int] = None) -> None:
        """Exchange mode, round-complete gossip (:meth:`bcfl.parallel.gossip.MailboxGossip.
        _refresh_aux`): ``d_c = sum_j w_j c_j`` with every term from the same applied round
        (the client's own control variate enters with weight ``W_cc - 1``); with round-tagged
        corrections it is filed under that round (two slots per client)."""
        if not (self.enabled and self.exchange):
            return
        d = self.buf[c]
        if self.corr_lag is not None and round_idx is not None:
            if c not in self.ring:
                self.ring[c] = [self.buf[c], torch.zeros_like(self.buf[c])]
                self.ring_round[c] = [-1, -1]
            slot = int(round_idx) % 2
            d = self.ring[c][slot]
            self.ring_round[c][slot] = int(round_idx)
        if views:   # self weight 0: d is overwritten (the kernel never reads it)
            ops.gossip_mix_(d, list(views), 0.0, [float(w) for w in weights])
        else:
            d.zero_()
        self.ready[c] = True
        self.lr_sum.pop(c, None)

    def after_exchange(self, c: int, self_w: float, views: Sequence[torch.Tensor],
                       weights: Sequence[float]) -> None:
        """:meth:`begin` + :meth:`end` without a model mix in between."""
        self.begin(c, self_w, views, weights)
        self.end(c)

    # ---- resume -------------------------------------------------------------------------
    def state_dict(self) -> Optional[dict]:
        if not self.enabled:
            return None
        st = {"buf": {int(c): t.detach().cpu().clone() for c, t in self.buf.items()},
              "ready": {int(c): bool(v) for c, v in self.ready.items()}}
        if self.exchange:
            st["cv"] = {int(c): t.detach().cpu().clone() for c, t in self.cv.items()}
        if self.ring:   # round-tagged corrections (slot 0 is buf itself)
            st["ring1"] = {int(c): r[1].detach().cpu().clone() for c, r in self.ring.items()}
            st["ring_round"] = {int(c): list(v) for c, v in self.ring_round.items()}
        return st

    @torch.no_grad()
    def load_state_dict(self, st: Optional[dict]) -> None:
        if not self.enabled or not st:
            return
        for c, t in st["buf"].items():
            self.buf[int(c)].copy_(t)
        for c, v in st["ready"].items():
            self.ready[int(c)] = bool(v)
        if self.exchange and "cv" in st:
            for c, t in st["cv"].items():
                self.cv[int(c)].copy_(t)
        for c, t in st.get("ring1", {}).items():
            c = int(c)
            self.ring[c] = [self.buf[c], t.to(self.buf[c].device).clone()]
            rr = st["ring_round"]
            self.ring_round[c] = [int(x) for x in rr.get(c, rr.get(str(c), [-1, -1]))]
