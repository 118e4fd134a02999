#!/usr/bin/env python
"""Headline benchmark: per-round wall-clock (+ final accuracy) of BERT-base, 8-client async P2P
gossip, Non-IID — BASELINE.json's metric on BASELINE.json config 3.

One "step" = one federated ROUND of an 8-client federation: every client trains one local epoch
(240 samples = 8 batches of 32, reference ``serverless_NonIID_IMDB.py:59``), evaluates on its 60
local test rows, publishes its model into its peers' one-sided hipIpc mailboxes (async: the copies
to every peer run concurrently on side streams; receivers mix the newest complete snapshot — with
drift correction across ranks, each client's SCAFFOLD control variate travels in the same
post, so the federation control variate is exact for whatever snapshot round is mixed),
every received payload is re-hashed and checked against its sender's committed Merkle root
before it is mixed (only at N > 1: with all 8 clients on one rank nothing crosses a process),
every client model is scored on its stride of a class-balanced 1000-row global draw (overlapped
with the next round on a side stream), every update is chained into the ledger, and the model is
checkpointed (async).

Scaling: the federation always has 8 clients (the config names 8); N GPUs host 8/N clients each
(strong scaling over GPUs). ``value`` = seconds per round for the whole job (max over ranks).
The JSON also carries device-time phases per round (HIP events, min / max over ranks), the
overlapped (hidden) side-stream time, process-start-to-end latency (the reference's "Latency"),
and with N > 1 the measured mailbox post bandwidth, staleness and verification counts.

    python bench.py                                   # 1 GPU, 8 virtual clients
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

T_IMPORT = time.time()

# reference serverless IMDB latency (All_graphs_IMDB_dataset.ipynb:748): 27.8 min @5 workers,
# 40 min @10 workers over 20 rounds -> 1.39 / 2.00 min/round; linear interpolation at 8 clients:
BASELINE_S_PER_ROUND = (27.8 + (40.0 - 27.8) * (8 - 5) / (10 - 5)) / 20.0 * 60.0  # 105.36 s
# reference final global accuracy, serverless Non-IID IMDB (All_graphs_IMDB_dataset.ipynb:1142)
BASELINE_FINAL_ACC = 0.54
ACCURACY_NOTE = (
    "synthetic IMDB-shaped data + random-init BERT-base; final_accuracy is scored on a "
    "class-balanced 1000-row global draw (final_majority_rate = what a constant predictor "
    "scores). Label-sharded Non-IID clients (each client sees ONE class) collapse to the majority "
    "rate under plain gossip averaging; the bench's protocol adds SCAFFOLD-style client-drift "
    "correction (update-space control variates fused into AdamW, no extra communication, "
    "bcfl/fl/drift.py) with the reference's fresh AdamW per round. 25-round curves on MI355X with "
    "and without it: profiles/accuracy_curves_scaffold_mi355x.json (benchmarks/accuracy_curves.py)")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--preset", default="baseline3_learnable",
                    help="baseline3_learnable (random-init protocol) | baseline3_bert_serverless_noniid "
                         "(reference hyper-parameters: lr 5e-5, fresh AdamW per round)")
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--mode", default="serverless")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--sync", action="store_true", help="synchronous gossip instead of async")
    ap.add_argument("--no-ledger", action="store_true")
    ap.add_argument("--no-ckpt", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--lanes", type=int, default=0, help="concurrent client lanes per GPU (0 = auto)")
    ap.add_argument("--transport", default="auto",
                    help="serverless gossip transport: auto (N > 1: one-sided hipIpc mailboxes; N = 1: "
                         "loopback = every client its own virtual rank, the multi-rank async protocol "
                         "in one process) | mailbox | loopback | rccl")
    ap.add_argument("--overlap-wgrad", type=int, default=-1, help="1/0 force, -1 auto")
    ap.add_argument("--anomaly-filter", default=None,
                    help="override the preset's update anomaly filter (none|pagerank|modz|both)")
    ap.add_argument("--no-info-passing", action="store_true",
                    help="skip the post-run information-passing measurement (N > 1)")
    ap.add_argument("--global-test-samples", type=int, default=0,
                    help="override the global evaluation draw (experiments only; 0 = preset)")
    ap.add_argument("--batch-size", type=int, default=0,
                    help="override the preset's local batch size (0 = preset)")
    ap.add_argument("--micro-batches", type=int, default=0,
                    help="ranks training one client at a time: 2 = concurrent micro-batches, 1 = off, 0 = auto")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra FLConfig override (JSON value), e.g. --set max_grad_norm=1.0")
    return ap.parse_args()


def _overrides(items):
    out = {}
    for it in items:
        k, _, v = it.partition("=")
        try:
            out[k.strip()] = json.loads(v)
        except json.JSONDecodeError:
            out[k.strip()] = v
    return out


def _launch_ranks(a) -> int:
    """``--gpus N`` without a torchrun environment: start N ranks (one process per GPU) as a
    CHILD ``torch.distributed.run`` job and return its exit code. Nothing here has touched the GPU
    yet (no torch import), and the parent waits instead of exec'ing."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def _heartbeat(rank: int, what: str, every_s: float = 30.0) -> list:
    """Rank 0: a daemon thread prints what the bench is doing to stderr every ``every_s`` seconds
    (a Llama-3-8B federation takes minutes to build and ~15 s per round; the printing never
    touches the GPU). Returns the mutable status cell."""
    import threading
    cell = [what]
    if rank != 0:
        return cell
    t0 = time.time()

    def run():
        while True:
            time.sleep(every_s)
            print(f"[bench] {time.time() - t0:.0f}s: {cell[0]}", file=sys.stderr, flush=True)
    threading.Thread(target=run, daemon=True).start()
    return cell


MODEL_NAMES = {"bert-base": "BERT-base", "biobert": "BioBERT", "albert-base-v2": "ALBERT-base-v2",
               "distilbert": "DistilBERT", "llama3-8b-lora": "Llama-3-8B LoRA",
               "tiny-bert": "tiny-BERT", "tiny-llama-lora": "tiny-Llama LoRA"}


def metric_name(cfg) -> str:
    """BASELINE.json's metric string for the bench's config (the default run names exactly
    "per-round wall-clock + final accuracy, BERT-base 8-client async P2P Non-IID")."""
    from bcfl.fl.drift import LABEL_SKEWED
    mode = ("server FedAvg" if cfg.mode == "server" else
            "async P2P" if cfg.async_gossip else "sync P2P")
    part = "Non-IID" if cfg.partition in LABEL_SKEWED else "IID"
    return (f"per-round wall-clock + final accuracy, {MODEL_NAMES.get(cfg.model, cfg.model)} "
            f"{cfg.num_clients}-client {mode} {part}")


def _protocol(fed, timed) -> dict:
    """What the round's exchange actually mixed: exchange kind (``state`` =
    neighbours' model states, ``delta`` = their cumulative updates, each applied once), how it is
    applied, the transport, the mean staleness of the applied neighbour updates over the timed
    rounds, and how many received updates were re-hashed and verified against their sender's
    committed Merkle root."""
    g = fed.gossip
    if g is None:
        return {"exchange": "fedavg", "transport": fed.cfg.server_transport}
    st = [float(h.get("stale_rounds") or 0.0) for h in timed]
    verified = 0
    if fed.ledger is not None:
        verified = sum(1 for b in fed.ledger.blocks() if b["kind"] == "verify" and b["verdict"] == "accept")
    out = {"exchange": getattr(g, "exchange", "state"),
           "apply": (getattr(g, "apply_mode", None) if getattr(g, "exchange", "") == "delta" else None),
           "transport": fed.transport,
           "virtual_ranks": bool(getattr(g, "virtual", False)),
           "mix_staleness_rounds": (sum(st) / len(st)) if st else 0.0,
           "verified_receives": verified}
    tr = getattr(g, "transport", None)
    if hasattr(tr, "stats"):
        out["loopback"] = tr.stats()
    return out


def _async_mix_desc(fed) -> str:
    g = fed.gossip
    delta = getattr(g, "exchange", "state") == "delta"
    complete = getattr(g, "apply_mode", "") == "complete"
    d = ("neighbours' cumulative updates applied once each" + (
        (", every source's round-T update together once the round is complete (own included), "
         + ("between local steps" if getattr(g, "apply_on_arrival", False) else "at the round end"))
        if complete else
        ", on arrival between local steps" if getattr(g, "apply_on_arrival", False) else
        ", at the round end") if delta else "newest complete snapshot of each neighbour")
    if getattr(g, "virtual", False):
        lag = g.transport.lag
        d += (f" (in-process virtual ranks: every post visible {lag[0]}-{lag[1]} local steps "
              "after it was made)")
    lead = int(fed.cfg.gossip_max_lead)
    d += (f"; bounded staleness: waits only while a neighbour is > {lead} rounds behind"
          if lead > 0 and fed.rt.distributed else "; never waits")
    if fed.drift.exchange:
        d += " + exchanged SCAFFOLD control variates (stale-exact)"
    if delta and getattr(fed, "keep_opt", False) and not fed.cfg.keep_optimizer_state:
        d += "; client AdamW moments kept across rounds"
    return d


def _rehearsal_cu_split() -> None:
    """``BCFL_REHEARSE_CUS=<compute units>``: ranks REHEARSED on one GPU each get a disjoint 1/N of
    its compute units (ROCr's ``HSA_CU_MASK``, set before the runtime initialises), so N processes
    behave like N equal, slower GPUs instead of time-slicing the whole chip — the pacing the 8-GPU
    run has (one rank per GPU), which is what the asynchronous gossip's staleness depends on."""
    cus = int(os.environ.get("BCFL_REHEARSE_CUS", "0") or 0)
    w, r = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))
    if cus <= 0 or w <= 1:
        return
    per = cus // w
    os.environ["HSA_CU_MASK"] = f"0:{r * per}-{(r + 1) * per - 1}"


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_launch_ranks(a))
    _rehearsal_cu_split()
    import bcfl  # noqa: F401  (sets the GEMM-library environment before torch initialises it)
    import torch
    from bcfl import ops
    from bcfl.config import get_preset
    from bcfl.fl import Federation
    from bcfl.parallel import dist as D

    rt = D.init_runtime(a.device)
    if os.environ.get("BCFL_REHEARSE_CUS") and rt.world > 1 and torch.cuda.is_available():
        # N ranks share one GPU's HBM: cap each caching allocator (it keeps ~2x its peak cached
        # across its streams) so N of them plus the mailboxes fit
        torch.cuda.set_per_process_memory_fraction(0.7 / rt.world)
    if rt.world != a.gpus:
        raise SystemExit(f"bench.py --gpus {a.gpus} but the job has WORLD_SIZE={rt.world}: "
                         "launch one rank per GPU (torch.distributed.run --nproc-per-node N)")
    out = a.out or os.path.join("runs", "bench", f"n{rt.world}")
    transport = a.transport
    if transport == "auto" and a.mode == "serverless" and not a.sync:
        # N = 1: the 8 clients run the SAME asynchronous protocol as on 8 GPUs (delta exchange,
        # round-complete application, exchanged control variates), each client its own virtual
        # rank whose posts reach the others 1-2 local steps late (the round-4
        # single-process bench mixed same-round states, a synchronous algorithm)
        transport = "loopback" if rt.world == 1 else "mailbox"
    lanes = a.lanes
    if transport == "loopback" and lanes == 0 and "8b" not in a.model.lower():
        # one lane (HIP stream) per virtual rank; an 8B model keeps the federation's activation-
        # memory cap (2 lanes: ~45 GB of saved activations per lane at batch 32)
        lanes = a.clients
    tr_kw = {} if transport == "auto" else {"gossip_transport": transport}
    kw = dict(model=a.model, num_clients=a.clients, num_rounds=a.warmup + a.steps, mode=a.mode,
              async_gossip=not a.sync, ledger=not a.no_ledger,
              save_every=0 if a.no_ckpt else 1, out_dir=out, reference_prints=False,
              device=a.device, client_lanes=lanes, micro_batches=a.micro_batches,
              overlap_wgrad=None if a.overlap_wgrad < 0 else bool(a.overlap_wgrad), **tr_kw)
    if a.lr is not None:
        kw["lr"] = a.lr
    if a.batch_size > 0:
        kw["batch_size"] = a.batch_size
    if a.global_test_samples > 0:
        kw["global_test_samples"] = a.global_test_samples
    if a.anomaly_filter:
        kw["anomaly_filter"] = a.anomaly_filter
    kw.update(_overrides(a.set))     # --set wins
    cfg = get_preset(a.preset, **kw)
    hb = _heartbeat(rt.rank, "building the federation")
    fed = Federation(cfg, verbose=False)
    for r in range(a.warmup):
        hb[0] = f"warm-up round {r}"
        fed.run_round(r)
    fed.drain()
    hb[0] = "timed rounds"
    if fed.is_cuda and rt.world > 1:  # device memory per rank (ranks may share one GPU)
        free, total = torch.cuda.mem_get_info(fed.device)
        print(f"[bench] rank {rt.rank}: {torch.cuda.memory_reserved(fed.device) / 2**30:.1f} GiB "
              f"reserved by torch, device {(total - free) / 2**30:.1f} / {total / 2**30:.1f} GiB used",
              file=sys.stderr, flush=True)
    D.barrier()
    if fed.is_cuda:
        torch.cuda.synchronize()
    tok0 = fed.tokens_trained
    t0 = time.perf_counter()
    for r in range(a.warmup, a.warmup + a.steps):
        fed.run_round(r)
    fed.drain()  # the last async exchange is part of the timed work
    if fed.ckpt is not None:
        fed.ckpt.wait()  # ... and so is the last checkpoint write
    D.barrier()
    if fed.is_cuda:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt = D.max_over_ranks(dt)
    fed.timer.resolve(block=True)
    fa = fed.federation_accuracy()  # collective in a multi-rank run: every rank calls it
    tokens = float(fed.tokens_trained - tok0)
    tok_t = torch.tensor([tokens], dtype=torch.float64, device=fed.device)
    D.all_reduce_(tok_t)
    tokens = float(tok_t.item())
    final_acc = fa.get("accuracy") if fa else (fed.global_accuracies[-1] if fed.global_accuracies else None)
    last = fed.history[-1]
    s_per_round = dt / a.steps
    phases = {k: v for k, v in last.items() if k.startswith("t_")}
    dev_phases = {k: v for k, v in last.items() if k.startswith("dev_t_")}
    timed = [h for h in fed.history if a.warmup <= h.get("round", -1) < a.warmup + a.steps]
    dev_mean, host_mean = {}, {}
    for h in timed:
        for k, v in h.items():
            if k.startswith("dev_t_") or k.startswith("t_hidden_") or k == "t_overlap_hidden":
                dev_mean[k] = dev_mean.get(k, 0.0) + v / max(len(timed), 1)
            elif k.startswith("t_"):
                host_mean[k] = host_mean.get(k, 0.0) + v / max(len(timed), 1)
    # per-rank spread of the timed rounds' mean device phases
    allr = D.all_gather_object(dev_mean) if rt.distributed else [dev_mean]
    spread = {k: {"min": min(d.get(k, 0.0) for d in allr), "max": max(d.get(k, 0.0) for d in allr)}
              for k in sorted(set().union(*allr))}
    multi = {}
    if rt.world > 1:
        ex = {"stale_rounds": [h.get("stale_rounds") for h in timed],
              "stale_max": max([float(h.get("stale_max") or 0.0) for h in timed] or [0.0]),
              "wait_s_total": sum(float(h.get("wait_s") or 0.0) for h in timed),
              "lead_wait_s_total": sum(float(h.get("lead_wait_s") or 0.0) for h in timed),
              "final_wait_s": sum(float(h.get("final_wait_s") or 0.0) for h in timed),
              "torn": sum(float(h.get("torn") or 0.0) for h in timed),
              "rejected_msgs": sum(float(h.get("rejected_msgs") or 0.0) for h in timed),
              "mixed": sum(float(h.get("mixed") or 0.0) for h in timed),
              # this rank's own communication: device time of the comm phase and wire bytes
              "dev_t_comm_mean_s": dev_mean.get("dev_t_comm", 0.0),
              "bytes_sent_per_round": (sum(float(h.get("bytes_sent") or 0.0) for h in timed)
                                       / max(len(timed), 1))}
        multi = {"per_rank": D.all_gather_object(ex)}
    # what one client update weighs on the wire (trainable parameters only: LoRA runs exchange
    # adapters) and what each rank actually sent per timed round (max over ranks)
    wire = 2 if (cfg.wire_dtype if cfg.mode == "serverless" else cfg.server_wire_dtype) == "bf16" else 4
    sent = [float(h.get("bytes_sent") or 0.0) for h in timed]
    exchange = {"trainable_params": int(fed.flat.num_params),
                "update_payload_bytes": int(fed.flat.numel) * wire,
                "wire_dtype": "bf16" if wire == 2 else "fp32",
                "bytes_sent_per_round_max_over_ranks": D.max_over_ranks(sum(sent) / max(len(sent), 1))}
    ck = fed.ckpt
    # measured peer-copy times of the mailbox posts (multi-rank runs: one model update to one
    # peer over xGMI), read before finish() closes the transport
    tr = getattr(fed.gossip, "transport", None)
    p2p = tr.post_stats() if tr is not None and hasattr(tr, "post_stats") else None
    info = None
    if rt.world > 1 and not a.no_info_passing:
        # outside the timed rounds: one client's model (the wire payload of the gossip engine)
        # from rank 0 to every peer over the mailbox transport, sequential (sync) vs concurrent
        # (async), measured and predicted, before / after PageRank removal
        from bcfl.trust.infopass import measure
        try:  # outside the timed region: never lose the bench line to this extra measurement
            info = measure(fed.flat.numel, sources=[0], iters=3)
        except Exception as e:  # mailbox setup failures are agreed on every rank
            info = {"error": f"{type(e).__name__}: {e}"}
    fed.finish()
    if rt.is_main:
        rec = {
            "metric": metric_name(cfg),
            "value": s_per_round,
            "unit": "s/round",
            "n_gpus": rt.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": s_per_round * 1000.0,
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": s_per_round / BASELINE_S_PER_ROUND,
            "speedup_vs_baseline": BASELINE_S_PER_ROUND / s_per_round,
            "baseline_s_per_round": BASELINE_S_PER_ROUND,
            "final_accuracy": final_acc,
            "final_accuracy_scope": (
                f"mean over all {a.clients} client models, each scored on a disjoint "
                f"1/{a.clients} stride of the class-balanced {cfg.global_test_samples}-row draw "
                f"({int(fa.get('rows', 0))} rows, round {fa.get('round')}, gathered from "
                f"{fa.get('ranks')} rank(s))" if fa and cfg.mode == "serverless" and
                cfg.global_eval_models == "all" else
                "the global model on the draw" if cfg.mode == "server" else
                "each rank's first client model on the draw (rank 0 reported)"),
            "final_majority_rate": last.get("global_majority_rate"),
            "accuracy_curve": [round(float(x), 4) for x in fed.global_accuracies],
            "accuracy_curve_rounds": list(fed.global_accuracy_rounds),
            "accuracy_curve_scope": "rank 0's hosted client models on their strides of the draw, per round",
            "global_eval_rows": last.get("global_eval_rows"),
            "final_train_loss": last.get("train_loss"),
            "baseline_final_accuracy": BASELINE_FINAL_ACC,
            "accuracy_note": ACCURACY_NOTE,
            "accuracy_protocol": {"lr": cfg.lr, "lr_schedule": cfg.lr_schedule,
                                  "lr_warmup_steps": cfg.lr_warmup_steps,
                                  "keep_optimizer_state": bool(getattr(fed, "keep_opt", cfg.keep_optimizer_state)),
                                  "synthetic_signal": cfg.synthetic_signal,
                                  "drift_correction": fed.drift.mode,
                                  "rounds_trained": a.warmup + a.steps},
            "tokens_per_s": tokens / dt,
            "samples_per_s": a.clients * cfg.train_samples * a.steps / dt,
            "dtype": "bf16" if fed.dtype == torch.bfloat16 else "fp32",
            "data": "synthetic (IMDB-shaped lengths, label-sorted Non-IID shards, packed varlen); random-init weights",
            "config": {"model": a.model, "global_batch": cfg.batch_size * a.clients,
                       "seq_len": cfg.max_seq_len,
                       "parallelism": f"fl{a.clients}-clients-on-{rt.world}gpu",
                       "clients": a.clients, "mode": a.mode,
                       "gossip": "sync" if a.sync else "async", "partition": cfg.partition,
                       "gossip_mix": ("same-round snapshots (waits for every neighbour's "
                                      "round-r post)" if getattr(fed, "same_round_mix", False) else
                                      "same-round" if a.sync else
                                      _async_mix_desc(fed)),
                       "train_samples_per_client": cfg.train_samples, "ledger": cfg.ledger,
                       "client_lanes_per_gpu": len(fed.lanes) or 1,
                       "micro_batches_per_step": fed.micro_split,
                       "overlap_wgrad": ops.wgrad_overlap_enabled(),
                       "checkpoint_every_round": cfg.save_every == 1 and ck is not None
                                                 and ck.skipped == 0,
                       "gossip_transport": fed.transport,
                       "protocol": _protocol(fed, timed)},
            "checkpoints": {"saved": ck.saved if ck else 0, "skipped": ck.skipped if ck else 0},
            "exchange": exchange,
            "p2p_post_measured": p2p,
            "info_passing": info,
            "ledger": {"height": len(fed.ledger) if fed.ledger else 0,
                       "audit": fed.ledger_audit,
                       "rejected_msgs": last.get("rejected_msgs")},
            "last_round_phases_s": phases,
            "last_round_device_phases_s": dev_phases,
            "timed_rounds_device_phases_mean_s": dev_mean,
            "timed_rounds_host_phases_mean_s": host_mean,
            "device_phases_rank_spread_s": spread,
            "device_span_vs_wall": (dev_mean.get("dev_t_round", 0.0) / s_per_round) if s_per_round else None,
            "process_latency_s": {"import_to_end": time.time() - T_IMPORT,
                                  "note": "process start (module import) to the end of the "
                                          "timed rounds incl. model build, data synthesis and "
                                          "warm-up — the reference's 'Latency' "
                                          "(server_IID_IMDB.py:59-63,229-233)"},
            **({"multi_rank": multi} if multi else {}),
            "hbm_peak_gb": fed.history[-1].get("hbm_peak_gb"),
        }
        print(json.dumps(rec), flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
