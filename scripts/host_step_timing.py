"""Host issue time vs device time of the one-client training step (the per-GPU work of the 8-GPU
layout): is the step host-bound? Times each part of LocalTrainer.step on the host (no syncs
added) and brackets every step with HIP events, then prints per-part host means, the device step
time, and a cProfile of the timed rounds' hottest Python functions.

    python scripts/host_step_timing.py [rounds] [--clients 1] [--global-test-samples 125]
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    import bcfl  # noqa: F401
    import torch
    from bcfl import ops
    from bcfl.config import get_preset
    from bcfl.fl import Federation
    from bcfl.fl import trainer as T

    cfg = get_preset("baseline3_learnable", num_clients=1, num_rounds=5 + rounds, client_lanes=1,
                     gossip_transport="loopback", global_test_samples=125, reference_prints=False,
                     out_dir="runs/host_timing", save_every=1)
    fed = Federation(cfg, verbose=False)
    parts = {}
    dev_steps = []
    on = [False]

    def tick(name, t):
        now = time.perf_counter()
        if on[0]:
            parts.setdefault(name, []).append(now - t)
        return now

    def step(self, b, loss_acc):
        t = time.perf_counter()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        self.model.train()
        logits = self.model(b)
        t = tick("forward", t)
        loss = ops.cross_entropy(logits, b.labels)
        t = tick("loss", t)
        T.backward(loss)   # BCFL_AUTOGRAD_THREAD=1: autograd's worker thread
        t = tick("backward", t)
        ops.join_wgrad(self.flat.device)
        self.opt.step()
        t = tick("optimizer", t)
        self.flat.zero_grad()
        loss_acc += loss.detach()
        t = tick("zero_grad+acc", t)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        if on[0]:
            dev_steps.append((e0, e1))

    T.LocalTrainer.step = step
    orig_epoch = T.LocalTrainer.train_epoch

    def train_epoch(self, batches, lr_fn=None, step_hook=None):
        def hook():
            t = time.perf_counter()
            if step_hook is not None:
                step_hook()
            tick("step_hook", t)
        return orig_epoch(self, batches, lr_fn, hook)
    T.LocalTrainer.train_epoch = train_epoch

    for r in range(3):
        fed.run_round(r)
    fed.drain()
    torch.cuda.synchronize()
    on[0] = True
    t0 = time.perf_counter()
    rt = []
    for r in range(3, 3 + rounds):
        a = time.perf_counter()
        fed.run_round(r)
        rt.append(time.perf_counter() - a)
    fed.drain()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / rounds
    dev = [a.elapsed_time(b) * 1e-3 for a, b in dev_steps]
    n = len(dev)
    # device time from one step's end event to the next step's start event (the step boundary:
    # AdamW has been issued before the end event; within a round only, steps 8 per round)
    spr = n // max(rounds, 1)
    gaps = [dev_steps[i][1].elapsed_time(dev_steps[i + 1][0]) * 1e-3
            for i in range(n - 1) if (i + 1) % spr]
    out = {"rounds": rounds, "steps": n, "wall_s_per_round": wall,
           "host_issue_s_per_round": sum(rt) / rounds,
           "device_step_s_mean": sum(dev) / max(n, 1),
           "device_step_boundary_gap_s_mean": sum(gaps) / max(len(gaps), 1),
           "host_step_parts_s_mean": {k: sum(v) / max(len(v), 1) for k, v in parts.items()},
           "note": "no profiler in these rounds; the cProfile below ran on 2 further rounds"}
    out["host_step_total_s_mean"] = sum(v for k, v in out["host_step_parts_s_mean"].items())
    print(json.dumps(out, indent=1), flush=True)
    on[0] = False
    prof = cProfile.Profile()
    prof.enable()
    for r in range(3 + rounds, 5 + rounds):
        fed.run_round(r)
    prof.disable()
    fed.drain()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(70)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("cumtime").print_stats(60)
    print(s.getvalue())
    # who blocks the host on the device (host reads / synchronisations) per round
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.print_callers("method 'cpu'|synchronize|method 'item'|method 'tolist'")
    print(s.getvalue())


if __name__ == "__main__":
    main()
