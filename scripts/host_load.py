"""Is the bench round host-bound? Runs the bench federation and reports, per timed round, the
wall time and the CPU time of every thread of the process (psutil): with 8 client lanes a
GIL-serialised dispatch shows up as ~1 core of total Python-thread CPU at ~100 % of the wall."""
import json
import os
import sys
import time

import psutil

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bcfl  # noqa: E402,F401
import torch  # noqa: E402
from bcfl.config import get_preset  # noqa: E402
from bcfl.fl import Federation  # noqa: E402
from bcfl.parallel import dist as D  # noqa: E402

lanes = int(sys.argv[1]) if len(sys.argv) > 1 else 0
D.init_runtime("auto")
cfg = get_preset("baseline3_learnable", num_rounds=8, out_dir="runs/hostload", reference_prints=False,
                 client_lanes=lanes)
fed = Federation(cfg, verbose=False)
for r in range(3):
    fed.run_round(r)
fed.drain()
proc = psutil.Process()


def snap():
    return {t.id: t.user_time + t.system_time for t in proc.threads()}


res = []
for r in range(3, 8):
    torch.cuda.synchronize()
    s0, t0 = snap(), time.perf_counter()
    fed.run_round(r)
    torch.cuda.synchronize()
    s1, t1 = snap(), time.perf_counter()
    per = sorted(((s1[k] - s0.get(k, 0.0)) for k in s1), reverse=True)
    res.append({"wall_s": t1 - t0, "cpu_total_s": sum(per), "top_threads_s": [round(x, 4) for x in per[:12]],
                "phases": {k: round(v, 4) for k, v in fed.history[-1].items() if k.startswith("t_")}})
print(json.dumps({"lanes": lanes, "rounds": res}, indent=1))
