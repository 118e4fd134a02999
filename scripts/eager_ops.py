"""Which eager torch ops (and D2D copies) run in a bench round: torch.profiler over one round of
the bench federation, aggregated by op name + input shapes (host-side attribution of the
'torch eager kernels' and copyBuffer rows of the rocprof summary)."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bcfl  # noqa: F401,E402
from bcfl.config import get_preset
from bcfl.fl import Federation

# the N = 1 bench's federation: 8 clients as in-process virtual ranks, one lane each
cfg = get_preset("baseline3_learnable", save_every=1, out_dir="runs/eager", reference_prints=False,
                 gossip_transport=sys.argv[1] if len(sys.argv) > 1 else "loopback",
                 client_lanes=8)
fed = Federation(cfg, verbose=False)
for r in range(2):
    fed.run_round(r)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    fed.run_round(2)
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
def dev(e):
    return getattr(e, "self_device_time_total", getattr(e, "self_cuda_time_total", 0))


rows = [e for e in ka if (e.key.startswith("aten::") or "Memcpy" in e.key or "copy" in e.key.lower())
        and dev(e) > 0]
rows.sort(key=lambda e: -dev(e))
print(f"{'op':40s} {'count':>7s} {'dev_us':>10s}  shapes")
for e in rows[:160]:
    print(f"{e.key[:40]:40s} {e.count:7d} {dev(e):10.0f}  {str(e.input_shapes)[:110]}")
fed.finish()
