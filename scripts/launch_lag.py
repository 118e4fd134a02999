"""Summarise a rocprofv3 --hip-trace --kernel-trace run: per-kernel launch->start lag (is the host
ahead of the device?) and the device idle gaps attributed to host lateness. Writes a small JSON."""
import csv
import json
import sys

import numpy as np

d = sys.argv[1]
api = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
ker = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
launch = {int(r["Correlation_Id"]): (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
          for r in api if "Launch" in r["Function"]}
rows = []
for k in ker:
    c = int(k["Correlation_Id"])
    if c in launch:
        rows.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), launch[c][0], launch[c][1], k["Kernel_Name"]))
rows.sort()
# second half only (steady state)
rows = rows[len(rows) // 2:]
lag = np.array([s - le for s, e, ls, le, n in rows]) / 1e3
out = {"kernels": len(rows), "lag_us_percentiles": {p: float(np.percentile(lag, p)) for p in (1, 10, 50, 90)}}
# gaps where the next kernel was launched AFTER the previous kernel ended (host late)
late, late_sum, idle_sum = [], 0.0, 0.0
prev_end = rows[0][1]
for s, e, ls, le, n in rows[1:]:
    if s > prev_end:
        idle_sum += s - prev_end
        if le > prev_end:
            late_sum += min(s, le) - prev_end if le < s else s - prev_end
            late.append((n[:60], (s - prev_end) / 1e3))
    prev_end = max(prev_end, e)
span = rows[-1][1] - rows[0][0]
out.update(span_ms=span / 1e6, idle_ms=idle_sum / 1e6, host_late_idle_ms=late_sum / 1e6)
agg = {}
for n, g in late:
    agg[n] = agg.get(n, 0.0) + g
out["top_late_next_kernel_us"] = sorted(agg.items(), key=lambda x: -x[1])[:15]
# blocking API calls
blk = {}
for r in api:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if dur > 50:
        blk.setdefault(r["Function"], []).append(dur)
out["api_calls_over_50us"] = {k: [len(v), float(np.sum(v))] for k, v in blk.items()}
json.dump(out, open(f"{d}/lag_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
