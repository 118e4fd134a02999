"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel [start, end) intervals over the
trace's span, plus the largest idle gaps (is the device ever waiting on the host?). Several trace
files (one per rank process sharing the GPU) are merged into one timeline."""
import csv
import json
import sys

rows = [r for f in sys.argv[1:] for r in csv.DictReader(open(f))]
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
# skip the first 40 % of the trace (start-up, compilation, warm-up rounds)
t0 = iv[0][0] + int(0.4 * (iv[-1][1] - iv[0][0]))
iv = [(max(a, t0), b) for a, b in iv if b > t0]
busy, gaps, gap_at = 0, [], []
cs, ce = iv[0]
for a, b in iv[1:]:
    if a > ce:
        busy += ce - cs
        gaps.append(a - ce)
        gap_at.append((ce, a - ce))
        cs, ce = a, b
    else:
        ce = max(ce, b)
busy += ce - cs
span = iv[-1][1] - iv[0][0]
timeline = [(round((a0 - iv[0][0]) / 1e6, 2), round(g / 1e6, 3)) for a0, g in gap_at if g > 500_000]
gaps.sort(reverse=True)
print(json.dumps({"span_ms": span / 1e6, "busy_ms": busy / 1e6, "busy_frac": busy / span,
                  "idle_ms": (span - busy) / 1e6, "n_gaps": len(gaps),
                  "gaps_over_50us_ms": sum(g for g in gaps if g > 50_000) / 1e6,
                  "largest_gaps_us": [round(g / 1e3, 1) for g in gaps[:10]],
                  "gaps_over_0p5ms_at_ms": timeline}))
