#!/usr/bin/env python
"""The one-client round boundary on the device: every kernel dispatch (all queues) from the last
AdamW of a round's training to the first forward GEMM of the next round on the training queue, with start offsets,
durations, host launch times (with a HIP API trace) and the idle gaps of the busiest queue, from a
rocprofv3 kernel trace. Anchored on the
once-per-round ``delta_round_end_kernel``; prints every boundary of the trace (training-queue dispatches only).

    python scripts/round_boundary.py path/to/run_kernel_trace.csv"""
import collections
import csv
import sys


def short(n):
    for p in ("void ", "bcfl::", "at::native::", "(anonymous namespace)::"):
        n = n.replace(p, "")
    n = n.split("(")[0]
    return n[:64]


QUIET_OTHERS_OFF = False   # print the side queues' dispatches too


def host_api(path):
    """{correlation id: host API start} and the host's synchronising calls, from the HIP API
    trace next to the kernel trace (rocprofv3 --hip-trace), if there is one."""
    import glob
    import os
    cands = glob.glob(os.path.join(os.path.dirname(path), "*hip_api_trace.csv"))
    if not cands:
        return {}, []
    launch, syncs = {}, []
    for r in csv.DictReader(open(cands[0])):
        fn = r.get("Function", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        launch[r.get("Correlation_Id")] = (s, fn)
        if "Synchronize" in fn or "Memcpy" in fn or "WaitEvent" in fn or "Query" in fn:
            syncs.append((s, e, fn))
    syncs.sort()
    return launch, syncs


def main(path):
    launch, syncs = host_api(path)
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r.get("Queue_Id") or r.get("Stream_Id") or "?"
    rows.sort(key=lambda r: r["s"])
    anchors = [i for i, r in enumerate(rows) if "delta_round_end_kernel" in r["Kernel_Name"]]
    busiest = collections.Counter(r["q"] for r in rows).most_common(1)[0][0]
    for a in anchors:
        lo = a
        while lo > 0 and "adamw_mt_kernel" not in rows[lo]["Kernel_Name"]:
            lo -= 1
        hi = a
        while hi + 1 < len(rows) and not ("g8_kernel" in rows[hi]["Kernel_Name"]
                                          and rows[hi]["q"] == busiest
                                          and rows[hi]["s"] > rows[a]["e"] + 1000):
            hi += 1
        # the next round starts with its first forward GEMM on the training queue
        t0 = rows[lo]["s"]
        print(f"--- boundary at dispatch {a}: {hi - lo + 1} dispatches, "
              f"{(rows[hi]['s'] - t0) / 1e3:.1f} us from the last AdamW to the next forward GEMM")
        last_e = None
        idle = 0
        for r in rows[lo:hi + 1]:
            if r["q"] != busiest and not QUIET_OTHERS_OFF:
                continue
            gap = ""
            if r["q"] == busiest:
                if last_e is not None and r["s"] > last_e:
                    gap = f"  gap {(r['s'] - last_e) / 1e3:.1f}"
                    idle += r["s"] - last_e
                last_e = max(last_e or 0, r["e"])
            h = launch.get(r.get("Correlation_Id"))
            hs = f"{(h[0] - t0) / 1e3:9.1f}" if h else "        -"
            print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} host {hs}  q{r['q']:>3}  "
                  f"{short(r['Kernel_Name'])}{gap}")
        print(f"idle on the busiest queue (q{busiest}) inside the window: {idle / 1e3:.1f} us")
        t1 = rows[hi]["s"]
        print("host synchronising / waiting calls in the window (start, duration us):")
        for s0, e0, fn in syncs:
            if t0 - 20000_000 <= s0 <= t1:
                print(f"   {(s0 - t0) / 1e3:9.1f} {(e0 - s0) / 1e3:8.1f}  {fn}")


if __name__ == "__main__":
    main(sys.argv[1])
