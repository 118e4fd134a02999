#!/usr/bin/env python
"""Attribute runtime copy kernels (__amd_rocclr_copyBuffer / fillBuffer) in a rocprofv3 kernel
trace to their surroundings: for every copy dispatch, the previous and next kernel on the same
queue, its grid size (bytes moved ~ grid threads x 16), counted per (prev, next) pair.

    python scripts/copy_neighbors.py path/to/run_kernel_trace.csv"""
import collections
import csv
import sys


def short(n):
    n = n.split("(")[0]
    for p in ("void ", "bcfl::"):
        n = n.replace(p, "")
    return n[:70]


def main(path):
    rows = list(csv.DictReader(open(path)))
    q = collections.defaultdict(list)
    for r in rows:
        q[(r.get("Agent_Id"), r.get("Queue_Id"))].append(r)
    pairs = collections.Counter()
    dur = collections.Counter()
    grids = collections.defaultdict(list)
    for k, lst in q.items():
        lst.sort(key=lambda r: int(r["Start_Timestamp"]))
        for i, r in enumerate(lst):
            if "rocclr_copyBuffer" not in r["Kernel_Name"] and "rocclr_fillBuffer" not in r["Kernel_Name"]:
                continue
            prev = short(lst[i - 1]["Kernel_Name"]) if i else "-"
            nxt = short(lst[i + 1]["Kernel_Name"]) if i + 1 < len(lst) else "-"
            key = (short(r["Kernel_Name"]), prev, nxt)
            pairs[key] += 1
            dur[key] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            grids[key].append(int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0))
    print(f"{'n':>5} {'avg us':>8} {'grid med':>9}  copy | prev -> next")
    for key, n in pairs.most_common(40):
        g = sorted(grids[key])
        print(f"{n:5d} {dur[key] / n / 1e3:8.1f} {g[len(g) // 2]:9d}  {key[0]} | {key[1]} -> {key[2]}")


if __name__ == "__main__":
    main(sys.argv[1])
