#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats.csv into a markdown table (top kernels + categories).

    python scripts/summarize_prof.py gpurun_out/prof_v3/run_kernel_stats.csv > profiles/x.md
"""
import csv
import re
import sys


def short(n: str) -> str:
    m = re.search(r"bcfl::\(anonymous namespace\)::(\w+)(<[^>]*>)?", n)
    if m:
        return "bcfl::" + m.group(1) + (m.group(2) or "")
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        mt = re.search(r"MT(\d+x\d+x\d+)", n)
        return f"hipBLASLt GEMM MT{mt.group(1) if mt else '?'}"
    m = re.search(r"at::native::(\w+)", n)
    if m:
        return "torch::" + m.group(1)
    return n[:60]


def category(n: str) -> str:
    if "attn" in n:
        return "attention (bcfl HIP, MFMA)"
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "GEMM (hipBLASLt)"
    if "bcfl" in n:
        if re.search(r"g8_|wgrad|linear_|gemm|colsum", n):
            return "GEMM (bcfl MFMA: g8 / K9 wgrad + reductions)"
        if "ln" in n.lower() or "layernorm" in n.lower():
            return "LayerNorm family (bcfl)"
        if "adamw" in n:
            return "AdamW (bcfl multi-tensor)"
        return "other bcfl HIP kernels (act / xent / gossip / SHA / mix)"
    if "at::native" in n:
        return "torch eager kernels"
    return "runtime copies / fills"


def main(path, title=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title or path}\n")
    print(f"Total kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches\n")
    cats = {}
    for r in rows:
        c = category(r["Name"])
        cats[c] = cats.get(c, 0.0) + float(r["TotalDurationNs"])
    print("| category | ms | % |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda x: -x[1]):
        print(f"| {c} | {v / 1e6:.1f} | {100 * v / tot:.1f} |")
    print("\n| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    agg = {}
    for r in rows:
        k = short(r["Name"])
        a = agg.setdefault(k, [0, 0.0])
        a[0] += int(r["Calls"])
        a[1] += float(r["TotalDurationNs"])
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
        print(f"| `{k}` | {c} | {t / 1e6:.1f} | {t / c / 1e3:.1f} | {100 * t / tot:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
