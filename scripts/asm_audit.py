#!/usr/bin/env python
"""Audit a hipcc ``-save-temps`` gfx950 .s file: per kernel, VGPR / scratch use and the main-loop
synchronisation (MFMA / LDS-DMA / barrier counts, every vmcnt wait) — the checks
cdna_hip_programming.md §5.7 asks for after any edit of a pipelined kernel.

    python scripts/asm_audit.py /tmp/t/gemm8-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    s = open(path).read()
    meta = {}
    # metadata: .vgpr_count / .private_segment_fixed_size per kernel (YAML at the end)
    for blk in re.split(r"\n\s+- \.agpr_count", s):
        n = re.search(r"\.name:\s+(\S+)", blk)
        v = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        if n and v:
            meta[n.group(1)] = (int(v.group(1)), int(sc.group(1)) if sc else -1)
    funcs = re.split(r"\n(?=_Z\w+:[^\n]*\n)", s)
    for f in funcs:
        m = re.match(r"(_Z\w+):", f)
        if not m or filt not in m.group(1):
            continue
        name = m.group(1)
        body = f.split(".Lfunc_end")[0]
        lines = [l.strip() for l in body.split("\n")]
        cnt = lambda pat: sum(1 for l in lines if re.match(pat, l))  # noqa: E731
        vm = [l.split("vmcnt")[1].split(")")[0].strip("(") for l in lines if "vmcnt(" in l]
        v, sc = meta.get(name, (-1, -1))
        print(f"{name}\n  vgpr={v} scratch={sc} mfma={cnt(r'v_mfma')} "
              f"dma={cnt(r'buffer_load_dwordx4.* lds')} ds_read={cnt(r'ds_read')} "
              f"barrier={cnt(r's_barrier')} scratch_ops={cnt(r'scratch_')} vmcnt={vm}")


if __name__ == "__main__":
    main()
