"""Where do lane / overlap runs differ from one-lane training? For each weight-gradient kernel
(BCFL_WGRAD_G8 = 0 K9 / 1 gemm8) run the test_gpu_federation config as (lanes, overlap) =
(1, F) twice, (3, F), (1, T), (3, T) and print, per run, the max |diff| against the first (1, F)
run and the parameters (flat-buffer slices) that differ."""
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bcfl  # noqa: E402,F401
from test_gpu_federation import _run  # noqa: E402


def slices():
    from bcfl.models import build_model
    m = build_model("bert-base-2l", 2, device="meta")
    out, off = [], 0
    for n, p in m.named_parameters():  # FlatParams slots: 64-element aligned
        out.append((n, off, off + p.numel()))
        off += (p.numel() + 63) // 64 * 64
    return out


def main():
    names = slices()
    for kern in sys.argv[1:] or ["0", "1"]:
        os.environ["BCFL_WGRAD_G8"] = kern
        runs = [((1, False), 0), ((1, False), 1), ((3, False), 0), ((1, True), 0), ((3, True), 0)]
        outs = {}
        for (lanes, ov), rep in runs:
            outs[(lanes, ov, rep)] = _run(tempfile.mkdtemp(), lanes, ov)[0]
        ref = outs[(1, False, 0)]
        for k, v in outs.items():
            d = (v - ref).abs().amax(0) if v.dim() > 1 else (v - ref).abs()
            bad = [n for n, a, b in names if b <= d.numel() and float(d[a:b].max()) > 0]
            print(f"wgrad={kern} run={k} maxdiff={float(d.max()):.3e} differing={bad[:12]}"
                  f"{' ...' if len(bad) > 12 else ''} ({len(bad)} params)", flush=True)


if __name__ == "__main__":
    main()
