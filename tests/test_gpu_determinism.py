"""Bitwise reproducibility of concurrent client lanes (profiles/lanes_determinism_r6.json).

Four BERT-base replicas train a fixed batch with fixed dropout keys on four concurrent HIP
streams, iteration after iteration, with no optimizer step: every iteration must reproduce every
gradient bit of the replica's first. Before the LayerNorm kernels were built without packed-fp32
VALU ops, ~10 % of these iterations differed in two of the four lanes (scripts/kernel_determinism.py
is the long form of this test, with the probes that located the kernel)."""
import numpy as np
import pytest
import torch


@pytest.mark.gpu
@pytest.mark.parametrize("overlap_wgrad", [False, True])
def test_gpu_concurrent_lanes_gradients_bitwise_reproducible(overlap_wgrad):
    from bcfl import ops
    from bcfl.data.batching import make_packed_batch, pad_packed
    from bcfl.data.registry import load_split
    from bcfl.fl.trainer import backward
    from bcfl.models import build_model
    from bcfl.parallel.flat import FlatParams
    dev = torch.device("cuda", 0)
    prev = ops.wgrad_overlap_enabled()
    ops.set_wgrad_overlap(overlap_wgrad)
    try:
        torch.manual_seed(0)
        ds = load_split("imdb", "train", 30522, 512)
        lanes = []
        for i in range(4):
            m = build_model("bert-base", 2, device=dev, dtype=torch.bfloat16)
            flat = FlatParams.from_model(m, dev, torch.bfloat16)
            rows = np.random.default_rng(100 + i).choice(len(ds), 32, replace=False)
            b = pad_packed(make_packed_batch(ds, rows), 256).to(dev)
            lanes.append({"m": m, "flat": flat, "b": b, "s": torch.cuda.Stream(dev), "ref": None})
        rng = ops.rng.global_rng()
        bad = []
        for it in range(12):
            for k, ln in enumerate(lanes):
                with torch.cuda.stream(ln["s"]):
                    rng.load_state({"seed": 1234 + 7 * k, "counter": 99 + k})
                    ln["m"].train()
                    loss = ops.cross_entropy(ln["m"](ln["b"]), ln["b"].labels)
                    backward(loss)
                    ops.join_wgrad(dev)
                    ln["g"] = torch.cat([p.grad.reshape(-1).float() for p in ln["flat"].params])
                    ln["flat"].zero_grad()
            torch.cuda.synchronize()
            for k, ln in enumerate(lanes):
                if ln["ref"] is None:
                    ln["ref"] = ln["g"]
                elif not torch.equal(ln["g"], ln["ref"]):
                    bad.append((it, k, int((ln["g"] != ln["ref"]).sum())))
        assert not bad, f"(iteration, lane, gradient elements differing): {bad}"
    finally:
        ops.set_wgrad_overlap(prev)
