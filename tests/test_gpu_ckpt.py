"""AsyncCheckpointer ordering on the GPU: a save snapshots the master before any later writer on
the compute stream can change it, and the device->host copy is off the critical path."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_async_checkpoint_is_not_torn_by_later_writes(tmp_path):
    from bcfl.ckpt import AsyncCheckpointer, read_safetensors
    from bcfl.models import build_model
    from bcfl.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    model = build_model("bert-base-2l", 2, device=dev, dtype=torch.bfloat16, seed=0)
    flat = FlatParams.from_model(model, dev, torch.bfloat16)
    ck = AsyncCheckpointer(model, flat, async_=True)
    for rnd in range(3):
        flat.master.normal_()
        expect = flat.master.clone()
        assert ck.save([str(tmp_path / f"r{rnd}")], metadata={"round": str(rnd)})
        # the next round's writers, issued right away on the compute stream
        for _ in range(4):
            flat.master.mul_(-3.0).add_(1.0)
        ck.wait()
        torch.cuda.synchronize()
        assert torch.equal(ck.pinned[0], expect.cpu()), f"round {rnd}: checkpoint mixes rounds"
        sd = read_safetensors(os.path.join(tmp_path / f"r{rnd}", "model.safetensors"))
        assert len(sd) > 0
    assert ck.skipped == 0 and ck.saved == 3
