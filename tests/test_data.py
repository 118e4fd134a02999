"""Host data path: client loaders and the batch prefetcher's stage / upload split."""
import numpy as np
import torch


def test_loader_stage_then_upload_is_device_batches():
    """The prefetcher's split (host ``stage`` on a thread, ``upload`` at the round start) yields
    the batches ``device_batches`` builds in one go."""
    from bcfl.data.batching import ClientLoader
    from bcfl.data.registry import load_split
    ds = load_split("imdb", "train", 30522, 128)
    idx = np.arange(40)
    a = ClientLoader(ds, idx, 8, shuffle=True, seed=3).device_batches("cpu", epoch=5)
    ld = ClientLoader(ds, idx, 8, shuffle=True, seed=3)
    b = ld.upload(ld.stage(5, pin=False), "cpu")
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert torch.equal(x.input_ids, y.input_ids) and torch.equal(x.labels, y.labels)
        assert torch.equal(x.cu_seqlens, y.cu_seqlens)
