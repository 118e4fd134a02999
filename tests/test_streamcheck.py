"""The stream race detector (bcfl.utils.streamcheck): the vector-clock core on
abstract streams (CPU), and the torch / HIP integration with planted missing waits (GPU)."""
import pytest
import torch

from bcfl.utils.streamcheck import HBDetector

K = 0x1000   # one storage


def test_planted_missing_wait_is_a_race():
    d = HBDetector()
    d.access(1, K, 0, 100, True, "producer")
    d.access(2, K, 0, 100, False, "consumer")
    assert len(d.races) == 1
    assert "write-read" in str(d.races[0]) and "producer" in str(d.races[0])


def test_event_wait_orders_producer_and_consumer():
    d = HBDetector()
    d.access(1, K, 0, 100, True, "producer")
    d.record(1, 7)
    d.wait_event(2, 7)
    d.access(2, K, 0, 100, False, "consumer")
    d.access(2, K, 0, 100, True, "consumer writes back")
    assert d.races == []


def test_wait_stream_and_host_sync_order():
    d = HBDetector()
    d.access(1, K, 0, 100, True, "w1")
    d.wait_stream(2, 1)
    d.access(2, K, 0, 100, True, "w2")
    d.access(3, K + 1, 0, 8, True, "w3")
    d.host_stream(3)                     # e.g. a blocking .item() on stream 3
    d.access(1, K + 1, 0, 8, False, "r1")   # launched after the host saw stream 3 finish
    assert d.races == []


def test_wait_covers_only_what_preceded_the_record():
    d = HBDetector()
    d.record(1, 9)                       # event recorded BEFORE the write
    d.access(1, K, 0, 100, True, "late write")
    d.wait_event(2, 9)
    d.access(2, K, 0, 100, False, "reader")
    assert len(d.races) == 1


def test_write_after_read_needs_ordering_too():
    d = HBDetector()
    d.access(1, K, 0, 100, False, "reader on 1")
    d.access(2, K, 0, 100, True, "writer on 2")
    assert len(d.races) == 1 and "read-write" in str(d.races[0])


def test_disjoint_ranges_and_concurrent_reads_are_fine():
    d = HBDetector()
    d.access(1, K, 0, 100, True, "a")
    d.access(2, K, 100, 200, True, "b")       # the other half of the same buffer
    d.access(3, K + 1, 0, 64, False, "r")
    d.access(4, K + 1, 0, 64, False, "r")     # shared read-only operand
    assert d.races == []


def test_allocator_reuse_without_record_stream_is_caught():
    """A block one stream still reads, handed to a new allocation on another stream (the missing
    ``record_stream`` hazard), is a race; after ``record_stream`` (forget) it is not."""
    d = HBDetector()
    d.access(1, K, 0, 100, False, "side-stream read")
    d.access(2, K, 0, 100, False, "new tensor", fresh=True)
    assert len(d.races) == 1
    d2 = HBDetector()
    d2.access(1, K, 0, 100, False, "side-stream read")
    d2.forget(K)
    d2.access(2, K, 0, 100, False, "new tensor", fresh=True)
    assert d2.races == []


@pytest.mark.gpu
def test_gpu_planted_missing_wait_detected_through_torch_and_native():
    """Real HIP streams: a buffer written by bcfl's mix kernel on one stream and read by an ATen
    op on another without a wait is reported; with ``wait_stream`` it is not."""
    from bcfl import ops
    from bcfl.utils import streamcheck
    dev = torch.device("cuda", 0)
    a = torch.ones(1 << 20, device=dev)
    b = torch.ones(1 << 20, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    det = streamcheck.enable()
    try:
        with torch.cuda.stream(s1):
            ops.gossip_mix_(a, [b], 0.5, [0.5])      # native write of a on s1
        with torch.cuda.stream(s2):
            _ = a.sum()                              # planted: no wait on s1
        torch.cuda.synchronize()
        n_bad = len(det.races)
        with torch.cuda.stream(s1):
            ops.gossip_mix_(a, [b], 0.5, [0.5])
        s2.wait_stream(s1)
        with torch.cuda.stream(s2):
            _ = a.sum()
        torch.cuda.synchronize()
        n_after = len(det.races)
    finally:
        streamcheck.disable()
    assert n_bad >= 1, "the planted missing wait was not detected"
    assert n_after == n_bad, [str(r) for r in det.races[n_bad:]]
