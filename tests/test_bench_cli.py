"""bench.py contract on the CPU: ``--gpus N`` without a torchrun environment launches N ranks as a
child torch.distributed.run job and prints ONE JSON line with n_gpus = N (the driver's scaling
runs rely on this)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_bench_gpus2_cpu_rehearsal(tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--gpus", "2", "--model", "tiny-bert", "--steps", "1", "--warmup", "1",
                        "--no-ckpt", "--out", str(tmp_path / "b")],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["warmup"] == 1
    assert d["value"] > 0 and d["higher_is_better"] is False
    assert d["config"]["clients"] == 8 and d["config"]["gossip_transport"] == "mailbox"
