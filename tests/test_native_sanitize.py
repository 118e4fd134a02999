"""Host C++ components (SHA-256/Merkle, ledger, graph analytics) under ASan + UBSan.
GPU sanitizers are not available, so the sanitizer run covers the host runtime only."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_native_host_asan_ubsan(tmp_path):
    nat = os.path.join(ROOT, "bcfl", "csrc", "native")
    srcs = [s for s in sorted(glob.glob(os.path.join(nat, "*.cpp"))) if "bindings" not in s]
    exe = str(tmp_path / "sanitize_main")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-I", nat,
           os.path.join(ROOT, "tests", "native", "sanitize_main.cpp"), *srcs, "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: tolerate other preloaded libraries in the environment
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "self-test OK" in r.stdout
