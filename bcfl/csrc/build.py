"""In-tree build of bcfl's native code (no JIT cache: the .so files travel with the repo).

* ``bcfl/_host*.so`` — host runtime (SHA-256/Merkle, ledger, graph analytics): g++ + pybind11.
* ``bcfl/_C*.so``    — HIP/CDNA4 kernels for gfx950 + torch bindings: hipcc.

Usage: ``python -m bcfl.csrc.build [--host-only] [--jobs N] [--force]``.
Object files are cached under ``build/`` by source mtime; compiles run in parallel.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _run(cmd, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _py_includes():
    import pybind11
    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def build_host(force=False, verbose=False) -> str:
    srcs = sorted(glob.glob(os.path.join(HERE, "native", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(HERE, "native", "*.h")))
    out = os.path.join(PKG, "_host" + EXT_SUFFIX)
    if not force and not _stale(out, srcs + hdrs + [__file__]):
        return out
    inc = sum((["-I", p] for p in _py_includes()), [])
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
           "-Wall", "-Wno-sign-compare", *inc, "-I", os.path.join(HERE, "native"), *srcs, "-o",
           out + ".tmp"]
    _run(cmd, verbose)
    os.replace(out + ".tmp", out)
    return out


def _torch_flags():
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths
    incs = include_paths()
    libs = library_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libs, abi


# Per-file code-generation flags. ``-amdgpu-mfma-vgpr-form``: MFMA results land in ordinary VGPRs
# instead of AGPRs — the attention kernels post-process every score tile with VALU ops, so AGPR
# accumulators cost one v_accvgpr_read per element per tile; without them the flash-attention
# kernels need no AGPRs at all and reach 3 waves/SIMD instead of 2.
#
# layernorm.hip is built WITHOUT packed-fp32 VALU ops (v_pk_mul / v_pk_add / v_pk_fma_f32). With
# them, the LayerNorm backward kernel returned a different result for the last quarter of a wave
# (lanes 48-63: one 128-byte group of one row, values a few bf16 ulps off) in ~10 % of the steps
# when other client lanes ran concurrently — bitwise-identical inputs before and after the kernel,
# and a re-run of the same kernel on those inputs reproducing the reference. Load type, cache
# policy, acquire / release fences, the row pipeline, the cross-lane reduction and the block order
# made no difference; the build without packed fp32 made 320 / 320 four-lane iterations bitwise
# reproducible (scripts/kernel_determinism.py, profiles/lanes_determinism_r6.json). The kernels
# are HBM-bound, so the scalar VALU form costs little.
FILE_FLAGS = {
    "attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
    "layernorm.hip": ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"],
}


def build_kernels(force=False, verbose=False, jobs=8) -> str:
    kern = sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(HERE, "kernels", "*.h")))
    binding = os.path.join(HERE, "bindings.cpp")
    out = os.path.join(PKG, "_C" + EXT_SUFFIX)
    os.makedirs(BUILD, exist_ok=True)
    incs, libdirs, abi = _torch_flags()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", os.path.join(HERE, "kernels"),
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    jobs_list = []
    objs = []
    for s in kern:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s, *hdrs, __file__]):
            jobs_list.append([HIPCC, *common, "-ffp-contract=fast", "-munsafe-fp-atomics",
                              *FILE_FLAGS.get(os.path.basename(s), []), "-c", s, "-o", o])
    tinc = sum((["-isystem", p] for p in incs + _py_includes()), [])
    # C++ comm engine (torch-facing HIP: IPC mailboxes)
    comm = sorted(glob.glob(os.path.join(HERE, "comm", "*.hip")))
    chdrs = sorted(glob.glob(os.path.join(HERE, "comm", "*.h")))
    for s in comm:
        o = os.path.join(BUILD, "comm_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s, *chdrs, __file__]):
            jobs_list.append([HIPCC, *common, *tinc, "-I", HERE, "-DTORCH_EXTENSION_NAME=_C",
                              "-DTORCH_API_INCLUDE_EXTENSION_H", "-c", s, "-o", o])
    bo = os.path.join(BUILD, "bindings.o")
    objs.append(bo)
    if force or _stale(bo, [binding, *hdrs, *chdrs, __file__]):
        jobs_list.append([HIPCC, *common, *tinc, "-DTORCH_EXTENSION_NAME=_C",
                          "-DTORCH_API_INCLUDE_EXTENSION_H", "-c", binding, "-o", bo])
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for f in [ex.submit(_run, c, verbose) for c in jobs_list]:
                f.result()
    if force or jobs_list or _stale(out, objs):
        lib = sum((["-L", p, f"-Wl,-rpath,{p}"] for p in libdirs), [])
        # link to a temporary file and rename: a reader (an importing process, a tree snapshot)
        # never sees a half-written library
        tmp = out + ".tmp"
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, *lib,
               "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
               "-lamdhip64"]
        _run(cmd, verbose)
        os.replace(tmp, out)
    return out


def build_all(host_only=False, force=False, verbose=False, jobs=8):
    outs = [build_host(force, verbose)]
    if not host_only:
        outs.append(build_kernels(force, verbose, jobs))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host-only", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    for o in build_all(a.host_only, a.force, a.verbose, a.jobs):
        print("built", o)


if __name__ == "__main__":
    main()
