"""Build librfrt.so in-tree: hipcc --offload-arch=gfx950, one object per .hip, then link.

``python -m rf_ray_tracing_warp_amd.build`` (or ``__graft_entry__.build()``).  Objects are rebuilt
only when their source or a header is newer.  -ffp-contract=off is part of the arithmetic
contract (only explicit fmaf() fuse; see rt_device.h).  -fno-slp-vectorize: SLP packing into
v_pk_*_f32 buys no f32 throughput on gfx950 and costs register-shuffle moves in the triangle loop.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.environ.get("RFRT_BUILD_DIR") or os.path.join(PKG, "_build")
LIB = os.environ.get("RFRT_LIB_OUT") or os.path.join(PKG, "librfrt.so")
ARCH = os.environ.get("RFRT_ARCH", "gfx950")

# RFRT_EXTRA_CFLAGS (with RFRT_BUILD_DIR / RFRT_LIB_OUT): A/B variant libraries, e.g. tools/cov_variants.py
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off",
          "-fno-fast-math", "-fno-slp-vectorize", "-Wall", "-Wno-unused-function",
          f"-I{os.path.join(REPO, 'include')}"] + os.environ.get("RFRT_EXTRA_CFLAGS", "").split()


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build librfrt.so)")


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, verbose):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not _stale(obj, [src] + _headers()):
        return obj
    cmd = [hipcc(), "-c", src, "-o", obj] + CFLAGS
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    if _stale(LIB, objs):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
