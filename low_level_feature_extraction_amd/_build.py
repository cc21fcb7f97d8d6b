"""Builds libllfe.so (HIP, gfx950) in-tree with hipcc.

The library is plain C-ABI (include/llfe.h); no torch extension machinery is used, so
the same .so is what a cgo/JNI/ctypes caller would load.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libllfe.so")
SOURCES = ["llfe_api.cpp", "contours.cpp", "png_decode.cpp", "jpeg_decode.cpp", "stencil.hip", "stencil_stream.hip", "hysteresis.hip", "unique.hip", "kmeans.hip", "kmeans_big.hip", "resize.hip", "contours_gpu.hip",
           "cvresize.hip", "text.hip", "gather.hip"]
HEADERS = ["llfe_internal.h", "contours.h", "kmeans_common.h"]
# second builds of a source under another object name: (source, object stem, defines)
RECOMPILE = [("kmeans.hip", "kmeans_wide", ["-DLLFE_KM_WIDE=1", "-DLLFE_KM_THREADS=512", "-DLLFE_KM_UNROLL=4"])]
ARCH = os.environ.get("LLFE_OFFLOAD_ARCH", "gfx950")
# sources compiled with LLVM's iterative ILP scheduler (-amdgpu-sched-strategy=iterative-ilp):
# bit-identical, the stencil at 120 VGPRs without its 3 spills; round 6, four interleaved A/B
# pairs: headline +0.65 %, k_stencil 2.375 -> 2.336 ms isolated
ILP_SCHED = set(filter(None, os.environ.get("LLFE_ILP_SCHED", "stencil_stream.hip,kmeans.hip").split(",")))


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the llfe HIP backend cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "llfe.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    objs = []
    hipcc = _hipcc()
    common = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", f"-I{os.path.join(ROOT, 'include')}",
              "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
              *os.environ.get("LLFE_EXTRA_FLAGS", "").split()]  # (experiments only)
    tmpdir = os.path.join(PKG, "build")
    os.makedirs(tmpdir, exist_ok=True)
    procs = []
    for src, stem, defs in [(s, s, []) for s in SOURCES] + RECOMPILE:
        obj = os.path.join(tmpdir, stem + ".o" if stem != src else src + ".o")
        objs.append(obj)
        if src in ("contours.cpp", "png_decode.cpp", "jpeg_decode.cpp"):  # pure host code
            lang = ["-x", "c++"]
        else:
            lang = ["-x", "hip", f"--offload-arch={ARCH}"]
        extra = ["-fno-slp-vectorize"] if src == "stencil_stream.hip" else []  # keep the scalar fma chains scalar
        if src in ILP_SCHED:
            extra += ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
        cmd = [hipcc, *common, *lang, *extra, *defs, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = []
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((cmd, out.decode(errors="replace")))
        elif verbose and out:
            print(out.decode(errors="replace"), file=sys.stderr)
    if failed:
        msg = "\n\n".join(" ".join(c) + "\n" + o for c, o in failed)
        raise RuntimeError("libllfe build failed:\n" + msg)
    tmp = LIB + ".tmp"
    cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp, "-lpthread", "-lz", "-ldl"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
