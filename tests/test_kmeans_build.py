"""The k-means kernel's two builds and its LDS invariants (CPU: hipcc cross-compiles gfx950).

Round 6 runs k-means in 256-thread workgroups, four per CU, and hands batches whose attempts
all fit the GPU at once to a second build of kmeans.hip in 512-thread workgroups
(`launch_kmeans_wide`, DESIGN.md §3 "256-thread k-means workgroups").  The workgroup size is
a build knob (LLFE_KM_THREADS); a size whose shared-memory layout breaks -- 128 threads let
the k-means++ selection's step sums overflow the Lloyd accumulators they alias, which gave
wrong palettes on the GPU -- must fail to compile rather than run.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "low_level_feature_extraction_amd", "csrc", "kmeans.hip")
LIB = os.path.join(ROOT, "low_level_feature_extraction_amd", "libllfe.so")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    pytest.skip("hipcc not available")


def _compile(tmp_path, *defs):
    cmd = [_hipcc(), "-O0", "-std=c++17", f"-I{os.path.join(ROOT, 'include')}", "--offload-arch=gfx950",
           "--cuda-device-only", "-c", SRC, "-o", str(tmp_path / "k.o"), *defs]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600)


def test_too_narrow_workgroup_does_not_build(tmp_path):
    r = _compile(tmp_path, "-DLLFE_KM_THREADS=128")
    assert r.returncode != 0
    assert "selection step sums overflow the Lloyd accumulators" in r.stderr


def test_library_carries_both_widths():
    if not os.path.exists(LIB):
        pytest.skip("libllfe.so not built")
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    out = subprocess.run([nm, "-C", LIB], capture_output=True, text=True, check=True).stdout
    assert " T llfe::launch_kmeans(" in out
    assert " T llfe::launch_kmeans_wide(" in out
