"""The compiled shape of the stencil's LDS input ring (CPU: hipcc cross-compiles gfx950 here).

Round 6 moved the stencil's input rows into a per-wave LDS ring filled five steps ahead by
12-byte direct-to-LDS loads.  The compiler does not track those loads: the
kernel waits for a row with a hand-placed, counted ``s_waitcnt vmcnt(4)`` before it reads it
(at most four younger ring loads outstanding, vector-memory operations completing in order).
A ring read scheduled above its wait would read a row that has not landed yet -- wrong
results that come and go with memory timing.  This test pins, in the ISA of the kernel the
bench runs (k_stencil_stream<true, true>, built with _build.py's flags), that every ring
read (one ``ds_read_b96`` of the lane's 16-byte slot) comes after a ``vmcnt(4)`` wait with
no other ring read in between, once per unrolled row step, and that the rows arrive by
direct-to-LDS loads
(``global_load_lds_dwordx3`` for interior waves, ``buffer_load_dwordx3 ... lds`` for border
waves).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "low_level_feature_extraction_amd", "csrc", "stencil_stream.hip")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    pytest.skip("hipcc not available")


def _function(asm: str, mangled_part: str) -> str:
    m = re.search(r"^(_Z\S*" + mangled_part + r"\S*):", asm, re.M)
    assert m, f"{mangled_part} not in the ISA"
    start = m.start()
    return asm[start:asm.index("s_endpgm", start)]


def test_stencil_ring_reads_wait_for_their_rows(tmp_path):
    out = tmp_path / "stencil.s"
    cmd = [_hipcc(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
           f"-I{os.path.join(ROOT, 'include')}", "--offload-arch=gfx950", "--cuda-device-only", "-S", SRC,
           "-o", str(out)]
    from low_level_feature_extraction_amd import _build
    if "stencil_stream.hip" in _build.ILP_SCHED:
        cmd[1:1] = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    f = _function(out.read_text(), r"k_stencil_streamILb1ELb1E")
    lines = f.splitlines()
    assert sum("global_load_lds_dwordx3" in ln for ln in lines) >= 12, "interior rows: direct-to-LDS loads"
    assert sum(re.search(r"buffer_load_dwordx3 .* lds", ln) is not None for ln in lines) >= 12, \
        "border rows: range-checked buffer loads to LDS"
    events = []
    for ln in lines:
        if re.search(r"s_waitcnt vmcnt\(4\)", ln):
            events.append("W")
        elif re.search(r"\bds_read_b96\b|\bds_read2_b32\b", ln):
            events.append("R")
    reads = events.count("R")
    assert reads >= 12, "one ring read per unrolled row step"
    for i, e in enumerate(events):
        if e == "R":
            assert i > 0 and events[i - 1] == "W", "a ring read is not preceded by its vmcnt(4) wait"
