"""The compiled shape of k_ccl_runs' tile loop (CPU: hipcc cross-compiles gfx950 here).

Round 5's first k_ccl_runs broadcast its tile index from lane 0 with a shuffle inside a
per-wave loop; hipcc threaded the latch's ``lane != 0`` path straight back to that shuffle
(a nested loop skipping lane 0's atomic), so lanes 1-63 relabelled list entry 0's tile
without lane 0 and its root counter ran past the roots buffer ("The round-5
fault", profiles/r6/ccl_root_cause/).  The kept kernel takes its tiles from a workgroup
counter read from LDS between two barriers, with no cross-lane broadcast of the index.  This
test pins that structure in the ISA: one outer loop whose header holds the counter atomic,
both barriers and the LDS read of the base, and one nested loop (the wave's tiles of the
round) -- no second nested loop that could re-enter the barriers or a tile without the rest
of the wave.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "low_level_feature_extraction_amd", "csrc", "hysteresis.hip")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    pytest.skip("hipcc not available")


def _function(asm: str, name: str) -> str:
    m = re.search(r"^(_Z\S*" + name + r"\S*):", asm, re.M)
    assert m, f"{name} not in the ISA"
    start = m.start()
    end = asm.index("s_endpgm", start)
    return asm[start:end]


def test_k_ccl_runs_tile_loop_structure(tmp_path):
    out = tmp_path / "hyst.s"
    cmd = [_hipcc(), "-O3", "-std=c++17", "-ffp-contract=off", f"-I{os.path.join(ROOT, 'include')}",
           "--offload-arch=gfx950", "--cuda-device-only", "-S", SRC, "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    f = _function(out.read_text(), "k_ccl_runs")
    lines = f.splitlines()
    d1 = [i for i, ln in enumerate(lines) if "Loop Header: Depth=1" in ln]
    d2 = [i for i, ln in enumerate(lines) if "Loop Header: Depth=2" in ln]
    assert len(d1) == 1, "k_ccl_runs: expected one outer (work-counter) loop"
    assert len(d2) == 1, "k_ccl_runs: a second nested loop appeared (a threaded re-entry?)"
    head = lines[d1[0]:d2[0]]
    atom = [i for i, ln in enumerate(head) if "global_atomic_add" in ln]
    bars = [i for i, ln in enumerate(head) if re.search(r"\bs_barrier\b", ln)]
    lds = [i for i, ln in enumerate(head) if "ds_read_b32" in ln]
    assert atom and len(bars) == 2 and lds, "the work counter, both barriers and the base read sit in the outer header"
    assert atom[0] < bars[0] < lds[0] < bars[1], "atomic -> barrier -> LDS base read -> barrier"
    # the tile index never crosses lanes: no shuffle / readlane between the counter and the tiles
    assert not any(re.search(r"ds_bpermute|v_readlane|ds_swizzle", ln) for ln in head)
    assert not any(re.search(r"\bs_barrier\b", ln) for ln in lines[d2[0]:])
