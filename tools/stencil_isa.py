#!/usr/bin/env python3
"""Per-stage VALU instruction budget of k_stencil_stream<true, true> from its gfx950 ISA.

Builds stencil_stream.hip with -DLLFE_ST_MARK=1 (stage markers fenced by
sched_barrier, so no instruction crosses a stage boundary; the counts are those of the
shipped schedule up to that fencing) and counts, for each of the 12 unrolled row steps
of the main loop, the VALU instructions (v_*) per stage on the path an interior wave
takes (12-byte loads, no border REPLICATE, full-width stores), separately for the
candidate-only blocks (the Canny direction classes and NMS, run only on wave rows with
a pixel above LOW).  One row step of a wave = 64 lanes x 4 pixels = 256 pixels, 240 of
them output columns.

    python tools/stencil_isa.py [--asm file.s] [--json out.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "low_level_feature_extraction_amd", "csrc", "stencil_stream.hip")
KERNEL = "_ZN4llfe12_GLOBAL__N_116k_stencil_streamILb1ELb1E"


def build_asm(path, src=SRC):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-DLLFE_ST_MARK=1",
           f"-I{os.path.join(ROOT, 'include')}", "-x", "hip", "--offload-arch=gfx950", "--offload-device-only", "-S",
           f"-I{os.path.dirname(SRC)}", src, "-o", path]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def family(op):
    """Coarse opcode family of a VALU mnemonic (for the issue-cost column)."""
    if op.startswith("v_mov_b32_dpp") or "_dpp" in op:
        return "dpp"
    if op.startswith("v_mov") or op.startswith("v_cndmask"):
        return "mov/select"
    if op.startswith("v_pk_"):
        return "packed"
    if op.startswith(("v_perm", "v_alignbit", "v_bfe", "v_bfi", "v_lshl_or", "v_and_or", "v_or3", "v_lshl_add")):
        return "byte/bit"
    if op.startswith(("v_dot2", "v_mad", "v_fma", "v_mul")):
        return "mul/dot"
    if op.startswith(("v_cvt",)):
        return "convert"
    if op.startswith(("v_cmp", "v_max", "v_min", "v_sub", "v_add", "v_and", "v_or", "v_xor", "v_lshr", "v_lshl",
                      "v_ashr", "v_not")):
        return "alu"
    return "other"


def analyse(asm_text):
    lines = asm_text.splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    # the main row loop: from the first stage marker to the last
    marks = [i for i, l in enumerate(body) if ";@st " in l]
    seg = body[marks[0]:marks[-1] + 1]
    steps = []  # per row step: {stage: Counter(kind -> n)}
    cur = None
    stage = None
    block = []

    def flush_block():
        nonlocal block
        if cur is None or stage is None or not block:
            block = []
            return
        text = "\n".join(block)
        ops = [b.split()[0] for b in block if b.split() and b.split()[0].startswith("v_")]
        if re.search(r"global_load_(ubyte|ushort)|v_readlane|global_store_byte|;@rare", text):
            kind = "border"  # byte loads / REPLICATE / per-byte stores of border waves, and the
            # blocks the source marks rare (ST_RARE: border columns, REPLICATE rows, row -5..-1 fill)
        elif stage in ("direction",) or (stage == "nms" and "cand_block" in text):
            kind = "cand"
        else:
            kind = "path"
        for op in ops:
            cur[stage][kind] += 1
            cur[stage]["fam:" + kind + ":" + family(op)] += 1
        block = []

    for l in seg:
        s = l.strip()
        if s.startswith(";@rare"):
            block.append(s)
            continue
        m = re.match(r";@st (\w+)", s)
        if m:
            flush_block()
            name = m.group(1)
            if name == "load":
                cur = collections.defaultdict(collections.Counter)
                steps.append(cur)
            if name == "direction_end":
                name = "sobel"
            stage = name
            continue
        if re.match(r"\.LBB\d+_\d+:", s):
            flush_block()
            continue
        if s.startswith("s_cbranch") or s.startswith("s_branch"):
            block.append(s)
            flush_block()
            continue
        block.append(s)
    flush_block()
    return steps


def nms_blocks(asm_text):
    """Mark the NMS candidate block (the one the m_cand branch skips) by rewriting the
    asm: the block after the first conditional branch of each nms region up to the
    label it targets."""
    out = []
    lines = asm_text.splitlines()
    i = 0
    while i < len(lines):
        l = lines[i]
        out.append(l)
        if ";@st nms" in l:
            # find the two branches; the candidate block lies between the second branch and its target
            j = i + 1
            brs = []
            while j < len(lines) and len(brs) < 2 and ";@st" not in lines[j]:
                out.append(lines[j])
                if lines[j].strip().startswith("s_cbranch"):
                    brs.append(lines[j].strip().split()[-1])
                j += 1
            if len(brs) == 2:
                tgt = brs[1]
                while j < len(lines) and not lines[j].startswith(tgt + ":"):
                    out.append(lines[j] + " ; cand_block" if lines[j].strip().startswith("v_") else lines[j])
                    j += 1
            i = j
            continue
        i += 1
    return "\n".join(out)


ORDER = ["load", "gray", "blur5", "ring_gray", "edge", "gauss_row", "sobel", "direction", "nms", "store", "ring_mag",
         "gauss_col", "mean_mask_sum", "step_end"]
LABEL = {"load": "load issue + address", "gray": "BGR2GRAY", "blur5": "GaussianBlur 5x5",
         "ring_gray": "gray ring moves", "edge": "border flags / REPLICATE", "gauss_row": "Gauss11 CV_32F row pass",
         "sobel": "Sobel + |dx|+|dy| + candidate test", "direction": "Canny direction classes",
         "nms": "NMS + double threshold", "store": "class-map store", "ring_mag": "magnitude ring moves",
         "gauss_col": "Gauss11 column pass", "mean_mask_sum": "rint / mask / masked sum + count",
         "step_end": "loop control"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--json")
    ap.add_argument("--src", default=SRC)
    a = ap.parse_args()
    if a.asm:
        text = open(a.asm).read()
    else:
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "st.s")
            build_asm(p, a.src)
            text = open(p).read()
    steps = analyse(nms_blocks(text))
    n = len(steps)
    tot = collections.Counter()
    for st in steps:
        for stage, c in st.items():
            for k, v in c.items():
                tot[(stage, k)] += v
    rows = []
    path_sum = cand_sum = 0.0
    print(f"k_stencil_stream<true,true>: {n} unrolled row steps; VALU wave-instructions per step (= per 256 pixels)")
    print(f"{'stage':40s} {'every row':>10s} {'cand rows':>10s} {'border':>8s}   families (every row)")
    for stage in ORDER:
        p, c, b = tot[(stage, "path")] / n, tot[(stage, "cand")] / n, tot[(stage, "border")] / n
        fams = {k.split(":")[2]: round(v / n, 1) for (s, k), v in tot.items() if s == stage and k.startswith("fam:path:")}
        rows.append({"stage": stage, "label": LABEL[stage], "every_row": round(p, 2), "candidate_rows": round(c, 2),
                     "border_waves": round(b, 2), "families": fams})
        path_sum += p
        cand_sum += c
        print(f"{LABEL[stage]:40s} {p:10.1f} {c:10.1f} {b:8.1f}   {fams}")
    print(f"{'total':40s} {path_sum:10.1f} {cand_sum:10.1f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"kernel": "k_stencil_stream<true,true>", "steps": n, "per_256_pixels": rows,
                       "every_row_total": round(path_sum, 1), "candidate_rows_extra": round(cand_sum, 1)}, f, indent=1)


if __name__ == "__main__":
    main()
