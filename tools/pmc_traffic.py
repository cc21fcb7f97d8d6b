#!/usr/bin/env python3
"""Per-launch HBM traffic from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE run
separately, MI355X_MICROARCH.md §HBM / §PMC slots).

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR [VALU_DIR] > traffic.json

Each DIR holds run_counter_collection.csv from
``rocprofv3 --pmc <C> --kernel-trace -d DIR -o run --output-format csv -- python3 bench.py ...``.
Device kernels are folded into the logical launches libllfe times (k_hysteresis_dilate
= the four k_ccl_* kernels, k_kmeans = order + k-means + finalize); every logical
launch happens once per 256-image chunk, so per-launch traffic = total / chunks, with
chunks = the number of k_stencil (or k_kmeans_finalize) dispatches.

Corrections (gfx950): FETCH_SIZE and WRITE_SIZE are reported in KiB.  FETCH_SIZE counts
half the bytes of wide coalesced streaming reads (16 B / lane), so it is doubled for the
kernels that read that way (FETCH_X2); byte-wide readers are taken as reported (the
guide calls other widths uncalibrated -- checked here: k_color_bitmap's doubled fetch
equals its 3P input exactly, k_stencil's raw fetch lies between its 3P input and the
no-reuse halo bound 3P x 1.75, its doubled fetch would exceed that bound -- that was
the tiled round-1 stencil; the row-streaming one is a dword-per-lane streaming reader).
"""
from __future__ import annotations

import csv
import json
import os
import sys
from collections import defaultdict

# wide coalesced streaming readers: 16 B/lane (k-means, keys, scatter) and the
# row-streaming stencil's three coalesced dwords per lane (r2c: raw fetch 0.55 x its 3P
# input, doubled 1.09 x 3P = its 16/256-column + 10/270-row halo)
FETCH_X2 = {"k_kmeans", "k_uq_scatter", "k_stencil"}

LOGICAL = [  # (substring of the device kernel name, logical launch)
    ("k_stencil", "k_stencil"),
    ("shadow_reduce", "k_stencil"),
    ("k_ccl_", "k_hysteresis_dilate"),
    ("k_bits_dilate", "k_hysteresis_dilate"),
    ("k_uq_scatter", "k_uq_scatter"),
    ("k_uq_part", "k_uq_part"),
    ("k_uq_gather", "k_uq_gather"),
    ("k_kmeans", "k_kmeans"),
    ("k_resize", "k_resize"),
    ("k_reduce", "k_reduce"),
]


def logical(name: str):
    if name.startswith("void "):  # template kernels are reported with their return type
        name = name[5:]
    if not name.startswith("llfe::"):
        return None
    for sub, lg in LOGICAL:
        if sub in name:
            return lg
    return None


def load(d, counter):
    path = os.path.join(d, "run_counter_collection.csv")
    totals = defaultdict(float)
    dispatches = defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            totals[name] += float(row["Counter_Value"])
            dispatches[name].add(row.get("Dispatch_Id"))
    return totals, {k: len(v) for k, v in dispatches.items()}


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    ft, fd = load(fetch_dir, "FETCH_SIZE")
    wt, wd = load(write_dir, "WRITE_SIZE")

    def chunks(disp):
        for k, v in disp.items():
            if "k_stencil" in k or "k_kmeans_finalize" in k:
                return v
        return 1

    out = {"unit": "bytes per logical launch",
           "correction": "FETCH_SIZE KiB x 1024 (x 2 for FETCH_X2 kernels), WRITE_SIZE KiB x 1024", "kernels": {}}
    agg = defaultdict(lambda: {"fetch_kib_raw": 0.0, "write_kib_raw": 0.0})
    for k, v in ft.items():
        lg = logical(k)
        if lg:
            agg[lg]["fetch_kib_raw"] += v / chunks(fd)
    for k, v in wt.items():
        lg = logical(k)
        if lg:
            agg[lg]["write_kib_raw"] += v / chunks(wd)
    if len(sys.argv) > 3:  # SQ_INSTS_VALU pass: VALU wave-instructions per logical launch
        vt, vd = load(sys.argv[3], "SQ_INSTS_VALU")
        for k, v in vt.items():
            lg = logical(k)
            if lg:
                agg[lg]["valu_insts"] = agg[lg].get("valu_insts", 0.0) + v / chunks(vd)
    for lg, a in agg.items():
        a["bytes"] = a["fetch_kib_raw"] * 1024 * (2 if lg in FETCH_X2 else 1) + a["write_kib_raw"] * 1024
        out["kernels"][lg] = a
    out["dispatches_fetch_pass"] = {k: v for k, v in fd.items() if logical(k)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
