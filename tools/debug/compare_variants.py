"""Bit-identity check of two libllfe builds on the bench workload (debug tool):
python tools/debug/compare_variants.py VARIANT  -> compares libllfe_VARIANT.so with libllfe.so"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(variant, out):
    code = f"""
import sys, numpy as np, torch
sys.path.insert(0, {ROOT!r})
from low_level_feature_extraction_amd import synth
from low_level_feature_extraction_amd.backend import Backend
be = Backend.get(0)
imgs = synth.synth_batch(64, 1080, 1920, seed=77, device="cuda:0")
res = be.process(imgs, ("colors", "shapes", "shadows"), seed=5)
np.savez({out!r}, c=np.stack([np.pad(r.centers_rgb, ((0, 5 - len(r.centers_rgb)), (0, 0))) for r in res]),
         n=np.array([r.counts.sum() for r in res]), comp=np.array([r.compactness for r in res]),
         u=np.array([r.n_unique for r in res]), s=np.array([r.shadow_sum for r in res]),
         sh=np.array([len(r.shapes) for r in res]))
"""
    env = dict(os.environ)
    if variant:
        env["LLFE_LIB_VARIANT"] = variant
    subprocess.run([sys.executable, "-c", code], check=True, env=env)


def main():
    v = sys.argv[1]
    run(v, "/tmp/cmp_a.npz")
    run(None, "/tmp/cmp_b.npz")
    a, b = np.load("/tmp/cmp_a.npz"), np.load("/tmp/cmp_b.npz")
    ok = True
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        ok &= same
        print(k, "identical" if same else f"DIFFERENT ({(a[k] != b[k]).sum()} entries)")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
