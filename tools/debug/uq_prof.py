"""GPU box: hipEvent times of the unique-colour front kernels alone (llfe_color_unique)
on the bench batch (512 x 1080p, 50 % ui / 50 % photo, or LLFE_UQ_KIND=ui|photo), for
each libllfe variant in tools/debug/variants (or the in-tree build)."""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

if len(sys.argv) > 1 and sys.argv[1] == "--one":
    import torch

    from low_level_feature_extraction_amd import synth
    from low_level_feature_extraction_amd.backend import Backend

    kind = os.environ.get("LLFE_UQ_KIND")
    be = Backend.get(0)
    x = synth.synth_batch(512, 1080, 1920, seed=4321, device="cuda:0", **({"kind": kind} if kind else {}))
    for _ in range(2):
        be.color_unique(x, seed=1)
    torch.cuda.synchronize()
    be.set_profiling(True)
    for k in range(5):
        be.color_unique(x, seed=2 + k)
    torch.cuda.synchronize()
    st = be.kernel_stats()
    print(" ".join(f"{n.replace('k_uq_', '')} {v['total_ms'] / max(v['launches'], 1):.3f}" for n, v in st.items()))
    raise SystemExit(0)

lib = os.path.join(ROOT, "low_level_feature_extraction_amd", "libllfe.so")
variants = sorted(glob.glob(os.path.join(ROOT, "tools/debug/variants/libllfe_*.so"))) or [lib]
keep = lib + ".keep"
shutil.copy(lib, keep)
try:
    for v in variants:
        if v != lib:
            shutil.copy(v, lib)
        r = subprocess.run([sys.executable, __file__, "--one"], capture_output=True, text=True, timeout=300)
        print(f"{os.path.basename(v):28s}", r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-800:])
finally:
    shutil.copy(keep, lib)
    os.remove(keep)
