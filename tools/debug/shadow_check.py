"""GPU box: shadow (sum, count) of the fused stencil vs the oracle over sizes / classes,
with shapes on and off (k_stencil_stream<CLS, SHD> instantiations).  Prints mismatches."""
import sys

import numpy as np

sys.path.insert(0, ".")
from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402
from oracle import oracle as O  # noqa: E402

be = Backend.get(0)
sizes = [(270, 480), (540, 960), (1080, 1920), (1080, 3840), (2160, 1920), (2160, 3840)]
bad = 0
for (h, w) in sizes:
    imgs = np.stack([synth.synth_numpy(i, h, w, seed=7) for i in range(2)])
    exp = [O.shadow_stats(im) for im in imgs]
    for feats in (("shadows",), ("shapes", "shadows")):
        res = be.process(imgs, feats, seed=3)
        got = [(r.shadow_sum, r.shadow_count) for r in res]
        ok = got == [tuple(e) for e in exp]
        bad += not ok
        print(h, w, feats, "ok" if ok else f"MISMATCH got {got} exp {exp}", flush=True)
print("bad", bad)
