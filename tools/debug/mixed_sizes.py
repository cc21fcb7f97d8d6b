"""Debug: reproduce test_run_batch_mixed_sizes step by step with progress prints."""
import sys, time, faulthandler
sys.path.insert(0, '.')
faulthandler.dump_traceback_later(60, exit=True)
import numpy as np
from low_level_feature_extraction_amd import synth
from low_level_feature_extraction_amd.backend import Backend
be = Backend.get(0)
imgs = [synth.synth_numpy(i, 64 + 32 * (i % 2), 96, seed=8) for i in range(5)]
for feats in [("colors",), ("shapes",), ("shadows",), ("colors", "shapes", "shadows")]:
    for i, im in enumerate(imgs):
        t = time.time()
        print("call", feats, i, im.shape, flush=True)
        r = be.process(im[None], feats, seed=9, index_base=i)
        print("  ok %.3fs" % (time.time() - t), r[0].n_unique, len(r[0].shapes), flush=True)
print("done", flush=True)
