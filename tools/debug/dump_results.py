"""Dump the batch results of the in-tree libllfe.so on a fixed synthetic batch (debug:
bit-identity of two builds, see tools/debug/identity.sh)."""
import hashlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402

be = Backend.get(0)
imgs = synth.synth_batch(int(sys.argv[2]) if len(sys.argv) > 2 else 128, 1080, 1920, seed=77, device="cuda:0")
res = be.process(imgs, ("colors", "shapes", "shadows"), seed=5)
torch.cuda.synchronize()
np.savez(sys.argv[1], c=np.stack([np.pad(np.asarray(r.centers_rgb, np.int32), ((0, 5 - len(r.centers_rgb)), (0, 0))) for r in res]),
         n=np.stack([np.pad(np.asarray(r.counts, np.int64), (0, 5 - len(r.counts))) for r in res]),
         comp=np.array([r.compactness for r in res]), u=np.array([r.n_unique for r in res]),
         s=np.array([r.shadow_sum for r in res]), sc=np.array([r.shadow_count for r in res]),
         sh=np.array([len(r.shapes) for r in res]),
         shp=np.array([int(hashlib.sha1(repr(r.shapes).encode()).hexdigest()[:15], 16) for r in res], np.int64))
