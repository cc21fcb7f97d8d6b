"""GPU box: shadow stats of one batch through every entry point, repeated (race hunt)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from low_level_feature_extraction_amd import synth  # noqa: E402
from low_level_feature_extraction_amd.backend import Backend  # noqa: E402
from oracle import oracle as O  # noqa: E402

be = Backend.get(0)
h, w = int(sys.argv[1]), int(sys.argv[2])
imgs = np.stack([synth.synth_numpy(i, h, w, seed=7) for i in range(2)])
exp = [tuple(int(v) for v in O.shadow_stats(im)) for im in imgs]
if len(sys.argv) > 3:
    r = be.process(imgs, ("shadows",), seed=3)
    print("FIRST process host ", [(x.shadow_sum, x.shadow_count) for x in r])
dev = torch.from_numpy(imgs).cuda()
torch.cuda.synchronize()
print("exp", exp)
for rep in range(3):
    s, c = be.shadow_stats(imgs)
    print("shadow_stats host  ", [(int(a), int(b)) for a, b in zip(s, c)])
    s, c = be.shadow_stats(dev)
    print("shadow_stats device", [(int(a), int(b)) for a, b in zip(s, c)])
    r = be.process(imgs, ("shadows",), seed=3)
    print("process host       ", [(x.shadow_sum, x.shadow_count) for x in r])
    r = be.process(dev, ("shadows",), seed=3)
    print("process device     ", [(x.shadow_sum, x.shadow_count) for x in r])
    r = be.process(imgs[:1], ("shadows",), seed=3)
    print("process host n=1   ", [(x.shadow_sum, x.shadow_count) for x in r], flush=True)
