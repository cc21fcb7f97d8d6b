"""GPU box: the stencil (shapes + shadows) on a 512 x 1080p batch of one synthetic class
(argv[1]: ui | photo | mix), 3 launches; run under rocprofv3 --pmc to split the stencil's
VALU count by class (tools/debug/stencil_pmc_kind.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from low_level_feature_extraction_amd import backend as B, synth  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "mix"
x = synth.synth_batch(512, 1080, 1920, seed=2025, device="cuda:0", kind=None if kind == "mix" else kind)
torch.cuda.synchronize()
be = B.Backend.get(0)
for _ in range(3):
    be.process(x, ("shapes", "shadows"), seed=7)
torch.cuda.synchronize()
print("done", kind)
