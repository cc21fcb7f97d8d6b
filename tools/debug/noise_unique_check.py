import sys, numpy as np
sys.path.insert(0, '.')
from low_level_feature_extraction_amd.backend import Backend
from low_level_feature_extraction_amd import synth
from oracle import oracle as O
be = Backend.get(0)
imgs = np.stack([synth.synth_numpy(i, 1080, 1920, seed=2025) for i in range(8)])
_, u_dev = be.color_unique(imgs, seed=7)
noise = np.stack([O.numpy_noise(1080 * 1920, 11 + i).reshape(1080, 1920, 3) for i in range(8)])
_, u_np = be.color_unique(imgs, seed=7, noise=noise)
_, u_dev2 = be.color_unique(imgs, seed=8)
print("device", list(u_dev)); print("device2", list(u_dev2)); print("numpy ", list(u_np))
print("ratio dev/np", [round(a / b, 4) for a, b in zip(u_dev, u_np)])
