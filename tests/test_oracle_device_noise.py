"""The oracle's restatement of the product's production noise (orc_device_noise).

The reference draws ``np.random.normal(0, 0.5, (P, 3)).astype(np.int8)`` from the
process-global NumPy RNG (color_extractor.py:223-225); the product draws a seeded
stream of the same distribution on the device (unique.hip).  The GPU
tests pin the device stream to this restatement bit-exactly
(tests/test_gpu_served.py); here, on the CPU, the restatement is checked against the
reference's distribution and its per-image structure.
"""
import math

import numpy as np


def _tail(z):
    return 0.5 * math.erfc(-z / math.sqrt(2.0))  # P(Z <= z)


def test_distribution_matches_trunc_normal(orc):
    n = 1 << 20
    a = orc.device_noise(n, 12345, 7).astype(np.int64)
    assert a.shape == (n, 3)
    ref = np.random.RandomState(0).normal(0, 0.5, (n, 3)).astype(np.int8)  # the reference's draw
    # trunc(0.5 Z): |value| = 1 iff 2 <= |Z| < 4, 2 iff 4 <= |Z| < 6 (|Z| >= 6: ~1e-9, not drawn)
    p1, p2 = _tail(-2.0) - _tail(-4.0), _tail(-4.0)
    for ch in range(3):
        for val, p in [(-1, p1), (1, p1), (-2, p2), (2, p2)]:
            sd = math.sqrt(n * p * (1 - p))
            got = int((a[:, ch] == val).sum())
            want_ref = int((ref[:, ch] == val).sum())
            assert abs(got - n * p) <= 5 * sd + 3, (ch, val, got, n * p)
            assert abs(want_ref - n * p) <= 5 * sd + 3  # (the same bound holds for NumPy's own draw)
    assert set(np.unique(a)) <= {-2, -1, 0, 1, 2}
    # channels are independent: joint non-zero rate = product of the marginals
    nz = a != 0
    both = float((nz[:, 0] & nz[:, 1]).mean())
    assert abs(both - nz[:, 0].mean() * nz[:, 1].mean()) < 2e-4


def test_rotations_per_global_index(orc):
    """One field per (seed, size); image g reads it rotated by a multiple of 16 pixels."""
    P = 4096 + 5  # L = 4112
    L = (P + 15) // 16 * 16
    a = orc.device_noise(P, 99, 0)
    b = orc.device_noise(P, 99, 1)
    assert not np.array_equal(a, b)
    assert np.array_equal(orc.device_noise(P, 99, 1), b)  # deterministic
    assert not np.array_equal(orc.device_noise(P, 100, 0), a)  # the seed changes the field
    # at P = L every field pixel is read once: index 1's noise is index 0's rotated by
    # exactly one multiple of 16
    fa_full = orc.device_noise(L, 99, 0)
    fb_full = orc.device_noise(L, 99, 1)
    rot = [s for s in range(0, L, 16) if np.array_equal(np.roll(fa_full, -s, axis=0), fb_full)]
    assert len(rot) == 1


def test_small_and_empty(orc):
    assert orc.device_noise(0, 1, 0).shape == (0, 3)
    one = orc.device_noise(1, 1, 0)
    assert one.shape == (1, 3) and set(one.ravel()) <= {-2, -1, 0, 1, 2}
