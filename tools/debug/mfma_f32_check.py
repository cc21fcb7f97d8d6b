"""Compares v_mfma_f32_16x16x4_f32 results (tools/debug/mfma_f32_probe.hip) with rounding
models: sequential fma chains in k order / reverse order, products rounded then added,
one rounding of the exact sum, and pairwise trees.  Usage: mfma_f32_check.py file.bin"""
import sys
from fractions import Fraction

import numpy as np


def f32(x: Fraction) -> float:
    """Round an exact rational to the nearest f32 (ties to even)."""
    d = float(x)  # nearest double (correct rounding of the rational)
    f = np.float32(d)
    # double rounding fix: compare the two f32 neighbours around d exactly
    cand = [f, np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))]
    best = min(cand, key=lambda c: (abs(Fraction(float(c)) - x), int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1))
    return float(best)


def fma(a, b, c):
    return f32(Fraction(a) * Fraction(b) + Fraction(c))


def main(path):
    raw = np.fromfile(path, dtype=np.int32, count=2)
    T, chain = int(raw[0]), int(raw[1])
    data = np.fromfile(path, dtype=np.float32, offset=8)
    na = T * chain * 64
    A = data[:na].reshape(T, chain, 16, 4)
    B = data[na:2 * na].reshape(T, chain, 4, 16)
    C = data[2 * na:2 * na + T * 256].reshape(T, 16, 16)
    D = data[2 * na + T * 256:].reshape(T, 16, 16)
    models = {"fma k0..3": 0, "fma k3..0": 0, "round(exact sum) per instr": 0, "prod rounded, add k0..3": 0,
              "pairwise exact pairs, round, +c": 0, "exact 4-sum rounded, then +c rounded": 0}
    total = 0
    per_mode = {}
    rng = np.random.default_rng(0)
    for t in range(T):
        mode = t % 4
        for (m, n) in [tuple(x) for x in rng.integers(0, 16, size=(6, 2))]:
            got = float(D[t, m, n])
            res = {}
            for name in models:
                c = float(C[t, m, n])
                for j in range(chain):
                    p = [Fraction(float(A[t, j, m, k])) * Fraction(float(B[t, j, k, n])) for k in range(4)]
                    if name == "fma k0..3":
                        for k in range(4):
                            c = f32(p[k] + Fraction(c))
                    elif name == "fma k3..0":
                        for k in range(3, -1, -1):
                            c = f32(p[k] + Fraction(c))
                    elif name == "round(exact sum) per instr":
                        c = f32(sum(p) + Fraction(c))
                    elif name == "prod rounded, add k0..3":
                        for k in range(4):
                            c = f32(Fraction(f32(p[k])) + Fraction(c))
                    elif name == "pairwise exact pairs, round, +c":
                        s01 = f32(p[0] + p[1])
                        s23 = f32(p[2] + p[3])
                        c = f32(Fraction(f32(Fraction(s01) + Fraction(s23))) + Fraction(c))
                    else:
                        c = f32(Fraction(f32(sum(p))) + Fraction(c))
                res[name] = c
            total += 1
            pm = per_mode.setdefault(mode, {k: 0 for k in models} | {"n": 0})
            pm["n"] += 1
            for name, v in res.items():
                if v == got:
                    models[name] += 1
                    pm[name] += 1
    print(f"{total} outputs checked (chain of {chain} MFMAs each)")
    for name, v in models.items():
        print(f"  {name:40s} {v}/{total}")
    for mode, pm in sorted(per_mode.items()):
        print("mode", mode, {k: v for k, v in pm.items()})


if __name__ == "__main__":
    main(sys.argv[1])
