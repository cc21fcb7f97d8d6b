"""H2D bandwidth from pinned host memory: one copy vs the same bytes split over several
streams (SDMA engines), and the kernel-side read of pinned host memory is not measured.

    python tools/debug/h2d_bw.py [MiB]
"""
import sys
import time

import torch


def run(src, dst, parts, reps=5):
    streams = [torch.cuda.Stream() for _ in range(parts)]
    n = src.numel()
    cuts = [n * i // parts for i in range(parts + 1)]
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                dst[cuts[i]:cuts[i + 1]].copy_(src[cuts[i]:cuts[i + 1]], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return n / best / 1e9


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1600
    n = mib << 20
    src = torch.empty(n, dtype=torch.uint8).pin_memory()
    src.fill_(7)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    run(src, dst, 1, 2)
    for parts in (1, 2, 3, 4, 8):
        print(f"{mib} MiB H2D over {parts} stream(s): {run(src, dst, parts):6.1f} GB/s", flush=True)
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    src2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    # two independent full-size copies at once (two batches in flight)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(s1):
        dst.copy_(src, non_blocking=True)
    with torch.cuda.stream(s2):
        d2.copy_(src2, non_blocking=True)
    torch.cuda.synchronize()
    print(f"two {mib} MiB copies on two streams: {2 * n / (time.perf_counter() - t) / 1e9:6.1f} GB/s")


if __name__ == "__main__":
    main()
