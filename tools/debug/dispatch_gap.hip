// Does a kernel's scratch use delay workgroup dispatch?  Two copies of one busy kernel
// (512 threads, ~75 KB dynamic LDS, two workgroups per CU like k_kmeans; per-workgroup work
// drawn from a hash so durations vary), one with a dynamically indexed private array (scratch),
// one without.  Per workgroup: start / end wall clock and CU; the host prints the idle gap
// between a workgroup's end and the next start on the same CU.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/dgap tools/debug/dispatch_gap.hip && /tmp/dgap
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }

template <bool kScratch>
__global__ __launch_bounds__(512, 4) void k_busy(unsigned long long *rec, int base_iters, int sel) {
    extern __shared__ float lds[];
    const unsigned long long t0 = wall();
    unsigned h = blockIdx.x * 2654435761u;
    h ^= h >> 15;
    const int iters = sel < 0 ? base_iters : base_iters + (int)(h % (unsigned)base_iters) * 3;  // 1x .. 4x (sel < 0: all 1x)
    float acc = (float)threadIdx.x;
    float arr[16];
#pragma unroll
    for (int i = 0; i < 16; i++) arr[i] = acc + (float)i;
    for (int i = 0; i < iters; i++) {
        acc = fmaf(acc, 1.0000001f, 0.5f);
        if (kScratch) arr[(i + sel) & 15] += acc;
    }
    if (base_iters > 0) {
        lds[threadIdx.x & 63] = acc;
        __syncthreads();
        acc += lds[(threadIdx.x + 1) & 63];
    }
    if (kScratch) acc += arr[sel & 15];
    if (threadIdx.x == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        rec[4 * blockIdx.x] = t0;
        rec[4 * blockIdx.x + 1] = wall();
        rec[4 * blockIdx.x + 2] = hw;
        rec[4 * blockIdx.x + 3] = xcc;
    }
    if (acc == 1234.5f) rec[0] = 0;
}

template <bool kScratch>
static void run(const char *name, int nblk, int iters, size_t lds = 75 * 1024, int sel = 3) {
    unsigned long long *d;
    hipMalloc(&d, sizeof(unsigned long long) * 4 * nblk);
    hipFuncSetAttribute((const void *)k_busy<kScratch>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k_busy<kScratch>, dim3(nblk), dim3(512), lds, 0, d, iters, sel);
    hipDeviceSynchronize();
    std::vector<unsigned long long> r(4 * nblk);
    hipMemcpy(r.data(), d, r.size() * 8, hipMemcpyDeviceToHost);
    hipFree(d);
    std::map<unsigned long long, std::vector<std::pair<double, double>>> cu;
    double t_min = 1e300, t_max = 0, busy = 0;
    for (int b = 0; b < nblk; b++) {
        const double s = r[4 * b] / 100.0, e = r[4 * b + 1] / 100.0;  // us (100 MHz)
        const unsigned long long hw = r[4 * b + 2], x = r[4 * b + 3];
        const unsigned long long id = x * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15);
        cu[id].push_back({s, e});
        t_min = std::min(t_min, s);
        t_max = std::max(t_max, e);
        busy += e - s;
    }
    std::vector<double> gaps;
    for (auto &kv : cu) {
        auto v = kv.second;
        std::sort(v.begin(), v.end());
        std::vector<double> ends;
        for (size_t i = 0; i < v.size(); i++) {
            if (i >= 2) {
                double best = -1;
                for (double e : ends)
                    if (e <= v[i].first) best = std::max(best, e);
                if (best >= 0) gaps.push_back(v[i].first - best);
            }
            ends.push_back(v[i].second);
        }
    }
    std::sort(gaps.begin(), gaps.end());
    double mean = 0;
    for (double g : gaps) mean += g;
    mean /= std::max<size_t>(1, gaps.size());
    printf("%-10s lds %3zu KB sel %2d ", name, lds / 1024, sel);
    printf("blocks %d CUs %zu span %.2f ms, busy/slot %.2f ms (%zu slots), gap us: p50 %.1f p90 %.1f mean %.1f\n",
           nblk, cu.size(), (t_max - t_min) / 1e3, busy / 1e3 / (2.0 * cu.size()), 2 * cu.size(),
           gaps.empty() ? 0 : gaps[gaps.size() / 2], gaps.empty() ? 0 : gaps[gaps.size() * 9 / 10], mean);
}

int main() {
    hipFuncAttributes a{}, b{};
    hipFuncGetAttributes(&a, (const void *)k_busy<false>);
    hipFuncGetAttributes(&b, (const void *)k_busy<true>);
    printf("private bytes/lane: no-scratch %zu, scratch %zu\n", (size_t)a.localSizeBytes, (size_t)b.localSizeBytes);
    run<false>("varied", 5120, 20000, 75 * 1024, 3);
    run<false>("uniform", 5120, 50000, 75 * 1024, -1);
    run<false>("varied", 5120, 20000, 1024, 3);
    run<false>("uniform", 5120, 50000, 1024, -1);
    return 0;
}
