// Micro-benchmark: cost per point of the k-means labelling loop shapes on gfx950.
//   hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/debug/km_micro.hip -o /tmp/km_micro
// Variants (one 1024-thread workgroup per block of points, LDS lane-private accumulators):
//   0  plain: 4 keys per lane per step from one 16-B load
//   1  one key per lane per step (4-B loads), 8 steps per round
//   2  as 1 without the LDS atomics (labels summed into a register)
//   3  as 1 without memory (synthetic keys)
//   4  as 0 without the LDS atomics
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
struct CentP {
    f2 x[3], y[3], z[3];
};

__device__ __forceinline__ int label5p(uint32_t key, const CentP &c) {
    const float x = (float)((key >> 16) & 255u), y = (float)((key >> 8) & 255u), z = (float)(key & 255u);
    const f2 px = f2{x, x}, py = f2{y, y}, pz = f2{z, z};
    f2 d[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        const f2 t0 = px - c.x[j], t1 = py - c.y[j], t2 = pz - c.z[j];
        f2 dd = t0 * t0;
        dd = __builtin_elementwise_fma(t1, t1, dd);
        dd = __builtin_elementwise_fma(t2, t2, dd);
        d[j] = dd;
    }
    const float m = fminf(fminf(fminf(d[0].x, d[0].y), fminf(d[1].x, d[1].y)), d[2].x);
    int l = 4;
    l = d[1].y == m ? 3 : l;
    l = d[1].x == m ? 2 : l;
    l = d[0].y == m ? 1 : l;
    l = d[0].x == m ? 0 : l;
    return l;
}

constexpr int KT = 1024;

template <int V>
__global__ __launch_bounds__(KT) void k(const uint32_t *__restrict__ keys, int n_per_block, float cs,
                                        unsigned long long *out) {
    __shared__ unsigned long long accA[5][KT], accB[5][KT];
    __shared__ uint32_t tab[16][64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    CentP c;
#pragma unroll
    for (int j = 0; j < 3; j++) {
        c.x[j] = f2{cs * (40.f + 30 * j), cs * (55.f + 30 * j)};
        c.y[j] = f2{cs * (90.f - 10 * j), cs * (60.f + 7 * j)};
        c.z[j] = f2{cs * (20.f + 50 * j), j == 2 ? 1e30f : cs * (200.f - 40 * j)};
    }
    for (int k2 = 0; k2 < 5; k2++) accA[k2][tid] = accB[k2][tid] = 0;
    tab[wid][lane] = (uint32_t)lane * 64;
    const uint32_t *p = keys + (size_t)blockIdx.x * n_per_block;
    const int per_wave = n_per_block / 16;
    const uint32_t *pw = p + (size_t)wid * per_wave;
    unsigned long long reg = 0;
    for (int rep = 0; rep < 20; rep++) {
        if (V == 0 || V == 4) {
            for (int s = 0; s < per_wave / 256; s++) {
                const uint4 v = *(const uint4 *)(pw + s * 256 + lane * 4);
                const uint32_t kq[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const int l = label5p(kq[jj], c);
                    if (V == 0) {
                        atomicAdd(&accA[l][tid], (unsigned long long)((kq[jj] >> 16) & 255u) |
                                                     ((unsigned long long)((kq[jj] >> 8) & 255u) << 32));
                        atomicAdd(&accB[l][tid], (unsigned long long)(kq[jj] & 255u) | (1ull << 32));
                    } else {
                        reg += (unsigned long long)l + kq[jj];
                    }
                }
            }
        } else {
            for (int s = 0; s < per_wave / 64; s += 8) {
                uint32_t kq[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    uint32_t off = (uint32_t)(s + u) * 64;
                    if (V == 5) off = tab[wid][(s + u) & 63];  // LDS read per step
                    kq[u] = V == 3 ? ((uint32_t)(s + u) * 2654435761u + (uint32_t)lane * 40503u) & 0xFFFFFFu
                                   : pw[off + lane];
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int l = label5p(kq[u], c);
                    if (V == 2) {
                        reg += (unsigned long long)l + kq[u];
                    } else {
                        atomicAdd(&accA[l][tid], (unsigned long long)((kq[u] >> 16) & 255u) |
                                                     ((unsigned long long)((kq[u] >> 8) & 255u) << 32));
                        atomicAdd(&accB[l][tid], (unsigned long long)(kq[u] & 255u) | (1ull << 32));
                    }
                }
            }
        }
    }
    __syncthreads();
    unsigned long long s = reg;
    for (int k2 = 0; k2 < 5; k2++) s += accA[k2][tid] + accB[k2][tid];
    atomicAdd(out, s);
}

int main() {
    const int blocks = 256, npb = 1 << 18;  // 256 WGs x 262144 points
    std::vector<uint32_t> h((size_t)blocks * npb);
    uint32_t x = 12345;
    for (auto &v : h) {
        x = x * 1664525u + 1013904223u;
        v = (x >> 8) & 0xFFFFFFu;
    }
    uint32_t *d;
    unsigned long long *o;
    hipMalloc(&d, h.size() * 4);
    hipMalloc(&o, 8);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(KT), 0, 0, d, npb, 1.f, o);
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(KT), 0, 0, d, npb, 1.f, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double pts = (double)blocks * npb * 20;
        printf("%-40s %8.3f ms  %6.3f ns/point/WG-equivalent  %.2f Gpts/s\n", name, ms,
               ms * 1e6 / (pts / blocks), pts / ms / 1e6);
    };
    run(k<0>, "0 plain uint4 + atomics");
    run(k<4>, "4 plain uint4, no atomics");
    run(k<1>, "1 one key/lane + atomics");
    run(k<2>, "2 one key/lane, no atomics");
    run(k<3>, "3 one key/lane synthetic + atomics");
    run(k<5>, "5 one key/lane + per-step LDS read + atomics");
    return 0;
}
