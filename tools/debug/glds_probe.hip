// GPU box (round 6): layout and completion of 12-byte direct-to-LDS loads as the stencil's
// LDS input ring uses them.  One wave per block streams R rows of 64 x 12 bytes through a
// ring of D slots: the row for step t + D - 1 is issued at step t (global_load_lds_dwordx3, or
// buffer_load_dwordx3 ... lds), a store is issued every step, and step t reads its row back
// after s_waitcnt vmcnt(D - 2).  Mismatching words are counted per mode (ring lanes 16 bytes
// apart: k_layout shows a 12-byte load lands at lane * 16).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int D = 6, R = 64;

template <int MODE>
__global__ __launch_bounds__(64) void k_probe(const uint8_t *src, uint32_t *sink, int *bad, int n_bytes) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[D][256];  // 16 bytes a lane (measured below)
    const int lane = threadIdx.x;
    const uint8_t *base = src + (size_t)blockIdx.x * R * 768;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, n_bytes, 0x00020000);
    int nbad = 0;
    uint32_t acc = 0;
#pragma unroll
    for (int t0 = -(D - 1); t0 < R; t0 += 12) {
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int t = t0 + k;
            const int slot = ((t + D - 1) % D + D) % D;
            if (t + D - 1 < R && t + D - 1 >= 0) {
                if (MODE == 0)
                    __builtin_amdgcn_global_load_lds((const void *)(base + (size_t)(t + D - 1) * 768 + lane * 12),
                                                     (void *)&ring[slot][0], 12, 0, 0);
                else
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)&ring[slot][0], 12,
                                                             (int)(blockIdx.x * R * 768 + (t + D - 1) * 768 + lane * 12), 0, 0, 0);
            }
            if (t >= 0 && t < R) {
                __builtin_amdgcn_s_waitcnt(((D - 2) & 15) | (7 << 4) | (15 << 8));
                const int rs_ = ((t % D) + D) % D;
                const uint32_t *q = &ring[rs_][4 * lane];
                // expected bytes from the fill formula (no global loads of our own to wait for)
                uint32_t e[3] = {0u, 0u, 0u};
                const uint32_t i0 = blockIdx.x * R * 768u + (uint32_t)t * 768u + (uint32_t)lane * 12u;
#pragma unroll
                for (int bb = 0; bb < 12; bb++) e[bb >> 2] |= (uint32_t)(uint8_t)((i0 + bb) * 2654435761u >> 13) << (8 * (bb & 3));
                const uint32_t a = q[0], b = q[1], c = q[2];
                nbad += (a != e[0]) + (b != e[1]) + (c != e[2]);
                acc += a ^ b ^ c;
                sink[(size_t)blockIdx.x * 64 * R + t * 64 + lane] = acc;  // a store every step
            }
        }
    }
    atomicAdd(bad + MODE, nbad);
}

// the raw layout: one dwordx3 DMA (global and buffer forms) into a zeroed 2 KB LDS buffer, dumped
__global__ __launch_bounds__(64) void k_layout(const uint8_t *src, uint32_t *out, int n_bytes) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[2][512];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) (&buf[0][0])[i] = 0xEEEEEEEEu;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, n_bytes, 0x00020000);
    __builtin_amdgcn_global_load_lds((const void *)(src + lane * 12), (void *)&buf[0][0], 12, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void *)&buf[1][0], 12, lane * 12, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) out[i] = (&buf[0][0])[i];
}

int main() {
    const int blocks = 4096;
    const size_t n = (size_t)blocks * R * 768;
    uint8_t *h = (uint8_t *)malloc(n);
    for (size_t i = 0; i < n; i++) h[i] = (uint8_t)((uint32_t)i * 2654435761u >> 13);
    uint8_t *d;
    uint32_t *sink;
    int *bad;
    hipMalloc(&d, n);
    hipMalloc(&sink, (size_t)blocks * 64 * R * 4);
    hipMalloc(&bad, 8);
    hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(64), 0, 0, d, sink, bad, (int)n);
    hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(64), 0, 0, d, sink, bad, (int)n);
    uint32_t *lay;
    hipMalloc(&lay, 4096);
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, d, lay, (int)n);
    uint32_t hl[1024];
    hipMemcpy(hl, lay, 4096, hipMemcpyDeviceToHost);
    for (int form = 0; form < 2; form++) {
        const uint32_t *L = hl + 512 * form, *S = (const uint32_t *)h;
        int m12 = 0, m16 = 0, untouched = 0;
        for (int l = 0; l < 64; l++)
            for (int w = 0; w < 3; w++) {
                m12 += L[3 * l + w] == S[3 * l + w];
                m16 += L[4 * l + w] == S[3 * l + w];
            }
        for (int i = 0; i < 512; i++) untouched += L[i] == 0xEEEEEEEEu;
        printf("%s dwordx3 -> LDS: words matching at lane*12: %d / 192, at lane*16: %d / 192, untouched words of 512: %d\n",
               form ? "buffer" : "global", m12, m16, untouched);
    }
    int hb[2];
    hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost);
    printf("glds dwordx3 ring: %d bad words; buffer ... lds ring: %d bad words (of %zu)\n", hb[0], hb[1], n / 4);
    return hipDeviceSynchronize() != hipSuccess;
}
