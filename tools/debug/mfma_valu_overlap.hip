// Does v_mfma_f32_16x16x4_f32 run beside VALU FMAs, or does it share their issue /
// datapath?  Times VALU-only, MFMA-only and mixed loops (same counts) with hipEvents;
// the bf16 MFMA mix is the control (the matrix pipe proper).  Stencil redesign, DESIGN §3.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int MODE>  // 0 VALU, 1 f32 MFMA, 2 both, 3 bf16 MFMA, 4 bf16 MFMA + VALU,
                     // 5 / 6: odd waves VALU x2, even waves f32 / bf16 MFMA x2 (wave-specialised)
__global__ __launch_bounds__(256) void k(float *out, int iters, float s) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = threadIdx.x * 0.001f + i;
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    f32x4 d0 = c0, d1 = c0, d2 = c0, d3 = c0;
    const float a = s * threadIdx.x, b = s + threadIdx.x;
    bf16x8 ab;
#pragma unroll
    for (int i = 0; i < 8; i++) ab[i] = (__bf16)(a + i);
    const bool odd = (threadIdx.x >> 6) & 1;
    const int reps = MODE >= 5 ? 2 : 1;
    for (int it = 0; it < iters * reps; it++) {
        if (MODE == 1 || MODE == 2 || (MODE == 5 && !odd)) {
            // 8 f32 MFMAs (32 cyc/SIMD each) in 4 independent chains
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
        }
        if (MODE == 3 || MODE == 4 || (MODE == 6 && !odd)) {
            // 8 bf16 16x16x32 MFMAs (16 cyc/SIMD each)
            d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d3, 0, 0, 0);
            d0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d0, 0, 0, 0);
            d1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d1, 0, 0, 0);
            d2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d2, 0, 0, 0);
            d3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, ab, d3, 0, 0, 0);
        }
        if (MODE == 0 || MODE == 2 || MODE == 4 || (MODE >= 5 && odd)) {
            // 64 independent v_fma_f32 (4 cyc each per wave64)
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int i = 0; i < 16; i++) v[i] = __builtin_fmaf(v[i], 0.999f, s);
        }
    }
    float acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc += v[i];
    acc += c0[0] + c1[1] + c2[2] + c3[3] + d0[0] + d1[1] + d2[2] + d3[3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    float *out;
    const int blocks = 256 * 8, iters = 2000;  // 8 blocks of 4 waves per CU = 8 waves / SIMD
    hipMalloc(&out, sizeof(float) * blocks * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[7] = {"VALU 64 fma", "f32 MFMA x8", "f32 MFMA x8 + VALU 64 fma", "bf16 MFMA x8",
                            "bf16 MFMA x8 + VALU 64 fma",
                            "waves split: f32 MFMA x16 | VALU 128", "waves split: bf16 MFMA x16 | VALU 128"};
    for (int rep = 0; rep < 2; rep++)
        for (int m = 0; m < 7; m++) {
            hipEventRecord(e0);
            switch (m) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, out, iters, 1e-7f); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // cycles per iteration per SIMD at the measured clock: report ms only
            if (rep) printf("%-30s %8.3f ms\n", names[m], ms);
        }
    return 0;
}
