// Issue-rate microbenchmark: cycles per wave64 VALU instruction per SIMD for the
// instruction kinds the stencil / k-means kernels use, at 1 and 8 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/debug/valu_rate.hip -o /tmp/valu_rate && /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
template <int OP>
__global__ void k(unsigned *out, int iters) {
    unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 + 1, a5 = a0 + 2, a6 = a0 + 3, a7 = a0 + 4;
    unsigned b = blockIdx.x | 1;
    for (int i = 0; i < iters; i++) {
#define OP1(r)                                                                                          \
    if (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));                               \
    if (OP == 1) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(r) : "v"(b));                              \
    if (OP == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(b));                            \
    if (OP == 3) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r) : "v"(b));                          \
    if (OP == 4) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:1" : "+v"(r) : "v"(b));        \
    if (OP == 5) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(r) : "v"(b) : "s0", "s1");  \
    if (OP == 6) asm volatile("v_cvt_f32_ubyte1 %0, %1" : "+v"(r) : "v"(b));                            \
    if (OP == 7) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(r));                                      \
    if (OP == 8) asm volatile("v_dot2_u32_u16 %0, %1, %1, %0" : "+v"(r) : "v"(b));                      \
    if (OP == 9) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(r) : "v"(b));                      \
    if (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(r) : "v"(b));                       \
    if (OP == 11) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(r) : "v"(b)); \
    if (OP == 13) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 14) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 15) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(r));  \
    if (OP == 16) asm volatile("v_mov_b32 %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 17) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r) : "v"(b) : "vcc");  \
    if (OP == 18) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 19) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 20) asm volatile("v_max_i32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 21) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 22) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(b));  \
    if (OP == 24) asm volatile("v_add_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 25) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(r));  \
    if (OP == 26) asm volatile("v_rndne_f32 %0, %0" : "+v"(r));  \
    if (OP == 27) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(r), "v"(b) : "vcc");  \
    if (OP == 28) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(r) : "v"(b));  \
    if (OP == 29) asm volatile("v_dot4_u32_u8 %0, %1, %1, %0" : "+v"(r) : "v"(b));  \
    if (OP == 30) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 31) asm volatile("v_lshrrev_b32 %0, 1, %0" : "+v"(r));  \
    if (OP == 32) asm volatile("v_sad_u32 %0, %0, %1, %1" : "+v"(r) : "v"(b));  \
    if (OP == 34) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(r) : "v"(b)); \
    if (OP == 35) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 36) asm volatile("v_not_b32 %0, %0" : "+v"(r));  \
    if (OP == 37) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 38) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 39) asm volatile("v_max_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 40) asm volatile("v_min_f32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 41) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 42) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r) : "v"(b));  \
    if (OP == 43) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(r) : "v"(b));  \
    if (OP == 44) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(r) : "v"(b));  \
    if (OP == 45) asm volatile("v_pk_max_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 46) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 47) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 48) asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 49) asm volatile("v_max_u16 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 50) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(r) : "v"(b) : "vcc");  \
    if (OP == 51) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(r));  \
    if (OP == 52) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(r) : "v"(b));  \
    if (OP == 53) asm volatile("v_add_u32 %0, s4, %0" : "+v"(r) : : "s4");  \
    if (OP == 54) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 55) asm volatile("v_mul_f32_e64 %0, -%0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 56) asm volatile("v_cvt_f32_ubyte0 %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 57) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "+v"(r) : "v"(b));  \
    if (OP == 58) asm volatile("v_and_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(r) : "v"(b));  \
    if (OP == 59) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(r) : "v"(b)); \
    if (OP == 60) asm volatile("v_fmac_f32 %0, %1, %1\n v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 61) asm volatile("v_perm_b32 %0, %0, %1, %1\n v_and_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 62) asm volatile("v_fmac_f32 %0, %1, %1\n v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 63) asm volatile("v_add_u32 %0, %0, %1\n v_mul_f32 %0, %0, %1" : "+v"(r) : "v"(b)); \
    if (OP == 64) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 65) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 66) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 67) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(r) : "v"(b));  \
    if (OP == 68) asm volatile("v_lshrrev_b32 %0, 16, %0\n v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(b));
        REP8(OP1(a0) OP1(a1) OP1(a2) OP1(a3) OP1(a4) OP1(a5) OP1(a6) OP1(a7))
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
template <int OP>
__global__ void kpk(unsigned *out, int iters) {  // v_pk_fma_f32 on 64-bit pairs
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a0 = {1.f * threadIdx.x, 2.f}, a1 = a0 + 1.f, a2 = a0 + 2.f, a3 = a0 + 3.f, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 b = {1.0001f, 0.9999f};
    for (int i = 0; i < iters; i++) {
#define OP2(r) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(r) : "v"(b));
        REP8(OP2(a0) OP2(a1) OP2(a2) OP2(a3) OP2(a4) OP2(a5) OP2(a6) OP2(a7))
    }
    f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = __float_as_uint(s.x + s.y);
}

static const char *names[] = {"v_add_u32", "v_fmac_f32", "v_pk_add_u16", "v_perm_b32", "v_mov_dpp", "v_cndmask_e64",
                              "v_cvt_f32_ubyte", "v_bfe_u32", "v_dot2_u32_u16", "v_alignbit", "v_lshl_or", "v_mad_u32_u24",
                              "v_pk_fma_f32", "v_and_b32", "v_or_b32", "v_lshlrev_b32", "v_mov_b32", "v_cndmask_e32", "v_add_f32", "v_mul_f32", "v_max_i32", "v_sub_u32", "v_add3_u32", "v_pk_add_f32", "v_add_u16", "v_cvt_f32_u32", "v_rndne_f32", "v_cmp_gt_u32", "v_med3_u32", "v_dot4_u32_u8", "v_mul_u32_u24", "v_lshrrev_b32", "v_sad_u32", "v_cvt_pk_u8_f32", "v_fma_f32", "v_pk_mul_f32", "v_xor_b32", "v_not_b32", "v_bfi_b32", "v_min_u32", "v_max_u32", "v_min_f32", "v_sub_f32", "v_lshlrev_b32_v", "v_lshrrev_b32_v", "v_ashrrev_i32", "v_pk_max_u16", "v_pk_sub_u16", "v_sub_u16", "v_mul_lo_u16", "v_max_u16", "v_add_co_u32", "v_cvt_u32_f32", "v_and_or_b32", "v_add_u32_sgpr", "v_add_u32_e64", "v_mul_f32_e64neg", "v_cvt_f32_ubyte0", "v_mov_b32_sdwa", "v_and_b32_sdwa", "v_add_u32_sdwa", "mix_fmac_add", "mix_perm_and", "mix_fmac_2add", "mix_add_mulf", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_hi_u32_u24", "v_bcnt_u32_b32", "v_xor_lshr_mix"};
template <int OP>
void run(unsigned *out, int wps) {
    const int blocks = 256 * wps, threads = 256, iters = 2000;  // 4 waves per block = one per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        if (OP != 12) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(threads), 0, 0, out, iters);
        else hipLaunchKernelGGL(kpk<0>, dim3(blocks), dim3(threads), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double insts_per_simd = (double)wps * iters * 64;  // per SIMD: wps waves x iters x 64 insts
    printf("%-16s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (%.3f ms)\n", names[OP >= 35 ? OP + 1 : OP], wps,
           ms * 1e-3 * 2.4e9 / insts_per_simd, ms);
}
template <int OP>
void both(unsigned *out) {
    run<OP>(out, 1);
    run<OP>(out, 8);
}
__global__ void kclk(unsigned long long *o) {
    unsigned long long c0 = clock64(), w0 = wall_clock64();
    unsigned a = threadIdx.x;
    for (int i = 0; i < 200000; i++) asm volatile("v_add_u32 %0, %0, %0" : "+v"(a));
    unsigned long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = c1 - c0; o[2 * blockIdx.x + 1] = (w1 - w0) + (a & 0); }
}
int main() {
    {
        unsigned long long *d, h[2];
        hipMalloc(&d, 2 * 2048 * 8);
        hipLaunchKernelGGL(kclk, dim3(2048), dim3(256), 0, 0, d);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        int rate = 0;
        hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
        printf("clock64 ticks %llu over wall ticks %llu (wall rate %d kHz): shader clock ~ %.3f GHz\n", h[0], h[1], rate,
               (double)h[0] / h[1] * rate * 1e-6);
    }
    unsigned *out;
    hipMalloc(&out, 256 * 8 * 256 * 4);
    both<0>(out); both<1>(out); both<64>(out); both<65>(out); both<66>(out); both<67>(out); both<68>(out);
    return 0;
}
