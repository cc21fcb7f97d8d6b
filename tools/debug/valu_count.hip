// Calibration of the PMC counter SQ_INSTS_VALU on gfx950: one wave per kernel issues
// exactly 1024 instructions of one kind (straight-line inline asm, no loop), so the
// counter per launch says how many "VALU instructions" one such instruction counts as.
//   hipcc -O3 --offload-arch=gfx950 tools/debug/valu_count.hip -o /tmp/valu_count
//   rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d out -- /tmp/valu_count
#include <hip/hip_runtime.h>
#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)
#define R1024(x) R16(R16(R4(x)))

template <int OP>
__global__ void k_count(unsigned *out) {
    unsigned r = threadIdx.x, b = blockIdx.x | 1;
    float f = (float)r, g = 1.0f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p = {f, f}, q = {g, g};
    if (OP == 0) { R1024(asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));) }
    if (OP == 1) { R1024(asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p) : "v"(q));) }
    if (OP == 2) { R1024(asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(b));) }
    if (OP == 3) { R1024(asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 bound_ctrl:1" : "+v"(r) : "v"(b));) }
    if (OP == 4) { R1024(asm volatile("v_dot2_u32_u16 %0, %1, %1, %0" : "+v"(r) : "v"(b));) }
    if (OP == 5) { R1024(asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(r) : "v"(b));) }
    if (OP == 6) { R1024(asm volatile("v_cvt_f32_ubyte1 %0, %1" : "+v"(f) : "v"(b));) }
    if (OP == 7) { R1024(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"(g));) }
    if (OP == 8) { R1024(asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p) : "v"(q));) }
    if (OP == 9) { R1024(asm volatile("v_mov_b32 %0, %1" : "+v"(r) : "v"(b));) }
    if (OP == 10) { R1024(asm volatile("s_add_u32 %0, %0, 1" : "+s"(b));) }  // SALU: expect 0 VALU
    out[blockIdx.x * 64 + threadIdx.x] = r + (unsigned)f + (unsigned)p.x + (unsigned)p.y + b;
}

int main() {
    unsigned *d;
    hipMalloc(&d, 64 * 64 * sizeof(unsigned));
    // 1 wave per launch, then 64 waves (1 per CU ... spread) to check the counter scales
    for (int waves : {1, 64}) {
        hipLaunchKernelGGL(k_count<0>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<1>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<2>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<3>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<4>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<5>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<6>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<7>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<8>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<9>, dim3(waves), dim3(64), 0, 0, d);
        hipLaunchKernelGGL(k_count<10>, dim3(waves), dim3(64), 0, 0, d);
    }
    hipDeviceSynchronize();
    printf("launched: ops 0..10 (add_u32, pk_fma_f32, pk_add_u16, mov_dpp, dot2_u32_u16, perm, cvt_f32_ubyte1, "
           "fma_f32, pk_add_f32, mov_b32, s_add_u32) x 1024 per wave, at 1 and 64 waves\n");
    hipFree(d);
    return 0;
}
