// Probe of v_mfma_f32_16x16x4_f32 numerics (stencil redesign: can the CV_32F Gauss11 row
// pass -- s = fma(x[t], k[t], s), t = 0..10 -- run on the matrix pipe bit-exactly?).
// Writes A, B, C and the MFMA result of many random 16x16x4 products to a binary file;
// tools/debug/mfma_f32_check.py compares them with candidate rounding models.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// one wave per trial: lane l holds A[l&15][l>>4], B[l>>4][l&15], C[4(l>>4)+i][l&15]
__global__ void k_probe(const float *A, const float *B, const float *C, float *D, int chain) {
    const int l = threadIdx.x, t = blockIdx.x;
    f32x4 c;
    for (int i = 0; i < 4; i++) c[i] = C[(size_t)t * 256 + (4 * (l >> 4) + i) * 16 + (l & 15)];
    for (int j = 0; j < chain; j++) {
        const float a = A[((size_t)t * chain + j) * 64 + (l & 15) * 4 + (l >> 4)];   // A[m][k], 16 x 4
        const float b = B[((size_t)t * chain + j) * 64 + (l >> 4) * 16 + (l & 15)];  // B[k][n], 4 x 16
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    for (int i = 0; i < 4; i++) D[(size_t)t * 256 + (4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main(int argc, char **argv) {
    const int T = 2048, chain = 3;
    std::vector<float> A((size_t)T * chain * 64), B((size_t)T * chain * 64), C((size_t)T * 256), D((size_t)T * 256);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    auto frand = [&](int emin, int emax) {  // random sign-positive float, random exponent, full mantissa
        const uint64_t r = rnd();
        const int e = emin + (int)(r % (uint64_t)(emax - emin + 1));
        const uint32_t bits = (uint32_t)((e + 127) << 23) | (uint32_t)((r >> 20) & 0x7fffff);
        float f;
        __builtin_memcpy(&f, &bits, 4);
        return f;
    };
    for (int t = 0; t < T; t++) {
        const int mode = t % 4;  // 0: stencil-like, 1: wide exponents, 2: cancellation, 3: mixed signs
        for (size_t i = 0; i < (size_t)chain * 64; i++) {
            float a, b;
            if (mode == 0) {
                a = frand(-12, -1);
                b = (float)(rnd() % 256);
            } else if (mode == 1) {
                a = frand(-20, 10);
                b = frand(-20, 10);
            } else if (mode == 2) {
                a = frand(-2, 2) * ((rnd() & 1) ? 1.f : -1.f);
                b = frand(8, 12);
            } else {
                a = frand(-6, 6) * ((rnd() & 1) ? 1.f : -1.f);
                b = frand(-6, 6) * ((rnd() & 1) ? 1.f : -1.f);
            }
            A[(size_t)t * chain * 64 + i] = a;
            B[(size_t)t * chain * 64 + i] = b;
        }
        for (int i = 0; i < 256; i++) C[(size_t)t * 256 + i] = mode == 0 ? frand(-4, 7) : frand(-10, 12) * ((rnd() & 1) ? 1.f : -1.f);
    }
    float *dA, *dB, *dC, *dD;
    hipMalloc(&dA, A.size() * 4);
    hipMalloc(&dB, B.size() * 4);
    hipMalloc(&dC, C.size() * 4);
    hipMalloc(&dD, D.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, chain);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 1;
    }
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    FILE *f = fopen(argc > 1 ? argv[1] : "mfma_f32_probe.bin", "wb");
    const int hdr[2] = {T, chain};
    fwrite(hdr, 4, 2, f);
    fwrite(A.data(), 4, A.size(), f);
    fwrite(B.data(), 4, B.size(), f);
    fwrite(C.data(), 4, C.size(), f);
    fwrite(D.data(), 4, D.size(), f);
    fclose(f);
    printf("wrote %d trials\n", T);
    return 0;
}
