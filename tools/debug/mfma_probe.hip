// Probe of gfx950 MFMA operand layouts and f16 accumulation numerics (stencil redesign
// prototype).  Prints which lane->element hypotheses reproduce A*B.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// hyp 0: lane l holds k = 16*(l>>4) + j   (j = 0..15)
// hyp 1: k = 8*(l>>4) + j for j<8, 32 + 8*(l>>4) + (j-8) for j>=8
__device__ int kmap_i8_16(int l, int j, int hyp) {
    if (hyp == 0) return 16 * (l >> 4) + j;
    return j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8);
}

__global__ void k_i8_16x16x64(const int8_t *A, const int8_t *B, int32_t *D, int hyp) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; j++) {
        const int k = kmap_i8_16(l, j, hyp);
        a[j] = A[(l & 15) * 64 + k];   // A[m][k], 16 x 64
        b[j] = B[k * 16 + (l & 15)];   // B[k][n], 64 x 16
    }
    i32x4 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    i32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];  // row = 4g + r, col = l & 15
}

__device__ int kmap_i8_32(int l, int j, int hyp) {
    if (hyp == 0) return 16 * (l >> 5) + j;
    return j < 8 ? 8 * (l >> 5) + j : 16 + 8 * (l >> 5) + (j - 8);
}

__global__ void k_i8_32x32x32(const int8_t *A, const int8_t *B, int32_t *D, int hyp) {
    const int l = threadIdx.x;
    int8_t a[16], b[16];
    for (int j = 0; j < 16; j++) {
        const int k = kmap_i8_32(l, j, hyp);
        a[j] = A[(l & 31) * 32 + k];
        b[j] = B[k * 32 + (l & 31)];
    }
    i32x4 av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 16; r++) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

// f16 16x16x32: lane l holds A[l&15][8*(l>>4)+j]
__global__ void k_f16(const _Float16 *A, const _Float16 *B, const float *C, float *D) {
    const int l = threadIdx.x;
    f16x8 a, b;
    for (int j = 0; j < 8; j++) {
        const int k = 8 * (l >> 4) + j;
        a[j] = A[(l & 15) * 32 + k];
        b[j] = B[k * 16 + (l & 15)];
    }
    f32x4 c;
    for (int r = 0; r < 4; r++) c[r] = C[(4 * (l >> 4) + r) * 16 + (l & 15)];
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

template <typename T, typename F>
static void run_int(const char *name, int M, int N, int K, F launch, int nhyp) {
    std::vector<int8_t> A(M * K), B(K * N);
    uint32_t s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (int8_t)((s >> 24) - 128); };
    for (auto &v : A) v = rnd();
    for (auto &v : B) v = rnd();
    std::vector<int32_t> ref(M * N, 0);
    for (int m = 0; m < M; m++)
        for (int n = 0; n < N; n++) {
            int acc = 0;
            for (int k = 0; k < K; k++) acc += A[m * K + k] * B[k * N + n];
            ref[m * N + n] = acc;
        }
    int8_t *dA, *dB;
    int32_t *dD;
    hipMalloc(&dA, A.size());
    hipMalloc(&dB, B.size());
    hipMalloc(&dD, M * N * 4);
    hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
    for (int h = 0; h < nhyp; h++) {
        hipMemset(dD, 0, M * N * 4);
        launch(dA, dB, dD, h);
        std::vector<int32_t> got(M * N);
        hipMemcpy(got.data(), dD, M * N * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < M * N; i++) bad += got[i] != ref[i];
        printf("%s hyp %d: %d / %d mismatches\n", name, h, bad, M * N);
    }
    hipFree(dA);
    hipFree(dB);
    hipFree(dD);
}

int main() {
    run_int<int8_t>("i8_16x16x64", 16, 16, 64, [](int8_t *a, int8_t *b, int32_t *d, int h) {
        hipLaunchKernelGGL(k_i8_16x16x64, dim3(1), dim3(64), 0, 0, a, b, d, h); hipDeviceSynchronize(); }, 2);
    run_int<int8_t>("i8_32x32x32", 32, 32, 32, [](int8_t *a, int8_t *b, int32_t *d, int h) {
        hipLaunchKernelGGL(k_i8_32x32x32, dim3(1), dim3(64), 0, 0, a, b, d, h); hipDeviceSynchronize(); }, 2);
    // f16 numerics: D[0][n] = C + sum_k A[0][k] B[k][n]
    const int M = 16, N = 16, K = 32;
    std::vector<_Float16> A(M * K, (_Float16)0), B(K * N, (_Float16)0);
    std::vector<float> C(M * N, 0.f);
    // case columns:
    // n=0: products 2048*2048 (=2^22), 0.25*0.5 (=0.125), -2048*2048  -> exact 0.125, chained f32 0
    // n=1: C = 2^22, products 0.125, -2^22 (C first)                   -> exact 0.125
    // n=2: products 0.125 at k=31 after +-2^22 at k=0,1                -> order test
    // n=3: 32 products of 1/3-ish values: compare with f32 chain and exact
    // n=4: products 2^22 at k=0, 0.125 at k=8 (next group of 8), -2^22 at k=16
    // n=5: C = 0.125, products 2^22, -2^22
    auto setA = [&](int k, float v) { A[0 * K + k] = (_Float16)v; };
    for (int k = 0; k < K; k++) setA(k, 1.0f);
    auto setB = [&](int k, int n, float v) { B[k * N + n] = (_Float16)v; };
    // A[0][k] = 1 except where noted; use B to carry values (f16 exact values)
    setA(0, 2048.f); setB(0, 0, 2048.f); setA(1, 0.25f); setB(1, 0, 0.5f); setA(2, -2048.f); setB(2, 0, 2048.f);
    C[1] = 4194304.f; setB(1, 1, 0.125f); setA(2, -2048.f); setB(2, 1, 2048.f);
    setB(0, 2, 2048.f); setB(2, 2, 2048.f); setB(31, 2, 0.125f);  // k=0: 2048*2048, k=2: -2048*2048 (A[0][2]=-2048)
    setB(0, 4, 2048.f); setB(8, 4, 0.125f); setA(16, -2048.f); setB(16, 4, 2048.f);
    C[5] = 0.125f; setB(0, 5, 2048.f); setB(2, 5, 2048.f);
    uint32_t s = 777;
    for (int k = 0; k < K; k++) {
        s = s * 1664525u + 1013904223u;
        setB(k, 3, (float)((s >> 20) & 1023) / 7.0f);
    }
    _Float16 *dA, *dB;
    float *dC, *dD;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, C.size() * 4);
    hipMalloc(&dD, C.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_f16, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    std::vector<float> D(M * N);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    for (int n = 0; n < 6; n++) {
        double ex = C[n];
        float ch = C[n];
        for (int k = 0; k < K; k++) {
            ex += (double)(float)A[k] * (double)(float)B[k * N + n];
            ch = fmaf((float)A[k], (float)B[k * N + n], ch);
        }
        printf("f16 col %d: mfma %.9g  exact %.9g  f32-fma-chain %.9g\n", n, D[n], ex, ch);
    }
    // random accuracy: many columns of random values in [0,255] x weights ~ gaussian
    return 0;
}
