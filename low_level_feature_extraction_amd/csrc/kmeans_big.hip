// cv2.kmeans(float32(unique_colors), K, None, (EPS+MAX_ITER, 200, 0.2), 10,
// KMEANS_PP_CENTERS) for K = min(n_colors, U) in (5, LLFE_MAX_COLORS]
// (app/services/analyze/color_extractor.py:180-197, extract_colors(n_colors=...) :203).
//
// The /analyze endpoint always asks for 5 colours (analyze.py:101), which the cube-table
// kernel (kmeans.hip) serves; this kernel is the general-K path of the drop-in.  It
// restates the same OpenCV semantics (kmeans.hip header) on the plain sorted key list,
// with the centres in LDS and every per-centre loop bounded by the runtime K:
//  * k-means++ (generateCentersPP): D(p) = min over the chosen centres, exact integers;
//    per 256-point step sums of D / of the trial sums T_j = min(D, d(., t_j)) go to
//    four scratch slots, the selection prefix(D) >= p walks the step sums and resolves
//    inside one step;
//  * Lloyd: labels by the first minimum of the float32 normL2Sqr; the points of a wave
//    step that share a label are reduced together (sorted keys: a 64-point row holds a
//    few labels), so the per-wave accumulators see one LDS update per (row, label);
//    empty clusters take the farthest point of the biggest cluster;
//  * compactness: sum of normL2Sqr to the final centres with the last labels.
// One 512-thread workgroup per (image, attempt), in the LPT order of k_kmeans_order.
#include "kmeans_common.h"

namespace llfe {
namespace {

using namespace km;

constexpr int BT = 512;      // threads per (image, attempt)
constexpr int BW = BT / 64;  // waves
constexpr int BSTEP = 256;   // points per wave step (64 lanes x 4)

struct BigSmem {
    float c[kMaxColors][3];      // Lloyd centres (labelling)
    float cprev[kMaxColors][3];  // centres of the last labelling
    int icc[kMaxColors][3];      // k-means++ chosen centres
    long long sums[kMaxColors][3];
    int counts[kMaxColors];
    unsigned long long wacc[BW][kMaxColors][2];  // per wave: x | y << 32, z | n << 32
    unsigned long long wtot[BW][3];
    unsigned long long scan_w[BW];
    int found_step[3];
    unsigned long long found_excl[3];
    int ci[3];
    double dred[BW];
    double maxd[BW];
    int maxi[BW];
    int moved_idx[kMaxColors];
    int moved_lbl[kMaxColors];
    int n_moved;
    int flag;
};

__device__ __forceinline__ float fkey(uint32_t k, int c) { return (float)((k >> (16 - 8 * c)) & 255u); }

// D(p) = min over the first kk chosen centres, for the lane's 4 points
__device__ __forceinline__ void dmin4(const BigSmem &sm, const uint32_t (&kq)[4], int kk, uint32_t (&D)[4]) {
#pragma unroll
    for (int q = 0; q < 4; q++) D[q] = 0xFFFFFFFFu;
    for (int m = 0; m < kk; m++) {
        const int cx = sm.icc[m][0], cy = sm.icc[m][1], cz = sm.icc[m][2];
#pragma unroll
        for (int q = 0; q < 4; q++)
            D[q] = min(D[q], (uint32_t)d2i(key_r(kq[q]), key_g(kq[q]), key_b(kq[q]), cx, cy, cz));
    }
}

// first-minimum label of the lane's 4 points over K centres (float normL2Sqr)
__device__ __forceinline__ void label4(const float (*c)[3], int K, const uint32_t (&kq)[4], int (&l)[4]) {
    float best[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        best[q] = __builtin_inff();
        l[q] = 0;
    }
    for (int k = 0; k < K; k++) {
        const float cx = c[k][0], cy = c[k][1], cz = c[k][2];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float d = d2f(fkey(kq[q], 0), fkey(kq[q], 1), fkey(kq[q], 2), cx, cy, cz);
            const bool lt = d < best[q];
            best[q] = lt ? d : best[q];
            l[q] = lt ? k : l[q];
        }
    }
}

__device__ __forceinline__ int moved_label(const BigSmem &sm, int i, int l) {
    for (int m = 0; m < sm.n_moved; m++)
        if (sm.moved_idx[m] == i) l = sm.moved_lbl[m];
    return l;
}

__global__ __launch_bounds__(BT) void k_kmeans_big(const uint32_t *__restrict__ keys, long long key_stride,
                                                   const long long *__restrict__ n_unique, int n_colors,
                                                   unsigned long long seed, ImgIndex index,
                                                   const int *__restrict__ order, uint32_t *__restrict__ scratch,
                                                   long long scratch_stride, KmeansAttemptOut *__restrict__ out) {
    __shared__ BigSmem sm;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int img = order[blockIdx.x / kAttempts];
    const int att = blockIdx.x % kAttempts;
    const int N = (int)n_unique[img];
    const int K = min(n_colors, N);
    KmeansAttemptOut *o = out + (size_t)img * kAttempts + att;
    if (K <= 1) {  // (k_kmeans_finalize returns the unique colours)
        if (tid == 0) {
            o->compactness = 0.0;
            o->iters = 0;
        }
        return;
    }
    const uint32_t *pts = keys + (size_t)img * key_stride;
    const int M = (N + BSTEP - 1) / BSTEP;  // steps
    const int Mw = (M + BW - 1) / BW;
    const int sb = min(M, wid * Mw), se = min(M, sb + Mw);
    uint32_t *ss = scratch + ((size_t)img * kAttempts + att) * (size_t)scratch_stride;
    auto slot = [&](int q) { return ss + (size_t)q * (size_t)M; };
    // the lane's 4 keys of step s (zeros past N) and how many are points
    auto load4 = [&](int s, uint32_t (&kq)[4]) {
        const int i0 = s * BSTEP + lane * 4;
        int cnt = 4;
        if (i0 + 4 <= N) {
            const uint4 v = *(const uint4 *)(pts + i0);
            kq[0] = v.x;
            kq[1] = v.y;
            kq[2] = v.z;
            kq[3] = v.w;
        } else {
            cnt = max(0, N - i0);
#pragma unroll
            for (int q = 0; q < 4; q++) kq[q] = q < cnt ? pts[i0 + q] : 0u;
        }
        return cnt;
    };
    uint64_t rng = attempt_rng(seed, index.at(img), att, K);

    // ------------------------------------------------ k-means++ (generateCentersPP)
    {
        const uint32_t k0 = pts[cvrng_next(rng) % (uint32_t)N];
        if (tid == 0) {
            sm.icc[0][0] = key_r(k0);
            sm.icc[0][1] = key_g(k0);
            sm.icc[0][2] = key_b(k0);
        }
    }
    __syncthreads();
    int cur = 0;
    unsigned long long sum0 = 0;
    {
        unsigned long long wt = 0;
        for (int s = sb; s < se; s++) {
            uint32_t kq[4], D[4];
            const int cnt = load4(s, kq);
            dmin4(sm, kq, 1, D);
            uint32_t ls = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) ls += q < cnt ? D[q] : 0u;
            const uint32_t st = wave_sum(ls);
            if (lane == 0) slot(0)[s] = st;
            wt += st;
        }
        if (lane == 0) sm.wtot[wid][0] = wt;
    }
    __syncthreads();
    for (int w = 0; w < BW; w++) sum0 += sm.wtot[w][0];
    __syncthreads();
    for (int kk = 1; kk < K; kk++) {
        double p[3];
#pragma unroll
        for (int j = 0; j < 3; j++) p[j] = cvrng_double(rng) * (double)sum0;
        // ---- the step holding prefix(D) >= p_j: thread-contiguous step ranges, block scan
        {
            const uint32_t *scur = slot(cur);
            const int q = (M + BT - 1) / BT;
            const int t0 = min(M, tid * q), t1 = min(M, t0 + q);
            unsigned long long R = 0;
            for (int s = t0; s < t1; s++) R += scur[s];
            unsigned long long x = R;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned long long y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            if (lane == 63) sm.scan_w[wid] = x;
            if (tid < 3) {
                sm.found_step[tid] = -1;
                sm.ci[tid] = -1;
            }
            __syncthreads();
            unsigned long long pre = 0;
            for (int w = 0; w < wid; w++) pre += sm.scan_w[w];
            const unsigned long long excl = pre + x - R;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                if (p[j] > 0 && (double)excl < p[j] && p[j] <= (double)(excl + R)) {
                    unsigned long long e = excl;
                    for (int s = t0; s < t1; s++) {
                        const unsigned long long v = scur[s];
                        if ((double)(e + v) >= p[j]) {
                            sm.found_step[j] = s;
                            sm.found_excl[j] = e;
                            break;
                        }
                        e += v;
                    }
                }
            }
            __syncthreads();
        }
        // ---- waves 0..2 resolve the point inside the found step
        if (wid < 3) {
            const int j = wid;
            const double pj = j == 0 ? p[0] : (j == 1 ? p[1] : p[2]);
            if (!(pj > 0)) {
                if (lane == 0) sm.ci[j] = 0;
            } else if (sm.found_step[j] < 0) {
                if (lane == 0) sm.ci[j] = N - 1;
            } else {
                const int s = sm.found_step[j];
                uint32_t kq[4], D[4];
                const int cnt = load4(s, kq);
                dmin4(sm, kq, kk, D);
                uint32_t lsum = 0;
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    D[qq] = qq < cnt ? D[qq] : 0u;
                    lsum += D[qq];
                }
                unsigned long long x = lsum;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const unsigned long long y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                unsigned long long e = sm.found_excl[j] + x - lsum;
                int hit = -1;
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    e += D[qq];
                    if (hit < 0 && qq < cnt && (double)e >= pj) hit = qq;
                }
                const unsigned long long bal = __ballot(hit >= 0);
                const int first = bal ? (int)__builtin_ctzll(bal) : 0;
                const int hitj = __shfl(hit, first);
                if (lane == 0) sm.ci[j] = bal ? min(s * BSTEP + first * 4 + hitj, N - 1) : N - 1;
            }
        }
        __syncthreads();
        int tx[3], ty[3], tz[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const uint32_t k = pts[sm.ci[j]];
            tx[j] = key_r(k);
            ty[j] = key_g(k);
            tz[j] = key_b(k);
        }
        // ---- trial pass: T_j = min(D, d(., t_j)), step sums into the three free slots
        const int sl0 = cur == 0 ? 1 : 0, sl1 = cur <= 1 ? 2 : 1, sl2 = cur <= 2 ? 3 : 2;
        unsigned long long wt0 = 0, wt1 = 0, wt2 = 0;
        for (int s = sb; s < se; s++) {
            uint32_t kq[4], D[4];
            const int cnt = load4(s, kq);
            dmin4(sm, kq, kk, D);
            uint32_t l0 = 0, l1 = 0, l2 = 0;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                if (qq >= cnt) break;
                const int r = key_r(kq[qq]), g = key_g(kq[qq]), b = key_b(kq[qq]);
                l0 += min(D[qq], (uint32_t)d2i(r, g, b, tx[0], ty[0], tz[0]));
                l1 += min(D[qq], (uint32_t)d2i(r, g, b, tx[1], ty[1], tz[1]));
                l2 += min(D[qq], (uint32_t)d2i(r, g, b, tx[2], ty[2], tz[2]));
            }
            const uint32_t a0 = wave_sum(l0), a1 = wave_sum(l1), a2 = wave_sum(l2);
            if (lane == 0) {
                slot(sl0)[s] = a0;
                slot(sl1)[s] = a1;
                slot(sl2)[s] = a2;
            }
            wt0 += a0;
            wt1 += a1;
            wt2 += a2;
        }
        if (lane == 0) {
            sm.wtot[wid][0] = wt0;
            sm.wtot[wid][1] = wt1;
            sm.wtot[wid][2] = wt2;
        }
        __syncthreads();
        unsigned long long S[3] = {0, 0, 0};
        for (int w = 0; w < BW; w++)
            for (int j = 0; j < 3; j++) S[j] += sm.wtot[w][j];
        int best = 0;
        for (int j = 1; j < 3; j++)
            if ((double)S[j] < (double)S[best]) best = j;  // first on ties
        sum0 = S[best];
        cur = best == 0 ? sl0 : (best == 1 ? sl1 : sl2);
        __syncthreads();
        if (tid == 0) {
            sm.icc[kk][0] = best == 0 ? tx[0] : (best == 1 ? tx[1] : tx[2]);
            sm.icc[kk][1] = best == 0 ? ty[0] : (best == 1 ? ty[1] : ty[2]);
            sm.icc[kk][2] = best == 0 ? tz[0] : (best == 1 ? tz[1] : tz[2]);
        }
        __syncthreads();
    }

    // ------------------------------------------------ Lloyd iterations
    if (tid < K * 3) {
        const int k = tid / 3, j = tid % 3;
        sm.c[k][j] = (float)sm.icc[k][j];
    }
    __syncthreads();
    int iter = 1;
    const double eps2 = 0.2 * 0.2;
    for (;;) {
        for (int q = tid; q < BW * kMaxColors * 2; q += BT) (&sm.wacc[0][0][0])[q] = 0;
        __syncthreads();
        for (int s = sb; s < se; s++) {
            uint32_t kq[4];
            int l[4];
            const int cnt = load4(s, kq);
            label4(sm.c, K, kq, l);
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const bool valid = qq < cnt;
                const unsigned long long a = (unsigned long long)key_r(kq[qq]) | ((unsigned long long)key_g(kq[qq]) << 32);
                const unsigned long long b = (unsigned long long)key_b(kq[qq]) | (1ull << 32);
                unsigned long long act = __ballot(valid);
                // the row's points that share a label are summed together (few labels per row)
                while (act) {
                    const int l0 = __builtin_amdgcn_readlane(l[qq], (int)__builtin_ctzll(act));
                    const bool mine = valid && l[qq] == l0;
                    act &= ~__ballot(mine);
                    const unsigned long long va = wave_sum(mine ? a : 0ull), vb = wave_sum(mine ? b : 0ull);
                    if (lane == 0) {
                        sm.wacc[wid][l0][0] += va;
                        sm.wacc[wid][l0][1] += vb;
                    }
                }
            }
        }
        __syncthreads();
        if (tid < K * 4) {
            const int k = tid >> 2, comp = tid & 3;
            unsigned long long acc = 0;
            for (int w = 0; w < BW; w++) {
                const unsigned long long v = sm.wacc[w][k][comp >> 1];
                acc += (comp & 1) ? (v >> 32) : (v & 0xFFFFFFFFull);
            }
            if (comp < 3) sm.sums[k][comp] = (long long)acc;
            else sm.counts[k] = (int)acc;
        } else if (tid >= 128 && tid < 128 + K * 3) {
            const int q = tid - 128, k = q / 3, j = q % 3;
            sm.cprev[k][j] = sm.c[k][j];
        } else if (tid == 256) {
            sm.n_moved = 0;
        }
        __syncthreads();

        // ---- empty clusters: move the farthest point of the biggest cluster (rare)
        for (int ek = 0; ek < K; ek++) {
            if (sm.counts[ek] != 0) continue;  // uniform
            int max_k = 0;
            for (int k1 = 1; k1 < K; k1++)
                if (sm.counts[max_k] < sm.counts[k1]) max_k = k1;
            const float scale = 1.f / (float)sm.counts[max_k];
            const float bx = (float)sm.sums[max_k][0] * scale, by = (float)sm.sums[max_k][1] * scale,
                        bz = (float)sm.sums[max_k][2] * scale;
            double md = -1.0;
            int mi = -1;
            for (int s = sb; s < se; s++) {
                uint32_t kq[4];
                int l[4];
                const int cnt = load4(s, kq);
                label4(sm.cprev, K, kq, l);
                for (int qq = 0; qq < cnt; qq++) {
                    const int i = s * BSTEP + lane * 4 + qq;
                    if (moved_label(sm, i, l[qq]) != max_k) continue;
                    const double d = (double)d2f(fkey(kq[qq], 0), fkey(kq[qq], 1), fkey(kq[qq], 2), bx, by, bz);
                    if (md <= d) {
                        md = d;
                        mi = i;
                    }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const double od = __shfl_xor(md, off);
                const int oi = __shfl_xor(mi, off);
                if (od > md || (od == md && oi > mi)) {
                    md = od;
                    mi = oi;
                }
            }
            if (lane == 0) {
                sm.maxd[wid] = md;
                sm.maxi[wid] = mi;
            }
            __syncthreads();
            if (tid == 0) {
                double bd2 = -1.0;
                int bi = -1;
                for (int w = 0; w < BW; w++)
                    if (sm.maxd[w] > bd2 || (sm.maxd[w] == bd2 && sm.maxi[w] > bi)) {
                        bd2 = sm.maxd[w];
                        bi = sm.maxi[w];
                    }
                if (bi >= 0) {
                    const uint32_t k = pts[bi];
                    sm.counts[max_k]--;
                    sm.counts[ek]++;
                    sm.sums[max_k][0] -= key_r(k);
                    sm.sums[max_k][1] -= key_g(k);
                    sm.sums[max_k][2] -= key_b(k);
                    sm.sums[ek][0] += key_r(k);
                    sm.sums[ek][1] += key_g(k);
                    sm.sums[ek][2] += key_b(k);
                    sm.moved_idx[sm.n_moved] = bi;
                    sm.moved_lbl[sm.n_moved] = ek;
                    sm.n_moved++;
                }
            }
            __syncthreads();
        }
        if (tid == 0) {
            double max_shift = 0.0;
            for (int k = 0; k < K; k++) {
                const float scale = 1.f / (float)sm.counts[k];
                double dist = 0.0;
                for (int j = 0; j < 3; j++) {
                    const float v = (float)sm.sums[k][j] * scale;
                    sm.c[k][j] = v;
                    const double t = (double)(v - sm.cprev[k][j]);
                    dist += t * t;
                }
                max_shift = fmax(max_shift, dist);
            }
            sm.flag = (iter + 1 == 100 || max_shift <= eps2) ? 1 : 0;
        }
        iter++;
        __syncthreads();
        if (sm.flag) break;
    }

    // ------------------------------------------------ compactness with the last labels
    double acc = 0.0;
    const bool moved = sm.n_moved > 0;
    for (int s = sb; s < se; s++) {
        uint32_t kq[4];
        int l[4];
        const int cnt = load4(s, kq);
        label4(sm.cprev, K, kq, l);
        for (int qq = 0; qq < cnt; qq++) {
            int lb = l[qq];
            if (moved) lb = moved_label(sm, s * BSTEP + lane * 4 + qq, lb);
            acc += (double)d2f(fkey(kq[qq], 0), fkey(kq[qq], 1), fkey(kq[qq], 2), sm.c[lb][0], sm.c[lb][1], sm.c[lb][2]);
        }
    }
    acc = wave_sum(acc);
    if (lane == 0) sm.dred[wid] = acc;
    __syncthreads();
    if (tid == 0) {
        double compactness = 0.0;
        for (int w = 0; w < BW; w++) compactness += sm.dred[w];
        o->compactness = compactness;
        o->iters = iter;
        o->bytes = 4ull * (unsigned long long)N * (unsigned long long)(K + iter);
        o->pp_pts = 0;
        o->pad = 0;
        o->n_cubes = 0;
        o->t_sel = 0;
        o->ll_pts = 0;
        o->t_sw = 0;
        o->drift_hist = 0;
        for (int k = 0; k < K; k++) {
            for (int j = 0; j < 3; j++) o->centers[k][j] = sm.c[k][j];
            o->counts[k] = sm.counts[k];
        }
    }
}

}  // namespace

hipError_t launch_kmeans_big(const uint32_t *keys, int64_t key_stride, const int64_t *n_unique, int n, int n_colors,
                             uint64_t seed, ImgIndex index, const int32_t *order, uint32_t *scratch,
                             int64_t scratch_stride, KmeansAttemptOut *attempts, hipStream_t s) {
    if (n_colors > kMaxColors) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_kmeans_big, dim3(n * kAttempts), dim3(BT), 0, s, keys, (long long)key_stride,
                       (const long long *)n_unique, n_colors, (unsigned long long)seed, index, order,
                       scratch, (long long)scratch_stride, attempts);
    return hipGetLastError();
}

}  // namespace llfe
