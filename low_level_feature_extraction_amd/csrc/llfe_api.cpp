// C ABI of libllfe.so (include/llfe.h): context, workspace and the batch pipeline
// that replaces the native work behind ColorExtractor.extract_colors,
// ShapeAnalyzer.analyze_shapes and ShadowAnalyzer.analyze_shadow_level.
//
// Per chunk of images (all on the caller's stream):
//   stencil (gray/blur5/Canny-NMS/adaptive mean)  -> class map + shadow sums
//   hysteresis as connected components (4 launches) fused with dilate + bit-pack
//   -> D2H (1 bit / pixel)
//   colour bitmap -> compaction -> k-means (10 attempts / image) -> D2H 64 B / image
//   host thread pool: external contours + shape geometry from the packed masks
#include <dlfcn.h>
#include <sched.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/llfe.h"
#include "contours.h"
#include "llfe_internal.h"

using namespace llfe;

namespace {

// ------------------------------------------------------------------ thread pool
class Pool {
  public:
    explicit Pool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this] { run(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    // run f(i) for i in [0, n) on the pool (+ calling thread), wait for all
    void parallel_for(int n, const std::function<void(int, int)> &f) {
        if (n <= 0) return;
        std::atomic<int> next{0};
        int done = 0;  // guarded by m_: the waiter checks it under the same lock, so a
                       // completion can never slip between its check and its sleep
        int workers = std::min((int)th_.size(), n);
        auto job = [&](int wid) {
            for (int i; (i = next.fetch_add(1)) < n;) f(i, wid);
        };
        {
            std::lock_guard<std::mutex> g(m_);
            for (int w = 0; w < workers; w++)
                q_.push_back([&, w] {
                    job(w + 1);
                    std::lock_guard<std::mutex> g2(m_);
                    done++;
                    cv_done_.notify_all();
                });
        }
        cv_.notify_all();
        job(0);
        std::unique_lock<std::mutex> lk(m_);
        cv_done_.wait(lk, [&] { return done == workers; });
    }

  private:
    void run() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                f = std::move(q_.back());
                q_.pop_back();
            }
            f();
        }
    }
    std::vector<std::thread> th_;
    std::vector<std::function<void()>> q_;
    std::mutex m_;
    std::condition_variable cv_, cv_done_;
    bool stop_ = false;
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count, bool zero = false) {
        if (count <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc((void **)&p, count * sizeof(T));
        if (e != hipSuccess) return e;
        n = count;
        if (zero) e = hipMemset(p, 0, count * sizeof(T));
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { release(); }
};

template <typename T>
struct HostBuf {
    T *p = nullptr;
    size_t n = 0;
    hipError_t ensure(size_t count) {
        if (count <= n) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipHostMalloc((void **)&p, count * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    ~HostBuf() { release(); }
};

// CV_32F Gaussian kernel of getGaussianKernel(n, sigma<=0): bit-exact softdouble
// construction (sigma = 0.15 n + 0.35, normalised, centre = 1/sum) cast to float.
void gauss_kernel_f32(int n, float *out) {
    double sigma = (double)n * 0.15 + 0.35;
    double scale2 = -0.125 / (sigma * sigma);
    int n2 = (n - 1) / 2;
    double vals[32], sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        vals[i] = std::exp((double)(x * x) * scale2);
        sum += vals[i];
    }
    sum = sum * 2.0 + 1.0;
    double mul = 1.0 / sum;
    for (int i = 0; i < n2; i++) out[i] = out[n - 1 - i] = (float)(vals[i] * mul);
    out[n2] = (float)(1.0 * mul);
}

// Pillow precompute_coeffs (LANCZOS, support 3) -> 22-bit fixed point
int pil_coeffs(int in_size, double in0, double in1, int out_size, std::vector<int32_t> &bounds,
               std::vector<int32_t> &kk) {
    double scale = (in1 - in0) / out_size;
    double filterscale = scale < 1.0 ? 1.0 : scale;
    double support = 3.0 * filterscale;
    int ksize = (int)std::ceil(support) * 2 + 1;
    bounds.assign((size_t)out_size * 2, 0);
    kk.assign((size_t)out_size * ksize, 0);
    std::vector<double> k(ksize);
    auto sinc = [](double x) {
        if (x == 0.0) return 1.0;
        x = x * M_PI;
        return std::sin(x) / x;
    };
    auto lanczos = [&](double x) { return (-3.0 <= x && x < 3.0) ? sinc(x) * sinc(x / 3) : 0.0; };
    for (int xx = 0; xx < out_size; xx++) {
        double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0, ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        int x = 0;
        for (; x < xmax; x++) {
            double wv = lanczos((x + xmin - center + 0.5) * ss);
            k[x] = wv;
            ww += wv;
        }
        for (x = 0; x < xmax; x++)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; x++) k[x] = 0;
        for (x = 0; x < ksize; x++) {
            double v = k[x] * (1 << 22);
            kk[(size_t)xx * ksize + x] = v < 0 ? (int32_t)(-0.5 + v) : (int32_t)(0.5 + v);
        }
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = xmax;
    }
    return ksize;
}

// batches in flight at once (llfe_submit_batch; LLFE_INFLIGHT picks 2 or 3)
constexpr int kMaxSlots = 3;

// device workspace of one chunk in flight
struct Work {
    DevBuf<uint8_t> d_in, d_cls, d_sroot, d_tflag;  // d_tflag: the stencil's hysteresis tile flags
    bool tflag_valid = false;  // d_tflag belongs to the class map in d_cls (stencil_params)
    DevBuf<int8_t> d_noise, d_nfield;  // d_nfield: the launch's noise field (unique.hip)
    DevBuf<uint64_t> d_bits, d_ebits;
    DevBuf<unsigned long long> d_shadow;
    DevBuf<int> d_order, d_parent, d_nroots, d_ftlist, d_ptlist;
    DevBuf<uint16_t> d_lab, d_roots;
    DevBuf<uint32_t> d_raw, d_keys, d_kscratch, d_pmeta, d_tstrong, d_segtab;  // d_segtab: k_uq_scatter's run table
    DevBuf<CubeEnt> d_segcubes, d_cubes;
    DevBuf<CellEnt> d_segcells, d_cells;
    DevBuf<SupEnt> d_sups;
    DevBuf<int32_t> d_ncubes, d_ncells, d_nsups;
    DevBuf<int64_t> d_nuniq;
    DevBuf<KmeansAttemptOut> d_att;
    int km_n = 0, km_colors = 0;  // images / n_colors of the last k-means launch (d_att)
    DevBuf<KmeansImageOut> d_kout;
    DevBuf<long long> d_index;  // per-image global indices of the chunk (llfe_batch.indices)
    // GPU contours (contours_gpu.hip); capacities grow when a pass overflows them
    DevBuf<uint64_t> d_ct_planes;
    DevBuf<CtComp> d_ct_comps;
    DevBuf<uint8_t> d_ct_acc;
    DevBuf<int2> d_ct_pts, d_ct_refs, d_ct_stage;
    DevBuf<CtCounters> d_ct_ctr;
    DevBuf<int> d_ct_info;
    DevBuf<llfe_shape> d_ct_shapes;
    CtCaps ct_min{0, 0, 0, 0};  // grown minimum capacities (0 = defaults)
};

// hipEvent pairs around launches (enabled by llfe_set_profiling)
struct Profiler {
    struct Rec {
        int kid, slot;
        hipEvent_t a, b;
        double bytes;
    };
    struct Stat {
        std::string name;
        int64_t launches = 0;
        double ms = 0, bytes = 0;
    };
    bool on = false;
    static constexpr int kStageSlot = -3;  // records of the stage entry points (caller's stream)
    int cur_slot = 0;  // slot of the work being enqueued (records are collected per slot)
    std::vector<hipEvent_t> all, free_;
    std::vector<Rec> pending;
    std::vector<Stat> stats;
    // debug (LLFE_TIMELINE=file): every collected record's start / end in ms after `base`,
    // an event recorded when profiling was switched on (tools/debug/pipe_timeline.py)
    hipEvent_t base = nullptr;
    FILE *tl = nullptr;
    hipEvent_t ev() {
        if (free_.empty()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            all.push_back(e);
            return e;
        }
        hipEvent_t e = free_.back();
        free_.pop_back();
        return e;
    }
    int kid(const char *name) {
        for (size_t i = 0; i < stats.size(); i++)
            if (stats[i].name == name) return (int)i;
        stats.push_back(Stat{name});
        return (int)stats.size() - 1;
    }
    hipEvent_t begin(hipStream_t s) {
        if (!on) return nullptr;
        hipEvent_t a = ev();
        if (a) (void)hipEventRecord(a, s);
        return a;
    }
    void end(hipEvent_t a, hipStream_t s, const char *name, double bytes) {
        if (!on || !a) return;
        hipEvent_t b = ev();
        if (!b) {
            free_.push_back(a);
            return;
        }
        (void)hipEventRecord(b, s);
        pending.push_back(Rec{kid(name), cur_slot, a, b, bytes});
    }
    // records of slot `slot` (-1: every slot, -2: every record) whose end event has
    // completed; a record still pending keeps its events (a recycled event still in
    // flight would time a later launch wrongly)
    void collect(int slot = -1) {
        size_t keep = 0;
        for (size_t i = 0; i < pending.size(); i++) {
            Rec &r = pending[i];
            const bool mine = slot == -2 || (slot == -1 ? r.slot >= 0 : r.slot == slot);
            if (!mine || hipEventQuery(r.b) != hipSuccess) {
                pending[keep++] = r;
                continue;
            }
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
                stats[r.kid].launches++;
                stats[r.kid].ms += ms;
                stats[r.kid].bytes += r.bytes;
                float t0 = 0.f;
                if (tl && base && hipEventElapsedTime(&t0, base, r.a) == hipSuccess)
                    fprintf(tl, "%s %d %.4f %.4f\n", stats[r.kid].name.c_str(), r.slot, t0, t0 + ms);
            }
            free_.push_back(r.a);
            free_.push_back(r.b);
        }
        pending.resize(keep);
        if (tl) fflush(tl);
    }
    // bytes known only after the launch completed (k-means sweeps)
    void add_bytes(const char *name, double bytes) {
        if (on) stats[kid(name)].bytes += bytes;
    }
    void reset() {
        for (auto &r : pending) {
            free_.push_back(r.a);
            free_.push_back(r.b);
        }
        pending.clear();
        stats.clear();
    }
    ~Profiler() {
        for (auto e : all) (void)hipEventDestroy(e);
        if (base) (void)hipEventDestroy(base);
        if (tl) fclose(tl);
    }
};

size_t shadow_tiles(int n, int h, int w) { return stencil_parts(n, h, w); }

// Images per device pass.  One pass per call when the workspace allows it: a bigger
// pass amortises the k-means launch's tail (its longest attempts run 100 Lloyd
// iterations) over more work (512 x 1080p per pass: +10 % images/s over 256).  The
// workspace is ~16 B per pixel + the 5 MB per-image partition cube and cell tables + the
// gathered cube / cell tables (<= 4 MiB + 1 MiB), held
// within LLFE_WORKSPACE_GB (default 24 GB of the 288 GB of HBM) PER IN-FLIGHT SLOT: every
// slot of llfe_set_inflight owns one such workspace, so depth 3 takes about 3x the budget.
int chunk_for(int h, int w) {
    double gb = 24.0;
    if (const char *e = getenv("LLFE_WORKSPACE_GB"); e && atof(e) > 0) gb = atof(e);
    const double P = (double)h * (double)w;
    const double cubes = std::min(P, (double)kMaxCubes), cells = std::min(cubes, (double)kParts * kCellsPerPart);
    const double per_image = 16.0 * P +  // keys, segments, class map, labels, masks
                             (double)kParts * (kCubesPerPart * sizeof(CubeEnt) + kCellsPerPart * sizeof(CellEnt)) +
                             cubes * sizeof(CubeEnt) + 2.0 * cells * sizeof(CellEnt);  // the gathered tables
    const double n = gb * 1e9 / per_image;
    return (int)std::max(1.0, std::min(n, (double)kMaxKmeansBatch));
}

// CPUs this process may run on: the affinity mask (sched_getaffinity), capped by a
// cgroup v2 cpu.max quota -- std::thread::hardware_concurrency() counts the whole node
int usable_cpus() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char quota[64] = {0};
        long long period = 0;
        if (fscanf(f, "%63s %lld", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0) {
            const long long q = atoll(quota) / period;
            if (q >= 1 && q < n) n = (int)q;
        }
        fclose(f);
    }
    return std::max(1, n);
}

// host cores per GPU process: the rank's own share when placement.bind() pinned it to its
// GPU's NUMA node (LLFE_RANK_CPUS), else the usable cores shared by the LOCAL_WORLD_SIZE
// ranks torchrun starts on the node
int cores_per_process() {
    if (const char *rc = getenv("LLFE_RANK_CPUS"); rc && atoi(rc) > 0) return atoi(rc);
    int local = 1;
    if (const char *lw = getenv("LOCAL_WORLD_SIZE"); lw && atoi(lw) > 0) local = atoi(lw);
    return std::max(1, usable_cpus() / local);
}

int default_threads() {
    const char *e = getenv("LLFE_HOST_THREADS");
    if (e && atoi(e) > 0) return atoi(e);
    return std::max(1, std::min(cores_per_process(), 16));
}

}  // namespace

struct llfe_ctx {
    int device = 0;
    std::string err;
    Pool *pool = nullptr;
    Profiler prof;
    double host_ct_ms = 0;       // llfe_host_contour_stats
    int64_t host_ct_images = 0;
    StencilParams sp{};
    // device workspace
    // per-slot device workspaces (up to kMaxSlots batches in flight: llfe_submit_batch)
    Work ws[kMaxSlots];
    hipStream_t streams[kMaxSlots] = {};
    hipStream_t col_streams[kMaxSlots] = {};  // colour path of workspace q
    hipEvent_t start_ev = nullptr, stream_done[kMaxSlots] = {};
    // asynchronous submissions (llfe_submit_batch / llfe_collect_batch): slot = ticket % inflight_max
    int inflight_max = 2;
    struct Pending {
        bool busy = false, done = false;
        llfe_batch b{};
        uint32_t features = 0;
        std::vector<llfe_image_result> res;
        std::vector<llfe_shape> shp;
        std::vector<int64_t> idx;  // llfe_submit_images: the images' global indices (b.indices)
    };
    Pending inflight[kMaxSlots];
    bool any_inflight() const {
        for (const Pending &p : inflight)
            if (p.busy) return true;
        return false;
    }
    int64_t next_ticket = 0, next_collect = 0;
    DevBuf<uint8_t> d_rsz_tmp, d_rsz_src;
    DevBuf<uint8_t> d_ragged;       // llfe_process_images: one size group's packed images
    DevBuf<int8_t> d_ragged_noise;
    DevBuf<int32_t> d_coef;
    DevBuf<uint8_t> d_text;                  // llfe_text_binary: gray, then its upscale
    DevBuf<unsigned long long> d_text_hist;  // 256 bins + threshold + count of 255s
    // pinned host staging; the per-chunk results are double-buffered so the host can
    // trace chunk c's contours while the GPU runs chunk c + 1
    HostBuf<uint64_t> h_bits_s[kMaxSlots];
    // GPU contours: per-image (components, ref base, contours, kept, shape base),
    // counters and shape records of each slot
    // contours on the GPU (contours_gpu.hip) or on the host pool from the D2H'd mask
    // (default: the host pool runs them while the GPU is in k-means, which measured
    // faster on one MI355X; LLFE_CONTOURS=gpu or llfe_set_contour_mode switch)
    bool gpu_contours = false;
    bool slot_gpu_ct[kMaxSlots] = {};  // mode each in-flight slot was enqueued with
    HostBuf<int> h_ct_info_s[kMaxSlots];
    HostBuf<CtCounters> h_ct_ctr_s[kMaxSlots];
    HostBuf<llfe_shape> h_ct_shapes_s[kMaxSlots];
    int64_t h_ct_shape_cap[kMaxSlots] = {};
    HostBuf<unsigned long long> h_shadow_s[kMaxSlots];
    HostBuf<KmeansImageOut> h_kout_s[kMaxSlots];
    hipEvent_t chunk_done[kMaxSlots] = {};
    hipEvent_t input_ready = nullptr, colour_done = nullptr;  // intra-chunk stream split
    bool concurrent = true;           // llfe_set_concurrency
    hipEvent_t mask_done[kMaxSlots] = {};  // shapes/shadows results are on the host
    // host-input copies of successive chunks / batches are chained (h2d_done of the last
    // one): with two batches in flight, batch k + 1's H2D then starts after batch k's
    // instead of splitting PCIe with it, so batch k's kernels start at half the latency
    hipEvent_t h2d_done = nullptr;
    bool h2d_pending = false;
    // the mask / shadow D2H runs on its own stream so the colour stage starts right after
    // the hysteresis kernels; mask_ready[slot] orders it after them, and a workspace is
    // not overwritten before the D2H that last read it (w_mask_slot) has finished
    hipStream_t copy_stream = nullptr;
    hipEvent_t mask_ready[kMaxSlots] = {};
    int w_mask_slot[kMaxSlots] = {-1, -1, -1};
    HostBuf<KmeansImageOut> h_kout;
    // llfe_submit_images: per slot, the gather table (n source addresses, n row pitches)
    HostBuf<uint64_t> h_gather_s[kMaxSlots];
    DevBuf<uint64_t> d_gather_s[kMaxSlots];
    Work *km_last = nullptr;  // workspace of the last k-means launch (llfe_kmeans_attempts)
    // per-thread host scratch
    std::vector<std::vector<int8_t>> work;
    std::vector<Contours> cont;
    std::vector<ShapeScratch> shs;
    std::vector<std::vector<llfe_shape>> img_shapes;
    std::vector<int32_t> img_ncont;
    int64_t host_fallbacks = 0;  // GPU-contour chunks traced on the host instead
    // llfe_set_contour_mode(LLFE_CONTOURS_GPU_FORCE_FALLBACK): every GPU-traced chunk is
    // redone on the host path (diagnostic: exercises the fallback)
    bool force_ct_fallback = false;

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
};

#define HIPCHK(ctx, expr)                                                                                   \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess) return (ctx)->fail(LLFE_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                                 __FILE__, __LINE__);                                       \
    } while (0)

// launch `expr` bracketed by profiler events (name, algorithmic HBM bytes)
#define TIMED(ctx, s, name, bytes, expr)                  \
    do {                                                  \
        hipEvent_t ev_a_ = (ctx)->prof.begin(s);          \
        HIPCHK(ctx, expr);                                \
        (ctx)->prof.end(ev_a_, s, name, (double)(bytes)); \
    } while (0)

namespace {

// The stage entry points run on workspace 0, slot 0's host buffers and the caller's
// stream: refused while submitted batches (one of which may own workspace 0) are not
// collected.  Their profiler records carry the stage tag, so llfe_collect_batch never
// takes them for a slot's.
int stage_enter(llfe_ctx *ctx, const char *fn) {
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "%s with submitted batches not yet collected", fn);
    ctx->prof.cur_slot = Profiler::kStageSlot;
    return LLFE_OK;
}

int stage_input(llfe_ctx *ctx, Work &W, const llfe_batch *b, int i0, int n, const uint8_t **d_img, const int8_t **d_noise,
                hipStream_t s) {
    size_t P3 = (size_t)b->height * b->width * 3;
    const bool h2d = !b->on_device || (b->noise && !b->noise_on_device);
    if (h2d && ctx->h2d_pending) HIPCHK(ctx, hipStreamWaitEvent(s, ctx->h2d_done, 0));
    if (b->on_device) {
        *d_img = b->data + (size_t)i0 * P3;
    } else {
        HIPCHK(ctx, W.d_in.ensure(P3 * n));
        HIPCHK(ctx, hipMemcpyAsync(W.d_in.p, b->data + (size_t)i0 * P3, P3 * n, hipMemcpyHostToDevice, s));
        *d_img = W.d_in.p;
    }
    *d_noise = nullptr;
    if (b->noise) {
        if (b->noise_on_device) {
            *d_noise = b->noise + (size_t)i0 * P3;
        } else {
            HIPCHK(ctx, W.d_noise.ensure(P3 * n));
            HIPCHK(ctx, hipMemcpyAsync(W.d_noise.p, b->noise + (size_t)i0 * P3, P3 * n, hipMemcpyHostToDevice, s));
            *d_noise = W.d_noise.p;
        }
    }
    if (h2d) {
        HIPCHK(ctx, hipEventRecord(ctx->h2d_done, s));
        ctx->h2d_pending = true;
    }
    return LLFE_OK;
}

// The hysteresis workspace of an n x h x w batch, grown on demand.
int hyst_work(llfe_ctx *ctx, Work &W, int n, int h, int w, HystWork *out) {
    const size_t ids = hysteresis_ids(n, h, w);
    const size_t tiles = (size_t)tiles_x(w) * tiles_y(h) * n;
    HIPCHK(ctx, W.d_lab.ensure((size_t)n * h * w));
    HIPCHK(ctx, W.d_parent.ensure(ids));
    HIPCHK(ctx, W.d_sroot.ensure(ids));
    HIPCHK(ctx, W.d_roots.ensure(ids));
    HIPCHK(ctx, W.d_nroots.ensure(tiles));
    HIPCHK(ctx, W.d_tstrong.ensure(hysteresis_tiles(n, h, w) * hysteresis_tile_words()));
    HIPCHK(ctx, W.d_ebits.ensure((size_t)n * h * words_per_row(w)));
    HIPCHK(ctx, W.d_ftlist.ensure(tiles + 2));
    HIPCHK(ctx, W.d_ptlist.ensure(tiles + 1));
    *out = HystWork{W.d_lab.p,     W.d_parent.p, W.d_sroot.p,       W.d_roots.p,   W.d_nroots.p,
                    W.d_tstrong.p, W.d_ebits.p,
                    W.tflag_valid ? W.d_tflag.p : nullptr, W.d_ftlist.p + 2, W.d_ftlist.p,
                    W.d_ptlist.p};
    W.tflag_valid = false;  // (one hysteresis pass per stencil launch)
    return LLFE_OK;
}

// The stencil parameters of a class-map launch into W.d_cls: the hysteresis tile flags
// (zeroed here, on s) that let the hysteresis skip the tiles without a Canny candidate.
int stencil_params(llfe_ctx *ctx, Work &W, int n, int h, int w, hipStream_t s, StencilParams *sp) {
    *sp = ctx->sp;
    W.tflag_valid = false;
    // LLFE_HYST_TILE_FLAGS=0: no flags, the hysteresis visits every tile (its test path)
    if (const char *e = getenv("LLFE_HYST_TILE_FLAGS"))
        if (!strcmp(e, "0")) return LLFE_OK;
    const size_t tiles = (size_t)n * tiles_x(w) * ((h + 63) / 64);
    HIPCHK(ctx, W.d_tflag.ensure(tiles));
    HIPCHK(ctx, hipMemsetAsync(W.d_tflag.p, 0, tiles, s));
    sp->tflag = W.d_tflag.p;
    W.tflag_valid = true;
    return LLFE_OK;
}

// Canny hysteresis (connected components) + dilate + pack of W.d_cls.
int run_hysteresis_dilate(llfe_ctx *ctx, Work &W, int n, int h, int w, uint64_t *bits, uint8_t *mask_u8, hipStream_t s) {
    HystWork wk;
    const int rc = hyst_work(ctx, W, n, h, w, &wk);
    if (rc) return rc;
    // algorithmic bytes (which folds hysteresis into the fused 4P stencil
    // front): what any implementation of this stage must move -- the class map read (P) and
    // the bit-packed dilated mask written (P/8).  The CC labels and tile bitmaps it also
    // reads and writes are the implementation's (PMC saw ~2.4 P per image, round 4).
    TIMED(ctx, s, "k_hysteresis_dilate", (double)n * h * w * (1 + 0.125),
          launch_hysteresis_dilate(W.d_cls.p, n, h, w, wk, bits, mask_u8, s));
    return LLFE_OK;
}

// External contours + shape records of W.d_bits on the GPU (hysteresis workspace reused)
int run_contours(llfe_ctx *ctx, Work &W, int n, int h, int w, const uint64_t *bits, hipStream_t s) {
    CtCaps c = contours_default_caps(n, h, w);
    c.comps = std::max(c.comps, W.ct_min.comps);
    c.pts = std::max(c.pts, W.ct_min.pts);
    c.refs = std::max(c.refs, W.ct_min.refs);
    c.shapes = std::max(c.shapes, W.ct_min.shapes);
    const size_t ids = hysteresis_ids(n, h, w);
    HIPCHK(ctx, W.d_lab.ensure((size_t)n * h * w));
    HIPCHK(ctx, W.d_parent.ensure(ids));
    HIPCHK(ctx, W.d_roots.ensure(ids));
    HIPCHK(ctx, W.d_nroots.ensure((size_t)tiles_x(w) * tiles_y(h) * n));
    HIPCHK(ctx, W.d_ct_planes.ensure(5 * contours_plane_words(n, h, w)));
    HIPCHK(ctx, W.d_ct_comps.ensure(c.comps));
    HIPCHK(ctx, W.d_ct_acc.ensure(c.comps));
    HIPCHK(ctx, W.d_ct_pts.ensure(c.pts));
    HIPCHK(ctx, W.d_ct_refs.ensure(c.refs));
    HIPCHK(ctx, W.d_ct_stage.ensure((size_t)kCtTraceBlocks * kCtStage));
    HIPCHK(ctx, W.d_ct_ctr.ensure(1));
    HIPCHK(ctx, W.d_ct_info.ensure((size_t)n * kCtInfo));
    HIPCHK(ctx, W.d_ct_shapes.ensure(c.shapes));
    CtWork wk{W.d_lab.p, W.d_parent.p, W.d_roots.p, W.d_nroots.p, W.d_ct_planes.p, W.d_ct_comps.p, W.d_ct_acc.p,
              W.d_ct_pts.p, W.d_ct_refs.p, W.d_ct_stage.p, W.d_ct_ctr.p, W.d_ct_info.p, W.d_ct_shapes.p, c};
    // algorithmic bytes: mask bits read by components + scan, labels written and read
    TIMED(ctx, s, "k_contours", (double)n * h * w * (0.25 + 4.0), launch_contours(bits, n, h, w, wk, s));
    return LLFE_OK;
}

// enqueue the D2H of a contour pass's results into host slot `slot` on stream cs
int copy_contours(llfe_ctx *ctx, Work &W, int n, int slot, hipStream_t cs) {
    HIPCHK(ctx, ctx->h_ct_info_s[slot].ensure((size_t)n * kCtInfo));
    HIPCHK(ctx, ctx->h_ct_ctr_s[slot].ensure(1));
    HIPCHK(ctx, ctx->h_ct_shapes_s[slot].ensure(W.d_ct_shapes.n));
    ctx->h_ct_shape_cap[slot] = (int64_t)W.d_ct_shapes.n;
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_ct_info_s[slot].p, W.d_ct_info.p, sizeof(int) * n * kCtInfo,
                               hipMemcpyDeviceToHost, cs));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_ct_ctr_s[slot].p, W.d_ct_ctr.p, sizeof(CtCounters), hipMemcpyDeviceToHost, cs));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_ct_shapes_s[slot].p, W.d_ct_shapes.p, sizeof(llfe_shape) * W.d_ct_shapes.n,
                               hipMemcpyDeviceToHost, cs));
    return LLFE_OK;
}

// grow the contour capacities after an overflowing pass (counters hold what was asked)
void grow_contour_caps(Work &W, int n, int h, int w, const CtCounters &ct) {
    const CtCaps d = contours_default_caps(n, h, w);
    CtCaps &m = W.ct_min;
    auto up = [](int64_t cur, int64_t dflt, int64_t need) { return std::max({2 * std::max(cur, dflt), need + need / 4}); };
    if (ct.flags & kCtOverflowComps) m.comps = up(m.comps, d.comps, (int64_t)ct.comps + (int64_t)n * kCtQuirkCap);
    if (ct.flags & kCtOverflowPts) m.pts = up(m.pts, d.pts, (int64_t)ct.pts);
    if (ct.flags & (kCtOverflowRefs | kCtOverflowComps))
        m.refs = up(m.refs, d.refs, std::max<int64_t>(m.comps, d.comps) + (int64_t)n * kCtQuirkCap);
    if (ct.flags & kCtOverflowShapes) m.shapes = up(m.shapes, d.shapes, (int64_t)ct.shapes);
}

// contiguous_keys: also gather each image's unique keys into W.d_keys in np.unique order
// (llfe_color_unique's output, the general-K k-means); otherwise they stay where k_uq_part
// wrote them (W.d_raw, partition R at the prefix of the partition pixel counts) and the cube
// k-means reads them there (KmeansCubes::part_hist)
int color_stage(llfe_ctx *ctx, Work &W, const uint8_t *img, const uint64_t *img_tab, const int8_t *noise, int n, int h,
                int w, uint64_t seed, ImgIndex index, bool contiguous_keys, hipStream_t s) {
    // unique colours -> W.d_keys (sorted, key_stride) + cube table for k-means
    const int64_t P = (int64_t)h * w;
    const int64_t key_stride = (std::max<int64_t>(P, 1) + 3) & ~int64_t(3);
    const int64_t cube_stride = std::min<int64_t>(key_stride, kMaxCubes);
    const int64_t cell_stride = std::min<int64_t>(cube_stride, (int64_t)kParts * kCellsPerPart);
    HIPCHK(ctx, W.d_raw.ensure((size_t)n * key_stride));
    HIPCHK(ctx, W.d_keys.ensure((size_t)n * key_stride));
    HIPCHK(ctx, W.d_segcubes.ensure((size_t)n * kParts * kCubesPerPart));
    HIPCHK(ctx, W.d_cubes.ensure((size_t)n * cube_stride));
    HIPCHK(ctx, W.d_segcells.ensure((size_t)n * kParts * kCellsPerPart));
    HIPCHK(ctx, W.d_cells.ensure((size_t)n * cell_stride));
    HIPCHK(ctx, W.d_ncells.ensure(n));
    HIPCHK(ctx, W.d_sups.ensure((size_t)n * cell_stride));
    HIPCHK(ctx, W.d_nsups.ensure(n));
    HIPCHK(ctx, W.d_pmeta.ensure((size_t)n * kParts * 5));
    HIPCHK(ctx, W.d_nuniq.ensure(n));
    HIPCHK(ctx, W.d_ncubes.ensure(n));
    // (d_pmeta: hist, cl, uq, cc, cs; k-means reads uq)
    uint32_t *hist = W.d_pmeta.p, *cl = hist + (size_t)n * kParts, *uq = hist + (size_t)2 * n * kParts,
             *cc = uq + (size_t)n * kParts, *cs = cc + (size_t)n * kParts;
    HIPCHK(ctx, hipMemsetAsync(hist, 0, sizeof(uint32_t) * n * kParts, s));
    HIPCHK(ctx, W.d_segtab.ensure((size_t)n * uq_tab_words(P)));
    if (!noise) {
        HIPCHK(ctx, W.d_nfield.ensure((size_t)noise_field_pixels(P)));
        HIPCHK(ctx, launch_uq_noise(noise, W.d_nfield.p, P, seed, s));
    }
    // Algorithmic bytes (colour pass 3P + 4 MiB + 8U per image): the scatter
    // is charged the input read (3P, + 3P of parity noise when given), k_uq_part the 2^24-bit
    // presence bitmap's clear + scan (4 MiB; held in LDS here) and the unique-key write (4U),
    // k_uq_gather the key read (4U); the step segments written and read back between the
    // scatter and k_uq_part (4P each way) are the implementation's, not counted.
    // keys -> per-step segments sorted by partition + run table + partition totals
    TIMED(ctx, s, "k_uq_scatter", (double)n * P * (noise ? 6 : 3),
          launch_uq_scatter(img, img_tab, noise, W.d_nfield.p, n, h, w, seed, index, key_stride, hist, W.d_segtab.p,
                            W.d_keys.p, s));
    // the partitions' sorted unique keys go to the (free) d_raw
    TIMED(ctx, s, "k_uq_part", (double)n * 4194304.0,
          launch_uq_part(W.d_keys.p, n, key_stride, P, hist, W.d_segtab.p, W.d_raw.p, W.d_segcubes.p,
                         W.d_segcells.p, uq, cc, cl, cs, s));
    TIMED(ctx, s, "k_uq_gather", 0,
          launch_uq_gather(W.d_raw.p, n, key_stride, hist, uq, cc, cl, cs, W.d_segcubes.p, W.d_segcells.p,
                           W.d_keys.p, W.d_cubes.p, W.d_cells.p, W.d_sups.p, cube_stride, cell_stride,
                           cell_stride, W.d_nuniq.p, W.d_ncubes.p, W.d_ncells.p, W.d_nsups.p, contiguous_keys, s));
    return LLFE_OK;
}

int kmeans_stage(llfe_ctx *ctx, Work &W, const uint32_t *keys, int64_t key_stride, const int64_t *d_nuniq, int n,
                 int n_colors, uint64_t seed, ImgIndex index, const KmeansCubes &cubes, hipStream_t s) {
    if (n_colors < 1 || n_colors > kMaxColors)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "n_colors must be in [1, LLFE_MAX_COLORS]");
    const int64_t sstride = kmeans_scratch_stride(key_stride);
    HIPCHK(ctx, W.d_order.ensure((size_t)n + 2));  // LPT order + the two work-queue counters
    HIPCHK(ctx, W.d_kscratch.ensure((size_t)n * kAttempts * sstride));
    HIPCHK(ctx, W.d_att.ensure((size_t)n * kAttempts));
    HIPCHK(ctx, W.d_kout.ensure(n));
    W.km_n = n;
    W.km_colors = n_colors;
    ctx->km_last = &W;
    // per-image cv::RNG state = splitmix64(seed + global index) is derived on the device
    TIMED(ctx, s, "k_kmeans", 0,
          launch_kmeans(keys, key_stride, d_nuniq, n, n_colors, seed, index, W.d_order.p, W.d_kscratch.p,
                        sstride, W.d_att.p, W.d_kout.p, cubes, s));
    if (const char *path = getenv("LLFE_KM_TRACE")) {  // debug: per-attempt timeline + U
        std::vector<KmeansAttemptOut> att((size_t)n * kAttempts);
        std::vector<int64_t> nu(n);
        HIPCHK(ctx, hipMemcpyAsync(att.data(), W.d_att.p, sizeof(KmeansAttemptOut) * att.size(),
                                   hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipMemcpyAsync(nu.data(), d_nuniq, sizeof(int64_t) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipStreamSynchronize(s));
        if (FILE *f = fopen(path, "a")) {
            for (int i = 0; i < n; i++)
                for (int a = 0; a < kAttempts; a++) {
                    const KmeansAttemptOut &o = att[(size_t)i * kAttempts + a];
                    fprintf(f, "%d %d %lld %d %llu %llu %u %u %llu %llu %llu %u %u %d %llu %llu %llu 0 0 %llu %llu %u %u\n", i, a, (long long)nu[i], o.iters,
                            (unsigned long long)o.t_start, (unsigned long long)o.t_end, o.hw_id, o.xcc_id,
                            (unsigned long long)o.t_pp, (unsigned long long)o.t_lloyd, (unsigned long long)o.bytes, o.pp_pts, o.n_cubes, o.pad, (unsigned long long)o.t_sel,
                            (unsigned long long)o.ll_pts, (unsigned long long)o.t_sw, (unsigned long long)o.drift_hist,
                            (unsigned long long)o.t_lstart, o.hw_id2, o.xcc_id2);
                }
            fclose(f);
        }
    }
    return LLFE_OK;
}

// ColorExtractor.is_light_color (color_extractor.py:67-71), in the reference's order
bool is_light_color(int r, int g, int b) {
    const double R = r / 255.0, G = g / 255.0, B = b / 255.0;
    return 0.2126 * R + 0.7152 * G + 0.0722 * B > 0.6;
}

// extract_colors' palette rules (color_extractor.py:231-284) on r's centres and counts:
// frequency order (stable on ties; np.argsort(-counts)'s tie order is host-dependent in the
// reference), hex, '#ffffff' / '#000000' dropped, primary, three accents
// (padded with the last, or the primary), background by the primary's luminance
void fill_palette(llfe_image_result &r) {
    const int K = r.n_colors;
    int ord[kMaxColors];
    for (int i = 0; i < K; i++) ord[i] = i;
    if (K > 1) std::stable_sort(ord, ord + K, [&](int a, int b) { return r.counts[a] > r.counts[b]; });
    char hex[kMaxColors][8];
    int rgb[kMaxColors][3];
    int nh = 0;
    for (int i = 0; i < K; i++) {
        const uint8_t *c = r.centers_rgb[ord[i]];
        if ((c[0] == 255 && c[1] == 255 && c[2] == 255) || (c[0] == 0 && c[1] == 0 && c[2] == 0)) continue;
        std::snprintf(hex[nh], 8, "#%02x%02x%02x", c[0], c[1], c[2]);
        rgb[nh][0] = c[0], rgb[nh][1] = c[1], rgb[nh][2] = c[2];
        nh++;
    }
    if (nh == 0) {  // nothing left: the contrasting colour for white (:245-256)
        const char *bg = is_light_color(255, 255, 255) ? "#000000" : "#FFFFFF";
        std::snprintf(r.primary, 8, "%s", bg);
        std::snprintf(r.background, 8, "%s", bg);
        for (auto &a : r.accent) std::snprintf(a, 8, "%s", bg);
        return;
    }
    std::snprintf(r.primary, 8, "%s", hex[0]);
    int na = 0;
    for (int i = 1; i < nh && na < 3; i++)
        if (std::strcmp(hex[i], hex[0]) != 0) std::snprintf(r.accent[na++], 8, "%s", hex[i]);
    for (; na < 3; na++) std::snprintf(r.accent[na], 8, "%s", na ? r.accent[na - 1] : r.primary);
    std::snprintf(r.background, 8, "%s", is_light_color(rgb[0][0], rgb[0][1], rgb[0][2]) ? "#000000" : "#FFFFFF");
}

// ShadowAnalyzer.analyze_shadow_level's decision (shadow pyc @L22-31): 0 Low, 1 Moderate, 2 High
int32_t shadow_level(uint64_t sum, uint64_t count) {
    if (count == 0) return 0;
    const double avg_darkness = 255.0 - (double)sum / (double)count;
    return avg_darkness < 30 ? 0 : (avg_darkness < 60 ? 1 : 2);
}

void fill_color_result(const KmeansImageOut &k, llfe_image_result &r) {
    r.n_colors = k.k;
    for (int c = 0; c < kMaxColors; c++) {
        r.counts[c] = k.counts[c];
        for (int j = 0; j < 3; j++) r.centers_rgb[c][j] = k.centers_rgb[c][j];
    }
    r.n_unique = k.n_unique;
    r.compactness = k.compactness;
    fill_palette(r);
}

bool valid_dims(int n, int h, int w) { return n >= 0 && h > 0 && w > 0 && (int64_t)h * w < (1LL << 31); }

// global indices of images [i0, i0 + n) of a batch: index_base + i, or the caller's list
// (uploaded on stream s into the workspace)
int chunk_index(llfe_ctx *ctx, Work &W, const llfe_batch *b, int i0, int n, hipStream_t s, ImgIndex *out) {
    *out = ImgIndex{b->index_base + i0, nullptr};
    if (b->indices && n > 0) {
        HIPCHK(ctx, W.d_index.ensure((size_t)n));
        HIPCHK(ctx, hipMemcpyAsync(W.d_index.p, b->indices + i0, sizeof(long long) * n, hipMemcpyHostToDevice, s));
        out->idx = W.d_index.p;
    }
    return LLFE_OK;
}

// Device half of one chunk, on slot `slot`'s stream and workspace: every kernel, then
// the D2H of the per-image results into host slot `slot`, with events the host half
// waits on.
// img_tab (device, llfe_submit_images): image i of the chunk at img_tab[i], read in place by
// the scatter and the stencil (b->data then only names the first image)
int enqueue_chunk(llfe_ctx *ctx, const llfe_batch *b, uint32_t features, uint64_t seed, int i0, int n, int slot,
                  int q, const uint64_t *img_tab = nullptr) {
    ctx->prof.cur_slot = slot;
    Work &W = ctx->ws[q];
    hipStream_t s = ctx->streams[q];
    const int h = b->height, w = b->width, wpr = words_per_row(w);
    const bool want_col = features & LLFE_FEATURE_COLORS, want_shp = features & LLFE_FEATURE_SHAPES,
               want_shd = features & LLFE_FEATURE_SHADOWS;
    const int64_t P = (int64_t)h * w;
    const int64_t key_stride = (std::max<int64_t>(P, 1) + 3) & ~int64_t(3);
    const int n_colors = b->n_colors ? b->n_colors : kMaxK;
    const uint8_t *img;
    const int8_t *noise;
    int rc = stage_input(ctx, W, b, i0, n, &img, &noise, s);
    if (rc) return rc;
    ImgIndex index;
    rc = chunk_index(ctx, W, b, i0, n, s, &index);
    if (rc) return rc;
    // the colour path (unique colours + k-means) runs on the second stream, concurrently
    // with shapes / shadows (both only read the input).  Measured (512 x 1080p): shapes
    // alongside the colour front 13.1k images/s; shapes held back to share the GPU with
    // k-means 12.8k -- the stencil waves slow the k-means attempts more than they fill
    // its tail.
    hipStream_t col_s = s;
    if (want_col && ctx->concurrent && (want_shp || want_shd)) {
        col_s = ctx->col_streams[q];
        HIPCHK(ctx, hipEventRecord(ctx->input_ready, s));
        HIPCHK(ctx, hipStreamWaitEvent(col_s, ctx->input_ready, 0));
    }
    // colour front (unique colours), then shapes / shadows (on the other stream), then
    // k-means
    if (want_col) {
        rc = color_stage(ctx, W, img, img_tab, noise, n, h, w, seed, index, /*contiguous_keys=*/n_colors > kMaxK, col_s);
        if (rc) return rc;
    }
    // d_shadow / d_bits of this workspace may still be in the previous chunk's D2H
    if (ctx->w_mask_slot[q] >= 0) HIPCHK(ctx, hipStreamWaitEvent(s, ctx->mask_done[ctx->w_mask_slot[q]], 0));
    if (want_shp || want_shd) {
        HIPCHK(ctx, W.d_shadow.ensure(2 * (size_t)n + shadow_tiles(n, h, w)));
        StencilParams sp = ctx->sp;
        if (want_shp) {
            HIPCHK(ctx, W.d_cls.ensure((size_t)n * P));
            rc = stencil_params(ctx, W, n, h, w, s, &sp);  // (starts from ctx->sp)
            if (rc) return rc;
        }
        // after stencil_params: the stencil reads an in-place batch through its table (with
        // the packed-batch addressing, image i >= 1 would lie past image 0's allocation)
        sp.img_tab = img_tab;
        TIMED(ctx, s, "k_stencil", (double)n * P * (3 + (want_shp ? 1 : 0)),
              launch_stencil(img, n, h, w, want_shp ? W.d_cls.p : nullptr, nullptr,
                             want_shd ? W.d_shadow.p : nullptr, want_shd ? W.d_shadow.p + n : nullptr,
                             (uint2 *)(W.d_shadow.p + 2 * n), sp, s));
    }
    // shapes + shadows go to the host (event mask_done) while the GPU is still in this
    // chunk's colour stage, so contour tracing overlaps k-means
    const bool gpu_ct = ctx->gpu_contours && w <= kCtMaxWidth && h <= kCtMaxHeight;
    ctx->slot_gpu_ct[slot] = gpu_ct;
    if (want_shp) {
        HIPCHK(ctx, W.d_bits.ensure((size_t)n * h * wpr));
        if (!gpu_ct) HIPCHK(ctx, ctx->h_bits_s[slot].ensure((size_t)n * h * wpr));
        rc = run_hysteresis_dilate(ctx, W, n, h, w, W.d_bits.p, nullptr, s);
        if (rc) return rc;
        if (gpu_ct) {
            rc = run_contours(ctx, W, n, h, w, W.d_bits.p, s);
            if (rc) return rc;
        }
    }
    if (want_shd) HIPCHK(ctx, ctx->h_shadow_s[slot].ensure(2 * (size_t)n));
    if (want_shp || want_shd) {
        hipStream_t cs = ctx->copy_stream;
        HIPCHK(ctx, hipEventRecord(ctx->mask_ready[slot], s));
        HIPCHK(ctx, hipStreamWaitEvent(cs, ctx->mask_ready[slot], 0));
        if (want_shp && gpu_ct) {
            rc = copy_contours(ctx, W, n, slot, cs);
            if (rc) return rc;
        } else if (want_shp) {
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_bits_s[slot].p, W.d_bits.p, sizeof(uint64_t) * n * h * wpr,
                                       hipMemcpyDeviceToHost, cs));
        }
        if (want_shd)
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_shadow_s[slot].p, W.d_shadow.p, sizeof(unsigned long long) * 2 * n,
                                       hipMemcpyDeviceToHost, cs));
        HIPCHK(ctx, hipEventRecord(ctx->mask_done[slot], cs));
        ctx->w_mask_slot[q] = slot;
    } else {
        HIPCHK(ctx, hipEventRecord(ctx->mask_done[slot], s));
    }
    if (want_col) {
        // (n_colors <= 5: the keys in k_uq_part's segmented layout, W.d_raw)
        const bool seg = n_colors <= kMaxK;
        const KmeansCubes cubes{W.d_cubes.p, std::min<int64_t>(key_stride, kMaxCubes), W.d_ncubes.p,
                                W.d_pmeta.p + (size_t)2 * n * kParts, W.d_cells.p, W.d_ncells.p,
                                std::min<int64_t>(std::min<int64_t>(key_stride, kMaxCubes), (int64_t)kParts * kCellsPerPart),
                                seg ? W.d_pmeta.p : nullptr, W.d_sups.p, W.d_nsups.p,
                                std::min<int64_t>(std::min<int64_t>(key_stride, kMaxCubes), (int64_t)kParts * kCellsPerPart)};
        rc = kmeans_stage(ctx, W, seg ? W.d_raw.p : W.d_keys.p, key_stride, W.d_nuniq.p, n, n_colors, seed, index,
                          cubes, col_s);
        if (rc) return rc;
        HIPCHK(ctx, ctx->h_kout_s[slot].ensure(n));
        HIPCHK(ctx, hipMemcpyAsync(ctx->h_kout_s[slot].p, W.d_kout.p, sizeof(KmeansImageOut) * n,
                                   hipMemcpyDeviceToHost, col_s));
        if (col_s != s) {  // the chunk (and the next chunk's use of this workspace) ends after both
            HIPCHK(ctx, hipEventRecord(ctx->colour_done, col_s));
            HIPCHK(ctx, hipStreamWaitEvent(s, ctx->colour_done, 0));
        }
    }
    HIPCHK(ctx, hipEventRecord(ctx->chunk_done[slot], s));
    return LLFE_OK;
}

// Shape records of n images from their bit-packed dilated masks (hb, host) on the
// context's thread pool: external contours + the analyze_shapes loop (contours.cpp).
void host_shapes_from_bits(llfe_ctx *ctx, const uint64_t *hb, int n, int h, int w, int i0,
                           llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity,
                           int64_t &total_shapes) {
    const int wpr = words_per_row(w);
    ctx->img_shapes.resize(n);
    ctx->img_ncont.assign(n, 0);
    const auto t0 = std::chrono::steady_clock::now();
    ctx->pool->parallel_for(n, [&](int i, int wid) {
        external_contours_bits(hb + (size_t)i * h * wpr, h, w, wpr, ctx->work[wid], ctx->cont[wid]);
        ctx->img_ncont[i] = shapes_from_contours(ctx->cont[wid], ctx->shs[wid], ctx->img_shapes[i]);
    });
    ctx->host_ct_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->host_ct_images += n;
    for (int i = 0; i < n; i++) {
        llfe_image_result &r = results[i0 + i];
        r.shape_offset = total_shapes;
        r.n_shapes = (int32_t)ctx->img_shapes[i].size();
        r.n_contours = ctx->img_ncont[i];
        for (size_t k = 0; k < ctx->img_shapes[i].size(); k++) {
            if (shapes && total_shapes + (int64_t)k < shape_capacity) shapes[total_shapes + k] = ctx->img_shapes[i][k];
        }
        total_shapes += r.n_shapes;
    }
}

// Recompute the dilated masks of a chunk synchronously on workspace 0 (the device is
// idle after the hipDeviceSynchronize) -- the input is still the caller's.
int redo_masks(llfe_ctx *ctx, const llfe_batch *b, int i0, int n, hipStream_t s) {
    HIPCHK(ctx, hipDeviceSynchronize());
    Work &W = ctx->ws[0];
    const int h = b->height, w = b->width;
    const uint8_t *img;
    const int8_t *noise;
    llfe_batch nb = *b;
    nb.noise = nullptr;
    int rc = stage_input(ctx, W, &nb, i0, n, &img, &noise, s);
    if (rc) return rc;
    HIPCHK(ctx, W.d_cls.ensure((size_t)n * h * w));
    HIPCHK(ctx, W.d_bits.ensure((size_t)n * h * words_per_row(w)));
    StencilParams sp;
    if ((rc = stencil_params(ctx, W, n, h, w, s, &sp))) return rc;
    HIPCHK(ctx, launch_stencil(img, n, h, w, W.d_cls.p, nullptr, nullptr, nullptr, nullptr, sp, s));
    return run_hysteresis_dilate(ctx, W, n, h, w, W.d_bits.p, nullptr, s);
}

// Shape records of a chunk whose contours ran on the GPU (slot's host copies).  A pass
// that overflowed a capacity is redone for this chunk alone, synchronously, with the
// capacities grown from what its counters asked for.  A mask the GPU tracer does not
// handle (a border-following anomaly, a contour wider than its LDS window, a deeper
// Douglas-Peucker stack than it holds) is traced on the host pool instead: the chunk's
// masks are recomputed, copied back and run through the bit-identical host path, so
// one unusual image never fails its batch.
int gpu_shapes_of_chunk(llfe_ctx *ctx, const llfe_batch *b, int i0, int n, int slot, llfe_image_result *results,
                        llfe_shape *shapes, int64_t shape_capacity, int64_t &total_shapes) {
    const int h = b->height, w = b->width;
    for (int attempt = 0;; attempt++) {
        const CtCounters ct = *ctx->h_ct_ctr_s[slot].p;
        if ((ct.flags & (kCtBadTrace | kCtTooWide | kCtDpOverflow)) || ctx->force_ct_fallback) {
            hipStream_t s = ctx->streams[0];
            int rc = redo_masks(ctx, b, i0, n, s);
            if (rc) return rc;
            const size_t words = (size_t)n * h * words_per_row(w);
            HIPCHK(ctx, ctx->h_bits_s[slot].ensure(words));
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_bits_s[slot].p, ctx->ws[0].d_bits.p, sizeof(uint64_t) * words,
                                       hipMemcpyDeviceToHost, s));
            HIPCHK(ctx, hipStreamSynchronize(s));
            host_shapes_from_bits(ctx, ctx->h_bits_s[slot].p, n, h, w, i0, results, shapes, shape_capacity,
                                  total_shapes);
            ctx->host_fallbacks++;
            return LLFE_OK;
        }
        if (!(ct.flags & kCtOverflowMask)) break;
        if (attempt >= 8) return ctx->fail(LLFE_ERR_CAPACITY, "GPU contours: capacities still overflow (0x%x)", ct.flags);
        // redo the shapes path of this chunk on workspace 0 once the device is idle
        hipStream_t s = ctx->streams[0];
        int rc = redo_masks(ctx, b, i0, n, s);
        if (rc) return rc;
        Work &W = ctx->ws[0];
        grow_contour_caps(W, n, h, w, ct);
        rc = run_contours(ctx, W, n, h, w, W.d_bits.p, s);
        if (rc) return rc;
        rc = copy_contours(ctx, W, n, slot, s);
        if (rc) return rc;
        HIPCHK(ctx, hipStreamSynchronize(s));
    }
    const int *info = ctx->h_ct_info_s[slot].p;
    const llfe_shape *src = ctx->h_ct_shapes_s[slot].p;
    ctx->img_shapes.resize(n);
    ctx->img_ncont.assign(n, 0);
    for (int i = 0; i < n; i++) {
        llfe_image_result &r = results[i0 + i];
        const int nk = info[i * kCtInfo + 3], sb = info[i * kCtInfo + 4];
        r.shape_offset = total_shapes;
        r.n_shapes = nk;
        r.n_contours = info[i * kCtInfo + 2];
        ctx->img_ncont[i] = r.n_contours;
        ctx->img_shapes[i].assign(src + sb, src + sb + nk);
        if (shapes) {
            const int64_t room = std::max<int64_t>(0, std::min<int64_t>(nk, shape_capacity - total_shapes));
            if (room > 0) std::memcpy(shapes + total_shapes, src + sb, sizeof(llfe_shape) * (size_t)room);
        }
        total_shapes += nk;
    }
    return LLFE_OK;
}

// Host half of one chunk: wait for its slot, fill the result records, trace contours.
int finish_chunk(llfe_ctx *ctx, const llfe_batch *b, uint32_t features, int i0, int n, int slot,
                 llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity, int64_t &total_shapes) {
    const int h = b->height, w = b->width, wpr = words_per_row(w);
    const bool want_col = features & LLFE_FEATURE_COLORS, want_shp = features & LLFE_FEATURE_SHAPES,
               want_shd = features & LLFE_FEATURE_SHADOWS;
    // shapes + shadows are ready first (the GPU may still be in this chunk's colours)
    HIPCHK(ctx, hipEventSynchronize(ctx->mask_done[slot]));
    const unsigned long long *sh = ctx->h_shadow_s[slot].p;
    for (int i = 0; i < n; i++) {
        llfe_image_result &r = results[i0 + i];
        std::memset(&r, 0, sizeof r);
        r.shadow_level = -1;
        if (want_shd) {
            r.shadow_sum = sh[i];
            r.shadow_count = sh[n + i];
            r.shadow_level = shadow_level(r.shadow_sum, r.shadow_count);
        }
    }
    if (want_shp && ctx->slot_gpu_ct[slot]) {
        int rc = gpu_shapes_of_chunk(ctx, b, i0, n, slot, results, shapes, shape_capacity, total_shapes);
        if (rc) return rc;
    } else if (want_shp) {
        host_shapes_from_bits(ctx, ctx->h_bits_s[slot].p, n, h, w, i0, results, shapes, shape_capacity, total_shapes);
    }
    HIPCHK(ctx, hipEventSynchronize(ctx->chunk_done[slot]));
    if (want_col) {
        const KmeansImageOut *ko = ctx->h_kout_s[slot].p;
        for (int i = 0; i < n; i++) fill_color_result(ko[i], results[i0 + i]);
        if (ctx->prof.on) {
            double kb = 0, ub = 0;
            for (int i = 0; i < n; i++) {
                kb += (double)ko[i].bytes;
                ub += 4.0 * (double)ko[i].n_unique;
            }
            ctx->prof.add_bytes("k_kmeans", kb);
            // the unique keys: written once (k_uq_part, 4U of SURVEY.md 8d's 8U) and read
            // once -- by k_uq_gather when it makes them contiguous (n_colors > 5), else by
            // k-means itself where k_uq_part wrote them (its passes' 4U bytes)
            ctx->prof.add_bytes("k_uq_part", ub);
            if ((b->n_colors ? b->n_colors : kMaxK) > kMaxK) ctx->prof.add_bytes("k_uq_gather", ub);
        }
    }
    return LLFE_OK;
}

}  // namespace

extern "C" {

int llfe_abi_version(void) { return LLFE_ABI_VERSION; }

int llfe_default_host_threads(void) { return default_threads(); }

// path of the HIP runtime this library's HIP calls resolved to (dladdr of hipMalloc):
// a process must hold exactly one, shared with whatever produced its device pointers
// and stream handles (e.g. PyTorch-ROCm's torch/lib/libamdhip64.so)
const char *llfe_hip_runtime(void) {
    static std::string path;
    if (path.empty()) {
        Dl_info info{};
        hipError_t (*fn)(void **, size_t) = &hipMalloc;
        if (dladdr((void *)fn, &info) && info.dli_fname) path = info.dli_fname;
        else path = "?";
    }
    return path.c_str();
}

int llfe_init(int device, llfe_ctx **out) {
    if (!out) return LLFE_ERR_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return LLFE_ERR_HIP;
    if (device < 0 || device >= count) return LLFE_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return LLFE_ERR_HIP;
    llfe_ctx *c = new llfe_ctx();
    c->device = device;
    std::vector<hipEvent_t *> evs = {&c->start_ev, &c->input_ready, &c->colour_done, &c->h2d_done};
    // all streams at the default priority: a higher priority for the shapes streams or
    // for the colour streams measured neutral
    std::vector<hipStream_t *> sts = {&c->copy_stream};
    for (int q = 0; q < kMaxSlots; q++) {
        for (hipEvent_t *e : {&c->chunk_done[q], &c->mask_done[q], &c->stream_done[q], &c->mask_ready[q]})
            evs.push_back(e);
        sts.push_back(&c->streams[q]);
        sts.push_back(&c->col_streams[q]);
    }
    for (hipEvent_t *e : evs)
        if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
            llfe_destroy(c);
            return LLFE_ERR_HIP;
        }
    for (hipStream_t *st : sts)
        if (hipStreamCreateWithFlags(st, hipStreamNonBlocking) != hipSuccess) {
            llfe_destroy(c);
            return LLFE_ERR_HIP;
        }
    if (const char *fl = getenv("LLFE_INFLIGHT")) c->inflight_max = std::min(kMaxSlots, std::max(2, atoi(fl)));
    // contours on the host pool unless the process has too few host cores for them: a
    // "ui" 1080p image costs 0.28-0.36 ms of one core (round 3, llfe_host_contour_stats), so
    // 4 cores trace a 512-image 50 % ui step in ~23 ms, inside the ~28 ms GPU step (4 ranks on
    // 4 cores each: 19.3k images/s host vs 17.7k GPU contours, profiles/r3/multi/); below 4
    // the GPU path.  LLFE_CONTOURS=host / gpu overrides.
    c->gpu_contours = cores_per_process() < 4;
    if (const char *cm = getenv("LLFE_CONTOURS")) {
        if (!strcmp(cm, "gpu")) c->gpu_contours = true;
        if (!strcmp(cm, "host")) c->gpu_contours = false;
    }
    gauss_kernel_f32(11, c->sp.k11);
    {
        static const float kG11[11] = {LLFE_GAUSS11_F32};
        if (std::memcmp(kG11, c->sp.k11, sizeof(kG11)) != 0) {  // (an invariant of this build)
            std::fprintf(stderr, "llfe: getGaussianKernel(11) differs from the stencil's constants\n");
            llfe_destroy(c);
            return LLFE_ERR_UNSUPPORTED;
        }
    }
    c->pool = new Pool(default_threads() - 1);
    int nt = c->pool->size() + 1;
    c->work.resize(nt);
    c->cont.resize(nt);
    c->shs.resize(nt);
    *out = c;
    return LLFE_OK;
}

int llfe_destroy(llfe_ctx *ctx) {
    if (!ctx) return LLFE_OK;
    (void)hipSetDevice(ctx->device);
    std::vector<hipEvent_t> evs = {ctx->start_ev, ctx->input_ready, ctx->colour_done, ctx->h2d_done};
    std::vector<hipStream_t> sts = {ctx->copy_stream};
    for (int q = 0; q < kMaxSlots; q++) {
        for (hipEvent_t e : {ctx->chunk_done[q], ctx->mask_done[q], ctx->stream_done[q], ctx->mask_ready[q]})
            evs.push_back(e);
        sts.push_back(ctx->streams[q]);
        sts.push_back(ctx->col_streams[q]);
    }
    for (hipStream_t st : sts)
        if (st) (void)hipStreamSynchronize(st);
    for (hipEvent_t e : evs)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t st : sts)
        if (st) (void)hipStreamDestroy(st);
    delete ctx->pool;
    delete ctx;  // DevBuf / HostBuf members free themselves
    return LLFE_OK;
}

const char *llfe_last_error(llfe_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int llfe_set_profiling(llfe_ctx *ctx, int enable) {
    if (!ctx) return LLFE_ERR_INVALID;
    if (enable) ctx->prof.reset();
    ctx->prof.on = enable != 0;
    if (enable) {
        if (const char *path = getenv("LLFE_TIMELINE")) {  // debug: absolute kernel intervals
            HIPCHK(ctx, hipSetDevice(ctx->device));
            if (!ctx->prof.base) HIPCHK(ctx, hipEventCreate(&ctx->prof.base));
            HIPCHK(ctx, hipEventRecord(ctx->prof.base, nullptr));
            HIPCHK(ctx, hipEventSynchronize(ctx->prof.base));
            if (!ctx->prof.tl) ctx->prof.tl = fopen(path, "a");
            if (ctx->prof.tl) fprintf(ctx->prof.tl, "# base\n");
        }
    }
    return LLFE_OK;
}

int llfe_set_contour_mode(llfe_ctx *ctx, int mode) {
    if (!ctx || (mode != LLFE_CONTOURS_HOST && mode != LLFE_CONTOURS_GPU && mode != LLFE_CONTOURS_GPU_FORCE_FALLBACK))
        return LLFE_ERR_INVALID;
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "llfe_set_contour_mode with submitted batches not yet collected");
    ctx->gpu_contours = mode != LLFE_CONTOURS_HOST;
    ctx->force_ct_fallback = mode == LLFE_CONTOURS_GPU_FORCE_FALLBACK;
    return LLFE_OK;
}

int llfe_get_contour_mode(llfe_ctx *ctx) {
    if (!ctx) return LLFE_ERR_INVALID;
    if (!ctx->gpu_contours) return LLFE_CONTOURS_HOST;
    return ctx->force_ct_fallback ? LLFE_CONTOURS_GPU_FORCE_FALLBACK : LLFE_CONTOURS_GPU;
}

int llfe_set_inflight(llfe_ctx *ctx, int32_t depth) {
    if (!ctx || depth < 2 || depth > kMaxSlots) return LLFE_ERR_INVALID;
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "llfe_set_inflight with submitted batches not yet collected");
    ctx->inflight_max = depth;
    return LLFE_OK;
}

int llfe_get_inflight(llfe_ctx *ctx) { return ctx ? ctx->inflight_max : LLFE_ERR_INVALID; }

int llfe_set_concurrency(llfe_ctx *ctx, int enable) {
    if (!ctx) return LLFE_ERR_INVALID;
    ctx->concurrent = enable != 0;
    return LLFE_OK;
}

int llfe_kernel_stats(llfe_ctx *ctx, llfe_kernel_stat *out, int32_t cap) {
    if (!ctx) return LLFE_ERR_INVALID;
    ctx->prof.collect(-2);  // every completed launch (stage entry points never wait on a slot)
    int n = (int)ctx->prof.stats.size();
    for (int i = 0; i < n && i < cap && out; i++) {
        const auto &st = ctx->prof.stats[i];
        std::memset(&out[i], 0, sizeof(llfe_kernel_stat));
        std::snprintf(out[i].name, sizeof(out[i].name), "%s", st.name.c_str());
        out[i].launches = st.launches;
        out[i].total_ms = st.ms;
        out[i].bytes = st.bytes;
    }
    return n;
}

int llfe_host_contour_stats(llfe_ctx *ctx, double *busy_ms, int64_t *images, int32_t *threads, int32_t reset) {
    if (!ctx) return LLFE_ERR_INVALID;
    if (busy_ms) *busy_ms = ctx->host_ct_ms;
    if (images) *images = ctx->host_ct_images;
    if (threads) *threads = ctx->pool ? ctx->pool->size() : 0;
    if (reset) {
        ctx->host_ct_ms = 0;
        ctx->host_ct_images = 0;
    }
    return LLFE_OK;
}

int llfe_process_batch(llfe_ctx *ctx, const llfe_batch *b, uint32_t features, uint64_t seed,
                       llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity,
                       int64_t *shapes_needed, llfe_stream stream) {
    if (!ctx || !b || !results) return LLFE_ERR_INVALID;
    if (!valid_dims(b->n, b->height, b->width) || (b->n > 0 && !b->data))
        return ctx->fail(LLFE_ERR_INVALID, "invalid batch n=%d h=%d w=%d", b->n, b->height, b->width);
    if (b->n_colors < 0 || b->n_colors > kMaxColors)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "n_colors=%d outside [1, %d]", b->n_colors, kMaxColors);
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "llfe_process_batch with submitted batches not yet collected");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    const bool want_shp = features & LLFE_FEATURE_SHAPES;
    int64_t total_shapes = 0;
    // two-slot software pipeline: enqueue chunk c on stream c & 1 (kernels + D2H into
    // slot c & 1), then finish chunk c - 1 on the host (contours, result records) while
    // the GPU runs c -- and the tail of c - 1's k-means shares the GPU with c.  Both
    // streams first wait for the caller's stream (inputs produced there).
    HIPCHK(ctx, hipEventRecord(ctx->start_ev, s));
    for (hipStream_t st : ctx->streams) HIPCHK(ctx, hipStreamWaitEvent(st, ctx->start_ev, 0));
    int prev_i0 = -1, prev_n = 0, slot = 0;
    const int chunk = chunk_for(b->height, b->width);
    for (int i0 = 0; i0 < b->n; i0 += chunk) {
        const int n = std::min(chunk, b->n - i0);
        int rc = enqueue_chunk(ctx, b, features, seed, i0, n, slot, 0);
        if (rc) return rc;
        if (prev_i0 >= 0) {
            rc = finish_chunk(ctx, b, features, prev_i0, prev_n, slot ^ 1, results, shapes, shape_capacity, total_shapes);
            if (rc) return rc;
        }
        prev_i0 = i0;
        prev_n = n;
        slot ^= 1;
    }
    if (prev_i0 >= 0) {
        int rc = finish_chunk(ctx, b, features, prev_i0, prev_n, slot ^ 1, results, shapes, shape_capacity, total_shapes);
        if (rc) return rc;
    }
    // (every chunk has been waited for; the caller's stream gets the same order)
    for (int q = 0; q < 2; q++) {
        HIPCHK(ctx, hipEventRecord(ctx->stream_done[q], ctx->streams[q]));
        HIPCHK(ctx, hipStreamWaitEvent(s, ctx->stream_done[q], 0));
    }
    ctx->prof.collect();
    if (shapes_needed) *shapes_needed = total_shapes;
    if (want_shp && total_shapes > shape_capacity)
        return ctx->fail(LLFE_ERR_CAPACITY, "shape capacity %lld < %lld", (long long)shape_capacity,
                         (long long)total_shapes);
    return LLFE_OK;
}

// Ragged batch: images grouped by (preprocessed) size in input order; each group is
// packed into a device buffer (2-D copies absorb row strides and host / device sources;
// images the preprocessing rule resizes go through cv2.resize on the GPU) and runs as
// ordinary batches that carry every image's own global index.
int llfe_process_images(llfe_ctx *ctx, const llfe_image_desc *images, int32_t n, uint32_t features,
                        int32_t preprocessing, int32_t n_colors, uint64_t seed, int64_t index_base,
                        llfe_image_result *results, llfe_shape *shapes, int64_t shape_capacity,
                        int64_t *shapes_needed, llfe_stream stream) {
    if (!ctx || n < 0 || (n > 0 && (!images || !results))) return LLFE_ERR_INVALID;
    if (preprocessing < LLFE_PRE_NONE || preprocessing > LLFE_PRE_PERFORMANCE)
        return ctx->fail(LLFE_ERR_INVALID, "preprocessing mode %d", preprocessing);
    if (n_colors < 0 || n_colors > kMaxColors)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "n_colors=%d outside [1, %d]", n_colors, kMaxColors);
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "llfe_process_images with submitted batches not yet collected");
    struct Item {
        int oh, ow, interp;
        bool resize;
    };
    std::vector<Item> it((size_t)n);
    const bool with_noise = n > 0 && images[0].noise;
    for (int i = 0; i < n; i++) {
        const llfe_image_desc &d = images[i];
        if (!d.data || !valid_dims(1, d.height, d.width) ||
            (d.row_stride != 0 && d.row_stride < 3 * (int64_t)d.width))
            return ctx->fail(LLFE_ERR_INVALID, "image %d: invalid descriptor (%d x %d, stride %lld)", i, d.height,
                             d.width, (long long)d.row_stride);
        if ((d.noise != nullptr) != with_noise)
            return ctx->fail(LLFE_ERR_INVALID, "parity noise must be given for every image or for none");
        Item &q = it[i];
        int ow = d.width, oh = d.height, interp = 0;
        const int r = llfe_preprocess_size(d.width, d.height, preprocessing, &ow, &oh, &interp);
        if (r < 0) return ctx->fail(LLFE_ERR_INVALID, "image %d: preprocessing size", i);
        q = Item{r ? oh : d.height, r ? ow : d.width, interp, r == 1};
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    // size groups, in order of first appearance; members in input order
    std::vector<std::pair<std::pair<int, int>, std::vector<int>>> groups;
    {
        std::map<std::pair<int, int>, size_t> gi;
        for (int i = 0; i < n; i++) {
            const auto key = std::make_pair(it[i].oh, it[i].ow);
            auto f = gi.find(key);
            if (f == gi.end()) {
                gi[key] = groups.size();
                groups.push_back({key, {i}});
            } else {
                groups[f->second].second.push_back(i);
            }
        }
    }
    const bool want_shp = features & LLFE_FEATURE_SHAPES;
    int64_t total_shapes = 0;
    bool short_cap = false;
    std::vector<llfe_image_result> res;
    std::vector<int64_t> gidx;
    for (const auto &g : groups) {
        const int oh = g.first.first, ow = g.first.second;
        const int64_t P3 = (int64_t)oh * ow * 3;
        // staging passes of at most two device chunks (the batch path pipelines them)
        const int per = std::max(1, 2 * chunk_for(oh, ow));
        for (size_t a = 0; a < g.second.size(); a += per) {
            const int nb = (int)std::min<size_t>(per, g.second.size() - a);
            HIPCHK(ctx, ctx->d_ragged.ensure((size_t)nb * P3));
            if (with_noise) HIPCHK(ctx, ctx->d_ragged_noise.ensure((size_t)nb * P3));
            gidx.resize(nb);
            for (int j = 0; j < nb; j++) {
                const int i = g.second[a + j];
                const llfe_image_desc &d = images[i];
                gidx[j] = index_base + i;
                const size_t pitch = d.row_stride ? (size_t)d.row_stride : (size_t)d.width * 3;
                const hipMemcpyKind kind = d.on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
                uint8_t *dst = ctx->d_ragged.p + (size_t)j * P3;
                if (!it[i].resize) {
                    HIPCHK(ctx, hipMemcpy2DAsync(dst, (size_t)ow * 3, d.data, pitch, (size_t)d.width * 3, d.height,
                                                 kind, s));
                } else {
                    HIPCHK(ctx, ctx->d_rsz_src.ensure((size_t)d.height * d.width * 3));
                    HIPCHK(ctx, hipMemcpy2DAsync(ctx->d_rsz_src.p, (size_t)d.width * 3, d.data, pitch,
                                                 (size_t)d.width * 3, d.height, kind, s));
                    const int rc = llfe_resize_cv(ctx, ctx->d_rsz_src.p, d.height, d.width, 3, dst, oh, ow,
                                                  it[i].interp, stream);
                    if (rc) return rc;
                }
                if (with_noise)
                    HIPCHK(ctx, hipMemcpyAsync(ctx->d_ragged_noise.p + (size_t)j * P3, d.noise, (size_t)P3,
                                               d.noise_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
            }
            llfe_batch bb{};
            bb.data = ctx->d_ragged.p;
            bb.n = nb;
            bb.height = oh;
            bb.width = ow;
            bb.on_device = 1;
            bb.noise = with_noise ? ctx->d_ragged_noise.p : nullptr;
            bb.noise_on_device = 1;
            bb.n_colors = n_colors;
            bb.index_base = index_base;
            bb.indices = gidx.data();
            res.assign((size_t)nb, llfe_image_result{});
            const int64_t left = std::max<int64_t>(0, shape_capacity - total_shapes);
            int64_t need = 0;
            const int rc = llfe_process_batch(ctx, &bb, features, seed, res.data(),
                                              shapes && left > 0 ? shapes + total_shapes : nullptr, left, &need,
                                              stream);
            if (rc == LLFE_ERR_CAPACITY) {
                short_cap = true;  // results are valid; keep counting what is needed
            } else if (rc) {
                return rc;
            }
            for (int j = 0; j < nb; j++) {
                llfe_image_result r = res[j];
                r.shape_offset += total_shapes;
                results[g.second[a + j]] = r;
            }
            total_shapes += need;
        }
    }
    if (shapes_needed) *shapes_needed = total_shapes;
    if (want_shp && (short_cap || total_shapes > shape_capacity))
        return ctx->fail(LLFE_ERR_CAPACITY, "shape capacity %lld < %lld", (long long)shape_capacity,
                         (long long)total_shapes);
    return LLFE_OK;
}

// Asynchronous form of llfe_process_batch: up to two batches in flight, each on its own
// workspace and stream pair, so batch k + 1's unique-colour and stencil kernels start in
// the tail of batch k's k-means launch (where most CUs are idle) instead of after it.
int llfe_submit_batch(llfe_ctx *ctx, const llfe_batch *b, uint32_t features, uint64_t seed, llfe_stream stream,
                      int64_t *ticket) {
    if (!ctx || !b || !ticket) return LLFE_ERR_INVALID;
    if (!valid_dims(b->n, b->height, b->width) || (b->n > 0 && !b->data))
        return ctx->fail(LLFE_ERR_INVALID, "invalid batch n=%d h=%d w=%d", b->n, b->height, b->width);
    if (b->n_colors < 0 || b->n_colors > kMaxColors)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "n_colors=%d outside [1, %d]", b->n_colors, kMaxColors);
    if (b->n > chunk_for(b->height, b->width))
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_submit_batch: n=%d exceeds one device pass (%d)", b->n,
                         chunk_for(b->height, b->width));
    const int slot = (int)(ctx->next_ticket % ctx->inflight_max);
    auto &pd = ctx->inflight[slot];
    if (pd.busy) return ctx->fail(LLFE_ERR_CAPACITY, "%d batches already in flight: collect one first", ctx->inflight_max);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, hipEventRecord(ctx->start_ev, s));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->streams[slot], ctx->start_ev, 0));
    if (b->n > 0) {
        int rc = enqueue_chunk(ctx, b, features, seed, 0, b->n, slot, slot);
        if (rc) return rc;
    }
    pd.busy = true;
    pd.done = false;
    pd.b = *b;
    pd.features = features;
    *ticket = ctx->next_ticket++;
    return LLFE_OK;
}

int llfe_batch_capacity(int32_t h, int32_t w) {
    if (!valid_dims(1, h, w)) return LLFE_ERR_INVALID;
    return chunk_for(h, w);
}

// The request path's micro-batch (MicroBatcher): separately allocated images of one size
// gathered into the slot's input buffer on the slot's stream, then the same device work
// as llfe_submit_batch, every image under its own global index.
int llfe_submit_images(llfe_ctx *ctx, const llfe_image_desc *images, int32_t n, uint32_t features, int32_t n_colors,
                       uint64_t seed, const int64_t *indices, llfe_stream stream, int64_t *ticket) {
    if (!ctx || !ticket || n < 1 || !images || !indices) return LLFE_ERR_INVALID;
    const int h = images[0].height, w = images[0].width;
    if (!valid_dims(n, h, w)) return ctx->fail(LLFE_ERR_INVALID, "invalid batch n=%d h=%d w=%d", n, h, w);
    if (n_colors < 0 || n_colors > kMaxColors)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "n_colors=%d outside [1, %d]", n_colors, kMaxColors);
    if (n > chunk_for(h, w))
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_submit_images: n=%d exceeds one device pass (%d)", n,
                         chunk_for(h, w));
    int nd = 0;
    for (int i = 0; i < n; i++) {
        const llfe_image_desc &d = images[i];
        if (!d.data || d.height != h || d.width != w || (d.row_stride != 0 && d.row_stride < 3 * (int64_t)w))
            return ctx->fail(LLFE_ERR_INVALID, "image %d: %d x %d stride %lld in a %d x %d submission", i, d.height,
                             d.width, (long long)d.row_stride, h, w);
        if (d.noise)
            return ctx->fail(LLFE_ERR_UNSUPPORTED, "image %d: parity noise goes through llfe_process_images", i);
        nd += d.on_device ? 1 : 0;
    }
    const int slot = (int)(ctx->next_ticket % ctx->inflight_max);
    auto &pd = ctx->inflight[slot];
    if (pd.busy) return ctx->fail(LLFE_ERR_CAPACITY, "%d batches already in flight: collect one first", ctx->inflight_max);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipEventRecord(ctx->start_ev, (hipStream_t)stream));
    hipStream_t q = ctx->streams[slot];
    HIPCHK(ctx, hipStreamWaitEvent(q, ctx->start_ev, 0));
    Work &W = ctx->ws[slot];
    const size_t P3 = (size_t)h * w * 3;
    ctx->prof.cur_slot = slot;
    // in place when every image is a packed, 16-B aligned device image: the scatter and the
    // stencil (the only readers of the input) take image i's address from a table; else (host
    // sources, strided rows, the GPU contour mode, whose capacity redo re-reads a packed
    // batch) the images are gathered into the slot's input buffer first
    bool in_place = nd == n && !ctx->gpu_contours;
    for (int i = 0; in_place && i < n; i++)
        in_place = (images[i].row_stride == 0 || images[i].row_stride == 3 * (int64_t)w) &&
                   (((uintptr_t)images[i].data) & 15) == 0;
    const uint64_t *d_tab = nullptr;
    if (nd == n) {
        // a table of addresses and pitches (pinned, per slot: the slot is not reused before
        // this ticket's collect), then one gather launch unless the kernels read in place
        HIPCHK(ctx, ctx->h_gather_s[slot].ensure(2 * (size_t)n));
        HIPCHK(ctx, ctx->d_gather_s[slot].ensure(2 * (size_t)n));
        uint64_t *tab = ctx->h_gather_s[slot].p;
        for (int i = 0; i < n; i++) {
            tab[i] = (uint64_t)(uintptr_t)images[i].data;
            tab[n + i] = (uint64_t)(images[i].row_stride ? images[i].row_stride : 3 * (int64_t)w);
        }
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_gather_s[slot].p, tab, sizeof(uint64_t) * 2 * n, hipMemcpyHostToDevice, q));
        if (in_place) {
            d_tab = ctx->d_gather_s[slot].p;
        } else {
            HIPCHK(ctx, W.d_in.ensure(P3 * n));
            TIMED(ctx, q, "k_gather_images", 2.0 * (double)P3 * n,
                  launch_gather_images(ctx->d_gather_s[slot].p, n, h, w, W.d_in.p, q));
        }
    } else {
        HIPCHK(ctx, W.d_in.ensure(P3 * n));
        for (int i = 0; i < n; i++) {
            const llfe_image_desc &d = images[i];
            const size_t pitch = d.row_stride ? (size_t)d.row_stride : (size_t)w * 3;
            HIPCHK(ctx, hipMemcpy2DAsync(W.d_in.p + (size_t)i * P3, (size_t)w * 3, d.data, pitch, (size_t)w * 3, h,
                                         d.on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, q));
        }
    }
    pd.idx.assign(indices, indices + n);
    llfe_batch b{};
    b.data = d_tab ? images[0].data : W.d_in.p;
    b.n = n;
    b.height = h;
    b.width = w;
    b.on_device = 1;
    b.n_colors = n_colors;
    b.indices = pd.idx.data();
    int rc = enqueue_chunk(ctx, &b, features, seed, 0, n, slot, slot, d_tab);
    if (rc) return rc;
    pd.busy = true;
    pd.done = false;
    pd.b = b;
    pd.features = features;
    *ticket = ctx->next_ticket++;
    return LLFE_OK;
}

int llfe_collect_batch(llfe_ctx *ctx, int64_t ticket, llfe_image_result *results, llfe_shape *shapes,
                       int64_t shape_capacity, int64_t *shapes_needed) {
    if (!ctx || !results) return LLFE_ERR_INVALID;
    if (ticket != ctx->next_collect) return ctx->fail(LLFE_ERR_INVALID, "collect tickets in submission order");
    const int slot = (int)(ticket % ctx->inflight_max);
    auto &pd = ctx->inflight[slot];
    if (!pd.busy) return ctx->fail(LLFE_ERR_INVALID, "ticket %lld was not submitted", (long long)ticket);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const int n = pd.b.n;
    if (!pd.done) {  // host half once; a retry after LLFE_ERR_CAPACITY only copies
        pd.res.assign((size_t)n, llfe_image_result{});
        int64_t total = 0;
        if (n > 0) {
            int rc = finish_chunk(ctx, &pd.b, pd.features, 0, n, slot, pd.res.data(), nullptr, 0, total);
            if (rc) return rc;
        }
        pd.shp.clear();
        if (pd.features & LLFE_FEATURE_SHAPES) {
            pd.shp.reserve((size_t)total);
            // finish_chunk left the per-image shapes in ctx->img_shapes
            for (int i = 0; i < n; i++)
                pd.shp.insert(pd.shp.end(), ctx->img_shapes[i].begin(), ctx->img_shapes[i].end());
        }
        ctx->prof.collect(slot);
        pd.done = true;
    }
    const int64_t total = (int64_t)pd.shp.size();
    if (shapes_needed) *shapes_needed = total;
    std::memcpy(results, pd.res.data(), sizeof(llfe_image_result) * (size_t)n);
    if (shapes) std::memcpy(shapes, pd.shp.data(), sizeof(llfe_shape) * (size_t)std::min(total, shape_capacity));
    if (total > shape_capacity)
        return ctx->fail(LLFE_ERR_CAPACITY, "shape capacity %lld < %lld", (long long)shape_capacity, (long long)total);
    pd.busy = false;
    ctx->next_collect++;
    return LLFE_OK;
}

int llfe_gray_blur5(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *blurred, int32_t n, int32_t h, int32_t w,
                    llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !blurred) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, launch_stencil(bgr, n, h, w, nullptr, blurred, nullptr, nullptr, nullptr, ctx->sp, (hipStream_t)stream));
    HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
    return LLFE_OK;
}

int llfe_edge_classes(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *classes, int32_t n, int32_t h, int32_t w,
                      llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !classes) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, launch_stencil(bgr, n, h, w, classes, nullptr, nullptr, nullptr, nullptr, ctx->sp, (hipStream_t)stream));
    HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
    return LLFE_OK;
}

int llfe_font_binary(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *mask, int32_t n, int32_t h, int32_t w,
                     llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !mask) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, launch_font_binary(bgr, n, h, w, mask, ctx->sp, (hipStream_t)stream));
    HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
    return LLFE_OK;
}

int llfe_text_size(int32_t h, int32_t w, int32_t *out_h, int32_t *out_w) {
    if (h <= 0 || w <= 0 || !out_h || !out_w) return LLFE_ERR_INVALID;
    if (h < 30 || w < 100) {  // scale = max(2, 300 / width, 100 / height) (Python floats)
        const double sc = std::max(std::max(2.0, 300.0 / w), 100.0 / h);
        if (w * sc >= 2147483647.0 || h * sc >= 2147483647.0) return LLFE_ERR_UNSUPPORTED;
        *out_w = (int32_t)std::lrint(w * sc);  // saturate_cast<int>(double): round half even
        *out_h = (int32_t)std::lrint(h * sc);
        return 1;
    }
    *out_h = h;
    *out_w = w;
    return 0;
}

// TextExtractor.preprocess_image (text_extractor.py:15-46): gray, INTER_CUBIC upscale
// of small images (cvresize.hip), Otsu binary and the mean > 127 inversion (text.hip)
int llfe_text_binary(llfe_ctx *ctx, const uint8_t *img, int32_t h, int32_t w, int32_t channels, uint8_t *out,
                     int32_t *threshold, llfe_stream stream) {
    if (!ctx || !img || !out || h <= 0 || w <= 0) return LLFE_ERR_INVALID;
    if (channels != 1 && channels != 3 && channels != 4)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_text_binary: %d channels (1, 3 or 4)", channels);
    int32_t oh, ow;
    const int up = llfe_text_size(h, w, &oh, &ow);
    if (up < 0 || !valid_dims(1, h, w) || !valid_dims(1, oh, ow))
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_text_binary: %d x %d (-> %d x %d) pixels", h, w, oh, ow);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    const long long n = (long long)h * w, n2 = (long long)oh * ow;
    HIPCHK(ctx, ctx->d_text.ensure((size_t)(n + (up ? n2 : 0))));
    HIPCHK(ctx, ctx->d_text_hist.ensure(258));
    uint8_t *gray = ctx->d_text.p, *g = gray;
    HIPCHK(ctx, launch_text_gray(img, n, channels, gray, s));
    if (up) {
        const double sc = std::max(std::max(2.0, 300.0 / w), 100.0 / h);
        CvResizePlan plan;
        if (cv_resize_plan_scaled(h, w, 1, oh, ow, sc, sc, kCvInterCubic, plan) != 0)
            return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_text_binary: resize plan");
        HIPCHK(ctx, ctx->d_coef.ensure(plan.tab.size()));
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_coef.p, plan.tab.data(), plan.tab.size() * sizeof(int32_t),
                                   hipMemcpyHostToDevice, s));
        g = gray + n;
        HIPCHK(ctx, launch_cv_resize(plan, gray, g, ctx->d_coef.p, s));
        HIPCHK(ctx, hipStreamSynchronize(s));  // the host table dies with `plan`
    }
    HIPCHK(ctx, launch_text_otsu_binary(g, n2, ctx->d_text_hist.p, out, s));
    if (threshold) {
        unsigned long long t = 0;
        HIPCHK(ctx, hipMemcpyAsync(&t, ctx->d_text_hist.p + 256, sizeof t, hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipStreamSynchronize(s));
        *threshold = (int32_t)t;
    } else {
        HIPCHK(ctx, hipStreamSynchronize(s));
    }
    return LLFE_OK;
}

int llfe_shape_mask(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *mask, int32_t n, int32_t h, int32_t w,
                    llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !mask) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    Work &W = ctx->ws[0];  // stage entry points run on the caller's stream, slot 0
    HIPCHK(ctx, W.d_cls.ensure((size_t)n * h * w));
    StencilParams sp;
    int rc = stencil_params(ctx, W, n, h, w, s, &sp);
    if (rc) return rc;
    HIPCHK(ctx, launch_stencil(bgr, n, h, w, W.d_cls.p, nullptr, nullptr, nullptr, nullptr, sp, s));
    rc = run_hysteresis_dilate(ctx, W, n, h, w, nullptr, mask, s);
    if (rc) return rc;
    HIPCHK(ctx, hipStreamSynchronize(s));
    ctx->prof.collect(-2);
    return LLFE_OK;
}

// Canny(blur5(gray), 50, 150) of the shapes path (shape pyc @L6-30) before the
// dilation: the stencil's edge classes, then the hysteresis components, as 0 / 255
int llfe_canny(llfe_ctx *ctx, const uint8_t *bgr, uint8_t *edges, int32_t n, int32_t h, int32_t w,
               llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !edges) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    Work &W = ctx->ws[0];
    HIPCHK(ctx, W.d_cls.ensure((size_t)n * h * w));
    StencilParams sp;
    int rc = stencil_params(ctx, W, n, h, w, s, &sp);
    if (rc) return rc;
    HIPCHK(ctx, launch_stencil(bgr, n, h, w, W.d_cls.p, nullptr, nullptr, nullptr, nullptr, sp, s));
    HystWork wk;
    rc = hyst_work(ctx, W, n, h, w, &wk);
    if (rc) return rc;
    HIPCHK(ctx, launch_canny_edges(W.d_cls.p, n, h, w, wk, edges, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
    return LLFE_OK;
}

// dilate(src, ones(3, 3)) of the shapes path (shape pyc @L6-30) on n u8 images
int llfe_dilate3(llfe_ctx *ctx, const uint8_t *src, uint8_t *dst, int32_t n, int32_t h, int32_t w,
                 llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !src || !dst || src == dst) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, launch_dilate3_u8(src, n, h, w, dst, (hipStream_t)stream));
    HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
    return LLFE_OK;
}

int llfe_shadow_stats(llfe_ctx *ctx, const uint8_t *bgr, uint64_t *sums, uint64_t *counts, int32_t n, int32_t h,
                      int32_t w, llfe_stream stream) {
    if (!ctx || !valid_dims(n, h, w) || !bgr || !sums || !counts) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    Work &W = ctx->ws[0];
    HIPCHK(ctx, W.d_shadow.ensure(2 * (size_t)n + shadow_tiles(n, h, w)));
    HIPCHK(ctx, launch_stencil(bgr, n, h, w, nullptr, nullptr, W.d_shadow.p, W.d_shadow.p + n,
                               (uint2 *)(W.d_shadow.p + 2 * n), ctx->sp, s));
    HIPCHK(ctx, hipMemcpyAsync(sums, W.d_shadow.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipMemcpyAsync(counts, W.d_shadow.p + n, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
    return LLFE_OK;
}

int llfe_color_unique(llfe_ctx *ctx, const llfe_batch *b, uint64_t seed, uint32_t *keys, int64_t *n_unique,
                      llfe_stream stream) {
    if (!ctx || !b || !keys || !n_unique || !valid_dims(b->n, b->height, b->width)) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    const int cmax = chunk_for(b->height, b->width);
    if (b->n > cmax) return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_color_unique: n > %d", cmax);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    Work &W = ctx->ws[0];
    const int h = b->height, w = b->width, n = b->n;
    const int64_t P = (int64_t)h * w;
    const int64_t key_stride = (std::max<int64_t>(P, 1) + 3) & ~int64_t(3);
    const uint8_t *img;
    const int8_t *noise;
    int rc = stage_input(ctx, W, b, 0, n, &img, &noise, s);
    if (rc) return rc;
    ImgIndex index;
    rc = chunk_index(ctx, W, b, 0, n, s, &index);
    if (rc) return rc;
    rc = color_stage(ctx, W, img, nullptr, noise, n, h, w, seed, index, /*contiguous_keys=*/true, s);
    if (rc) return rc;
    HIPCHK(ctx, hipMemcpy2DAsync(keys, sizeof(uint32_t) * P, W.d_keys.p, sizeof(uint32_t) * key_stride,
                                 sizeof(uint32_t) * P, n, hipMemcpyDeviceToDevice, s));
    HIPCHK(ctx, hipMemcpyAsync(n_unique, W.d_nuniq.p, sizeof(int64_t) * n, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
    return LLFE_OK;
}

int llfe_kmeans(llfe_ctx *ctx, const uint32_t *keys, int64_t key_stride, const int64_t *n_points, int32_t n,
                int32_t n_colors, uint64_t seed, int64_t index_base, llfe_image_result *results,
                llfe_stream stream) {
    if (!ctx || !keys || !n_points || !results || n < 0) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    if (key_stride % 4 || ((uintptr_t)keys & 15))
        return ctx->fail(LLFE_ERR_INVALID, "keys must be 16-byte aligned with key_stride % 4 == 0");
    if (n > kMaxKmeansBatch) return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_kmeans: n > %d", kMaxKmeansBatch);
    for (int i = 0; i < n; i++)
        if (n_points[i] < 0 || n_points[i] > key_stride) return ctx->fail(LLFE_ERR_INVALID, "n_points out of range");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    Work &W = ctx->ws[0];
    HIPCHK(ctx, W.d_nuniq.ensure(n));
    HIPCHK(ctx, hipMemcpyAsync(W.d_nuniq.p, n_points, sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
    const KmeansCubes none{nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0};  // plain sweeps over caller-supplied keys
    int rc = kmeans_stage(ctx, W, keys, key_stride, W.d_nuniq.p, n, n_colors, seed, ImgIndex{index_base, nullptr}, none, s);
    if (rc) return rc;
    HIPCHK(ctx, ctx->h_kout.ensure(n));
    HIPCHK(ctx, hipMemcpyAsync(ctx->h_kout.p, W.d_kout.p, sizeof(KmeansImageOut) * n, hipMemcpyDeviceToHost, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
    for (int i = 0; i < n; i++) {
        std::memset(&results[i], 0, sizeof(llfe_image_result));
        results[i].shadow_level = -1;
        fill_color_result(ctx->h_kout.p[i], results[i]);
    }
    return LLFE_OK;
}

int llfe_palette_rules(const uint8_t *centers_rgb, const int32_t *counts, int32_t k, llfe_image_result *r) {
    if (!r || k < 0 || k > kMaxColors || (k > 0 && (!centers_rgb || !counts))) return LLFE_ERR_INVALID;
    r->n_colors = k;
    for (int i = 0; i < k; i++) {
        r->counts[i] = counts[i];
        for (int j = 0; j < 3; j++) r->centers_rgb[i][j] = centers_rgb[3 * i + j];
    }
    fill_palette(*r);
    return LLFE_OK;
}

int llfe_kmeans_attempts(llfe_ctx *ctx, int32_t n, llfe_kmeans_attempt *out) {
    if (!ctx || !out || n < 0) return LLFE_ERR_INVALID;
    if (ctx->any_inflight())
        return ctx->fail(LLFE_ERR_INVALID, "llfe_kmeans_attempts with submitted batches not yet collected");
    // the workspace the last k-means launch ran on (slot 0 for the synchronous entry points,
    // the ticket's slot for llfe_submit_batch / llfe_submit_images)
    if (!ctx->km_last) return ctx->fail(LLFE_ERR_INVALID, "no k-means launch yet");
    Work &W = *ctx->km_last;
    if (n > W.km_n) return ctx->fail(LLFE_ERR_INVALID, "the last k-means launch had %d images", W.km_n);
    if (W.km_colors > kMaxK) return ctx->fail(LLFE_ERR_UNSUPPORTED, "attempt records only for n_colors <= %d", kMaxK);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    std::vector<KmeansAttemptOut> a((size_t)n * kAttempts);
    HIPCHK(ctx, hipDeviceSynchronize());
    HIPCHK(ctx, hipMemcpy(a.data(), W.d_att.p, sizeof(KmeansAttemptOut) * a.size(), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < a.size(); i++) {
        llfe_kmeans_attempt &r = out[i];
        std::memset(&r, 0, sizeof r);
        for (int k = 0; k < kMaxK; k++) {
            for (int j = 0; j < 3; j++) {
                r.pp_centers[k][j] = a[i].pp_centers[k][j];
                r.centers[k][j] = a[i].centers[k][j];
            }
            r.counts[k] = a[i].counts[k];
        }
        r.iters = a[i].iters;
        r.compactness = a[i].compactness;
    }
    return LLFE_OK;
}

namespace {
// Image.resize(size, LANCZOS, box) of n same-size packed device images
int resize_lanczos_n(llfe_ctx *ctx, const uint8_t *src, int n, int32_t h, int32_t w, int32_t ch, uint8_t *dst,
                     int32_t out_h, int32_t out_w, const double *box, hipStream_t s) {
    double bx0 = box ? box[0] : 0, by0 = box ? box[1] : 0, bx1 = box ? box[2] : w, by1 = box ? box[3] : h;
    bool need_h = out_w != w || bx0 != 0 || bx1 != out_w;
    bool need_v = out_h != h || by0 != 0 || by1 != out_h;
    std::vector<int32_t> bh, kh, bv, kv;
    int ksh = pil_coeffs(w, bx0, bx1, out_w, bh, kh);
    int ksv = pil_coeffs(h, by0, by1, out_h, bv, kv);
    int yfirst = bv[0], ylast = bv[2 * out_h - 2] + bv[2 * out_h - 1];
    // coefficient block: [bh | kh | bv | kv]
    size_t nb = bh.size() + kh.size() + bv.size() + kv.size();
    HIPCHK(ctx, ctx->d_coef.ensure(nb));
    std::vector<int32_t> all;
    all.reserve(nb);
    if (need_h)
        for (int i = 0; i < out_h; i++) bv[2 * i] -= yfirst;
    all.insert(all.end(), bh.begin(), bh.end());
    all.insert(all.end(), kh.begin(), kh.end());
    all.insert(all.end(), bv.begin(), bv.end());
    all.insert(all.end(), kv.begin(), kv.end());
    HIPCHK(ctx, hipMemcpyAsync(ctx->d_coef.p, all.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, s));
    const int32_t *dbh = ctx->d_coef.p, *dkh = dbh + bh.size(), *dbv = dkh + kh.size(), *dkv = dbv + bv.size();
    const long long in_img = (long long)h * w * ch, out_img = (long long)out_h * out_w * ch;
    if (!need_h && !need_v) {
        HIPCHK(ctx, hipMemcpyAsync(dst, src, (size_t)n * in_img, hipMemcpyDeviceToDevice, s));
    } else if (need_h && !need_v) {
        HIPCHK(ctx, launch_resize_h(src, h, w, ch, yfirst, ylast - yfirst, dst, out_w, dbh, dkh, ksh, s, n, in_img,
                                    out_img));
    } else if (!need_h) {
        HIPCHK(ctx, launch_resize_v(src, w, ch, dst, out_h, dbv, dkv, ksv, s, n, in_img, out_img));
    } else {
        const int rows = ylast - yfirst;
        const long long tmp_img = (long long)rows * out_w * ch;
        HIPCHK(ctx, ctx->d_rsz_tmp.ensure((size_t)n * tmp_img));
        HIPCHK(ctx, launch_resize_h(src, h, w, ch, yfirst, rows, ctx->d_rsz_tmp.p, out_w, dbh, dkh, ksh, s, n, in_img,
                                    tmp_img));
        HIPCHK(ctx, launch_resize_v(ctx->d_rsz_tmp.p, out_w, ch, dst, out_h, dbv, dkv, ksv, s, n, tmp_img, out_img));
    }
    HIPCHK(ctx, hipStreamSynchronize(s));  // host coefficient vectors die here
    return LLFE_OK;
}

// thumbnail((max_w, max_h), LANCZOS) incl. the reducing_gap=2.0 reduce() pre-pass, n images
int thumbnail_n(llfe_ctx *ctx, const uint8_t *src, int n, int32_t h, int32_t w, int32_t ch, int32_t max_w,
                int32_t max_h, uint8_t *dst, int64_t dst_capacity, int32_t *out_h, int32_t *out_w, hipStream_t s) {
    int32_t ow, oh;
    int rc = llfe_thumbnail_size(w, h, max_w, max_h, &ow, &oh);
    if (rc < 0) return ctx->fail(rc, "invalid thumbnail geometry");
    if ((int64_t)n * ow * oh * ch > dst_capacity) return ctx->fail(LLFE_ERR_CAPACITY, "thumbnail dst too small");
    *out_w = ow;
    *out_h = oh;
    if (rc == 0) {
        HIPCHK(ctx, hipMemcpyAsync(dst, src, (size_t)n * h * w * ch, hipMemcpyDeviceToDevice, s));
        HIPCHK(ctx, hipStreamSynchronize(s));
        return LLFE_OK;
    }
    // Image.resize(size, LANCZOS, box=None, reducing_gap=2.0)
    const double gap = 2.0;
    int fx = (int)((double)w / ow / gap), fy = (int)((double)h / oh / gap);
    if (fx < 1) fx = 1;
    if (fy < 1) fy = 1;
    if (fx > 1 || fy > 1) {
        // _get_safe_box of the full image is the full image itself
        const int rw = (w + fx - 1) / fx, rh = (h + fy - 1) / fy;
        const long long red_img = (long long)rw * rh * ch;
        HIPCHK(ctx, ctx->d_rsz_src.ensure((size_t)n * red_img));
        HIPCHK(ctx, launch_reduce(src, w, ch, 0, 0, w, h, fx, fy, ctx->d_rsz_src.p, rw, rh, s, n,
                                  (long long)h * w * ch, red_img));
        const double box[4] = {0.0, 0.0, (double)w / fx, (double)h / fy};
        return resize_lanczos_n(ctx, ctx->d_rsz_src.p, n, rh, rw, ch, dst, oh, ow, box, s);
    }
    return resize_lanczos_n(ctx, src, n, h, w, ch, dst, oh, ow, nullptr, s);
}
}  // namespace

int llfe_resize_lanczos_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, uint8_t *dst,
                            int32_t out_h, int32_t out_w, const double *box, llfe_stream stream) {
    if (!ctx || !src || !dst || h <= 0 || w <= 0 || ch <= 0 || out_h <= 0 || out_w <= 0) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    return resize_lanczos_n(ctx, src, 1, h, w, ch, dst, out_h, out_w, box, (hipStream_t)stream);
}

// PIL Image.thumbnail's preserve_aspect_ratio (Python float semantics).  Returns 1
// and the new size when a resize happens, 0 when the image already fits.
int llfe_thumbnail_size(int32_t w, int32_t h, int32_t max_w, int32_t max_h, int32_t *out_w, int32_t *out_h) {
    if (w <= 0 || h <= 0 || max_w <= 0 || max_h <= 0 || !out_w || !out_h) return LLFE_ERR_INVALID;
    *out_w = w;
    *out_h = h;
    int64_t x = max_w, y = max_h;
    if (x >= w && y >= h) return 0;
    const double aspect = (double)w / (double)h;
    if ((double)x / (double)y >= aspect) {
        double num = (double)y * aspect;
        int64_t f = (int64_t)std::floor(num), c = (int64_t)std::ceil(num);
        double kf = std::fabs(aspect - (double)f / (double)y), kc = std::fabs(aspect - (double)c / (double)y);
        x = std::max<int64_t>(kc < kf ? c : f, 1);  // min(floor, ceil, key=...) keeps floor on ties
    } else {
        double num = (double)x / aspect;
        int64_t f = (int64_t)std::floor(num), c = (int64_t)std::ceil(num);
        auto key = [&](int64_t n) { return n == 0 ? 0.0 : std::fabs(aspect - (double)x / (double)n); };
        y = std::max<int64_t>(key(c) < key(f) ? c : f, 1);
    }
    *out_w = (int32_t)x;
    *out_h = (int32_t)y;
    return (x != w || y != h) ? 1 : 0;
}

// ImageProcessor.auto_process_image's resize: PIL thumbnail((max_w, max_h), LANCZOS,
// reducing_gap=2.0) on a device u8 HWC image (image_processor.py:221-224).  dst must hold
// out_h * out_w * ch bytes (at most h * w * ch).
int llfe_thumbnail_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, int32_t max_w,
                       int32_t max_h, uint8_t *dst, int64_t dst_capacity, int32_t *out_h, int32_t *out_w,
                       llfe_stream stream) {
    if (!ctx || !src || !dst || !out_h || !out_w || ch <= 0) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    return thumbnail_n(ctx, src, 1, h, w, ch, max_w, max_h, dst, dst_capacity, out_h, out_w, (hipStream_t)stream);
}

int llfe_thumbnail_pil_batch(llfe_ctx *ctx, const uint8_t *src, int32_t n, int32_t h, int32_t w, int32_t ch,
                             int32_t max_w, int32_t max_h, uint8_t *dst, int64_t dst_capacity, int32_t *out_h,
                             int32_t *out_w, llfe_stream stream) {
    if (!ctx || n < 0 || (n > 0 && (!src || !dst)) || !out_h || !out_w || ch <= 0 || n > 65535)
        return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (n == 0) return llfe_thumbnail_size(w, h, max_w, max_h, out_w, out_h) < 0 ? LLFE_ERR_INVALID : LLFE_OK;
    return thumbnail_n(ctx, src, n, h, w, ch, max_w, max_h, dst, dst_capacity, out_h, out_w, (hipStream_t)stream);
}

// cv2.resize (validate_and_preprocess_image, utils.py:118-143); tables built on the host
// exactly as OpenCV builds them, one kernel evaluates the output (cvresize.hip)
int llfe_resize_cv(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, uint8_t *dst, int32_t out_h,
                   int32_t out_w, int32_t interpolation, llfe_stream stream) {
    if (!ctx || !src || !dst || h <= 0 || w <= 0 || ch <= 0 || out_h <= 0 || out_w <= 0) return LLFE_ERR_INVALID;
    if (ch > 4) return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_resize_cv: ch > 4");
    CvResizePlan plan;
    if (cv_resize_plan(h, w, ch, out_h, out_w, interpolation, plan) != 0)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "llfe_resize_cv: interpolation %d not supported", interpolation);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    const int32_t *dtab = nullptr;
    if (!plan.tab.empty()) {
        HIPCHK(ctx, ctx->d_coef.ensure(plan.tab.size()));
        HIPCHK(ctx, hipMemcpyAsync(ctx->d_coef.p, plan.tab.data(), plan.tab.size() * sizeof(int32_t),
                                   hipMemcpyHostToDevice, s));
        dtab = ctx->d_coef.p;
    }
    HIPCHK(ctx, launch_cv_resize(plan, src, dst, dtab, s));
    HIPCHK(ctx, hipStreamSynchronize(s));  // the host table dies here
    return LLFE_OK;
}

int llfe_preprocess_size(int32_t w, int32_t h, int32_t mode, int32_t *out_w, int32_t *out_h, int32_t *interpolation) {
    if (w <= 0 || h <= 0 || !out_w || !out_h || !interpolation) return LLFE_ERR_INVALID;
    int max_dim, interp;
    switch (mode) {
    case LLFE_PRE_AUTO: max_dim = 2000, interp = LLFE_CV_INTER_AREA; break;
    case LLFE_PRE_HIGH_QUALITY: max_dim = 4000, interp = LLFE_CV_INTER_LANCZOS4; break;
    case LLFE_PRE_PERFORMANCE: max_dim = 1000, interp = LLFE_CV_INTER_LINEAR; break;
    case LLFE_PRE_NONE: return 0;
    default: return LLFE_ERR_INVALID;
    }
    const int m = std::max(w, h);
    if (m <= max_dim) return 0;
    const double scale = (double)max_dim / m;  // Python: max_dim / max(h, w)
    *out_w = (int32_t)(w * scale);             // int(w * scale): truncation toward 0
    *out_h = (int32_t)(h * scale);
    *interpolation = interp;
    return 1;
}

int llfe_reduce_pil(llfe_ctx *ctx, const uint8_t *src, int32_t h, int32_t w, int32_t ch, int32_t fx, int32_t fy,
                    uint8_t *dst, llfe_stream stream) {
    if (!ctx || !src || !dst || h <= 0 || w <= 0 || ch <= 0 || fx <= 0 || fy <= 0) return LLFE_ERR_INVALID;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    const int rw = (w + fx - 1) / fx, rh = (h + fy - 1) / fy;
    HIPCHK(ctx, launch_reduce(src, w, ch, 0, 0, w, h, fx, fy, dst, rw, rh, s));
    HIPCHK(ctx, hipStreamSynchronize(s));
    return LLFE_OK;
}

int llfe_find_contours(const uint8_t *mask, int32_t h, int32_t w, int32_t *points, int64_t points_capacity,
                       int32_t *offsets, int32_t offsets_capacity, int64_t *needed_points) {
    if (!mask || h <= 0 || w <= 0) return LLFE_ERR_INVALID;
    std::vector<int8_t> work;
    Contours c;
    external_contours_u8(mask, h, w, work, c);
    const int nc = (int)c.start.size() - 1;
    const int64_t npts = (int64_t)c.xy.size() / 2;
    if (needed_points) *needed_points = npts;
    if (npts > points_capacity || nc + 1 > offsets_capacity) return LLFE_ERR_CAPACITY;
    // output in cv2 order (newest first)
    int64_t wpos = 0;
    offsets[0] = 0;
    for (int k = 0; k < nc; k++) {
        int src = nc - 1 - k;
        int64_t a = c.start[src], b2 = c.start[src + 1];
        std::memcpy(points + 2 * wpos, c.xy.data() + 2 * a, sizeof(int32_t) * 2 * (b2 - a));
        wpos += b2 - a;
        offsets[k + 1] = (int32_t)wpos;
    }
    return nc;
}

namespace {
// host u8 masks -> bit-packed on the device -> GPU contour pass on workspace 0 (synchronous;
// capacities grown until nothing overflows).  Leaves the results in W.d_ct_* and
// slot 0's host copies.
int gpu_contours_of_masks(llfe_ctx *ctx, const uint8_t *masks, int n, int h, int w) {
    if (w > kCtMaxWidth || h > kCtMaxHeight)
        return ctx->fail(LLFE_ERR_UNSUPPORTED, "GPU contours need width <= %d and height <= %d", kCtMaxWidth,
                         kCtMaxHeight);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipDeviceSynchronize());
    Work &W = ctx->ws[0];
    hipStream_t s = ctx->streams[0];
    const int wpr = words_per_row(w);
    std::vector<uint64_t> bits((size_t)n * h * wpr, 0ull);
    for (size_t r = 0; r < (size_t)n * h; r++)
        for (int x = 0; x < w; x++)
            if (masks[r * w + x]) bits[r * wpr + (x >> 6)] |= 1ull << (x & 63);
    HIPCHK(ctx, W.d_bits.ensure(bits.size()));
    HIPCHK(ctx, hipMemcpyAsync(W.d_bits.p, bits.data(), sizeof(uint64_t) * bits.size(), hipMemcpyHostToDevice, s));
    for (int attempt = 0;; attempt++) {
        int rc = run_contours(ctx, W, n, h, w, W.d_bits.p, s);
        if (rc) return rc;
        rc = copy_contours(ctx, W, n, 0, s);
        if (rc) return rc;
        HIPCHK(ctx, hipStreamSynchronize(s));
        const CtCounters ct = *ctx->h_ct_ctr_s[0].p;
        if (ct.flags & (kCtBadTrace | kCtTooWide | kCtDpOverflow))
            return ctx->fail(LLFE_ERR_UNSUPPORTED, "GPU contours: unsupported mask (flags 0x%x)", ct.flags);
        if (!(ct.flags & kCtOverflowMask)) return LLFE_OK;
        if (attempt >= 8) return ctx->fail(LLFE_ERR_CAPACITY, "GPU contours: capacities still overflow");
        grow_contour_caps(W, n, h, w, ct);
    }
}
}  // namespace

int llfe_find_contours_gpu(llfe_ctx *ctx, const uint8_t *mask, int32_t h, int32_t w, int32_t *points,
                           int64_t points_capacity, int32_t *offsets, int32_t offsets_capacity,
                           int64_t *needed_points) {
    if (!ctx || !mask || h <= 0 || w <= 0 || !valid_dims(1, h, w)) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    int rc = gpu_contours_of_masks(ctx, mask, 1, h, w);
    if (rc) return rc;
    Work &W = ctx->ws[0];
    const CtCounters ct = *ctx->h_ct_ctr_s[0].p;
    const int *info = ctx->h_ct_info_s[0].p;
    const int base = info[1], nc = info[2];
    std::vector<int2> refs(nc);
    std::vector<CtComp> comps(ct.comps);
    std::vector<int2> pts(ct.pts);
    if (nc) HIPCHK(ctx, hipMemcpy(refs.data(), W.d_ct_refs.p + base, sizeof(int2) * nc, hipMemcpyDeviceToHost));
    if (ct.comps) HIPCHK(ctx, hipMemcpy(comps.data(), W.d_ct_comps.p, sizeof(CtComp) * ct.comps, hipMemcpyDeviceToHost));
    if (ct.pts) HIPCHK(ctx, hipMemcpy(pts.data(), W.d_ct_pts.p, sizeof(int2) * ct.pts, hipMemcpyDeviceToHost));
    int64_t npts = 0;
    for (int k = 0; k < nc; k++) npts += comps[refs[k].x].nv;
    if (needed_points) *needed_points = npts;
    if (npts > points_capacity || nc + 1 > offsets_capacity) return LLFE_ERR_CAPACITY;
    int64_t wpos = 0;  // cv2 order: newest first
    offsets[0] = 0;
    for (int k = 0; k < nc; k++) {
        const CtComp &c = comps[refs[nc - 1 - k].x];
        for (uint32_t v = 0; v < c.nv; v++) {
            points[2 * (wpos + v)] = pts[c.off + v].x;
            points[2 * (wpos + v) + 1] = pts[c.off + v].y;
        }
        wpos += c.nv;
        offsets[k + 1] = (int32_t)wpos;
    }
    return nc;
}

int llfe_shapes_from_masks_gpu(llfe_ctx *ctx, const uint8_t *masks, int32_t n, int32_t h, int32_t w,
                               llfe_shape *shapes, int64_t capacity, int32_t *n_shapes, int32_t *n_contours,
                               int64_t *needed) {
    if (!ctx || !masks || !valid_dims(n, h, w) || n <= 0) return LLFE_ERR_INVALID;
    if (int rc_ = stage_enter(ctx, __func__)) return rc_;
    int rc = gpu_contours_of_masks(ctx, masks, n, h, w);
    if (rc) return rc;
    const int *info = ctx->h_ct_info_s[0].p;
    const llfe_shape *src = ctx->h_ct_shapes_s[0].p;
    int64_t total = 0;
    for (int i = 0; i < n; i++) {
        const int nk = info[i * kCtInfo + 3], sb = info[i * kCtInfo + 4];
        if (n_shapes) n_shapes[i] = nk;
        if (n_contours) n_contours[i] = info[i * kCtInfo + 2];
        for (int k = 0; k < nk; k++)
            if (shapes && total + k < capacity) shapes[total + k] = src[sb + k];
        total += nk;
    }
    if (needed) *needed = total;
    return total > capacity ? LLFE_ERR_CAPACITY : LLFE_OK;
}

double llfe_border_radius(const int32_t *points, int32_t n, double epsilon_factor) {
    if (!points || n <= 0) return 0.0;
    ShapeScratch sc;
    return border_radius(points, n, epsilon_factor, sc);
}

int llfe_classify_contour(const int32_t *points, int32_t n, llfe_shape *out) {
    if (!points || n <= 0 || !out) return n == 0 ? 0 : LLFE_ERR_INVALID;
    ShapeScratch sc;
    return classify_contour(points, n, sc, *out) ? 1 : 0;
}

int llfe_shapes_from_mask(const uint8_t *mask, int32_t h, int32_t w, llfe_shape *shapes, int32_t capacity,
                          int32_t *n_contours) {
    if (!mask || h <= 0 || w <= 0) return LLFE_ERR_INVALID;
    std::vector<int8_t> work;
    Contours c;
    ShapeScratch sc;
    std::vector<llfe_shape> out;
    external_contours_u8(mask, h, w, work, c);
    int nc = shapes_from_contours(c, sc, out);
    if (n_contours) *n_contours = nc;
    if ((int64_t)out.size() > capacity) return LLFE_ERR_CAPACITY;
    for (size_t i = 0; i < out.size(); i++) shapes[i] = out[i];
    return (int)out.size();
}

}  // extern "C"
