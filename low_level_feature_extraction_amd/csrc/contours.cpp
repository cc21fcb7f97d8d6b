// Host-side shape analysis of the dilated Canny mask (product code).
//
// ShapeAnalyzer.analyze_shapes (shape pyc @L125-189): the mask produced on the GPU is
// copied back bit-packed; this file runs findContours(RETR_EXTERNAL,
// CHAIN_APPROX_SIMPLE) (@L140) and the per-contour geometry of the loop @L144-181:
// contourArea, boundingRect, arcLength, approxPolyDP (0.04 / 0.02 * perimeter) and
// the convex-hull area used by detect_border_radius (@L32-61).  The border following
// restates OpenCV's Suzuki-Abe implementation (1-pixel zero frame, 2 / 2|-128 border
// marks, contours returned newest-first) so the shape list order matches cv2.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "contours.h"

namespace llfe {

namespace {

// chain-code directions: 0 = +x, counter-clockwise on screen (y grows downward)
constexpr int kDx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
constexpr int kDy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

// Follow the outer border whose first raster pixel is `i0` (padded image of row
// pitch `pitch`); appends the CHAIN_APPROX_SIMPLE vertices (unpadded coordinates).
void trace_outer(int8_t *im, int pitch, int64_t i0, int x, int y, std::vector<int32_t> &xy) {
    int64_t d[16];
    const int64_t p = pitch;
    const int64_t base[8] = {1, -p + 1, -p, -p - 1, -1, p - 1, p, p + 1};
    for (int k = 0; k < 16; k++) d[k] = base[k & 7];
    constexpr int8_t kMark = 2;
    constexpr int8_t kMarkRight = (int8_t)(2 | -128);

    int s = 4;
    int64_t i1 = i0;
    // clockwise search (from up-left) for the last pixel of the border
    do {
        s = (s - 1) & 7;
        i1 = i0 + d[s];
    } while (im[i1] == 0 && s != 4);
    if (s == 4 && im[i1] == 0) {  // isolated pixel
        im[i0] = kMarkRight;
        xy.push_back(x);
        xy.push_back(y);
        return;
    }
    int64_t i3 = i0, i4 = 0;
    int prev_s = s ^ 4;
    for (;;) {
        const int s_end = s;
        while (s < 15) {
            i4 = i3 + d[++s];
            if (im[i4] != 0) break;
        }
        s &= 7;
        // right neighbour examined and empty -> "right bound" mark
        if ((unsigned)(s - 1) < (unsigned)s_end)
            im[i3] = kMarkRight;
        else if (im[i3] == 1)
            im[i3] = kMark;
        if (s != prev_s) {
            xy.push_back(x);
            xy.push_back(y);
            prev_s = s;
        }
        x += kDx[s];
        y += kDy[s];
        if (i4 == i0 && i3 == i1) break;
        i3 = i4;
        s = (s + 4) & 7;
    }
}

// Raster scan of the padded {0,1} image in OpenCV's order (RETR_EXTERNAL: holes and
// borders enclosed by an already traced border are skipped).  `bits` (optional) is the
// mask bit-packed (bit x & 63 of word x >> 6 of row y - 1): runs of zeros seen with
// prev == 0 change no scan state, so they are skipped a word at a time.
void scan_external(int8_t *im, int h, int w, const uint8_t *row_nonzero, Contours &out,
                   const uint64_t *bits = nullptr, int wpr = 0) {
    const int pitch = w + 2;
    for (int y = 1; y <= h; y++) {
        if (row_nonzero && !row_nonzero[y - 1]) continue;  // nothing can start or mark here
        int8_t *row = im + (int64_t)y * pitch;
        const uint64_t *rb = bits ? bits + (size_t)(y - 1) * wpr : nullptr;
        int lnbd = 0;
        int prev = 0;
        for (int x = 1; x <= w; x++) {
            if (rb && prev == 0) {  // jump to the next nonzero pixel (bit x - 1 onwards)
                int q = (x - 1) >> 6;
                uint64_t word = rb[q] & (~0ull << ((x - 1) & 63));
                while (!word && ++q < wpr) word = rb[q];
                if (!word) break;
                x = q * 64 + __builtin_ctzll(word) + 1;
                if (x > w) break;
            }
            int v = row[x];
            if (v == prev) continue;
            bool start = false;
            if (prev == 0 && v == 1) {
                start = row[lnbd] <= 0;  // not inside a border already found on this row
            } else if (v == 0 && prev >= 1) {
                if (prev & -2) lnbd = x - 1;  // hole start: skipped in RETR_EXTERNAL
            }
            if (start) {
                out.start.push_back((int64_t)(out.xy.size() / 2));
                trace_outer(im, pitch, (int64_t)y * pitch + x, x - 1, y - 1, out.xy);
                prev = row[x];
                continue;
            }
            prev = v;
            if (prev & -2) lnbd = x;
        }
    }
}

// byte i of kExpand[b] = bit i of b (0 / 1)
struct ExpandTable {
    uint64_t t[256];
    ExpandTable() {
        for (int b = 0; b < 256; b++) {
            uint64_t v = 0;
            for (int i = 0; i < 8; i++) v |= (uint64_t)((b >> i) & 1) << (8 * i);
            t[b] = v;
        }
    }
};
const ExpandTable kExpand;

}  // namespace

// mask: u8 (nonzero = edge), h x w.  `work` is reused scratch.
void external_contours_u8(const uint8_t *mask, int h, int w, std::vector<int8_t> &work, Contours &out) {
    const int pitch = w + 2;
    work.assign((size_t)pitch * (h + 2), 0);
    std::vector<uint8_t> nz(h, 0);
    for (int y = 0; y < h; y++) {
        const uint8_t *m = mask + (size_t)y * w;
        int8_t *r = work.data() + (size_t)(y + 1) * pitch + 1;
        uint8_t any = 0;
        for (int x = 0; x < w; x++) {
            int8_t b = m[x] ? 1 : 0;
            r[x] = b;
            any |= (uint8_t)b;
        }
        nz[y] = any;
    }
    out.xy.clear();
    out.start.clear();
    scan_external(work.data(), h, w, nz.data(), out);
    out.start.push_back((int64_t)(out.xy.size() / 2));
}

// bits: h rows x wpr u64 words, bit (x & 63) of word (x >> 6).  The padded int8 plane
// stays all-zero between images (`work` is per-thread scratch): only the 64-pixel words
// with a set bit are expanded, and exactly those are zeroed again afterwards (borders
// only mark foreground pixels, which lie in them) -- a ui-like 1080p mask touches ~1/10
// of the plane instead of rewriting all 2 MB of it.
void external_contours_bits(const uint64_t *bits, int h, int w, int wpr, std::vector<int8_t> &work,
                            Contours &out) {
    const int pitch = w + 2;
    const size_t need = (size_t)pitch * (h + 2);
    if (work.size() != need) work.assign(need, 0);
    thread_local std::vector<uint8_t> nz;
    thread_local std::vector<uint64_t> words;  // (y << 32 | q) of expanded words
    nz.assign(h, 0);
    words.clear();
    for (int y = 0; y < h; y++) {
        const uint64_t *wrow = bits + (size_t)y * wpr;
        int8_t *r = work.data() + (size_t)(y + 1) * pitch + 1;
        for (int q = 0; q < wpr; q++) {
            const uint64_t v = wrow[q];
            if (!v) continue;
            nz[y] = 1;
            words.push_back((uint64_t)y << 32 | (uint32_t)q);
            const int x0 = q * 64, n = std::min(64, w - x0);
            int8_t *dst = r + x0;
            if (n == 64) {
                for (int k = 0; k < 8; k++) {
                    const uint64_t e = kExpand.t[(v >> (8 * k)) & 255];
                    std::memcpy(dst + 8 * k, &e, 8);
                }
            } else {
                for (int b2 = 0; b2 < n; b2++) dst[b2] = (int8_t)((v >> b2) & 1);
            }
        }
    }
    out.xy.clear();
    out.start.clear();
    scan_external(work.data(), h, w, nz.data(), out, bits, wpr);
    out.start.push_back((int64_t)(out.xy.size() / 2));
    for (uint64_t yq : words) {
        const int y = (int)(yq >> 32), q = (int)(uint32_t)yq, x0 = q * 64;
        std::memset(work.data() + (size_t)(y + 1) * pitch + 1 + x0, 0, (size_t)std::min(64, w - x0));
    }
}

// ---------------------------------------------------------------- geometry
// cv::contourArea(oriented=false): |sum(prev.x*p.y - prev.y*p.x)| / 2 in double
double poly_area(const int32_t *p, int n) {
    if (n <= 0) return 0.0;
    double a = 0.0;
    double px = p[2 * (n - 1)], py = p[2 * (n - 1) + 1];
    for (int i = 0; i < n; i++) {
        double x = p[2 * i], y = p[2 * i + 1];
        a += px * y - py * x;
        px = x;
        py = y;
    }
    return std::fabs(a * 0.5);
}

// cv::arcLength(closed=true): float segment lengths (sqrtf) summed in double
double closed_perimeter(const int32_t *p, int n) {
    if (n <= 1) return 0.0;
    double per = 0.0;
    float px = (float)p[2 * (n - 1)], py = (float)p[2 * (n - 1) + 1];
    for (int i = 0; i < n; i++) {
        float x = (float)p[2 * i], y = (float)p[2 * i + 1];
        float dx = x - px, dy = y - py;
        per += (double)std::sqrt(dx * dx + dy * dy);
        px = x;
        py = y;
    }
    return per;
}

// cv::approxPolyDP(closed=true) vertex count (OpenCV's iterative Douglas-Peucker with
// farthest-point seeding and the collinear clean-up pass).  The seeding (three
// farthest-point sweeps) does not depend on epsilon, so one DpSeed serves both calls
// of classify_contour (0.02 and 0.04 x perimeter).
struct DpSeed {
    int pos, rs_start, sx, sy;
    double maxd;
};
static DpSeed dp_seed(const int32_t *src, int count) {
    DpSeed sd{0, 0, 0, 0, 0.0};
    int pos = 0, rs_start = 0, sx = 0, sy = 0;
    double maxd = 0;
    for (int it = 0; it < 3; it++) {  // two (approximately) farthest points
        maxd = 0;
        pos = (pos + rs_start) % count;
        sx = src[2 * pos];
        sy = src[2 * pos + 1];
        if (++pos >= count) pos = 0;
        for (int j = 1; j < count; j++) {
            const int x = src[2 * pos], y = src[2 * pos + 1];
            if (++pos >= count) pos = 0;
            double dx = x - sx, dy = y - sy, d = dx * dx + dy * dy;
            if (d > maxd) {
                maxd = d;
                rs_start = j;
            }
        }
    }
    sd.pos = pos;
    sd.rs_start = rs_start;
    sd.sx = sx;
    sd.sy = sy;
    sd.maxd = maxd;
    return sd;
}
int dp_vertex_count(const int32_t *src, int count, double eps, std::vector<int32_t> &dst,
                    std::vector<int> &stack, const DpSeed *seed = nullptr) {
    if (count == 0) return 0;
    dst.resize((size_t)2 * count + 2);
    stack.clear();
    auto rd = [&](const int32_t *arr, int &pos, int &x, int &y) {
        x = arr[2 * pos];
        y = arr[2 * pos + 1];
        if (++pos >= count) pos = 0;
    };
    eps *= eps;
    int nout = 0;
    const DpSeed sd = seed ? *seed : dp_seed(src, count);
    int pos = sd.pos, rs_start = sd.rs_start;
    int sx = sd.sx, sy = sd.sy, x = 0, y = 0;
    const bool le_eps = sd.maxd <= eps;
    if (!le_eps) {
        int a = pos % count;
        int b = (rs_start + a) % count;
        // push right slice (b, a) then slice (a, b): processed slice first
        stack.push_back(b);
        stack.push_back(a);
        stack.push_back(a);
        stack.push_back(b);
    } else {
        dst[2 * nout] = sx;
        dst[2 * nout + 1] = sy;
        nout++;
    }
    while (!stack.empty()) {
        int send = stack.back();
        stack.pop_back();
        int sstart = stack.back();
        stack.pop_back();
        int ex = src[2 * send], ey = src[2 * send + 1];
        pos = sstart;
        rd(src, pos, sx, sy);
        bool ok;
        int split = 0;
        if (pos != send) {
            double dx = ex - sx, dy = ey - sy, maxd = 0;
            while (pos != send) {
                rd(src, pos, x, y);
                double d = std::fabs((y - sy) * dx - (x - sx) * dy);
                if (d > maxd) {
                    maxd = d;
                    split = (pos + count - 1) % count;
                }
            }
            ok = maxd * maxd <= eps * (dx * dx + dy * dy);
        } else {
            ok = true;
            sx = src[2 * sstart];
            sy = src[2 * sstart + 1];
        }
        if (ok) {
            dst[2 * nout] = sx;
            dst[2 * nout + 1] = sy;
            nout++;
        } else {
            stack.push_back(split);
            stack.push_back(send);
            stack.push_back(sstart);
            stack.push_back(split);
        }
    }
    // clean-up of [almost] collinear points (closed contour)
    const int cnt = nout;
    int newc = nout;
    pos = cnt - 1;
    auto rdd = [&](int &pp, int &xx, int &yy) {
        xx = dst[2 * pp];
        yy = dst[2 * pp + 1];
        if (++pp >= cnt) pp = 0;
    };
    int px, py;
    rdd(pos, sx, sy);
    int wpos = pos;
    rdd(pos, px, py);
    for (int i = 0; i < cnt && newc > 2; i++) {
        int qx, qy;
        rdd(pos, qx, qy);
        double dx = qx - sx, dy = qy - sy;
        double d = std::fabs((px - sx) * dy - (py - sy) * dx);
        double sip = (double)(px - sx) * (qx - px) + (double)(py - sy) * (qy - py);
        if (d * d <= 0.5 * eps * (dx * dx + dy * dy) && dx != 0 && dy != 0 && sip >= 0) {
            newc--;
            dst[2 * wpos] = sx = qx;
            dst[2 * wpos + 1] = sy = qy;
            if (++wpos >= cnt) wpos = 0;
            rdd(pos, px, py);
            i++;
            continue;
        }
        dst[2 * wpos] = sx = px;
        dst[2 * wpos + 1] = sy = py;
        if (++wpos >= cnt) wpos = 0;
        px = qx;
        py = qy;
    }
    return newc;
}

// area of the convex hull (any correct hull gives the same area; Andrew's chain).  Only
// a column's lowest and highest point can be a hull vertex, so when the contour is not
// much wider than it has points, the chain runs over the column extremes in column order
// (one pass to bucket, no sort); the hull -- and so the area sum -- is the same.
double hull_area(const int32_t *p, int n, std::vector<int64_t> &tmp, std::vector<int64_t> &hull) {
    if (n < 3) return 0.0;
    int xmin = p[0], xmax = p[0];
    for (int i = 1; i < n; i++) {
        xmin = std::min(xmin, p[2 * i]);
        xmax = std::max(xmax, p[2 * i]);
    }
    const int64_t span = (int64_t)xmax - xmin + 1;
    if (span <= 4 * (int64_t)n) {
        // hull[c] = lowest | highest y + 2^30 of column xmin + c (low / high 32 bits), 0 = empty
        hull.assign((size_t)span, 0);
        for (int i = 0; i < n; i++) {
            const uint32_t y = (uint32_t)(p[2 * i + 1] + 0x40000000);
            int64_t &v = hull[(size_t)(p[2 * i] - xmin)];
            const uint32_t lo = (uint32_t)v, hi = (uint32_t)((uint64_t)v >> 32);
            v = v == 0 ? (int64_t)(((uint64_t)y << 32) | y)
                       : (int64_t)(((uint64_t)std::max(hi, y) << 32) | std::min(lo, y));
        }
        tmp.resize((size_t)2 * span);
        int m = 0;
        for (int64_t c = 0; c < span; c++) {
            const uint64_t v = (uint64_t)hull[(size_t)c];
            if (!v) continue;
            const int64_t xk = (int64_t)(xmin + c) << 32;
            const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
            tmp[(size_t)m++] = xk | lo;
            if (hi != lo) tmp[(size_t)m++] = xk | hi;
        }
        n = m;  // the column extremes, sorted by (x, y)
    } else {
        tmp.resize(n);
        for (int i = 0; i < n; i++) tmp[i] = ((int64_t)p[2 * i] << 32) | (uint32_t)(p[2 * i + 1] + 0x40000000);
        std::sort(tmp.begin(), tmp.end());
    }
    if (n < 3) return 0.0;
    auto X = [](int64_t v) { return (int64_t)(v >> 32); };
    auto Y = [](int64_t v) { return (int64_t)(uint32_t)v - 0x40000000; };
    auto cross = [&](int64_t o, int64_t a, int64_t b) {
        return (X(a) - X(o)) * (Y(b) - Y(o)) - (Y(a) - Y(o)) * (X(b) - X(o));
    };
    hull.assign((size_t)2 * n + 1, 0);
    int k = 0;
    for (int i = 0; i < n; i++) {
        while (k >= 2 && cross(hull[k - 2], hull[k - 1], tmp[i]) <= 0) k--;
        hull[k++] = tmp[i];
    }
    for (int i = n - 2, t = k + 1; i >= 0; i--) {
        while (k >= t && cross(hull[k - 2], hull[k - 1], tmp[i]) <= 0) k--;
        hull[k++] = tmp[i];
    }
    int m = k - 1;
    if (m < 3) return 0.0;
    double a = 0.0;
    for (int i = 0; i < m; i++) {
        int j = (i + m - 1) % m;
        a += (double)X(hull[j]) * (double)Y(hull[i]) - (double)Y(hull[j]) * (double)X(hull[i]);
    }
    return std::fabs(a * 0.5);
}

// detect_border_radius (shape pyc @L32-61) given the contour's arcLength and contourArea
static double border_radius_pa(const int32_t *p, int n, double epsilon_factor, double perimeter, double area,
                               ShapeScratch &sc, const DpSeed *seed = nullptr) {
    if (dp_vertex_count(p, n, epsilon_factor * perimeter, sc.dp, sc.stack, seed) > 4) {
        double ha = hull_area(p, n, sc.t0, sc.t1);
        if (ha > 0) return std::max(0.0, (1 - area / ha) * 50.0);
    }
    return 0.0;
}

double border_radius(const int32_t *p, int n, double epsilon_factor, ShapeScratch &sc) {
    return border_radius_pa(p, n, epsilon_factor, closed_perimeter(p, n), poly_area(p, n), sc);
}

// One iteration of the analyze_shapes loop (shape pyc @L146-181). Returns false when
// the contour is dropped (contourArea < 100).
bool classify_contour(const int32_t *p, int n, ShapeScratch &sc, llfe_shape &out) {
    const double area = poly_area(p, n);
    if (area < 100) return false;
    int xmin = p[0], xmax = p[0], ymin = p[1], ymax = p[1];
    for (int i = 1; i < n; i++) {
        xmin = std::min(xmin, p[2 * i]);
        xmax = std::max(xmax, p[2 * i]);
        ymin = std::min(ymin, p[2 * i + 1]);
        ymax = std::max(ymax, p[2 * i + 1]);
    }
    const double perimeter = closed_perimeter(p, n);
    const DpSeed seed = dp_seed(p, n);
    const double br = border_radius_pa(p, n, 0.02, perimeter, area, sc, &seed);
    const int nv = dp_vertex_count(p, n, 0.04 * perimeter, sc.dp, sc.stack, &seed);
    int type = LLFE_SHAPE_UNKNOWN;
    if (nv == 3) {
        type = LLFE_SHAPE_TRIANGLE;
    } else if (nv == 4) {
        type = LLFE_SHAPE_RECTANGLE;
    } else if (nv > 4) {
        if (perimeter > 0) {
            const double four_pi = 4 * 3.141592653589793;
            double circularity = four_pi * area / (perimeter * perimeter);
            type = circularity > 0.8 ? LLFE_SHAPE_CIRCLE : LLFE_SHAPE_POLYGON;
        }
    }
    out.type = type;
    out.x = xmin;
    out.y = ymin;
    out.width = xmax - xmin + 1;
    out.height = ymax - ymin + 1;
    out.pad_ = 0;
    out.border_radius = br;
    out.area = area;
    return true;
}

// all shapes of one image, in cv2's output order (newest contour first)
int shapes_from_contours(const Contours &c, ShapeScratch &sc, std::vector<llfe_shape> &out) {
    const int nc = (int)c.start.size() - 1;
    out.clear();
    for (int k = nc - 1; k >= 0; k--) {
        const int64_t a = c.start[k], b = c.start[k + 1];
        llfe_shape s;
        if (classify_contour(c.xy.data() + 2 * a, (int)(b - a), sc, s)) out.push_back(s);
    }
    return nc;
}

}  // namespace llfe
