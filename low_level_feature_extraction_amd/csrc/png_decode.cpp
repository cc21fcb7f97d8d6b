// Host PNG decoding for the decode step in front of the hot path: cv2.imdecode(buf,
// IMREAD_COLOR) at app/services/analyze/utils.py:108-109 and
// app/services/analyze/image_processor.py:208-211 (at ~10k 1080p
// images/s per GPU the host decode, not the GPU, bounds the end-to-end rate).
//
// IMREAD_COLOR semantics (as decode.py's Pillow path): 8-bit BGR out, alpha dropped (not
// composited), grey expanded, palette looked up, 16-bit samples reduced to their high
// byte.  Critical-chunk CRCs are checked (corrupt input is an error, as in libpng).
// Interlaced images and sub-byte depths return LLFE_ERR_UNSUPPORTED and are decoded by
// the caller's fallback (Pillow).
//
// Inflate uses libdeflate when the image provides libdeflate.so.0 (whole-stream, ~1.6x
// zlib's speed) and zlib otherwise; each row's filter is undone out of place into a
// ping-pong row pair (SSE2: Up 16 bytes per step, Sub / Average / Paeth one 3- or 4-byte
// pixel per step), then the row is converted straight into the NHWC batch (RGB -> BGR by
// SSSE3 shuffles where the CPU has them).
// A batch fans out over std::threads, one image per task.
#include <dlfcn.h>
#include <emmintrin.h>
#include <tmmintrin.h>
#include <zlib.h>

#include <cstdio>
#include <cstdlib>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "llfe.h"

namespace {

// ---------------------------------------------------------------- libdeflate (optional)
struct Deflate {
    void *(*alloc)() = nullptr;
    void (*free_)(void *) = nullptr;
    int (*zlib_dec)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
    uint32_t (*crc32)(uint32_t, const void *, size_t) = nullptr;
    bool ok = false;
    Deflate() {
        if (const char *off = getenv("LLFE_NO_LIBDEFLATE"); off && *off == '1') return;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (void *(*)())dlsym(h, "libdeflate_alloc_decompressor");
        free_ = (void (*)(void *))dlsym(h, "libdeflate_free_decompressor");
        zlib_dec = (int (*)(void *, const void *, size_t, void *, size_t, size_t *))dlsym(h, "libdeflate_zlib_decompress");
        crc32 = (uint32_t(*)(uint32_t, const void *, size_t))dlsym(h, "libdeflate_crc32");
        ok = alloc && free_ && zlib_dec && crc32;
    }
};
const Deflate &deflate() {
    static Deflate d;
    return d;
}

uint32_t crc(const uint8_t *p, size_t n) {
    const Deflate &d = deflate();
    if (d.ok) return d.crc32(0, p, n);
    uLong c = crc32(0L, Z_NULL, 0);
    while (n) {  // zlib's length is a uInt
        const uInt k = (uInt)std::min<size_t>(n, 1u << 30);
        c = crc32(c, p, k);
        p += k;
        n -= k;
    }
    return (uint32_t)c;
}

inline uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct Png {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    const uint8_t *plte = nullptr;
    uint32_t plte_n = 0;
    std::vector<std::pair<const uint8_t *, size_t>> idat;
    int channels() const { return ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : 4; }
};

// chunk walk; info_only stops after IHDR
int parse(const uint8_t *d, size_t n, Png &png, bool info_only) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || memcmp(d, sig, 8) != 0) return LLFE_ERR_INVALID;
    size_t p = 8;
    bool ihdr = false, iend = false;
    while (p + 12 <= n) {
        const uint32_t len = be32(d + p);
        const uint8_t *type = d + p + 4, *body = d + p + 8;
        if (len > n - p - 12) return LLFE_ERR_INVALID;
        const bool critical = !(type[0] & 32);
        if (critical && crc(type, (size_t)len + 4) != be32(body + len)) return LLFE_ERR_INVALID;
        if (!memcmp(type, "IHDR", 4)) {
            if (len != 13 || ihdr) return LLFE_ERR_INVALID;
            png.w = be32(body);
            png.h = be32(body + 4);
            png.depth = body[8];
            png.ctype = body[9];
            png.interlace = body[12];
            if (!png.w || !png.h || body[10] || body[11] || png.interlace > 1) return LLFE_ERR_INVALID;
            const int c = png.ctype, b = png.depth;
            const bool valid = (c == 0 && (b == 1 || b == 2 || b == 4 || b == 8 || b == 16)) ||
                               (c == 3 && (b == 1 || b == 2 || b == 4 || b == 8)) ||
                               ((c == 2 || c == 4 || c == 6) && (b == 8 || b == 16));
            if (!valid) return LLFE_ERR_INVALID;
            ihdr = true;
            if (info_only) return LLFE_OK;
        } else if (!ihdr) {
            return LLFE_ERR_INVALID;
        } else if (!memcmp(type, "PLTE", 4)) {
            if (len % 3 || len > 768) return LLFE_ERR_INVALID;
            png.plte = body;
            png.plte_n = len / 3;
        } else if (!memcmp(type, "IDAT", 4)) {
            png.idat.emplace_back(body, (size_t)len);
        } else if (!memcmp(type, "IEND", 4)) {
            iend = true;
            break;
        } else if (critical) {
            return LLFE_ERR_UNSUPPORTED;  // unknown critical chunk
        }
        p += (size_t)len + 12;
    }
    if (!ihdr || png.idat.empty()) return LLFE_ERR_INVALID;
    (void)iend;  // a missing IEND after complete image data is tolerated (as libpng does)
    if (png.ctype == 3 && !png.plte) return LLFE_ERR_INVALID;
    if (png.interlace || png.depth < 8) return LLFE_ERR_UNSUPPORTED;
    return LLFE_OK;
}

// zlib stream of the concatenated IDAT payloads -> exactly `out_n` bytes
bool inflate_idat(const Png &png, uint8_t *out, size_t out_n, std::vector<uint8_t> &cat) {
    const Deflate &d = deflate();
    if (d.ok) {
        const uint8_t *src = png.idat[0].first;
        size_t src_n = png.idat[0].second;
        if (png.idat.size() > 1) {
            size_t tot = 0;
            for (auto &c : png.idat) tot += c.second;
            cat.resize(tot);
            size_t o = 0;
            for (auto &c : png.idat) {
                memcpy(cat.data() + o, c.first, c.second);
                o += c.second;
            }
            src = cat.data();
            src_n = tot;
        }
        thread_local struct Dec {
            void *p = nullptr;
            ~Dec() {
                if (p) deflate().free_(p);
            }
        } dec;
        if (!dec.p) dec.p = d.alloc();
        size_t got = 0;
        if (dec.p) {
            const int rc = d.zlib_dec(dec.p, src, src_n, out, out_n, &got);
            if (rc == 0 && got == out_n) return true;
            if (rc == 1) return false;  // LIBDEFLATE_BAD_DATA
        }
        // short / over-long streams: zlib below decides exactly as a streaming reader would
    }
    z_stream z{};
    if (inflateInit(&z) != Z_OK) return false;
    z.next_out = out;
    z.avail_out = (uInt)out_n;
    int rc = Z_OK;
    for (size_t i = 0; i < png.idat.size() && z.avail_out; i++) {
        z.next_in = const_cast<Bytef *>(png.idat[i].first);
        z.avail_in = (uInt)png.idat[i].second;
        while (z.avail_in && z.avail_out) {
            rc = inflate(&z, Z_NO_FLUSH);
            if (rc == Z_STREAM_END) break;
            if (rc != Z_OK) {
                inflateEnd(&z);
                return false;
            }
        }
        if (rc == Z_STREAM_END) break;
    }
    const bool full = z.avail_out == 0;
    inflateEnd(&z);
    return full;  // trailing data after a complete image is ignored (libpng warns only)
}

inline uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    return (uint8_t)((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c));
}

// Undo one row's filter out of place: src = the filtered row (inflated buffer), dst = the
// row's unfiltered bytes, prior = the previous row's dst (nullptr for row 0).  Pixels move
// through whole 4-byte loads and stores (for BPP 3 the fourth byte is the next pixel's,
// rewritten by the next step; src and dst are padded): 3-byte copies through a stack
// temporary stall store forwarding at ~13 ns per pixel.  Sub is a per-byte add without
// carries in a 32-bit register (SWAR); Average and Paeth one pixel per step in 16-bit SSE2
// lanes (the left neighbour is a dependency).
inline uint32_t ld32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline void st32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

template <int BPP>
void unfilter_px(int f, uint8_t *__restrict dst, const uint8_t *__restrict src, const uint8_t *__restrict prior,
                 size_t n) {
    constexpr uint32_t keep = BPP == 4 ? 0xffffffffu : 0x00ffffffu;
    if (f == 1) {
        uint32_t a = 0;
        for (size_t i = 0; i < n; i += BPP) {
            const uint32_t x = ld32(src + i);
            const uint32_t s = ((x & 0x7f7f7f7fu) + (a & 0x7f7f7f7fu)) ^ ((x ^ a) & 0x80808080u);
            a = s & keep;
            st32(dst + i, s);
        }
        return;
    }
    const __m128i z = _mm_setzero_si128();
    auto ld = [](const uint8_t *p) { return _mm_cvtsi32_si128((int)ld32(p)); };
    auto st = [](uint8_t *p, __m128i v) { st32(p, (uint32_t)_mm_cvtsi128_si32(v)); };
    __m128i a = z, c = z;
    if (f == 3) {
        for (size_t i = 0; i < n; i += BPP) {
            const __m128i b = prior ? _mm_unpacklo_epi8(ld(prior + i), z) : z;
            const __m128i avg = _mm_srli_epi16(_mm_add_epi16(_mm_unpacklo_epi8(a, z), b), 1);
            a = _mm_add_epi8(ld(src + i), _mm_packus_epi16(avg, avg));
            st(dst + i, a);
        }
    } else {  // f == 4, Paeth
        for (size_t i = 0; i < n; i += BPP) {
            const __m128i b = prior ? _mm_unpacklo_epi8(ld(prior + i), z) : z;
            const __m128i a16 = _mm_unpacklo_epi8(a, z);
            // pa = |b - c|, pb = |a - c|, pc = |a + b - 2c|
            const __m128i bc = _mm_sub_epi16(b, c), ac = _mm_sub_epi16(a16, c);
            const __m128i pa = _mm_max_epi16(bc, _mm_sub_epi16(z, bc));
            const __m128i pb = _mm_max_epi16(ac, _mm_sub_epi16(z, ac));
            const __m128i s = _mm_add_epi16(bc, ac);
            const __m128i pc = _mm_max_epi16(s, _mm_sub_epi16(z, s));
            // a if pa <= pb && pa <= pc, else b if pb <= pc, else c
            const __m128i use_a = _mm_andnot_si128(_mm_or_si128(_mm_cmpgt_epi16(pa, pb), _mm_cmpgt_epi16(pa, pc)),
                                                   _mm_set1_epi16(-1));
            const __m128i use_b = _mm_andnot_si128(_mm_cmpgt_epi16(pb, pc), _mm_set1_epi16(-1));
            const __m128i bc_sel = _mm_or_si128(_mm_and_si128(use_b, b), _mm_andnot_si128(use_b, c));
            const __m128i pred = _mm_or_si128(_mm_and_si128(use_a, a16), _mm_andnot_si128(use_a, bc_sel));
            a = _mm_add_epi8(ld(src + i), _mm_packus_epi16(pred, pred));
            st(dst + i, a);
            c = b;
        }
    }
    (void)keep;
}

bool unfilter(int f, uint8_t *__restrict dst, const uint8_t *__restrict src, const uint8_t *__restrict prior, size_t n,
              int bpp) {
    switch (f) {
    case 0:
        memcpy(dst, src, n);
        return true;
    case 2:
        if (!prior) {
            memcpy(dst, src, n);
            return true;
        }
        {
            size_t i = 0;
            for (; i + 16 <= n; i += 16)
                _mm_storeu_si128((__m128i *)(dst + i), _mm_add_epi8(_mm_loadu_si128((const __m128i *)(src + i)),
                                                                    _mm_loadu_si128((const __m128i *)(prior + i))));
            for (; i < n; i++) dst[i] = (uint8_t)(src[i] + prior[i]);
        }
        return true;
    case 1:
    case 3:
    case 4:
        if (bpp == 3 && n % 3 == 0) {
            unfilter_px<3>(f, dst, src, prior, n);
            return true;
        }
        if (bpp == 4 && n % 4 == 0) {
            unfilter_px<4>(f, dst, src, prior, n);
            return true;
        }
        for (size_t i = 0; i < n; i++) {
            const int a = i >= (size_t)bpp ? dst[i - bpp] : 0, b = prior ? prior[i] : 0,
                      c = (prior && i >= (size_t)bpp) ? prior[i - bpp] : 0;
            const int pr = f == 1 ? a : (f == 3 ? (a + b) >> 1 : paeth(a, b, c));
            dst[i] = (uint8_t)(src[i] + pr);
        }
        return true;
    default:
        return false;
    }
}

// 8-bit RGB -> BGR, 16 pixels per step with SSSE3 byte shuffles (runtime-dispatched)
__attribute__((target("ssse3"))) size_t rgb_to_bgr_ssse3(const uint8_t *s, uint8_t *o, size_t w) {
    // out bytes of 16 px = in bytes with R and B swapped inside each 3-byte pixel; the
    // three 16-byte output vectors each take bytes from at most two input vectors
    const __m128i m00 = _mm_setr_epi8(2, 1, 0, 5, 4, 3, 8, 7, 6, 11, 10, 9, 14, 13, 12, -1);
    const __m128i m01 = _mm_setr_epi8(-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 1);
    const __m128i m10 = _mm_setr_epi8(-1, 15, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m128i m11 = _mm_setr_epi8(0, -1, 4, 3, 2, 7, 6, 5, 10, 9, 8, 13, 12, 11, -1, 15);
    const __m128i m12 = _mm_setr_epi8(-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, -1);
    const __m128i m21 = _mm_setr_epi8(14, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m128i m22 = _mm_setr_epi8(-1, 3, 2, 1, 6, 5, 4, 9, 8, 7, 12, 11, 10, 15, 14, 13);
    size_t x = 0;
    for (; x + 16 <= w; x += 16, s += 48, o += 48) {
        const __m128i a = _mm_loadu_si128((const __m128i *)s), b = _mm_loadu_si128((const __m128i *)(s + 16)),
                      c = _mm_loadu_si128((const __m128i *)(s + 32));
        _mm_storeu_si128((__m128i *)o, _mm_or_si128(_mm_shuffle_epi8(a, m00), _mm_shuffle_epi8(b, m01)));
        _mm_storeu_si128((__m128i *)(o + 16), _mm_or_si128(_mm_or_si128(_mm_shuffle_epi8(a, m10), _mm_shuffle_epi8(b, m11)),
                                                          _mm_shuffle_epi8(c, m12)));
        _mm_storeu_si128((__m128i *)(o + 32), _mm_or_si128(_mm_shuffle_epi8(b, m21), _mm_shuffle_epi8(c, m22)));
    }
    return x;
}

bool have_ssse3() {
    static const bool ok = __builtin_cpu_supports("ssse3");
    return ok;
}

// one unfiltered row -> BGR
void row_to_bgr(const Png &png, const uint8_t *s, uint8_t *o) {
    const uint32_t w = png.w;
    const int hb = png.depth == 16 ? 2 : 1;  // high byte first (big-endian samples)
    switch (png.ctype) {
    case 2: {
        uint32_t x = 0;
        if (hb == 1 && have_ssse3()) {
            x = (uint32_t)rgb_to_bgr_ssse3(s, o, w);
            s += 3 * (size_t)x;
            o += 3 * (size_t)x;
        }
        for (; x < w; x++, s += 3 * hb, o += 3) {
            o[0] = s[2 * hb];
            o[1] = s[hb];
            o[2] = s[0];
        }
        break;
    }
    case 6:
        for (uint32_t x = 0; x < w; x++, s += 4 * hb, o += 3) {
            o[0] = s[2 * hb];
            o[1] = s[hb];
            o[2] = s[0];
        }
        break;
    case 0:
        for (uint32_t x = 0; x < w; x++, s += hb, o += 3) o[0] = o[1] = o[2] = s[0];
        break;
    case 4:
        for (uint32_t x = 0; x < w; x++, s += 2 * hb, o += 3) o[0] = o[1] = o[2] = s[0];
        break;
    case 3:
        for (uint32_t x = 0; x < w; x++, s++, o += 3) {
            const uint32_t i = s[0];
            if (i < png.plte_n) {
                o[0] = png.plte[3 * i + 2];
                o[1] = png.plte[3 * i + 1];
                o[2] = png.plte[3 * i];
            } else {
                o[0] = o[1] = o[2] = 0;
            }
        }
        break;
    }
}

// 8-bit RGB rows unfiltered straight into the BGR output: every PNG filter is per channel
// (Sub / Avg / Paeth take the same channel of the left, upper and upper-left pixels), so it
// commutes with the R <-> B swap, and the swapped rows can be unfiltered against the previous
// BGR output row.  One pass over the row instead of unfilter + convert (round 4: the two
// were 11 % of a 1080p decode, inflate the rest).  No store passes the row's last byte: the
// row after it may be another image, decoded by another thread.
inline uint32_t rgb_bgr32(uint32_t x) { return __builtin_bswap32(x) >> 8; }  // R G B . -> B G R 0
inline void st24(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
}

__attribute__((target("ssse3"))) size_t up_bgr_ssse3(const uint8_t *s, const uint8_t *prior, uint8_t *o, size_t w) {
    const __m128i m00 = _mm_setr_epi8(2, 1, 0, 5, 4, 3, 8, 7, 6, 11, 10, 9, 14, 13, 12, -1);
    const __m128i m01 = _mm_setr_epi8(-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 1);
    const __m128i m10 = _mm_setr_epi8(-1, 15, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m128i m11 = _mm_setr_epi8(0, -1, 4, 3, 2, 7, 6, 5, 10, 9, 8, 13, 12, 11, -1, 15);
    const __m128i m12 = _mm_setr_epi8(-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0, -1);
    const __m128i m21 = _mm_setr_epi8(14, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
    const __m128i m22 = _mm_setr_epi8(-1, 3, 2, 1, 6, 5, 4, 9, 8, 7, 12, 11, 10, 15, 14, 13);
    size_t x = 0;
    const bool up = prior != nullptr;
    for (; x + 16 <= w; x += 16, s += 48, o += 48, prior += up ? 48 : 0) {
        const __m128i a = _mm_loadu_si128((const __m128i *)s), b = _mm_loadu_si128((const __m128i *)(s + 16)),
                      c = _mm_loadu_si128((const __m128i *)(s + 32));
        const __m128i o0 = _mm_or_si128(_mm_shuffle_epi8(a, m00), _mm_shuffle_epi8(b, m01));
        const __m128i o1 = _mm_or_si128(_mm_or_si128(_mm_shuffle_epi8(a, m10), _mm_shuffle_epi8(b, m11)),
                                        _mm_shuffle_epi8(c, m12));
        const __m128i o2 = _mm_or_si128(_mm_shuffle_epi8(b, m21), _mm_shuffle_epi8(c, m22));
        if (up) {
            _mm_storeu_si128((__m128i *)o, _mm_add_epi8(o0, _mm_loadu_si128((const __m128i *)prior)));
            _mm_storeu_si128((__m128i *)(o + 16), _mm_add_epi8(o1, _mm_loadu_si128((const __m128i *)(prior + 16))));
            _mm_storeu_si128((__m128i *)(o + 32), _mm_add_epi8(o2, _mm_loadu_si128((const __m128i *)(prior + 32))));
        } else {
            _mm_storeu_si128((__m128i *)o, o0);
            _mm_storeu_si128((__m128i *)(o + 16), o1);
            _mm_storeu_si128((__m128i *)(o + 32), o2);
        }
    }
    return x;
}

// src: the filtered RGB row (inflated buffer, readable 4 bytes past its end), dst: the BGR
// output row, prior: the previous BGR output row (nullptr for row 0); w >= 1 pixels.  dst is
// not __restrict: prior is the row before it in the same buffer, and the last pixel's
// 4-byte load of prior reaches dst[0] (a discarded lane, but the memory is shared).
bool unfilter_rgb_to_bgr(int f, uint8_t *dst, const uint8_t *__restrict src, const uint8_t *prior,
                         size_t w) {
    if (f < 0 || f > 4) return false;
    size_t x = 0;
    if (f == 0 || f == 2) {  // None, Up: no left dependency, 16 pixels per step
        const uint8_t *pr = f == 2 ? prior : nullptr;
        if (have_ssse3()) x = up_bgr_ssse3(src, pr, dst, w);
        for (; x < w; x++) {
            const size_t i = 3 * x;
            for (int c = 0; c < 3; c++) dst[i + c] = (uint8_t)(src[i + 2 - c] + (pr ? pr[i + c] : 0));
        }
        return true;
    }
    if (f == 1) {  // Sub: per-byte adds without carries (SWAR)
        uint32_t a = 0;
        for (; x < w; x++) {
            const uint32_t v = rgb_bgr32(ld32(src + 3 * x));
            a = ((v & 0x7f7f7f7fu) + (a & 0x7f7f7f7fu)) ^ ((v ^ a) & 0x80808080u);
            if (x + 1 < w) st32(dst + 3 * x, a);
            else st24(dst + 3 * x, a);
            a &= 0x00ffffffu;
        }
        return true;
    }
    const __m128i z = _mm_setzero_si128();
    auto ldp = [&](size_t i) {  // the previous row's pixel (4-byte load inside the image:
        // prior's row is followed by dst's)
        return prior ? _mm_unpacklo_epi8(_mm_cvtsi32_si128((int)ld32(prior + i)), z) : z;
    };
    auto put = [&](size_t xx, __m128i v) {
        const uint32_t u = (uint32_t)_mm_cvtsi128_si32(v);
        if (xx + 1 < w) st32(dst + 3 * xx, u);
        else st24(dst + 3 * xx, u);
    };
    __m128i a = z, c = z;
    if (f == 3) {
        for (; x < w; x++) {
            const __m128i b = ldp(3 * x);
            const __m128i avg = _mm_srli_epi16(_mm_add_epi16(_mm_unpacklo_epi8(a, z), b), 1);
            a = _mm_add_epi8(_mm_cvtsi32_si128((int)rgb_bgr32(ld32(src + 3 * x))), _mm_packus_epi16(avg, avg));
            put(x, a);
        }
    } else {  // Paeth
        for (; x < w; x++) {
            const __m128i b = ldp(3 * x);
            const __m128i a16 = _mm_unpacklo_epi8(a, z);
            const __m128i bc = _mm_sub_epi16(b, c), ac = _mm_sub_epi16(a16, c);
            const __m128i pa = _mm_max_epi16(bc, _mm_sub_epi16(z, bc));
            const __m128i pb = _mm_max_epi16(ac, _mm_sub_epi16(z, ac));
            const __m128i sm = _mm_add_epi16(bc, ac);
            const __m128i pc = _mm_max_epi16(sm, _mm_sub_epi16(z, sm));
            const __m128i use_a = _mm_andnot_si128(_mm_or_si128(_mm_cmpgt_epi16(pa, pb), _mm_cmpgt_epi16(pa, pc)),
                                                   _mm_set1_epi16(-1));
            const __m128i use_b = _mm_andnot_si128(_mm_cmpgt_epi16(pb, pc), _mm_set1_epi16(-1));
            const __m128i bc_sel = _mm_or_si128(_mm_and_si128(use_b, b), _mm_andnot_si128(use_b, c));
            const __m128i pred = _mm_or_si128(_mm_and_si128(use_a, a16), _mm_andnot_si128(use_a, bc_sel));
            a = _mm_add_epi8(_mm_cvtsi32_si128((int)rgb_bgr32(ld32(src + 3 * x))), _mm_packus_epi16(pred, pred));
            put(x, a);
            c = b;
        }
    }
    return true;
}

// cv2.imdecode refuses images above CV_IO_MAX_IMAGE_PIXELS (default 2^30 pixels,
// OPENCV_IO_MAX_IMAGE_PIXELS overrides): here LLFE_MAX_PIXELS, checked from the header
// before anything is allocated
uint64_t max_pixels() {
    static const uint64_t m = [] {
        const char *e = getenv("LLFE_MAX_PIXELS");
        const long long v = e ? atoll(e) : 0;
        return v > 0 ? (uint64_t)v : (uint64_t)1 << 30;
    }();
    return m;
}

// thread-local scratch above this size is released after each image, so one huge
// decode does not pin its peak allocation in every decode thread
constexpr size_t kKeepScratch = (size_t)64 << 20;

int decode_one(const uint8_t *data, size_t size, int32_t h, int32_t w, uint8_t *out) {
    Png png;
    int rc = parse(data, size, png, false);
    if (rc) return rc;
    if ((int64_t)png.h != h || (int64_t)png.w != w) return LLFE_ERR_CAPACITY;
    if ((uint64_t)png.w * png.h > max_pixels()) return LLFE_ERR_INVALID;
    const int bpp = png.channels() * png.depth / 8;
    const size_t rowb = (size_t)png.w * bpp, stride = rowb + 1, raw_n = stride * png.h;
    // a zlib stream inflates at most ~1032:1: a declared size the IDAT payload cannot
    // reach is corrupt -- rejected before the raw buffer is committed
    size_t idat_n = 0;
    for (auto &c : png.idat) idat_n += c.second;
    if (raw_n / 1032 > idat_n + 64) return LLFE_ERR_INVALID;
    thread_local std::vector<uint8_t> raw, cat, rows;
    raw.resize(raw_n + 16);       // (4-byte pixel loads read one byte past a row)
    rows.resize(2 * (rowb + 16));  // two unfiltered rows, ping-pong (this row, prior), padded
    rc = inflate_idat(png, raw.data(), raw_n, cat) ? LLFE_OK : LLFE_ERR_INVALID;
    const bool fused = png.ctype == 2 && png.depth == 8;  // RGB8: unfilter into BGR in one pass
    for (uint32_t y = 0; fused && rc == LLFE_OK && y < png.h; y++) {
        const uint8_t *r = raw.data() + y * stride;
        uint8_t *o = out + (size_t)y * png.w * 3;
        if (!unfilter_rgb_to_bgr(r[0], o, r + 1, y ? o - (size_t)png.w * 3 : nullptr, png.w)) rc = LLFE_ERR_INVALID;
    }
    for (uint32_t y = 0; !fused && rc == LLFE_OK && y < png.h; y++) {
        const uint8_t *r = raw.data() + y * stride;
        uint8_t *cur = rows.data() + (y & 1) * (rowb + 16);
        const uint8_t *prior = y ? rows.data() + ((y - 1) & 1) * (rowb + 16) : nullptr;
        if (!unfilter(r[0], cur, r + 1, prior, rowb, bpp)) rc = LLFE_ERR_INVALID;
        else row_to_bgr(png, cur, out + (size_t)y * png.w * 3);
    }
    if (raw.capacity() > kKeepScratch) std::vector<uint8_t>().swap(raw);
    if (cat.capacity() > kKeepScratch) std::vector<uint8_t>().swap(cat);
    if (rows.capacity() > kKeepScratch) std::vector<uint8_t>().swap(rows);
    return rc;
}

}  // namespace

extern "C" int llfe_png_info(const uint8_t *data, uint64_t size, int32_t *width, int32_t *height) {
    if (!data || !width || !height) return LLFE_ERR_INVALID;
    Png png;
    const int rc = parse(data, (size_t)size, png, true);
    if (rc) return rc;
    if (png.w > 0x7FFFFFFFu || png.h > 0x7FFFFFFFu) return LLFE_ERR_UNSUPPORTED;
    *width = (int32_t)png.w;
    *height = (int32_t)png.h;
    if ((uint64_t)png.w * png.h > max_pixels()) return LLFE_ERR_CAPACITY;
    return LLFE_OK;
}

// ---------------------------------------------------------------- format dispatch
int llfe_jpeg_info_one(const uint8_t *data, size_t size, int32_t *w, int32_t *h, int *ncomp);
bool llfe_jpeg_available();

extern "C" int llfe_decoder_info(char *buf, int32_t cap) {
    if (!buf || cap <= 0) return LLFE_ERR_INVALID;
    const int n = snprintf(buf, (size_t)cap, "png=%s;jpeg=%s", deflate().ok ? "libdeflate" : "zlib",
                           llfe_jpeg_available() ? "libjpeg.so.8" : "pillow");
    return n < cap ? LLFE_OK : LLFE_ERR_CAPACITY;
}
int llfe_jpeg_decode_one(const uint8_t *data, size_t size, int32_t h, int32_t w, uint8_t *out);

namespace {
constexpr uint8_t kPngSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
bool is_png(const uint8_t *d, size_t n) { return n >= 8 && !memcmp(d, kPngSig, 8); }
bool is_jpeg(const uint8_t *d, size_t n) { return n >= 3 && d[0] == 0xFF && d[1] == 0xD8 && d[2] == 0xFF; }

int decode_any(const uint8_t *d, size_t n, int32_t h, int32_t w, uint8_t *out) {
    if (is_png(d, n)) return decode_one(d, n, h, w, out);
    if (is_jpeg(d, n)) {
        if ((uint64_t)(uint32_t)w * (uint32_t)h > max_pixels()) return LLFE_ERR_INVALID;
        return llfe_jpeg_decode_one(d, n, h, w, out);
    }
    return LLFE_ERR_UNSUPPORTED;
}
}  // namespace

extern "C" int llfe_image_info(const uint8_t *data, uint64_t size, int32_t *width, int32_t *height) {
    if (!data || !width || !height) return LLFE_ERR_INVALID;
    if (is_png(data, (size_t)size)) return llfe_png_info(data, size, width, height);
    if (!is_jpeg(data, (size_t)size)) return LLFE_ERR_UNSUPPORTED;
    int nc = 0;
    const int rc = llfe_jpeg_info_one(data, (size_t)size, width, height, &nc);
    if (rc) return rc;
    if ((uint64_t)(uint32_t)*width * (uint32_t)*height > max_pixels()) return LLFE_ERR_CAPACITY;
    return LLFE_OK;
}

namespace {
template <typename F>
int decode_fanout(const uint8_t *const *data, const uint64_t *sizes, int32_t n, int32_t height, int32_t width,
                  uint8_t *out_bgr, int32_t *status, int32_t threads, F one) {
    if (n < 0 || (n && (!data || !sizes || !out_bgr || !status)) || height <= 0 || width <= 0) return LLFE_ERR_INVALID;
    const size_t img_bytes = (size_t)height * width * 3;
    const int nt = std::max(1, std::min<int>(threads > 0 ? threads : 1, n));
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int i; (i = next.fetch_add(1)) < n;) {
            int rc;
            try {
                rc = data[i] ? one(data[i], (size_t)sizes[i], height, width, out_bgr + (size_t)i * img_bytes)
                             : LLFE_ERR_INVALID;
            } catch (const std::bad_alloc &) {
                rc = LLFE_ERR_OOM;
            }
            status[i] = rc;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    for (int i = 0; i < n; i++)
        if (status[i]) return status[i];
    return LLFE_OK;
}
}  // namespace

extern "C" int llfe_decode_png_batch(const uint8_t *const *data, const uint64_t *sizes, int32_t n, int32_t height,
                                     int32_t width, uint8_t *out_bgr, int32_t *status, int32_t threads) {
    return decode_fanout(data, sizes, n, height, width, out_bgr, status, threads, decode_one);
}

extern "C" int llfe_decode_batch(const uint8_t *const *data, const uint64_t *sizes, int32_t n, int32_t height,
                                 int32_t width, uint8_t *out_bgr, int32_t *status, int32_t threads) {
    return decode_fanout(data, sizes, n, height, width, out_bgr, status, threads, decode_any);
}
