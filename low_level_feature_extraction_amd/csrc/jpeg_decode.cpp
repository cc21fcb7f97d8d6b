// Host JPEG decoding for the decode step in front of the hot path: cv2.imdecode(buf,
// IMREAD_COLOR) at app/services/analyze/utils.py:108-109 and
// app/services/analyze/image_processor.py:208-211.
//
// OpenCV decodes JPEG with libjpeg(-turbo): default (ISLOW) IDCT, fancy upsampling,
// output colour space JCS_EXT_BGR for 1- and 3-component images (grfmt_jpeg.cpp
// JpegDecoder::readData), so the BGR bytes are libjpeg's own colour conversion.  This
// file drives the system libjpeg-turbo (libjpeg.so.8, the same codec family OpenCV
// and Pillow bundle) through dlopen -- no headers are installed in the image, so the
// few API types used are declared below for the JPEG_LIB_VERSION 80 ABI.
// jpeg_CreateDecompress checks the struct size against the library's own, so a
// layout mismatch is reported as LLFE_ERR_UNSUPPORTED (the caller then falls back to
// Pillow), never as corrupted memory.
//
// Cases handed back to the caller (LLFE_ERR_UNSUPPORTED): 4-component (CMYK / YCCK)
// images (OpenCV converts those with its own CMYK formula) and images with an EXIF
// orientation other than 1 (imdecode applies the rotation; decode.py does it with
// Pillow's exif_transpose).  Corrupt data that libjpeg rejects is LLFE_ERR_INVALID.
#include <dlfcn.h>
#include <setjmp.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "llfe.h"

namespace llfe_jpeg {

typedef int jboolean;  // libjpeg's `boolean`
typedef unsigned int JDIMENSION;
constexpr int kJpegLibVersion = 80;
constexpr int JCS_GRAYSCALE = 1, JCS_RGB = 2, JCS_YCbCr = 3, JCS_EXT_BGR = 8;

struct ErrorMgr {  // struct jpeg_error_mgr
    void (*error_exit)(void *cinfo);
    void (*emit_message)(void *cinfo, int msg_level);
    void (*output_message)(void *cinfo);
    void (*format_message)(void *cinfo, char *buffer);
    void (*reset_error_mgr)(void *cinfo);
    int msg_code;
    union {
        int i[8];
        char s[80];
    } msg_parm;
    int trace_level;
    long num_warnings;
    const char *const *jpeg_message_table;
    int last_jpeg_message;
    const char *const *addon_message_table;
    int first_addon_message;
    int last_addon_message;
};

struct Decompress {  // struct jpeg_decompress_struct, JPEG_LIB_VERSION 80
    ErrorMgr *err;
    void *mem, *progress, *client_data;
    jboolean is_decompressor;
    int global_state;
    void *src;
    JDIMENSION image_width, image_height;
    int num_components, jpeg_color_space, out_color_space;
    unsigned int scale_num, scale_denom;
    double output_gamma;
    jboolean buffered_image, raw_data_out;
    int dct_method;
    jboolean do_fancy_upsampling, do_block_smoothing, quantize_colors;
    int dither_mode;
    jboolean two_pass_quantize;
    int desired_number_of_colors;
    jboolean enable_1pass_quant, enable_external_quant, enable_2pass_quant;
    JDIMENSION output_width, output_height;
    int out_color_components, output_components, rec_outbuf_height, actual_number_of_colors;
    void *colormap;
    JDIMENSION output_scanline;
    int input_scan_number;
    JDIMENSION input_iMCU_row;
    int output_scan_number;
    JDIMENSION output_iMCU_row;
    void *coef_bits;
    void *quant_tbl_ptrs[4], *dc_huff_tbl_ptrs[4], *ac_huff_tbl_ptrs[4];
    int data_precision;
    void *comp_info;
    jboolean is_baseline, progressive_mode, arith_code;
    uint8_t arith_dc_L[16], arith_dc_U[16], arith_ac_K[16];
    unsigned int restart_interval;
    jboolean saw_JFIF_marker;
    uint8_t JFIF_major_version, JFIF_minor_version, density_unit;
    uint16_t X_density, Y_density;
    jboolean saw_Adobe_marker;
    uint8_t Adobe_transform;
    jboolean CCIR601_sampling;
    void *marker_list;
    int max_h_samp_factor, max_v_samp_factor, min_DCT_h_scaled_size, min_DCT_v_scaled_size;
    JDIMENSION total_iMCU_rows;
    void *sample_range_limit;
    int comps_in_scan;
    void *cur_comp_info[4];
    JDIMENSION MCUs_per_row, MCU_rows_in_scan;
    int blocks_in_MCU;
    int MCU_membership[10];
    int Ss, Se, Ah, Al;
    int block_size;
    const int *natural_order;
    int lim_Se;
    int unread_marker;
    void *master, *main, *coef, *post, *inputctl, *marker, *entropy, *idct, *upsample, *cconvert, *cquantize;
};

struct Api {
    ErrorMgr *(*std_error)(ErrorMgr *) = nullptr;
    void (*create)(Decompress *, int, size_t) = nullptr;
    void (*destroy)(Decompress *) = nullptr;
    void (*mem_src)(Decompress *, const unsigned char *, unsigned long) = nullptr;
    int (*read_header)(Decompress *, jboolean) = nullptr;
    jboolean (*start)(Decompress *) = nullptr;
    JDIMENSION (*read_scanlines)(Decompress *, uint8_t **, JDIMENSION) = nullptr;
    jboolean (*finish)(Decompress *) = nullptr;
    bool ok = false;
    Api() {
        if (const char *off = getenv("LLFE_NO_LIBJPEG"); off && *off == '1') return;
        void *h = dlopen("libjpeg.so.8", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        std_error = (ErrorMgr * (*)(ErrorMgr *)) dlsym(h, "jpeg_std_error");
        create = (void (*)(Decompress *, int, size_t))dlsym(h, "jpeg_CreateDecompress");
        destroy = (void (*)(Decompress *))dlsym(h, "jpeg_destroy_decompress");
        mem_src = (void (*)(Decompress *, const unsigned char *, unsigned long))dlsym(h, "jpeg_mem_src");
        read_header = (int (*)(Decompress *, jboolean))dlsym(h, "jpeg_read_header");
        start = (jboolean(*)(Decompress *))dlsym(h, "jpeg_start_decompress");
        read_scanlines = (JDIMENSION(*)(Decompress *, uint8_t **, JDIMENSION))dlsym(h, "jpeg_read_scanlines");
        finish = (jboolean(*)(Decompress *))dlsym(h, "jpeg_finish_decompress");
        ok = std_error && create && destroy && mem_src && read_header && start && read_scanlines && finish;
        if (ok) ok = abi_matches();
    }
    // jpeg_CreateDecompress rejects a JPEG_LIB_VERSION or struct size that differs from
    // the library's own (JERR_BAD_LIB_VERSION / JERR_BAD_STRUCT_SIZE): probed once, so a
    // mismatch disables this decoder instead of failing every image as "corrupt"
    bool abi_matches();
};
const Api &api() {
    static Api a;
    return a;
}

struct Err {
    ErrorMgr mgr;
    char pad[256];  // slack in case the library's error manager is larger than declared
    jmp_buf jb;
    int code;
};

void on_error(void *cinfo) {
    Err *e = (Err *)((Decompress *)cinfo)->err;
    e->code = LLFE_ERR_INVALID;
    longjmp(e->jb, 1);
}
void on_output(void *) {}  // warnings (e.g. "Corrupt JPEG data: premature end") are not errors

bool Api::abi_matches() {
    Decompress ci;
    Err err;
    memset(&ci, 0, sizeof ci);
    ci.err = std_error(&err.mgr);
    err.mgr.error_exit = on_error;
    err.mgr.output_message = on_output;
    if (setjmp(err.jb)) return false;
    create(&ci, kJpegLibVersion, sizeof(Decompress));
    destroy(&ci);
    return true;
}

inline uint16_t rd16(const uint8_t *p, bool le) { return le ? (uint16_t)(p[0] | p[1] << 8) : (uint16_t)(p[0] << 8 | p[1]); }
inline uint32_t rd32(const uint8_t *p, bool le) {
    return le ? (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24
              : (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}

// EXIF orientation (tag 0x0112 of IFD0 in the first APP1 "Exif" segment), 1 if absent
int exif_orientation(const uint8_t *d, size_t n) {
    size_t p = 2;
    while (p + 4 <= n && d[p] == 0xFF) {
        const uint8_t m = d[p + 1];
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) {
            p += 2;
            continue;
        }
        if (m == 0xDA || m == 0xD9) break;  // SOS / EOI: no more header segments
        const size_t len = (size_t)d[p + 2] << 8 | d[p + 3];
        if (len < 2 || p + 2 + len > n) break;
        const uint8_t *s = d + p + 4;
        const size_t sl = len - 2;
        if (m == 0xE1 && sl >= 14 && !memcmp(s, "Exif\0\0", 6)) {
            const uint8_t *t = s + 6;
            const size_t tl = sl - 6;
            const bool le = t[0] == 'I';
            if (!(t[0] == t[1] && (t[0] == 'I' || t[0] == 'M'))) return 1;
            const uint32_t ifd = rd32(t + 4, le);
            if ((size_t)ifd + 2 > tl) return 1;
            const int cnt = rd16(t + ifd, le);
            for (int k = 0; k < cnt; k++) {
                const size_t e = (size_t)ifd + 2 + 12 * (size_t)k;
                if (e + 12 > tl) break;
                if (rd16(t + e, le) == 0x0112) return rd16(t + e + 8, le);
            }
            return 1;
        }
        p += 2 + len;
    }
    return 1;
}

// header only (sizes); returns LLFE_OK / error code
int info(const uint8_t *data, size_t size, int32_t *w, int32_t *h, int *ncomp) {
    const Api &A = api();
    if (!A.ok) return LLFE_ERR_UNSUPPORTED;
    Decompress ci;
    Err err;
    memset(&ci, 0, sizeof ci);
    ci.err = A.std_error(&err.mgr);
    err.mgr.error_exit = on_error;
    err.mgr.output_message = on_output;
    err.code = 0;
    if (setjmp(err.jb)) {
        A.destroy(&ci);
        return err.code;
    }
    A.create(&ci, kJpegLibVersion, sizeof(Decompress));
    A.mem_src(&ci, data, (unsigned long)size);
    A.read_header(&ci, 1);
    *w = (int32_t)ci.image_width;
    *h = (int32_t)ci.image_height;
    *ncomp = ci.num_components;
    A.destroy(&ci);
    return LLFE_OK;
}

// full decode into out (h x w x 3 BGR); `rows` is caller scratch for row pointers
int decode(const uint8_t *data, size_t size, int32_t h, int32_t w, uint8_t *out, std::vector<uint8_t *> &rows) {
    const Api &A = api();
    if (!A.ok) return LLFE_ERR_UNSUPPORTED;
    if (exif_orientation(data, size) != 1) return LLFE_ERR_UNSUPPORTED;
    rows.resize((size_t)h);
    for (int32_t y = 0; y < h; y++) rows[(size_t)y] = out + (size_t)y * w * 3;
    uint8_t **rp = rows.data();
    Decompress ci;
    Err err;
    memset(&ci, 0, sizeof ci);
    ci.err = A.std_error(&err.mgr);
    err.mgr.error_exit = on_error;
    err.mgr.output_message = on_output;
    err.code = 0;
    volatile int rc = LLFE_OK;
    if (setjmp(err.jb)) {
        A.destroy(&ci);
        return err.code;
    }
    A.create(&ci, kJpegLibVersion, sizeof(Decompress));
    A.mem_src(&ci, data, (unsigned long)size);
    A.read_header(&ci, 1);
    if (ci.num_components != 1 && ci.num_components != 3) {
        rc = LLFE_ERR_UNSUPPORTED;
    } else if ((int32_t)ci.image_width != w || (int32_t)ci.image_height != h) {
        rc = LLFE_ERR_CAPACITY;
    } else {
        ci.out_color_space = JCS_EXT_BGR;  // grfmt_jpeg.cpp: JCS_EXT_BGR, 3 components
        ci.out_color_components = 3;
        A.start(&ci);
        if ((int32_t)ci.output_width != w || (int32_t)ci.output_height != h || ci.output_components != 3) {
            rc = LLFE_ERR_UNSUPPORTED;
        } else {
            while (ci.output_scanline < ci.output_height) {
                const JDIMENSION before = ci.output_scanline;
                A.read_scanlines(&ci, rp + before, ci.output_height - before);
                if (ci.output_scanline == before) break;
            }
            A.finish(&ci);
        }
    }
    A.destroy(&ci);
    return rc;
}

}  // namespace llfe_jpeg

// used by png_decode.cpp's format-dispatching batch decoder
bool llfe_jpeg_available() { return llfe_jpeg::api().ok; }

int llfe_jpeg_info_one(const uint8_t *data, size_t size, int32_t *w, int32_t *h, int *ncomp) {
    return llfe_jpeg::info(data, size, w, h, ncomp);
}
int llfe_jpeg_decode_one(const uint8_t *data, size_t size, int32_t h, int32_t w, uint8_t *out) {
    thread_local std::vector<uint8_t *> rows;
    const int rc = llfe_jpeg::decode(data, size, h, w, out, rows);
    if (rows.capacity() > (1u << 16)) std::vector<uint8_t *>().swap(rows);
    return rc;
}
