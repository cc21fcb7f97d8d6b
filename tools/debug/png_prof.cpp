// Host profile of the native PNG decoder's phases (inflate / unfilter / BGR convert) on
// one file, single thread: tools/debug/png_prof <file.png> [reps]
#include "../../low_level_feature_extraction_amd/csrc/png_decode.cpp"

#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>

int main(int argc, char **argv) {
    std::ifstream f(argv[1], std::ios::binary);
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), {});
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    Png png;
    if (parse(d.data(), d.size(), png, false)) return 1;
    const int bpp = png.channels() * png.depth / 8;
    const size_t rowb = (size_t)png.w * bpp, stride = rowb + 1, raw_n = stride * png.h;
    std::vector<uint8_t> raw(raw_n + 16), cat, out((size_t)png.w * png.h * 3), un(raw_n + 16);
    int hist[5] = {0};
    double tf[5] = {0};
    double t_inf = 0, t_unf = 0, t_cvt = 0, t_all = 0, t_fus = 0;
    using C = std::chrono::steady_clock;
    for (int r = 0; r < reps; r++) {
        auto a = C::now();
        inflate_idat(png, raw.data(), raw_n, cat);
        auto b = C::now();
        for (uint32_t y = 0; y < png.h; y++) {
            uint8_t *row = raw.data() + y * stride;
            if (r == 0 && row[0] < 5) hist[row[0]]++;
            auto q0 = C::now();
            unfilter(row[0], un.data() + y * stride, row + 1, y ? un.data() + (y - 1) * stride : nullptr, rowb, bpp);
            if (row[0] < 5) tf[row[0]] += std::chrono::duration<double, std::milli>(C::now() - q0).count();
        }
        auto c = C::now();
        for (uint32_t y = 0; y < png.h; y++) row_to_bgr(png, un.data() + y * stride, out.data() + (size_t)y * png.w * 3);
        auto e = C::now();
        decode_one(d.data(), d.size(), png.h, png.w, out.data());
        auto g = C::now();
        if (png.ctype == 2 && png.depth == 8)
            for (uint32_t y = 0; y < png.h; y++) {
                uint8_t *o = out.data() + (size_t)y * png.w * 3;
                unfilter_rgb_to_bgr(raw[y * stride], o, raw.data() + y * stride + 1, y ? o - (size_t)png.w * 3 : nullptr, png.w);
            }
        t_fus += std::chrono::duration<double, std::milli>(C::now() - g).count();
        t_inf += std::chrono::duration<double, std::milli>(b - a).count();
        t_unf += std::chrono::duration<double, std::milli>(c - b).count();
        t_cvt += std::chrono::duration<double, std::milli>(e - c).count();
        t_all += std::chrono::duration<double, std::milli>(g - e).count();
    }
    printf("%s %ux%u ctype %d bytes %zu libdeflate %d | inflate %.2f ms unfilter %.2f ms convert %.2f ms | decode_one %.2f ms | filters none/sub/up/avg/paeth %d/%d/%d/%d/%d\n",
           argv[1], png.w, png.h, png.ctype, d.size(), (int)deflate().ok, t_inf / reps, t_unf / reps, t_cvt / reps,
           t_all / reps, hist[0], hist[1], hist[2], hist[3], hist[4]);
    printf("  fused unfilter + convert (RGB8) %.2f ms\n", t_fus / reps);
    printf("  per filter ms: none %.2f sub %.2f up %.2f avg %.2f paeth %.2f\n", tf[0] / reps, tf[1] / reps, tf[2] / reps, tf[3] / reps, tf[4] / reps);
}
