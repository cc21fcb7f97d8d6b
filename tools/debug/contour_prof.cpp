// Host profile of the contour pass on a dilated Canny mask (h x w u8 file): bit packing,
// expansion + raster scan + border following, and the shape geometry.
//   tools/debug/contour_prof mask.bin h w [reps]
#include "../../low_level_feature_extraction_amd/csrc/contours.cpp"

#include <chrono>
#include <cstdio>
#include <fstream>
#include <iterator>

int main(int argc, char **argv) {
    std::ifstream f(argv[1], std::ios::binary);
    std::vector<uint8_t> m((std::istreambuf_iterator<char>(f)), {});
    const int h = atoi(argv[2]), w = atoi(argv[3]), reps = argc > 4 ? atoi(argv[4]) : 20;
    const int wpr = (w + 63) / 64;
    std::vector<uint64_t> bits((size_t)h * wpr, 0);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            if (m[(size_t)y * w + x]) bits[(size_t)y * wpr + (x >> 6)] |= 1ull << (x & 63);
    std::vector<int8_t> work;
    llfe::Contours c;
    llfe::ShapeScratch sc;
    std::vector<llfe_shape> shapes;
    using C = std::chrono::steady_clock;
    double t_trace = 1e30, t_geo = 1e30;  // min over reps (shared, noisy host)
    for (int r = 0; r < reps; r++) {
        auto a = C::now();
        llfe::external_contours_bits(bits.data(), h, w, wpr, work, c);
        auto b = C::now();
        llfe::shapes_from_contours(c, sc, shapes);
        auto e = C::now();
        t_trace = std::min(t_trace, std::chrono::duration<double, std::milli>(b - a).count());
        t_geo = std::min(t_geo, std::chrono::duration<double, std::milli>(e - b).count());
    }
    size_t nv = c.xy.size() / 2;
    printf("%s: contours %zu vertices %zu shapes %zu | expand+scan+trace %.3f ms   geometry %.3f ms (min of reps)\n",
           argv[1], c.start.size() - 1, nv, shapes.size(), t_trace, t_geo);
}
