// Host-side contour structures shared by contours.cpp and llfe_api.cpp.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/llfe.h"

namespace llfe {

struct Contours {
    std::vector<int32_t> xy;     // x,y pairs in raster discovery order
    std::vector<int64_t> start;  // first point of each contour (+ end sentinel)
};

struct ShapeScratch {
    std::vector<int32_t> dp;
    std::vector<int> stack;
    std::vector<int64_t> t0, t1;
};

void external_contours_u8(const uint8_t *mask, int h, int w, std::vector<int8_t> &work, Contours &out);
void external_contours_bits(const uint64_t *bits, int h, int w, int wpr, std::vector<int8_t> &work, Contours &out);
bool classify_contour(const int32_t *p, int n, ShapeScratch &sc, llfe_shape &out);
double border_radius(const int32_t *p, int n, double epsilon_factor, ShapeScratch &sc);
int shapes_from_contours(const Contours &c, ShapeScratch &sc, std::vector<llfe_shape> &out);

}  // namespace llfe
