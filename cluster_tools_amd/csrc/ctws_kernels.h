// ctws_kernels.h — declarations of the gfx950 kernels (defined in k_*.hip).
#pragma once

#include "ctws_dev.h"

namespace ctws {

struct PrepParams {
    float threshold;
    int invert;
    int agg;
    int px2;
};
struct EdtColParams {
    int axis;
    int p2;
    int final_pass;
    int per_slice;
    uint32_t max_dist;
};
struct HmapParams {
    float a, b;
    int per_slice;
};
struct GaussParams {
    int axis;
    int r;
    int hmap_src;
};
struct FilterParams {
    uint32_t size_filter;
    int tz, ty, tx;  // flood tile extents: tiles holding a freed voxel are activated in act
    uint32_t* act;
};

// k_edt.hip
__global__ void k_input_minmax(const BlockDesc*, BlockStat*);
__global__ void k_prep_edt_x(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
template <int KMAX>
__global__ void k_prep_edt_x_reg(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
template <int W>
__global__ void k_edt_col(const BlockDesc*, BlockStat*, EdtColParams, const uint32_t*, uint32_t*, float*, uint32_t*,
                          uint32_t*);
__global__ void k_dt_slice_stats(const BlockDesc*, const BlockStat*, const float*, uint32_t*, uint32_t*);
__global__ void k_set_active(const BlockDesc*, BlockStat*, int);

// k_gauss.hip
__global__ void k_hmap(const BlockDesc*, const BlockStat*, HmapParams, const float*, const float*, const uint32_t*,
                       const uint32_t*, float*);
template <int W>
__global__ void k_gauss_col(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                            const float*, const uint32_t*, const uint32_t*, float*);
__global__ void k_gauss_row(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                            const float*, const uint32_t*, const uint32_t*, float*);
constexpr int kGaussMaxR = 12;  // sliding-window kernels for radius <= 12 (sigma < 4)
template <int W, int R>
__global__ void k_gauss_col_r(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                              const float*, const uint32_t*, const uint32_t*, float*);
template <int R>
__global__ void k_gauss_row_r(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                              const float*, const uint32_t*, const uint32_t*, float*);

// k_cc.hip
__global__ void k_localmax(const BlockDesc*, BlockStat*, const float*, uint8_t*, uint32_t*);
__global__ void k_plateau_union(const BlockDesc*, const BlockStat*, const float*, const uint8_t*, uint32_t*);
__global__ void k_plateau_flag(const BlockDesc*, const BlockStat*, uint8_t*, uint32_t*);
__global__ void k_seed_init(const BlockDesc*, const BlockStat*, const uint8_t*, const uint32_t*, uint32_t*);
__global__ void k_seed_union(const BlockDesc*, const BlockStat*, uint32_t*);
__global__ void k_flatten_roots(const BlockDesc*, const BlockStat*, int, uint32_t*, uint64_t*);
__global__ void k_bitmap_csum(const BlockDesc*, const BlockStat*, int, const uint64_t*, uint32_t*);
__global__ void k_chunk_scan(const BlockDesc*, BlockStat*, int, uint32_t*, int);
__global__ void k_word_prefix(const BlockDesc*, const BlockStat*, int, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_root_label(const BlockDesc*, const BlockStat*, int, uint32_t*, const uint64_t*, const uint32_t*);
__global__ void k_seed_label(const BlockDesc*, const BlockStat*, const uint32_t*, const float*, uint32_t*, uint64_t*,
                             uint8_t*, int);
__global__ void k_crop_init(const BlockDesc*, const BlockStat*, const uint32_t*, uint32_t*);
__global__ void k_crop_union(const BlockDesc*, const BlockStat*, const uint32_t*, uint32_t*);
__global__ void k_output(const BlockDesc*, BlockStat*, const uint32_t*, const uint32_t*, int, const uint64_t*, int,
                         const uint32_t*, const uint32_t*);

// k_flood.hip
template <int ND>
__global__ void k_flood(const BlockDesc*, const BlockStat*, const float*, uint64_t*, uint32_t*, const uint32_t*,
                        uint32_t*, uint32_t*);

template <int ND>
__global__ void k_flood_packed(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint8_t*,
                               const uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*);
constexpr int kLineWords = 24;
constexpr int kStatSlots = 64;  // flood statistics: counter[4 + slot * 4 + k]  // per tile: 8 words of line bits for each of x, y, z
__global__ void k_unpack_labels(const BlockDesc*, const BlockStat*, const uint64_t*, uint32_t*);
template <int ND>
__global__ void k_descent_tile(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, const uint32_t*,
                               uint32_t*);
__global__ void k_descent_init(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, uint64_t*, uint8_t*,
                               uint64_t*, uint64_t*, uint32_t*);
template <int ND, int U>
__global__ void k_frontier(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint64_t*,
                           const uint64_t*, uint64_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*, int);
__global__ void k_frontier_tiles(const BlockDesc*, const BlockStat*, const uint64_t*, uint32_t*, int, int, int);
template <int ND>
__global__ void k_flood_verify(const BlockDesc*, const BlockStat*, const float*, const uint64_t*, const uint32_t*,
                               const uint32_t*, uint32_t*);
__global__ void k_flood_reset(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, const uint32_t*,
                              uint64_t*, uint8_t*);

// k_post.hip
__global__ void k_slice_seed_base(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_hist_zero(const BlockDesc*, const BlockStat*, uint32_t*);
__global__ void k_hist(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, int, uint32_t*, int);
constexpr int kHistBins = 16384;  // largest LDS histogram of k_hist
__global__ void k_size_filter(const BlockDesc*, const BlockStat*, FilterParams, const uint32_t*, const uint8_t*,
                              const float*, uint32_t*, uint64_t*, uint8_t*, uint32_t*, int);
__global__ void k_slice_max(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, int, const uint32_t*,
                            uint32_t*);
__global__ void k_slice_offsets(const BlockDesc*, const BlockStat*, const uint32_t*, uint32_t*);
__global__ void k_finalize_ws(const BlockDesc*, const BlockStat*, const uint32_t*, const uint32_t*, const uint64_t*, int,
                              uint32_t*);

// k_pass2.hip (two-pass watershed, pass 2)
__global__ void k_p2_zero_dt(const BlockDesc*, const BlockStat*, float*);
__global__ void k_p2_values(const BlockDesc*, const BlockStat*, const uint32_t*, const uint32_t*, uint64_t*);
__global__ void k_p2_insert(const BlockDesc*, const BlockStat*, const uint64_t*, uint64_t*, uint32_t*, uint32_t*);
__global__ void k_p2_roots(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint64_t*);
__global__ void k_p2_label(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, const uint64_t*,
                           const uint32_t*, const float*, uint32_t*, uint64_t*, uint8_t*, uint32_t*, uint32_t*, int);
__global__ void k_p2_excl_zero(const BlockDesc*, const BlockStat*, uint8_t*);
__global__ void k_p2_excl(const BlockDesc*, const BlockStat*, const uint32_t*, uint8_t*);
__global__ void k_p2_check(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_p2_output(const BlockDesc*, BlockStat*, const uint32_t*, const uint32_t*, const uint32_t*,
                            const uint32_t*);
__global__ void k_slice_inmask(const BlockDesc*, const BlockStat*, uint32_t*);

}  // namespace ctws
