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
struct EdtRealParams {
    double pitch[3];
    int per_slice;  // 2-D dt: per-slice lines (y, x), dmax = Y^2 + X^2
    int real;       // 1: non-integer pitch (double temporary, maxDist = dmax); 0: float, ceil(dmax)
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
template <int KMAX, class T>
__global__ void k_prep_edt_x_co(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
template <class T>
__global__ void k_input_minmax_t(const BlockDesc*, BlockStat*);
constexpr int kEdtSearchCap = 48;  // bounded-search steps before a column goes to k_edt_col_fh
template <int W>
__global__ void k_edt_col(const BlockDesc*, BlockStat*, EdtColParams, const uint32_t*, uint32_t*, float*, uint32_t*,
                          uint32_t*, unsigned long long*, uint32_t*);
__global__ void k_sqrt_int_check(uint32_t, uint32_t, float*);
__global__ void k_edt_col_fh(const BlockDesc*, BlockStat*, EdtColParams, const uint32_t*, uint32_t*, float*, uint32_t*,
                             uint32_t*, const unsigned long long*, const uint32_t*);
template <class T>
__global__ void k_edt_real_init(const BlockDesc*, const BlockStat*, EdtRealParams, const uint32_t*, T*);
template <class T>
__global__ void k_edt_real_line(const BlockDesc*, const BlockStat*, int, EdtRealParams, int, T*, char*, int);
template <class T>
__global__ void k_edt_real_final(const BlockDesc*, BlockStat*, EdtRealParams, const T*, float*, uint32_t*, uint32_t*);
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
constexpr int kTapSlot = 4096;  // doubles per taps slot: radius <= 2047
constexpr int kGaussMaxR = 12;  // sliding-window kernels for radius <= 12 (sigma < 4)
template <int W, int R>
__global__ void k_gauss_col_r(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                              const float*, const uint32_t*, const uint32_t*, float*);
template <int R>
__global__ void k_gauss_row_r(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*, const float*,
                              const float*, const uint32_t*, const uint32_t*, float*);
// fused y + x passes on 2-D tiles: kGaussYxTY rows x (128 - 2R) columns per workgroup (the x pass
// maps 8 threads to each of the 32 rows)
constexpr int kGaussYxTY = 32;
template <int R>
__global__ void k_gauss_yx(const BlockDesc*, const BlockStat*, int, HmapParams, const double*, const double*,
                           const float*, const float*, const uint32_t*, const uint32_t*, float*);

// k_cc.hip
__global__ void k_localmax(const BlockDesc*, BlockStat*, const float*, uint8_t*, const uint32_t*, uint32_t*);
__global__ void k_plateau_flag(const BlockDesc*, const BlockStat*, uint8_t*, uint32_t*);
__global__ void k_flatten_tile_roots(const BlockDesc*, const BlockStat*, uint32_t*, const uint64_t*, uint64_t*);
__global__ void k_flatten_seeds(const BlockDesc*, const BlockStat*, uint32_t*, const uint64_t*, uint64_t*);
template <int ND>
__global__ void k_seed_members(const BlockDesc*, BlockStat*, const uint8_t*, const uint32_t*, uint32_t*, uint64_t*,
                               uint32_t*);
__global__ void k_seed_union2(const BlockDesc*, const BlockStat*, const uint8_t*, const uint32_t*, const uint32_t*,
                              uint32_t*);

// k_plateau.hip: the flood across a masked block's plateau (entries + min-plus run scans)
__global__ void k_plat_mark(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, uint64_t*, uint64_t*);
template <int ND>
__global__ void k_plat_entry(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint64_t*,
                             const uint32_t*);
__global__ void k_plat_scan_x(const BlockDesc*, const BlockStat*, uint64_t*, const uint64_t*, const uint32_t*);
template <int AX>
__global__ void k_plat_scan_col(const BlockDesc*, const BlockStat*, uint64_t*, const uint64_t*, const uint32_t*);
__global__ void k_plat_restore(const BlockDesc*, const BlockStat*, uint64_t*, const uint64_t*, uint64_t*);
__global__ void k_bitmap_csum(const BlockDesc*, const BlockStat*, int, const uint64_t*, uint32_t*);
__global__ void k_chunk_scan(const BlockDesc*, BlockStat*, int, uint32_t*, int);
__global__ void k_word_prefix(const BlockDesc*, const BlockStat*, int, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_root_label(const BlockDesc*, const BlockStat*, int, uint32_t*, const uint64_t*, const uint32_t*,
                             uint32_t*);
__global__ void k_seed_label(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, const float*,
                             uint32_t*, uint64_t*, uint8_t*, int);
__global__ void k_output(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*, int, const uint32_t*,
                         const uint32_t*, const uint32_t*, unsigned long long*, int);
__global__ void k_count_ids(const BlockDesc*, BlockStat*, const uint64_t*);

// k_tilecc.hip: LDS block-based union-find (plateaus, seed CC, halo-crop CC)
enum CcMode { CC_PLATEAU = 0, CC_SEED = 1, CC_CROP = 2 };
struct CcArgs {
    const float* v;        // PLATEAU: seed map
    const uint8_t* cls;    // PLATEAU / SEED: local-max classes (k_localmax)
    const uint32_t* Pp;    // SEED: plateau parents (is_max)
    const uint32_t* lab;   // CROP: flood labels (non-packed)
    const uint64_t* key;   // CROP: packed keys
    int packed;            // CROP
    uint64_t* troot;       // CROP: tile-root bitmap (inner C index, per block at fbase), zeroed;
                           // SEED: the members (seed voxels; outer rows), zeroed.  The seed forest's
                           // parents are written for members only: readers test this bitmap first
    uint64_t* xface;       // CROP: per tile, its low and high x columns as (root << 32 | label)
                           // (k_tile_cc writes, k_tile_merge's x face reads; per block at xcbase)
    const uint32_t* ptile; // PLATEAU: per tile, nonzero if it holds a plateau voxel (k_localmax;
                           // per block at ptbase)
};
template <int ND>
struct CcTile;
template <>
struct CcTile<3> {
    static constexpr int TZ = 4, TY = 16, TX = 32;
};
template <>
struct CcTile<2> {
    static constexpr int TZ = 1, TY = 32, TX = 64;
};
// the tile of one CC mode: 3-D plateau / seed CC in 8-deep tiles (half the z faces of
// k_tile_merge: config 4's seeds stage 11.98 -> 11.29 ms); the crop CC keeps 4-deep tiles
// (its k_tile_cc at 8 deep: 5.6 -> 7.7 ms per step, more than the merge saves)
template <int ND, int MODE>
struct CcTileM : CcTile<ND> {};
template <>
struct CcTileM<3, CC_PLATEAU> {
    static constexpr int TZ = 8, TY = 16, TX = 32;
};
template <>
struct CcTileM<3, CC_SEED> : CcTileM<3, CC_PLATEAU> {};
template <int ND, int MODE>
__global__ void k_tile_cc(const BlockDesc*, const BlockStat*, CcArgs, uint32_t*);
template <int ND>
__global__ void k_output_crop(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*);
template <int ND, int MODE>
__global__ void k_tile_merge(const BlockDesc*, const BlockStat*, CcArgs, uint32_t*);

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
                               const uint64_t*, uint32_t*);
template <int U>
__global__ void k_descent_init(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, uint64_t*, uint8_t*,
                               uint64_t*, uint64_t*, uint32_t*, uint32_t*);
template <int ND, int CW, int CY, int CZ>
__global__ void k_frontier(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint64_t*,
                           const uint64_t*, uint64_t*, const uint32_t*, uint32_t*, int, const uint32_t*,
                           const uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, int, int);
// k_eval.hip (VI / Rand contingency table)
__global__ void k_eval_add(const uint64_t*, const uint64_t*, int64_t, int, uint64_t*, unsigned long long*, int64_t,
                           uint64_t*, unsigned long long*, int64_t, uint64_t*, unsigned long long*, int64_t,
                           unsigned long long*);
__global__ void k_eval_reduce(const uint64_t*, const unsigned long long*, int64_t, const uint64_t*,
                              const unsigned long long*, int64_t, const uint64_t*, const unsigned long long*, int64_t,
                              const unsigned long long*, double*);
// k_seeded.hip (WatershedFromSeeds)
__global__ void k_fs_active(const BlockDesc*, BlockStat*, int);
__global__ void k_fs_insert(const BlockDesc*, BlockStat*, uint64_t*);
__global__ void k_fs_collect(const BlockDesc*, BlockStat*, const uint64_t*, uint32_t*);
__global__ void k_fs_offsets(const BlockDesc*, const BlockStat*, int, int*, int*);
__global__ void k_fs_rank(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_fs_label(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, const float*, uint32_t*,
                           uint64_t*, uint8_t*, int);
__global__ void k_fs_auto_label(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*, const uint32_t*,
                                const float*, uint32_t*, uint64_t*, uint8_t*, int);
__global__ void k_fs_output(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*, int, const uint32_t*,
                            const uint32_t*, int);
hipError_t fs_segmented_sort(void* tmp, size_t& bytes, const uint32_t* in, uint32_t* out, int n, int nseg,
                             const int* beg, const int* end, hipStream_t stream);
// per-chunk arrays (generations, queued marks) are indexed at fbase >> kChunkShift: a block's
// frontier words hold at least 2^kChunkShift words per chunk (every brick is 64 words)
constexpr int kChunkShift = 6;
template <int CW, int CY, int CZ>
__global__ void k_frontier_list0(const BlockDesc*, const BlockStat*, const uint64_t*, uint32_t*, uint32_t*);
__global__ void k_frontier_tiles(const BlockDesc*, const BlockStat*, const uint64_t*, uint32_t*, int, int, int);
template <int ND>
__global__ void k_flood_verify(const BlockDesc*, const BlockStat*, const float*, const uint64_t*, const uint64_t*,
                               uint32_t*);
constexpr int kWordWaves = 4;  // waves per workgroup of the word-tiled kernels
__global__ void k_flood_reset(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, const uint32_t*,
                              const uint64_t*, uint64_t*, uint8_t*);

// k_post.hip
__global__ void k_slice_seed_base(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint32_t*);
__global__ void k_hist_zero(const BlockDesc*, const BlockStat*, uint32_t*);
template <int PACKED>
__global__ void k_hist(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, uint32_t*, int);
constexpr int kHistBins = 16384;  // largest LDS histogram of k_hist
__global__ void k_size_filter(const BlockDesc*, const BlockStat*, FilterParams, const uint32_t*, const uint8_t*,
                              const float*, uint32_t*, uint64_t*, uint8_t*, uint32_t*, int);
__global__ void k_slice_max(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, int, const uint32_t*,
                            uint32_t*, int, int);
template <int PACKED>
__global__ void k_hist2d(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, const uint32_t*,
                         uint32_t*, int);
__global__ void k_sf_plan(const BlockDesc*, BlockStat*, uint32_t, const uint32_t*, const uint8_t*, const uint32_t*,
                          uint32_t*);
__global__ void k_sf_sparse(const BlockDesc*, const BlockStat*, uint32_t, const uint32_t*, const uint8_t*,
                            const uint32_t*, const float*, uint64_t*, uint8_t*, uint64_t*, uint64_t*);
__global__ void k_fixed_from_open(const BlockDesc*, const BlockStat*, const uint64_t*, uint8_t*);
template <int U>
__global__ void k_regrow_init(const BlockDesc*, const BlockStat*, uint32_t, const uint32_t*, const uint8_t*,
                              const float*, uint64_t*, uint8_t*, uint64_t*, uint64_t*, uint32_t*);
__global__ void k_auto_minima(const BlockDesc*, const BlockStat*, const float*, const uint32_t*, uint64_t*);
__global__ void k_auto_seed_set(const BlockDesc*, BlockStat*, const float*, const uint32_t*, const uint64_t*,
                                const uint32_t*, const uint32_t*, uint64_t*, uint8_t*, uint64_t*, uint64_t*, uint32_t*);
__global__ void k_slice_offsets(const BlockDesc*, const BlockStat*, const uint32_t*, uint32_t*);
__global__ void k_finalize_ws(const BlockDesc*, const BlockStat*, const uint32_t*, const uint32_t*, const uint64_t*, int,
                              uint32_t*);

// k_pass2.hip (two-pass watershed, pass 2)
__global__ void k_p2_zero_dt(const BlockDesc*, const BlockStat*, float*);
__global__ void k_p2_insert(const BlockDesc*, BlockStat*, uint64_t*, uint32_t*, const uint32_t*, const uint64_t*,
                            const uint32_t*, const uint32_t*);
__global__ void k_p2_roots(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, uint64_t*);
__global__ void k_p2_label(const BlockDesc*, const BlockStat*, const uint64_t*, const uint32_t*, const uint64_t*,
                           const uint32_t*, const float*, uint32_t*, uint64_t*, uint8_t*, uint32_t*, uint32_t*, int, int,
                           const uint32_t*, const uint64_t*, const uint32_t*, const uint32_t*, uint8_t*);
__global__ void k_p2_excl_zero(const BlockDesc*, const BlockStat*, uint8_t*);
__global__ void k_p2_excl(const BlockDesc*, const BlockStat*, const uint32_t*, uint8_t*);
__global__ void k_p2_check(const BlockDesc*, BlockStat*, const uint64_t*, const uint32_t*);
__global__ void k_p2_output(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*, int, const uint32_t*,
                            const uint32_t*, const uint32_t*);
__global__ void k_slice_inmask(const BlockDesc*, const BlockStat*, uint32_t*);

// k_relabel.hip (RelabelWorkflow: sorted uniques, assignment-table lookup)
__global__ void k_copy_to_host(const uint4*, uint4*, size_t);
__global__ void k_u64_range(const uint64_t*, int64_t, unsigned long long*);
__global__ void k_u64_bits(const uint64_t*, int64_t, uint64_t, unsigned long long*);
__global__ void k_bits_chunk_count(const uint64_t*, int64_t, uint32_t*);
__global__ void k_scan_chunks(const uint32_t*, int64_t, uint64_t*);
__global__ void k_bits_compact(const uint64_t*, int64_t, const uint64_t*, uint64_t, uint64_t, uint64_t*);
__global__ void k_u64_lookup(uint64_t*, int64_t, const uint64_t*, const uint64_t*, int64_t, unsigned long long*);
hipError_t u64_sort(void* tmp, size_t& bytes, const uint64_t* in, uint64_t* out, int64_t n, hipStream_t stream);
hipError_t u64_runs(void* tmp, size_t& bytes, const uint64_t* sorted, uint64_t* uniq, uint64_t* counts,
                    uint64_t* n_runs, int64_t n, hipStream_t stream);

// k_threshcc.hip (ThresholdedComponents: BlockComponents)
struct TcParams {
    int nz, ny, nx;
    int mode;       // 0 greater, 1 less, 2 equal
    int normalize;  // 1: vu.normalize before the threshold (min / max from k_tc_minmax)
    float thr;      // the threshold as float32
};
__global__ void k_tc_minmax(const float*, int64_t, uint32_t*);
__global__ void k_tc_tile(const float*, const uint8_t*, TcParams, const uint32_t*, uint32_t*, uint32_t*);
__global__ void k_tc_merge(TcParams, uint32_t*);
__global__ void k_tc_roots(const uint32_t*, int64_t, uint64_t*);
__global__ void k_tc_wordoff(const uint64_t*, int64_t, const uint64_t*, uint32_t*);
__global__ void k_tc_label(const uint32_t*, int64_t, const uint64_t*, const uint32_t*, uint64_t*);
template <class T>
__global__ void k_tc_to_f32(const T*, int64_t, float*);
template <class T>
__global__ void k_tc_raw_members(const T*, int64_t, int, double, float*);
__global__ void k_tc_normalize(float*, int64_t, const uint32_t*);
__global__ void k_tc_gauss(const float*, float*, int, int, int, int, const double*, int);

}  // namespace ctws
