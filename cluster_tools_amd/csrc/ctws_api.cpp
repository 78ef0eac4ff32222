// ctws_api.cpp — host side of libctws.so: the C-ABI of include/ctws.h.
//
// Replaces the block loop of the reference job entry (cluster_tools/watershed/watershed.py:
// 380-381, `for block_id in block_list: _ws_block(...)`) with batched launches: all blocks of
// a batch go through one pipeline of gfx950 kernels (grid.y = block), so even a single job
// fills the 256 CUs.  The caller keeps the dataset I/O and the "processed block" log protocol.
//
// Pipeline per batch (kernel files in brackets):
//   input min/max -> normalize + threshold + EDT x  [k_edt]     (_read_data, _apply_dt)
//   EDT y [, z] -> dt, dt min/max                    [k_edt]
//   Gaussian(sigma_seeds) of dt                      [k_gauss]   (_make_seeds)
//   hmap + Gaussian(sigma_weights)                   [k_gauss]   (_make_hmap)
//   local maxima, plateaus, seed CC, scan-order ids  [k_cc]
//   seeded flood                                     [k_flood]   (watershedsNew)
//   size filter + regrow flood                       [k_post, k_flood] (apply_size_filter)
//   2-D slice offsets / mask                         [k_post]    (_apply_watershed)
//   halo crop CC + uint64 offset                     [k_cc]      (_ws_block :326-341)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <type_traits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <climits>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/ctws.h"
#include "ctws_kernels.h"
#include "host_pool.h"

using namespace ctws;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct Workspace {
    int64_t cap_vox = 0, cap_words = 0, cap_chunks = 0, cap_slices = 0, cap_tiles = 0, cap_blocks = 0;
    float *fin = nullptr, *dt = nullptr, *A = nullptr, *Bf = nullptr, *sm = nullptr, *hm = nullptr;
    uint8_t* cls = nullptr;
    uint32_t *P = nullptr, *PF = nullptr, *lab = nullptr;
    uint64_t* key = nullptr;
    uint64_t* W = nullptr;
    uint32_t *Wp = nullptr, *csum = nullptr;
    uint32_t *smin = nullptr, *smax = nullptr, *sb = nullptr, *slmax = nullptr, *soff = nullptr, *surv = nullptr;
    uint32_t *act0 = nullptr, *act1 = nullptr, *lines0 = nullptr, *lines1 = nullptr;
    BlockDesc* desc = nullptr;
    BlockStat* stat = nullptr;
    uint32_t* counter = nullptr;
    double* taps = nullptr;  // [6][128]
    // pass 2 (two-pass watershed) relabel hash
    int64_t cap_hash = 0;
    uint64_t* hkey = nullptr;
    uint32_t* hpos = nullptr;
    uint32_t* p2err = nullptr;
    // frontier bitmaps of the descent flood
    int64_t cap_front = 0;
    uint64_t *front0 = nullptr, *front1 = nullptr, *fopen = nullptr;
    uint64_t* fplat = nullptr;   // plateau fill (k_plateau.hip): the plateau voxels
    uint64_t* fseed = nullptr;   // seed CC members (the seed forest's parents are written for members only)
    uint32_t* plev = nullptr;    // per block: the plateau height (0: none)
    uint32_t* fflags = nullptr;
    uint32_t *fchunk0 = nullptr, *fchunk1 = nullptr;  // per 64-word chunk: generation of its last change
    uint32_t *wl0 = nullptr, *wl1 = nullptr, *qgen = nullptr;  // chunk worklists, queued generation
    uint32_t* wlcnt = nullptr;  // worklist length per iteration
    int64_t cap_fstat = 0;
    uint32_t* fstat = nullptr;  // CTWS_TRACE statistics: open voxels, frontier visits per block
};

constexpr int kCounterBytes = 4 * (4 + 4 * kStatSlots);  // flood flag + statistics slots
constexpr int kFrontierBatch = 8;        // frontier iterations per host check
constexpr int kFrontierWavesHost = 4;    // waves per workgroup of k_frontier (kFrontierWaves)
constexpr int kFrontierMaxIters = 256;   // then the tile flood takes over
constexpr int kFrontierMaxItersCap = 4096;  // CTWS_FRONTIER_ITERS upper bound (worklist counters)

}  // namespace

struct ctws_handle {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    Workspace ws;
    uint32_t* h_counter = nullptr;  // pinned
    double* h_taps = nullptr;       // pinned [6][128]
    std::vector<std::pair<const char*, float>> timings;
    std::vector<hipEvent_t> events;
    hipEvent_t fev[2] = {nullptr, nullptr};
    uint64_t flood_tiles = 0, flood_iters = 0, flood_lines = 0;
    // host-pointer staging
    DevBuf st_in, st_mask, st_init, st_out;
    // host-pointer path: two slots of pinned host staging + device staging, copy streams
    struct HostSlot {
        void* pin_in = nullptr;  // inputs | masks | initial seeds of a batch, packed
        size_t pin_in_bytes = 0;
        void* pin_out = nullptr;  // uint64 outputs of a batch
        size_t pin_out_bytes = 0;
        DevBuf d_in, d_out;
        hipEvent_t ev_h2d = nullptr, ev_comp = nullptr, ev_d2h = nullptr;
        hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // CTWS_TRACE: the batch's upload, timed
        std::vector<hipEvent_t> ev_blk;  // per block of the batch: its output downloaded
    } hslot[2];
    hipStream_t s_in = nullptr, s_out = nullptr;
    // relabel (k_relabel.hip)
    DevBuf rl_lab, rl_bits, rl_cnt, rl_offs, rl_out, rl_keys, rl_vals, rl_red;
    DevBuf rl_sorted, rl_uniq, rl_counts, rl_tmp;  // sort-based unique
    int64_t rl_ntable = 0;  // entries of the resident assignment table (rl_keys / rl_vals)
    // EDT: counters (64 B) + columns queued for the lower-envelope pass (k_edt_col_fh)
    DevBuf edt_fh;
    DevBuf xface;  // crop CC: the tiles' x columns (CcArgs::xface)
    DevBuf ptile;  // plateau CC: per-tile plateau flags (CcArgs::ptile)
    DevBuf edt_scratch;  // k_edt_real_line: per-thread parabola stacks
    // WatershedFromSeeds (k_seeded.hip): distinct seed values, sorted values, segment offsets, sort temp
    DevBuf fs_vals, fs_sorted, fs_off, fs_tmp;
    // ThresholdedComponents (k_threshcc.hip): forest, root bitmap, chunk counts / offsets, word
    // offsets, min / max + any flag, host-pointer staging
    DevBuf tc_P, tc_bits, tc_cnt, tc_offs, tc_woff, tc_red, tc_in, tc_mask, tc_out, tc_raw, tc_tmp, tc_taps;
    // evaluation (k_eval.hip): gt / seg / pair hash tables with counts, state, sums, staging
    DevBuf ev_ka, ev_ca, ev_kb, ev_cb, ev_kp, ev_cp, ev_state, ev_out, ev_stage;
    int64_t ev_cap_a = 0, ev_cap_b = 0, ev_cap_p = 0;
    // test hooks
    int stop_after = 0;
    int trace = 0;       // CTWS_TRACE=1: per-round flood statistics on stderr
    int no_descent = 0;  // CTWS_NO_DESCENT=1: flood from the seeds alone (test hook)
    int seed_tilecc = 0;  // CTWS_SEED_TILECC=1: the seed CC by tiles (else k_seed_members / k_seed_union2)
    int no_fallback = 0; // CTWS_NO_FALLBACK=1: keep a failed descent result (debugging)
    // CTWS_FORCE_WIDE=1: every flood on the wide keys (k_flood, 32-bit d; tests).  wide_rerun:
    // run_batch is re-running blocks whose packed flood reported a saturated d (dsat)
    int force_wide = 0;
    int wide_rerun = 0;
    int sf_sparse = 1;  // CTWS_SF_SPARSE=0: the size filter's regrow initialisation scans every block
    int verify = 1;      // CTWS_VERIFY: 1 (default) check the flood fixpoint + fallback, 2 fail on a violation (tests), 0 off
    int prep_lds = 0;    // CTWS_PREP_LDS=1: LDS row kernel for the x pass at every row length (tests)
    int plateau_fill = 1;  // CTWS_PLATEAU_FILL=0: masked blocks' plateaus relaxed hop by hop (k_plateau.hip)
    int output_tile = 1;   // CTWS_OUTPUT_TILE=0: cropped blocks through the word-tiled k_output
    int gauss_w = 0;            // CTWS_GAUSS_W (8, 16, 32): x positions per sliding-window column tile
    int gauss_yx = 1;           // CTWS_GAUSS_YX=0: separate y and x passes instead of the fused tile kernel
    int words_per_wave = 32;    // CTWS_WORDS_PER_WAVE: words per wave of the word-tiled kernels
    // CTWS_D2H_WGS: workgroups of a device-to-host copy kernel; 0 (default): hipMemcpyAsync on the
    // SDMA engines.  r03 (uint32 downloads, config 3): the copy kernel's workgroups slowed the
    // concurrent compute from 94 to 140 ms per step (host-resident 7.69 vs 6.08 Gvoxel/s)
    int d2h_wgs = 0;
    int pack_threads = 6;       // CTWS_PACK_THREADS: threads packing inputs into pinned staging
    int unpack_threads = 9;     // CTWS_UNPACK_THREADS: threads widening downloads into the outputs
    std::unique_ptr<ctws_host::WorkerPool> pack_pool, unpack_pool;
    int h2d_mode = 0;           // CTWS_H2D_MODE: 0 a copy per block as packed, 1 one copy per batch, 2 pull kernel
    int h2d_wgs = 64;           // CTWS_H2D_WGS: workgroups of the pull kernel (mode 2)
    int host_ramp = 1;          // CTWS_HOST_RAMP=0: equal batches (no smaller first / last batches)
    int host_batch_blocks = 0;  // CTWS_HOST_BATCH_BLOCKS: cap on blocks per host-path batch (0: voxel cap)
    int64_t host_batch_voxels = (int64_t)256 << 20;  // CTWS_HOST_BATCH_VOXELS: smaller batches pipeline better
    int edt_wz = 0;  // CTWS_EDT_WZ: the same for the z pass alone (3-D DT)
    int edt_w = 0;  // CTWS_EDT_W (8, 16, 32, 64): x positions per EDT column tile (0: by line length)
    // CTWS_FRONTIER_CHUNK2D / _3D "CWxCYxCZ": frontier chunk brick (words x rows x slices, 64 words).
    // 3-D batches with a mask: 1x32x2 was their default until round 5 (a masked region is one
    // flat plateau the flood crosses hop by hop, and wider bricks in y cut the launches: config 5
    // 104 -> 72 ms before the plateau fill); with the plateau fill and the alternating sweep
    // order 1x8x8 relaxes config 5 faster (39.6 -> 36.4 ms, 132 -> 101 launches per step)
    int fchunk2[3] = {1, 64, 1};
    int fchunk3[3] = {1, 8, 8};
    int fchunk3_masked[3] = {1, 8, 8};
    int fchunk3_env = 0;  // CTWS_FRONTIER_CHUNK3D given: used for every 3-D batch
    int fc_cur[3] = {1, 64, 1};  // the brick of the current batch (run_batch)
    int cur_max[3] = {0, 0, 0};  // largest outer block extents (Z, Y, X) of the current batch
    // CTWS_FRONTIER_GRID: workgroups of k_frontier (chunks in flight / 4).  1024 rather than 2048:
    // half the chunks in flight keep more of each chunk's lines in L2 between its local sweeps
    // (r04: config 3 relaxation 20.3 -> 18.5 ms per step; 512: 23.0 ms, too few waves)
    int frontier_grid = 1024;
    int frontier_dir = 1;    // CTWS_FRONTIER_DIR: local sweeps queue only the neighbours a change may lower
    int frontier_reps = 32;  // CTWS_FRONTIER_REPS: local sweeps per chunk and launch (r02 sweep: 4 -> 32 cut k_frontier 19%)
    int frontier_max_iters = kFrontierMaxIters;  // CTWS_FRONTIER_ITERS: then the tile flood finishes
    std::vector<BlockDesc> last_desc;
    // pass 2 (2-D): per block of the next run_batch, the slice offsets of its previous run (empty:
    // none); a block with a wrapped-id merge runs again until its offsets are self-consistent
    std::vector<std::vector<uint32_t>> p2_hints;
    DevBuf p2_hint_dev;
    int p2_depth = 0;
    std::vector<uint8_t> last_bare;  // run_batch: per block, an in-mask voxel got the bare offset
};

namespace {

#define HIPCHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            h->err = std::string(#expr) + ": " + hipGetErrorString(e_);                  \
            return CTWS_EHIP;                                                            \
        }                                                                                \
    } while (0)

#define LAUNCHCHK()                                                                      \
    do {                                                                                 \
        hipError_t e_ = hipGetLastError();                                               \
        if (e_ != hipSuccess) {                                                          \
            h->err = std::string("kernel launch: ") + hipGetErrorString(e_);             \
            return CTWS_EHIP;                                                            \
        }                                                                                \
    } while (0)

template <class T>
int dev_alloc(ctws_handle* h, T*& p, int64_t n) {
    if (p) {
        hipFree(p);
        p = nullptr;
    }
    if (n <= 0) n = 1;
    hipError_t e = hipMalloc((void**)&p, sizeof(T) * (size_t)n);
    if (e != hipSuccess) {
        h->err = std::string("hipMalloc(") + std::to_string(sizeof(T) * (size_t)n) + "): " + hipGetErrorString(e);
        p = nullptr;
        return CTWS_ENOMEM;
    }
    return CTWS_OK;
}

int grow(ctws_handle* h, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes) return CTWS_OK;
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    if (hipMalloc(&b.p, std::max<size_t>(bytes, 16)) != hipSuccess) {
        h->err = "hipMalloc staging failed (" + std::to_string(bytes) + " bytes)";
        return CTWS_ENOMEM;
    }
    b.bytes = bytes;
    return CTWS_OK;
}

int ensure_workspace(ctws_handle* h, int64_t vox, int64_t words, int64_t chunks, int64_t slices, int64_t tiles,
                     int64_t blocks, int64_t hash, int64_t front) {
    Workspace& w = h->ws;
    int r = CTWS_OK;
#define ALLOC(field, n) \
    if ((r = dev_alloc(h, w.field, (n))) != CTWS_OK) return r
    if (vox > w.cap_vox) {
        vox = std::max<int64_t>(vox, w.cap_vox + w.cap_vox / 4);
        ALLOC(fin, vox);
        ALLOC(dt, vox);
        ALLOC(A, vox);
        ALLOC(Bf, vox);
        ALLOC(sm, vox);
        ALLOC(hm, vox);
        ALLOC(cls, vox + 16);  // k_plateau_flag reads aligned 16-byte groups
        ALLOC(P, vox + 4);
        ALLOC(PF, vox + 4);
        ALLOC(lab, vox);
        ALLOC(key, vox);
        w.cap_vox = vox;
    }
    if (words > w.cap_words) {
        ALLOC(W, words);
        ALLOC(Wp, words);
        w.cap_words = words;
    }
    if (chunks > w.cap_chunks) {
        ALLOC(csum, chunks);
        w.cap_chunks = chunks;
    }
    if (slices > w.cap_slices) {
        ALLOC(smin, slices);
        ALLOC(smax, slices);
        ALLOC(sb, slices);
        ALLOC(slmax, slices);
        ALLOC(soff, slices);
        ALLOC(surv, slices);
        w.cap_slices = slices;
    }
    if (tiles > w.cap_tiles) {
        ALLOC(act0, tiles);
        ALLOC(act1, tiles);
        ALLOC(lines0, tiles * kLineWords);
        ALLOC(lines1, tiles * kLineWords);
        w.cap_tiles = tiles;
    }
    if (blocks > w.cap_blocks) {
        ALLOC(desc, blocks);
        ALLOC(stat, blocks);
        w.cap_blocks = blocks;
    }
    if (hash > w.cap_hash) {
        ALLOC(hkey, hash);
        ALLOC(hpos, hash);
        w.cap_hash = hash;
    }
    if (!w.p2err) ALLOC(p2err, 4);
    if (front > w.cap_front) {
        ALLOC(front0, front);
        ALLOC(front1, front);
        ALLOC(fopen, front);
        ALLOC(fplat, front);
        ALLOC(fseed, front);
        ALLOC(fchunk0, (front >> kChunkShift) + 1);
        ALLOC(fchunk1, (front >> kChunkShift) + 1);
        ALLOC(wl0, (front >> kChunkShift) + 1);
        ALLOC(wl1, (front >> kChunkShift) + 1);
        ALLOC(qgen, (front >> kChunkShift) + 1);
        w.cap_front = front;
    }
    if (!w.fflags) ALLOC(fflags, kFrontierBatch);
    if (!w.wlcnt) ALLOC(wlcnt, kFrontierMaxItersCap + 2);
    if (blocks > w.cap_fstat) {
        ALLOC(fstat, 3 * blocks);
        ALLOC(plev, blocks);
        w.cap_fstat = blocks;
    }
    if (!w.counter) ALLOC(counter, kCounterBytes / 4);
    if (!w.taps) ALLOC(taps, 6 * kTapSlot);
#undef ALLOC
    return CTWS_OK;
}

// vigra Kernel1D<double>::initGaussian(sigma, 1.0) (restated; taps for offsets -r..r)
std::vector<double> gaussian_taps(double sigma) {
    std::vector<double> k;
    if (sigma > 0.0) {
        const double sigma2 = -0.5 / sigma / sigma;
        const double norm = 1.0 / (std::sqrt(2.0 * M_PI) * sigma);
        int radius = (int)(3.0 * sigma + 0.5);
        if (radius == 0) radius = 1;
        for (double x = -(double)radius; x <= (double)radius; ++x) {
            const double x2 = x * x;
            k.push_back(norm * std::exp(x2 * sigma2));
        }
    } else {
        k.push_back(1.0);
    }
    double sum = 0.0;
    for (double v : k) sum += v;
    sum = 1.0 / sum;
    for (double& v : k) v = v * sum;
    return k;
}

struct BlockIO {
    const void* in;
    const uint8_t* mask;
    const uint64_t* init;
    uint64_t* out;
    uint32_t* out32 = nullptr;  // host path: compact uint32 codes (widened on the host)
};

struct Plan {
    // validated, derived configuration
    int nd_ws, dt_2d, pass2;
    int from_seeds;  // WatershedFromSeeds (watershed_from_seeds.py): given seeds, hmap = input
    int pitch[3];
    double pitchd[3];  // pixel_pitch as given
    bool real_pitch;   // a non-integer pitch: vigra's double-temporary distance path
    bool seeds_smooth, weights_smooth;
    double sig_seeds[3], sig_weights[3];
};

int make_plan(ctws_handle* h, const ctws_cfg* cfg, Plan& p) {
    p.from_seeds = 0;
    p.nd_ws = cfg->apply_ws_2d ? 2 : 3;
    p.dt_2d = cfg->apply_dt_2d ? 1 : 0;
    if (cfg->pass_id != 0 && cfg->pass_id != 1) {
        h->err = "pass_id must be 0 (_ws_block) or 1 (_ws_pass2)";
        return CTWS_EINVAL;
    }
    p.pass2 = cfg->pass_id == 1 ? 1 : 0;
    for (int k = 0; k < 3; ++k) {
        p.pitch[k] = 1;
        p.pitchd[k] = 1.0;
    }
    p.real_pitch = false;
    if (cfg->has_pixel_pitch) {
        if (p.dt_2d) {
            h->err = "apply_dt_2d requires pixel_pitch None (watershed.py:151)";
            return CTWS_EINVAL;
        }
        for (int k = 0; k < 3; ++k) {
            const double v = cfg->pixel_pitch[k];
            if (!(v > 0.0) || !std::isfinite(v)) {
                h->err = "pixel_pitch must be positive";
                return CTWS_EINVAL;
            }
            p.pitchd[k] = v;
            // vigra: int(pitch) != pitch selects the real-valued (double) path (multi_distance.hxx);
            // a large integer pitch stays integer: its dmax >= 2^24 selects the float path per batch
            // (run_batch), as the oracle's distance_transform does.  (The int copy is only read by
            // the exact integer path, which such a pitch never takes.)
            if (v != std::floor(v)) p.real_pitch = true;
            else p.pitch[k] = (int)std::min(v, 65536.0);
        }
    }
    auto sig = [&](const double* s, int is_list, double* out, bool& en) -> int {
        en = is_list ? true : (s[0] != 0.0);
        if (is_list && p.nd_ws == 2) {
            h->err = "per-axis sigma needs a 3-D watershed (volume_utils.py:97-98)";
            return CTWS_EINVAL;
        }
        for (int k = 0; k < 3; ++k) {
            out[k] = is_list ? s[k] : s[0];
            if (out[k] < 0.0) {
                h->err = "negative sigma";
                return CTWS_EINVAL;
            }
            if ((int)(3.0 * out[k] + 0.5) >= kTapSlot / 2) {
                h->err = "sigma too large (radius >= 2048)";
                return CTWS_EUNSUPPORTED;
            }
        }
        return CTWS_OK;
    };
    int r;
    if ((r = sig(cfg->sigma_seeds, cfg->sigma_seeds_is_list, p.sig_seeds, p.seeds_smooth)) != CTWS_OK) return r;
    if ((r = sig(cfg->sigma_weights, cfg->sigma_weights_is_list, p.sig_weights, p.weights_smooth)) != CTWS_OK)
        return r;
    return CTWS_OK;
}

int col_width(int L) { return L <= 512 ? 32 : (L <= 1024 ? 16 : 8); }

// dynamic LDS above 64 KiB needs the kernel's opt-in (gfx950: up to 160 KiB per workgroup)
constexpr size_t kMaxLds = 160 * 1024;
template <class K>
void lds_optin(K kern, size_t lds) {
    if (lds > 65536) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}
// The largest outer block extents the LDS line kernels take: a whole row in LDS (k_prep_edt_x:
// 16 B per voxel; k_gauss_row: 16 B per voxel + 1 KiB) and whole y / z columns 8 wide (k_edt_col<8>,
// k_gauss_col<8>: 32 B per position + 1 KiB).  Round 6: the former caps X <= 4096, Y, Z <= 2048
// were the 64 KiB default, not the hardware.
constexpr int kMaxRowX = (int)((kMaxLds - 1024) / 16);    // 10176
constexpr int kMaxColLen = (int)((kMaxLds - 1024) / 32);  // 5088
// EDT columns: 16 x positions (64-B row segments) beat 32 — half the LDS per tile, twice the
// tiles per CU, and the bounded search's per-lane trip counts vary less per wave (r01 sweep:
// y+z passes 1.60 ms at 32, 1.44 at 16, 1.77 at 8 for config 2)
// EDT column tile width: 32 x positions (full 128-B rows) while the column tile fits 32 KiB
// of LDS (config 4/5 z pass, 80-deep lines: 14.9 -> 13.8 / 14.3 -> 12.7 ms of EDT per step);
// 16 up to 1024-long lines (a 576-long y line at 32 wide, 74 KiB, measured 9.1 vs 5.6 ms)
int edt_col_width(int L) { return L <= 256 ? 32 : L <= 1024 ? 16 : 8; }

void record(ctws_handle* h, size_t idx) {
    while (h->events.size() <= idx) {
        hipEvent_t e;
        hipEventCreate(&e);
        h->events.push_back(e);
    }
    hipEventRecord(h->events[idx], h->stream);
}

// ---- Gaussian passes over the active axes, z -> y -> x --------------------------------------
#define CTWS_R12(M) M(1), M(2), M(3), M(4), M(5), M(6), M(7), M(8), M(9), M(10), M(11), M(12)
#define CTWS_ROWR(R) &k_gauss_row_r<R>
#define CTWS_COL32(R) &k_gauss_col_r<32, R>
#define CTWS_COL16(R) &k_gauss_col_r<16, R>
#define CTWS_COL8(R) &k_gauss_col_r<8, R>
using GaussKernel = decltype(&k_gauss_row_r<1>);
const GaussKernel kGaussRowR[kGaussMaxR + 1] = {nullptr, CTWS_R12(CTWS_ROWR)};
const GaussKernel kGaussColR32[kGaussMaxR + 1] = {nullptr, CTWS_R12(CTWS_COL32)};
const GaussKernel kGaussColR16[kGaussMaxR + 1] = {nullptr, CTWS_R12(CTWS_COL16)};
const GaussKernel kGaussColR8[kGaussMaxR + 1] = {nullptr, CTWS_R12(CTWS_COL8)};
#define CTWS_YX(R) &k_gauss_yx<R>
using GaussYxKernel = decltype(&k_gauss_yx<1>);
const GaussYxKernel kGaussYx[kGaussMaxR + 1] = {nullptr, CTWS_R12(CTWS_YX)};
#undef CTWS_YX
#undef CTWS_R12
#undef CTWS_ROWR
#undef CTWS_COL32
#undef CTWS_COL16
#undef CTWS_COL8

int run_gauss(ctws_handle* h, const Plan& pl, const double* sig, bool hmap_src, const float* src, float* dst,
              int nb, int maxZ, int maxY, int maxX, HmapParams hp, int taps_slot) {
    Workspace& w = h->ws;
    int axes[3], na = 0;
    for (int a = (pl.nd_ws == 3 ? 0 : 1); a < 3; ++a)
        if (sig[a] > 0.0) axes[na++] = a;
    if (na == 0) {
        if (hmap_src) {
            dim3 g((unsigned)std::min<int64_t>(((int64_t)maxZ * maxY * maxX + 255) / 256, 4096), nb);
            k_hmap<<<g, 256, 0, h->stream>>>(w.desc, w.stat, hp, w.fin, w.dt, w.smin, w.smax, dst);
            LAUNCHCHK();
        } else if (src != dst) {
            // identity smoothing: the caller reads `src`
        }
        return CTWS_OK;
    }
    const float* cur = src;
    for (int i = 0; i < na; ++i) {
        const int a = axes[i];
        auto taps = gaussian_taps(sig[a]);
        const int r = (int)taps.size() / 2;
        double* dtaps = w.taps + (taps_slot * 3 + a) * kTapSlot;
        double* htaps = h->h_taps + (taps_slot * 3 + a) * kTapSlot;
        std::memcpy(htaps, taps.data(), sizeof(double) * taps.size());
        HIPCHK(hipMemcpyAsync(dtaps, htaps, sizeof(double) * taps.size(), hipMemcpyHostToDevice, h->stream));
        float* out = (i == na - 1) ? dst : ((i % 2 == 0) ? w.A : w.Bf);
        GaussParams gp{a, r, (i == 0 && hmap_src) ? 1 : 0};
        const float* in = (i == 0 && hmap_src) ? w.fin : cur;
        // the last two axes y, x with one radius: fused tile kernel (k_gauss_yx)
        if (h->gauss_yx && a == 1 && i + 1 == na - 1 && axes[i + 1] == 2 && r >= 1 && r <= kGaussMaxR) {
            auto tx = gaussian_taps(sig[2]);
            if ((int)tx.size() / 2 == r) {
                double* dtx = w.taps + (taps_slot * 3 + 2) * kTapSlot;
                double* htx = h->h_taps + (taps_slot * 3 + 2) * kTapSlot;
                std::memcpy(htx, tx.data(), sizeof(double) * tx.size());
                HIPCHK(hipMemcpyAsync(dtx, htx, sizeof(double) * tx.size(), hipMemcpyHostToDevice, h->stream));
                const int TX = 128 - 2 * r;
                const int64_t ntiles = (int64_t)maxZ * ((maxY + kGaussYxTY - 1) / kGaussYxTY) * ((maxX + TX - 1) / TX);
                dim3 g((unsigned)ntiles, nb);
                hipLaunchKernelGGL(kGaussYx[r], g, dim3(256), 0, h->stream, w.desc, w.stat, gp.hmap_src, hp,
                                   (const double*)dtaps, (const double*)dtx, in, (const float*)w.dt,
                                   (const uint32_t*)w.smin, (const uint32_t*)w.smax, dst);
                LAUNCHCHK();
                return CTWS_OK;
            }
        }
        if (r >= 1 && r <= kGaussMaxR) {
            // sliding-window kernels (k_gauss.hip)
            if (a == 2 && maxX > 1024) {
                // rows longer than a wave's registers hold: the generic row kernel
                dim3 g((unsigned)(((int64_t)maxZ * maxY + 3) / 4), nb);
                const size_t lds = 2 * 128 * 4 + 4 * (size_t)maxX * 4;
                if (lds > 65536)  // gfx950: up to 160 KiB of LDS per workgroup, above 64 KiB by opt-in
                    (void)hipFuncSetAttribute((const void*)k_gauss_row, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)lds);
                k_gauss_row<<<g, 256, lds, h->stream>>>(w.desc, w.stat, gp, hp, dtaps, in, w.dt, w.smin, w.smax, out);
            } else if (a == 2) {
                // rows per wave shrink with X: size the grid for the widest block
                const int rpw = 64 / ((maxX + 15) / 16);
                dim3 g((unsigned)(((int64_t)maxZ * maxY + 4 * rpw - 1) / (4 * rpw)), nb);
                const size_t lds = 4 * 2 * (size_t)(64 * 17 + 64) * 4;
                hipLaunchKernelGGL(kGaussRowR[r], g, dim3(256), lds, h->stream, w.desc, w.stat, gp, hp,
                                   (const double*)dtaps, in, (const float*)w.dt, (const uint32_t*)w.smin,
                                   (const uint32_t*)w.smax, out);
            } else {
                const int Lm = a == 0 ? maxZ : maxY;
                const int other = a == 0 ? maxY : maxZ;
                const int W = h->gauss_w ? h->gauss_w : col_width(Lm);
                dim3 g((unsigned)((int64_t)other * ((maxX + W - 1) / W)), nb);
                const size_t lds = (size_t)Lm * W * 4;
                auto kern = W == 32 ? kGaussColR32[r] : (W == 16 ? kGaussColR16[r] : kGaussColR8[r]);
                lds_optin(kern, lds);
                hipLaunchKernelGGL(kern, g, dim3(256), lds, h->stream, w.desc, w.stat, gp, hp, (const double*)dtaps,
                                   in, (const float*)w.dt, (const uint32_t*)w.smin, (const uint32_t*)w.smax, out);
            }
        } else if (a == 2) {
            dim3 g((unsigned)(((int64_t)maxZ * maxY + 3) / 4), nb);
            const size_t lds = 2 * 128 * 4 + 4 * (size_t)maxX * 4;
            if (lds > 65536)
                (void)hipFuncSetAttribute((const void*)k_gauss_row, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            k_gauss_row<<<g, 256, lds, h->stream>>>(w.desc, w.stat, gp, hp, dtaps, in, w.dt, w.smin, w.smax, out);
        } else {
            const int Lm = a == 0 ? maxZ : maxY;
            const int other = a == 0 ? maxY : maxZ;
            const int W = col_width(Lm);
            dim3 g((unsigned)((int64_t)other * ((maxX + W - 1) / W)), nb);
            const size_t lds = 2 * 128 * 4 + (size_t)Lm * W * 4;
            if (W == 32) lds_optin(k_gauss_col<32>, lds);
            else if (W == 16) lds_optin(k_gauss_col<16>, lds);
            else lds_optin(k_gauss_col<8>, lds);
            if (W == 32)
                k_gauss_col<32><<<g, 256, lds, h->stream>>>(w.desc, w.stat, gp, hp, dtaps, in, w.dt, w.smin, w.smax,
                                                            out);
            else if (W == 16)
                k_gauss_col<16><<<g, 256, lds, h->stream>>>(w.desc, w.stat, gp, hp, dtaps, in, w.dt, w.smin, w.smax,
                                                            out);
            else
                k_gauss_col<8><<<g, 256, lds, h->stream>>>(w.desc, w.stat, gp, hp, dtaps, in, w.dt, w.smin, w.smax,
                                                           out);
        }
        LAUNCHCHK();
        cur = out;
    }
    return CTWS_OK;
}

int cdiv(int a, int b) { return (a + b - 1) / b; }

// ---- flood rounds until no tile is active -----------------------------------------------
// tile extents of k_flood_packed (PTile) and k_flood (FloodTile)
// frontier chunk bricks instantiated in k_flood.hip (CTWS_FRONTIER_SHAPES below): index or -1
// the built bricks: the defaults (2-D 1x64x1, 3-D 1x8x8, masked 3-D 1x32x2) and one alternative
// per dimension for the schedule-independence tests (tests/test_frontier_variants.py); the other
// shapes measured within +-0.1 ms of the defaults (r03) and were dropped from the build
int frontier_chunk_kind(int nd, int cw, int cy, int cz) {
    static const int shapes[5][4] = {{2, 1, 64, 1}, {2, 4, 16, 1}, {3, 1, 8, 8}, {3, 8, 8, 1}, {3, 1, 32, 2}};
    for (int k = 0; k < 5; ++k)
        if (shapes[k][0] == nd && shapes[k][1] == cw && shapes[k][2] == cy && shapes[k][3] == cz) return k;
    return -1;
}
bool frontier_chunk_ok(int nd, int cw, int cy, int cz) { return frontier_chunk_kind(nd, cw, cy, cz) >= 0; }

void flood_tile_dims(int nd, bool packed, int* tz, int* ty, int* tx) {
    *tz = nd == 3 ? (packed ? 16 : 4) : (packed ? 4 : 1);
    *ty = nd == 3 ? (packed ? 16 : 8) : 32;
    *tx = packed ? (nd == 3 ? 16 : 32) : 64;
}

// preset: act0 already holds the tiles to solve in the first round (regrow); otherwise all.
int run_flood(ctws_handle* h, int nd, bool packed, int nb, int max_tiles, int64_t ntiles, const float* hm,
              bool preset, int* rounds_out, float* kernel_ms) {
    Workspace& w = h->ws;
    if (!h->fev[0]) {
        hipEventCreate(&h->fev[0]);
        hipEventCreate(&h->fev[1]);
    }
    float kms = 0.f;
    uint32_t tiles_solved = 0, local_iters = 0;
    if (!preset) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)w.act0, 8u, (size_t)ntiles, h->stream));  // full solve
    HIPCHK(hipMemsetAsync(w.act1, 0, sizeof(uint32_t) * (size_t)ntiles, h->stream));
    HIPCHK(hipMemsetAsync(w.lines0, 0, sizeof(uint32_t) * kLineWords * (size_t)ntiles, h->stream));
    HIPCHK(hipMemsetAsync(w.lines1, 0, sizeof(uint32_t) * kLineWords * (size_t)ntiles, h->stream));
    uint32_t* cur = w.act0;
    uint32_t* nxt = w.act1;
    uint32_t* lcur = w.lines0;  // consumed (and cleared) by the packed kernel
    uint32_t* lnxt = w.lines1;
    dim3 g((unsigned)max_tiles, nb);
    int round = 0;
    for (; round < 1000000; ++round) {
        HIPCHK(hipMemsetAsync(w.counter, 0, kCounterBytes, h->stream));
        hipEventRecord(h->fev[0], h->stream);
        if (packed && nd == 3)
            k_flood_packed<3><<<g, 256, 0, h->stream>>>(w.desc, w.stat, hm, w.key, w.cls, cur, nxt, lcur, lnxt,
                                                        w.counter);
        else if (packed)
            k_flood_packed<2><<<g, 128, 0, h->stream>>>(w.desc, w.stat, hm, w.key, w.cls, cur, nxt, lcur, lnxt,
                                                        w.counter);
        else if (nd == 3)
            k_flood<3><<<g, 256, 0, h->stream>>>(w.desc, w.stat, hm, w.key, w.lab, cur, nxt, w.counter);
        else
            k_flood<2><<<g, 256, 0, h->stream>>>(w.desc, w.stat, hm, w.key, w.lab, cur, nxt, w.counter);
        LAUNCHCHK();
        hipEventRecord(h->fev[1], h->stream);
        HIPCHK(hipMemcpyAsync(h->h_counter, w.counter, kCounterBytes, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        for (int k = 1; k < 4; ++k) {
            uint32_t t = 0;
            for (int sl = 0; sl < kStatSlots; ++sl) t += h->h_counter[4 + sl * 4 + k];
            h->h_counter[k] = t;
        }
        float ms = 0.f;
        hipEventElapsedTime(&ms, h->fev[0], h->fev[1]);
        kms += ms;
        tiles_solved += h->h_counter[1];
        local_iters += h->h_counter[2];
        if (h->trace)
            fprintf(stderr, "[ctws] flood%s round %d: %.3f ms, tiles %u, sweeps %u, lines %u, next %u\n",
                    preset ? " (regrow)" : "", round, ms, h->h_counter[1], h->h_counter[2], h->h_counter[3],
                    h->h_counter[0]);
        h->flood_lines += h->h_counter[3];
        if (*h->h_counter == 0) break;
        HIPCHK(hipMemsetAsync(cur, 0, sizeof(uint32_t) * (size_t)ntiles, h->stream));
        std::swap(cur, nxt);
        std::swap(lcur, lnxt);
    }
    if (rounds_out) *rounds_out = round + 1;
    if (kernel_ms) *kernel_ms = kms;
    h->flood_tiles += tiles_solved;
    h->flood_iters += local_iters;
    return CTWS_OK;
}

// Frontier relaxation (k_frontier) from the open / changed bitmaps in w.fopen / w.front0 (written
// by k_descent_init for the first flood, by k_regrow_init for the size-filter regrow) until no
// key changes.  Batches of kFrontierBatch launches run between host checks of their flags; if
// it has not converged after frontier_max_iters iterations (very long equal-height paths) the
// tile flood finishes from the current keys.
int run_frontier(ctws_handle* h, const Plan& pl, int nb, int64_t TF, int max_tiles, int64_t TT, bool packed,
                 uint32_t* fst, int* iters_out, int* rounds_out, float* kms_out, bool regrow = false) {
    Workspace& w = h->ws;
    const int64_t nch = (TF >> kChunkShift) + 1;
    uint64_t* fb[2] = {w.front0, w.front1};  // changed bitmaps: iteration it reads fb[it & 1]
    uint32_t* gen[2] = {w.fchunk0, w.fchunk1};  // iteration it writes gen[it & 1], reads gen[(it + 1) & 1]
    uint32_t* wl[2] = {w.wl0, w.wl1};
    HIPCHK(hipMemsetAsync(w.fchunk0, 0, sizeof(uint32_t) * (size_t)nch, h->stream));
    HIPCHK(hipMemsetAsync(w.fchunk1, 0, sizeof(uint32_t) * (size_t)nch, h->stream));
    HIPCHK(hipMemsetAsync(w.qgen, 0, sizeof(uint32_t) * (size_t)nch, h->stream));
    HIPCHK(hipMemsetAsync(w.wlcnt, 0, sizeof(uint32_t) * (size_t)(h->frontier_max_iters + 2), h->stream));
    // iteration 0: every chunk with an open voxel
    const dim3 lg((unsigned)std::min<int64_t>((TF / nb + 64 * 64 * kFrontierWavesHost - 1) / (64 * 64 * kFrontierWavesHost) + 1,
                                              1024), nb);
    const int* fc = h->fc_cur;
    const int fkind = frontier_chunk_kind(pl.nd_ws, fc[0], fc[1], fc[2]);
#define CTWS_FRONTIER_SHAPES(X) X(0, 2, 1, 64, 1) X(1, 2, 4, 16, 1) X(2, 3, 1, 8, 8) X(3, 3, 8, 8, 1) X(4, 3, 1, 32, 2)
#define CTWS_LIST0(K, ND, CW, CY, CZ) \
    case K: k_frontier_list0<CW, CY, CZ><<<lg, 256, 0, h->stream>>>(w.desc, w.stat, w.fopen, wl[0], w.wlcnt); break;
    switch (fkind) {
        CTWS_FRONTIER_SHAPES(CTWS_LIST0)
        default: h->err = "bad frontier chunk"; return CTWS_EINVAL;
    }
#undef CTWS_LIST0
    LAUNCHCHK();
    // one wave per list entry; the largest list is every chunk of the batch
    const unsigned fg = (unsigned)std::min<int64_t>((nch + kFrontierWavesHost - 1) / kFrontierWavesHost, h->frontier_grid);
    bool converged = false;
    int fiters = 0;
    while (fiters < h->frontier_max_iters && !converged) {
        const int it0 = fiters;
        const int nl = std::min(kFrontierBatch, h->frontier_max_iters - it0);
        std::vector<hipEvent_t> tev;
        if (h->trace) {
            tev.resize(nl + 1);
            for (auto& e : tev) hipEventCreate(&e);
            hipEventRecord(tev[0], h->stream);
        }
        for (int k = 0; k < nl; ++k) {
            const int it = it0 + k;
#define CTWS_FRONTIER(K, ND, CW, CY, CZ)                                                                            \
    case K:                                                                                                         \
        k_frontier<ND, CW, CY, CZ><<<fg, 256, 0, h->stream>>>(                                                      \
            w.desc, w.stat, w.hm, w.key, w.fopen, fb[it & 1], fb[(it + 1) & 1], gen[(it + 1) & 1], gen[it & 1], it, \
            wl[it & 1], w.wlcnt + it, wl[(it + 1) & 1], w.wlcnt + it + 1, w.qgen, fst ? fst + nb : nullptr,         \
            h->frontier_reps, h->frontier_dir);                                                                     \
        break;
            switch (fkind) {
                CTWS_FRONTIER_SHAPES(CTWS_FRONTIER)
            }
#undef CTWS_FRONTIER
            if (h->trace) hipEventRecord(tev[k + 1], h->stream);
        }
        LAUNCHCHK();
        HIPCHK(hipMemcpyAsync(h->h_counter, w.wlcnt + it0, sizeof(uint32_t) * (nl + 1), hipMemcpyDeviceToHost,
                              h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        if (h->trace) {
            for (int k = 0; k < nl; ++k) {
                float ms = 0.f;
                hipEventElapsedTime(&ms, tev[k], tev[k + 1]);
                std::fprintf(stderr, "[ctws] frontier it %d: %u chunks, %.3f ms\n", it0 + k, h->h_counter[k], ms);
                if (!h->h_counter[k + 1]) break;
            }
            for (auto& e : tev) hipEventDestroy(e);
        }
        std::memmove(h->h_counter, h->h_counter + 1, sizeof(uint32_t) * nl);
        for (int k = 0; k < nl; ++k) {
            ++fiters;
            if (!h->h_counter[k]) {  // nothing queued for the next iteration
                converged = true;
                break;
            }
        }
    }
#undef CTWS_FRONTIER_SHAPES
    *iters_out += fiters;
    if (!converged) {
        int TZ, TY, TX;
        flood_tile_dims(pl.nd_ws, packed, &TZ, &TY, &TX);
        HIPCHK(hipMemsetAsync(w.act0, 0, sizeof(uint32_t) * (size_t)TT, h->stream));
        k_frontier_tiles<<<dim3((unsigned)std::min<int64_t>((TF / nb + 255) / 256 + 1, 4096), nb), 256, 0,
                           h->stream>>>(w.desc, w.stat, w.fopen, w.act0, TZ, TY, TX);
        // a sparse regrow (k_sf_sparse) left the survivors' seed flags as the first flood had
        // them: the tile flood needs every survivor fixed
        if (regrow) k_fixed_from_open<<<dim3(2048, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.fopen, w.cls);
        LAUNCHCHK();
        int rounds = 0;
        float kms = 0.f;
        int r = run_flood(h, pl.nd_ws, packed, nb, max_tiles, TT, w.hm, true, &rounds, &kms);
        if (r != CTWS_OK) return r;
        *rounds_out += rounds;
        *kms_out += kms;
    }
    return CTWS_OK;
}



void add_timing(ctws_handle* h, const char* name, float v);

int64_t words_of(int64_t n) { return n / 64 + 1; }
int64_t chunks_of(int64_t n) { return (words_of(n) + 255) / 256; }

// timings of one ctws_ws_blocks call: summed over its batches (counts too)
void add_timing(ctws_handle* h, const char* name, float v) {
    for (auto& t : h->timings)
        if (std::strcmp(t.first, name) == 0) {
            t.second += v;
            return;
        }
    h->timings.push_back({name, v});
}

// ---- WatershedFromSeeds seeds (k_seeded.hip) ----------------------------------------------
// The blocks' distinct seed values (hash), sorted per block (segmented radix sort), a label
// per value = 1 + its rank; blocks without any seed get the strict minima of the hmap
// (k_auto_minima + the bitmap rank, labels written by k_fs_auto_label once `packed` is known).
int fs_seeds(ctws_handle* h, const std::vector<BlockDesc>& desc, int nb, int64_t TH, int64_t TW, int64_t TS,
             int64_t maxH, int64_t maxRows, dim3 vg, dim3 wg) {
    Workspace& w = h->ws;
    int r;
    const size_t nh = (size_t)std::max<int64_t>(TH, 1);
    if ((r = grow(h, h->fs_vals, sizeof(uint32_t) * nh)) != CTWS_OK) return r;
    if ((r = grow(h, h->fs_sorted, sizeof(uint32_t) * nh)) != CTWS_OK) return r;
    if ((r = grow(h, h->fs_off, sizeof(int) * 2 * (size_t)nb)) != CTWS_OK) return r;
    uint32_t* vals = (uint32_t*)h->fs_vals.p;
    uint32_t* sorted = (uint32_t*)h->fs_sorted.p;
    int* off = (int*)h->fs_off.p;
    HIPCHK(hipMemsetAsync(w.hkey, 0xFF, sizeof(uint64_t) * nh, h->stream));
    k_fs_insert<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey);
    const dim3 hg((unsigned)std::min<int64_t>((maxH + 255) / 256, 4096), nb);
    k_fs_collect<<<hg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, vals);
    k_fs_offsets<<<(nb + 255) / 256, 256, 0, h->stream>>>(w.desc, w.stat, nb, off, off + nb);
    LAUNCHCHK();
    size_t tb = 0;
    HIPCHK(fs_segmented_sort(nullptr, tb, vals, sorted, (int)nh, nb, off, off + nb, h->stream));
    if ((r = grow(h, h->fs_tmp, tb)) != CTWS_OK) return r;
    HIPCHK(fs_segmented_sort(h->fs_tmp.p, tb, vals, sorted, (int)nh, nb, off, off + nb, h->stream));
    k_fs_rank<<<hg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, sorted, w.hpos);
    LAUNCHCHK();
    std::vector<BlockStat> st(nb);
    HIPCHK(hipMemcpyAsync(st.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    std::vector<uint32_t> surv((size_t)std::max<int64_t>(TS, 1), 1u);
    bool any = false;
    for (int i = 0; i < nb; ++i)
        if (st[i].n_seeds == 0) {
            surv[desc[i].sbase] = 0u;
            any = true;
        }
    HIPCHK(hipMemcpyAsync(w.surv, surv.data(), sizeof(uint32_t) * surv.size(), hipMemcpyHostToDevice, h->stream));
    if (any) {
        // watershedsNew with an all-zero seed image seeds from the strict minima of the hmap
        HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
        const dim3 ag((unsigned)std::min<int64_t>(maxRows, 65535), nb);
        k_auto_minima<<<ag, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.surv, w.W);
        k_bitmap_csum<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum);
        k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.csum, 2);
        k_word_prefix<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum, w.Wp);
        LAUNCHCHK();
    }
    // (surv stays in w.surv: k_fs_auto_label reads it; the size filter re-initialises it)
    return CTWS_OK;
}

// ---- one batch, all pointers on the device ------------------------------------------------
int run_batch(ctws_handle* h, const ctws_cfg* cfg, const Plan& pl, ctws_block* blocks, const BlockIO* io, int nb) {
    Workspace& w = h->ws;
    std::vector<BlockDesc> desc(nb);
    int64_t T = 0, TI = 0, TW = 0, TC = 0, TS = 0, TT = 0, TH = 0, TF = 0;
    int64_t maxH = 0, maxRows = 0, maxIRows = 0;
    int maxZ = 0, maxY = 0, maxX = 0, max_tiles = 0;
    int64_t maxN = 0, maxNI = 0;
    int maxIZ = 0, maxIY = 0, maxIX = 0;
    bool real_edt = pl.real_pitch;  // the batch's distances take vigra's real-valued path
    bool real_double = pl.real_pitch;  // ... with a double temporary (else float)
    const uint64_t bvol = (uint64_t)(cfg->block_shape[0] * cfg->block_shape[1] * cfg->block_shape[2]);
    {
        bool any_mask = false;
        for (int i = 0; i < nb; ++i) any_mask |= io[i].mask != nullptr;
        const int* fc = pl.nd_ws == 2 ? h->fchunk2 : (any_mask && !h->fchunk3_env ? h->fchunk3_masked : h->fchunk3);
        std::memcpy(h->fc_cur, fc, sizeof(h->fc_cur));
    }
    for (int i = 0; i < nb; ++i) {
        const ctws_block& b = blocks[i];
        BlockDesc& d = desc[i];
        std::memset(&d, 0, sizeof(d));
        d.Z = (int)b.outer_shape[0];
        d.Y = (int)b.outer_shape[1];
        d.X = (int)b.outer_shape[2];
        d.nd_ws = pl.nd_ws;
        d.N = (int64_t)d.Z * d.Y * d.X;
        d.base = T;
        d.iz0 = (int)b.inner_begin[0];
        d.iy0 = (int)b.inner_begin[1];
        d.ix0 = (int)b.inner_begin[2];
        d.IZ = (int)b.inner_shape[0];
        d.IY = (int)b.inner_shape[1];
        d.IX = (int)b.inner_shape[2];
        d.NI = (int64_t)d.IZ * d.IY * d.IX;
        d.crop = b.crop_relabel ? 1 : 0;
        d.ibase = T;  // inner arrays reuse the outer-sized parent array (NI <= N)
        d.wbase = TW;
        d.cbase = TC;
        d.sbase = TS;
        d.input = io[i].in;
        d.mask = io[i].mask;
        d.init = io[i].init;
        d.out = io[i].out;
        d.out32 = io[i].out32;
        d.n_channels = b.n_channels;
        d.dtype = b.input_dtype;
        if (b.n_channels > 0) {
            int cb = cfg->channel_begin, ce = cfg->channel_end < 0 ? b.n_channels : cfg->channel_end;
            if (cb < 0) cb += b.n_channels;
            if (ce > b.n_channels) ce = b.n_channels;
            if (cb > ce) cb = ce;
            d.c0 = cb;
            d.C = ce - cb;
            if (d.C <= 0) {
                h->err = "empty channel range";
                return CTWS_EINVAL;
            }
        } else {
            d.c0 = 0;
            d.C = 1;
        }
        d.id_offset = (uint64_t)b.block_id * bvol;
        d.pass2 = (uint32_t)pl.pass2;
        d.p2hint = -1;
        if (pl.pass2 || pl.from_seeds) {
            if (!d.init) {
                h->err = "pass 2 needs initial_seeds (ds_out[input_bb]) for every block";
                return CTWS_EINVAL;
            }
            int64_t cap = 4096;
            while (cap < d.N / 4) cap <<= 1;
            d.hbase = TH;
            d.hcap = cap;
            TH += cap;
        }
        d.maxd = (uint32_t)std::min<int64_t>((int64_t)pl.pitch[0] * pl.pitch[0] * d.Z * d.Z +
                                                 (int64_t)pl.pitch[1] * pl.pitch[1] * d.Y * d.Y +
                                                 (int64_t)pl.pitch[2] * pl.pitch[2] * d.X * d.X, 0xFFFFFFFFll);
        d.fbase = TF;
        // frontier bitmaps: rows padded to a multiple of 64, and at least 64 words per frontier
        // chunk brick (k_frontier), so that the per-chunk arrays can be indexed at fbase / 64
        {
            const int* fc = h->fc_cur;
            const int64_t wpr = (d.X + 63) / 64;
            const int64_t nch = ((wpr + fc[0] - 1) / fc[0]) * ((d.Y + fc[1] - 1) / fc[1]) * ((d.Z + fc[2] - 1) / fc[2]);
            TF += std::max((((int64_t)d.Z * d.Y + 63) / 64) * 64 * wpr, nch << kChunkShift);
        }
        T += d.N;
        TI += d.NI;
        TW += words_of(d.N);
        TC += chunks_of(d.N);
        TS += d.Z;
        maxZ = std::max(maxZ, d.Z);
        maxY = std::max(maxY, d.Y);
        maxX = std::max(maxX, d.X);
        maxN = std::max(maxN, d.N);
        maxNI = std::max(maxNI, d.NI);
        maxIZ = std::max(maxIZ, d.IZ);
        maxIY = std::max(maxIY, d.IY);
        maxIX = std::max(maxIX, d.IX);
        maxH = std::max(maxH, d.hcap);
        maxRows = std::max(maxRows, (int64_t)d.Z * d.Y);
        maxIRows = std::max(maxIRows, (int64_t)d.IZ * d.IY);
        // validation against what the kernels assume (run_blocks already failed such blocks
        // individually, block_refusal)
        if (d.X > kMaxRowX || d.Y > kMaxColLen || d.Z > kMaxColLen || d.N >= (1ll << 31)) {
            h->err = "outer block too large for the kernels (X <= 10176, Y, Z <= 5088, N < 2^31)";
            return CTWS_EUNSUPPORTED;
        }
        if (d.iz0 < 0 || d.iy0 < 0 || d.ix0 < 0 || d.iz0 + d.IZ > d.Z || d.iy0 + d.IY > d.Y || d.ix0 + d.IX > d.X ||
            d.IZ <= 0 || d.IY <= 0 || d.IX <= 0) {
            h->err = "inner block outside the outer block";
            return CTWS_EINVAL;
        }
        if (!d.input || (!d.out && !d.out32)) {
            h->err = "null input/output";
            return CTWS_EINVAL;
        }
        // vigra's convolveLine needs line length > kernel radius
        auto chk_len = [&](const double* sg, bool en) -> bool {
            if (!en) return true;
            const int lens[3] = {d.Z, d.Y, d.X};
            for (int a = (pl.nd_ws == 3 ? 0 : 1); a < 3; ++a) {
                if (sg[a] <= 0) continue;
                int r = (int)(3.0 * sg[a] + 0.5);
                if (r == 0) r = 1;
                if (lens[a] < r + 1) return false;
            }
            return true;
        };
        if (!chk_len(pl.sig_seeds, pl.seeds_smooth) || !chk_len(pl.sig_weights, pl.weights_smooth)) {
            h->err = "convolveLine(): kernel longer than line";
            return CTWS_EINVAL;
        }
        double dmax;
        if (pl.dt_2d) dmax = (double)d.Y * d.Y + (double)d.X * d.X;
        else
            dmax = std::pow(pl.pitchd[0] * d.Z, 2) + std::pow(pl.pitchd[1] * d.Y, 2) + std::pow(pl.pitchd[2] * d.X, 2);
        // dmax >= 2^24: float32 squared distances are no longer exact integers; vigra's float
        // arithmetic is then reproduced by the real-valued path (k_edt_real_*)
        if (dmax >= 16777216.0 && !pl.from_seeds) real_edt = true;
        if (dmax > 3.4028234663852886e38 && !pl.from_seeds) real_double = true;  // > FLT_MAX: double, as vigra
    }
    // flood tile grids: the largest (wide kernel) bounds the per-tile arrays
    auto set_tiles = [&](bool packed) {
        int TZ, TY, TX;
        flood_tile_dims(pl.nd_ws, packed, &TZ, &TY, &TX);
        TT = 0;
        max_tiles = 0;
        for (auto& d : desc) {
            d.tz = (d.Z + TZ - 1) / TZ;
            d.ty = (d.Y + TY - 1) / TY;
            d.tx = (d.X + TX - 1) / TX;
            d.tbase = (int)TT;
            TT += (int64_t)d.tz * d.ty * d.tx;
            max_tiles = std::max(max_tiles, d.tz * d.ty * d.tx);
        }
    };
    // crop CC: each cropped block's tiles get 2 x columns of (root, label) entries (k_tile_cc)
    int64_t TXF = 0;
    {
        const int ctz = pl.nd_ws == 3 ? CcTile<3>::TZ : CcTile<2>::TZ;
        const int cty = pl.nd_ws == 3 ? CcTile<3>::TY : CcTile<2>::TY;
        const int ctx = pl.nd_ws == 3 ? CcTile<3>::TX : CcTile<2>::TX;
        for (auto& d : desc) {
            d.xcbase = TXF;
            if (d.crop) TXF += (int64_t)cdiv(d.IZ, ctz) * cdiv(d.IY, cty) * cdiv(d.IX, ctx) * 2 * ctz * cty;
        }
    }
    // plateau CC: one flag per tile (k_localmax sets it for the tiles with a plateau voxel)
    int64_t TPT = 0;
    {
        const int ptz = pl.nd_ws == 3 ? CcTileM<3, CC_PLATEAU>::TZ : CcTileM<2, CC_PLATEAU>::TZ;
        const int pty = pl.nd_ws == 3 ? CcTileM<3, CC_PLATEAU>::TY : CcTileM<2, CC_PLATEAU>::TY;
        const int ptx = pl.nd_ws == 3 ? CcTileM<3, CC_PLATEAU>::TX : CcTileM<2, CC_PLATEAU>::TX;
        for (auto& d : desc) {
            d.ptbase = TPT;
            TPT += (int64_t)cdiv(d.Z, ptz) * cdiv(d.Y, pty) * cdiv(d.X, ptx);
        }
    }
    h->last_bare.assign(nb, 1);  // (a run stopped early by a test hook writes no labels)
    h->cur_max[0] = maxZ;
    h->cur_max[1] = maxY;
    h->cur_max[2] = maxX;
    set_tiles(true);
    const int64_t TT_packed = TT;
    set_tiles(false);
    const int64_t TT_wide = TT;
    set_tiles(true);
    int r;
    if ((r = ensure_workspace(h, T, TW, TC, TS, std::max(TT_packed, TT_wide), nb, TH, TF)) != CTWS_OK) return r;
    if (TXF && (r = grow(h, h->xface, sizeof(uint64_t) * (size_t)TXF)) != CTWS_OK) return r;
    if ((r = grow(h, h->ptile, sizeof(uint32_t) * (size_t)std::max<int64_t>(TPT, 1))) != CTWS_OK) return r;
    if (pl.pass2 && pl.nd_ws == 2 && (int)h->p2_hints.size() == nb) {
        std::vector<uint32_t> flat;
        for (int i = 0; i < nb; ++i) {
            if ((int)h->p2_hints[i].size() != desc[i].Z) continue;
            desc[i].p2hint = (int64_t)flat.size();
            flat.insert(flat.end(), h->p2_hints[i].begin(), h->p2_hints[i].end());
        }
        if (!flat.empty()) {
            if ((r = grow(h, h->p2_hint_dev, sizeof(uint32_t) * flat.size())) != CTWS_OK) return r;
            HIPCHK(hipMemcpy(h->p2_hint_dev.p, flat.data(), sizeof(uint32_t) * flat.size(), hipMemcpyHostToDevice));
        }
    }
    HIPCHK(hipMemcpyAsync(w.desc, desc.data(), sizeof(BlockDesc) * nb, hipMemcpyHostToDevice, h->stream));
    h->last_desc = desc;
    std::vector<BlockStat> st(nb);
    for (auto& s : st) {
        std::memset(&s, 0, sizeof(s));
        s.in_min = 0xFFFFFFFFu;
        s.dt_min = 0xFFFFFFFFu;
    }
    HIPCHK(hipMemcpyAsync(w.stat, st.data(), sizeof(BlockStat) * nb, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)w.smin, 0xFFFFFFFFu, (size_t)TS, h->stream));
    HIPCHK(hipMemsetAsync(w.smax, 0, sizeof(uint32_t) * TS, h->stream));
    HIPCHK(hipMemsetAsync(w.slmax, 0, sizeof(uint32_t) * TS, h->stream));
    HIPCHK(hipMemsetAsync(w.surv, 0, sizeof(uint32_t) * TS, h->stream));

    const dim3 vg((unsigned)std::min<int64_t>((maxN + 255) / 256, 4096), nb);
    const dim3 ig((unsigned)std::min<int64_t>((maxNI + 255) / 256, 4096), nb);
    // 4 voxels per thread (16-byte groups)
    const dim3 vg4((unsigned)std::min<int64_t>((maxN / 4 + 256) / 256, 4096), nb);
    const dim3 wg((unsigned)((words_of(maxN) + 255) / 256), nb);
    // row-tile kernels: kRows rows (z, y) per workgroup iteration
    const dim3 rg((unsigned)std::min<int64_t>((maxRows + kRows - 1) / kRows, 16384), nb);
    const dim3 rig((unsigned)std::min<int64_t>((maxIRows + kRows - 1) / kRows, 16384), nb);
    // word-tile kernels: one wave per 64-voxel row word, kWordWaves waves per workgroup
    // (h->words_per_wave words per wave: a workgroup per handful of words would make the
    // dispatch of ~10^6 workgroups the bottleneck)
    const int64_t wpw = (int64_t)kWordWaves * h->words_per_wave;
    // (x extents rounded to a multiple of 8: xcd_swizzle's id % 8 then labels one XCD per grid row)
    auto r8 = [](int64_t v) { return (unsigned)std::min<int64_t>(v > 8 ? (v + 7) / 8 * 8 : v, 65528); };
    // one workgroup per tile, rounded up to a multiple of 8 for xcd_swizzle (no cap: every tile
    // needs its workgroup; the extra ones return at once)
    auto tiles8 = [](int64_t v) { return (unsigned)(v > 8 ? (v + 7) / 8 * 8 : v); };
    const dim3 wtg(r8((maxRows * ((maxX + 63) / 64) + wpw - 1) / wpw), nb);
    const dim3 wtig(r8((maxIRows * ((maxIX + 63) / 64) + wpw - 1) / wpw), nb);
    size_t ev = 0;
    std::vector<const char*> names;
    auto mark = [&](const char* name) {
        record(h, ev++);
        names.push_back(name);
    };
    mark("start");

    // ---- normalize + threshold + EDT ------------------------------------------------------
    {
        // one raw dtype and 3-D datasets in the batch: the typed kernels (global loads in flight)
        int dt = desc[0].dtype;
        bool typed = !h->prep_lds && maxX <= 1024;
        bool all_exact = true;
        for (auto& d : desc) {
            typed &= d.dtype == dt && d.n_channels == 0;
            all_exact &= d.X == maxX && (d.X == 256 || d.X == 512 || d.X == 1024) && d.n_channels == 0 && d.dtype == 3;
        }
        dim3 g((unsigned)std::min<int64_t>((maxN + 65535) / 65536, 256), nb);
        if (typed) {
            dim3 gm((unsigned)std::min<int64_t>((maxN + 8 * 256 - 1) / (8 * 256), 1024), nb);
            if (dt == CTWS_U8) k_input_minmax_t<uint8_t><<<gm, 256, 0, h->stream>>>(w.desc, w.stat);
            else if (dt == CTWS_U16) k_input_minmax_t<uint16_t><<<gm, 256, 0, h->stream>>>(w.desc, w.stat);
            else if (dt == CTWS_F32) k_input_minmax_t<float><<<gm, 256, 0, h->stream>>>(w.desc, w.stat);
            else k_input_minmax_t<double><<<gm, 256, 0, h->stream>>>(w.desc, w.stat);
        } else {
            k_input_minmax<<<g, 256, 0, h->stream>>>(w.desc, w.stat);
        }
        LAUNCHCHK();
        // WatershedFromSeeds: _read_data without invert; the normalized input is the hmap
        PrepParams pp{(float)cfg->threshold, pl.from_seeds ? 0 : cfg->invert_inputs, cfg->agglomerate_channels,
                      pl.pitch[2] * pl.pitch[2]};
        float* fin_out = pl.from_seeds ? w.hm : w.fin;
        dim3 gx((unsigned)(((int64_t)maxZ * maxY + 3) / 4), nb);
        // rows up to 1024 voxels: one wave per row in registers.  f32 rows of exactly 64 K voxels
        // move as float4 with lanes owning consecutive voxels (k_prep_edt_x_reg); other rows use
        // the lane-interleaved coalesced layout (k_prep_edt_x_co)
        auto launch_co = [&](auto kmax_c) {
            constexpr int KM = decltype(kmax_c)::value;
            if (dt == CTWS_U8) k_prep_edt_x_co<KM, uint8_t><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
            else if (dt == CTWS_U16) k_prep_edt_x_co<KM, uint16_t><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
            else if (dt == CTWS_F32) k_prep_edt_x_co<KM, float><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
            else k_prep_edt_x_co<KM, double><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
        };
        if (typed && all_exact && maxX == 256)
            k_prep_edt_x_reg<4><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
        else if (typed && all_exact && maxX == 512)
            k_prep_edt_x_reg<8><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
        else if (typed && all_exact && maxX == 1024)
            k_prep_edt_x_reg<16><<<gx, 256, 0, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
        else if (typed && maxX <= 256)
            launch_co(std::integral_constant<int, 4>());
        else if (typed && maxX <= 512)
            launch_co(std::integral_constant<int, 8>());
        else if (typed && maxX <= 1024)
            launch_co(std::integral_constant<int, 16>());
        else {
            lds_optin(k_prep_edt_x, 4 * (size_t)maxX * 4);
            k_prep_edt_x<<<gx, 256, 4 * (size_t)maxX * 4, h->stream>>>(w.desc, w.stat, pp, fin_out, (uint32_t*)w.A);
        }
        LAUNCHCHK();
        if (pl.from_seeds) k_fs_active<<<(nb + 255) / 256, 256, 0, h->stream>>>(w.desc, w.stat, nb);
        else k_set_active<<<(nb + 255) / 256, 256, 0, h->stream>>>(w.desc, w.stat, nb);
        LAUNCHCHK();
    }
    mark("prep_edt_x");
    bool packed = true;
    uint32_t max_seeds = 0;  // sizes the LDS histogram of the size filter
    std::vector<BlockStat> s2(nb);
    const dim3 gsb((unsigned)((maxZ + 255) / 256), nb);
    if (pl.from_seeds) {
        if ((r = fs_seeds(h, desc, nb, TH, TW, TS, maxH, maxRows, vg, wg)) != CTWS_OK) return r;
    } else {
    if (real_edt) {
        // vigra's real-valued path: double temporary (non-integer pitch) or float (dmax >= 2^24)
        EdtRealParams er{{pl.pitchd[0], pl.pitchd[1], pl.pitchd[2]}, pl.dt_2d, real_double ? 1 : 0};
        const int nthr = 64 * 256;
        const int maxL = std::max(maxZ, std::max(maxY, maxX));
        const size_t esz = real_double ? 8 : 4;
        if ((r = grow(h, h->edt_scratch, (size_t)nthr * maxL * (2 * esz + 20))) != CTWS_OK) return r;
        char* scr = (char*)h->edt_scratch.p;
        auto run_real = [&](auto tag) {
            using T = decltype(tag);
            T* tmp = (T*)w.key;  // free until the flood
            k_edt_real_init<T><<<vg, 256, 0, h->stream>>>(w.desc, w.stat, er, (const uint32_t*)w.A, tmp);
            for (int a = pl.dt_2d ? 1 : 0; a < 3; ++a)
                k_edt_real_line<T><<<nthr / 256, 256, 0, h->stream>>>(w.desc, w.stat, nb, er, a, tmp, scr, maxL);
            k_edt_real_final<T><<<vg, 256, 0, h->stream>>>(w.desc, w.stat, er, tmp, w.dt, w.smin, w.smax);
        };
        if (real_double) run_real(double());
        else run_real(float());
        LAUNCHCHK();
        if (!pl.dt_2d && pl.nd_ws == 2) {
            dim3 gs((unsigned)maxZ, nb);
            k_dt_slice_stats<<<gs, 256, 0, h->stream>>>(w.desc, w.stat, w.dt, w.smin, w.smax);
            LAUNCHCHK();
        }
    } else {
        // y pass (final for a 2-D dt), then z pass (3-D dt)
        // (a forced width narrows until the column tile fits the LDS: the default already does)
        auto fit = [](int W, int L) {
            while (W > 8 && (size_t)L * W * 4 > kMaxLds) W /= 2;
            return W;
        };
        const int Wy = fit(h->edt_w ? h->edt_w : edt_col_width(maxY), maxY);
        EdtColParams ep{1, pl.pitch[1] * pl.pitch[1], pl.dt_2d, pl.dt_2d, 0u};
        dim3 gy((unsigned)((int64_t)maxZ * ((maxX + Wy - 1) / Wy)), nb);
        const size_t ldsy = (size_t)maxY * Wy * 4;
        // columns that may go to the lower-envelope pass: one entry each at most
        int64_t ncols = 0, ncols_z = 0;
        for (auto& d : desc) {
            ncols += (int64_t)d.Z * d.X;
            ncols_z += (int64_t)d.Y * d.X;
        }
        if (!pl.dt_2d) ncols = std::max(ncols, ncols_z);
        if ((r = grow(h, h->edt_fh, 64 + 8 * (size_t)ncols)) != CTWS_OK) return r;
        uint32_t* fh_cnt = (uint32_t*)h->edt_fh.p;
        unsigned long long* fh_list = (unsigned long long*)((char*)h->edt_fh.p + 64);
        HIPCHK(hipMemsetAsync(fh_cnt, 0, 64, h->stream));
        const unsigned gfh = (unsigned)std::min<int64_t>((ncols + 255) / 256, 1024);
        auto launch_col = [&](int W, dim3 g, size_t lds, EdtColParams p, const uint32_t* gin, uint32_t* gout,
                              uint32_t* cnt) {
            auto go = [&](auto kern) {
                lds_optin(kern, lds);
                kern<<<g, 256, lds, h->stream>>>(w.desc, w.stat, p, gin, gout, w.dt, w.smin, w.smax, fh_list, cnt);
            };
            if (W == 64) go(k_edt_col<64>);
            else if (W == 32) go(k_edt_col<32>);
            else if (W == 16) go(k_edt_col<16>);
            else go(k_edt_col<8>);
            k_edt_col_fh<<<gfh, 256, 0, h->stream>>>(w.desc, w.stat, p, gin, gout, w.dt, w.smin, w.smax, fh_list, cnt);
        };
        launch_col(Wy, gy, ldsy, ep, (uint32_t*)w.A, (uint32_t*)w.Bf, fh_cnt);
        LAUNCHCHK();
        if (!pl.dt_2d) {
            const int Wz = fit(h->edt_wz ? h->edt_wz : h->edt_w ? h->edt_w : edt_col_width(maxZ), maxZ);
            dim3 gz((unsigned)((int64_t)maxY * ((maxX + Wz - 1) / Wz)), nb);
            const size_t ldsz = (size_t)maxZ * Wz * 4;
            EdtColParams ez{2, pl.pitch[0] * pl.pitch[0], 1, 0, 0u};
            launch_col(Wz, gz, ldsz, ez, (uint32_t*)w.Bf, nullptr, fh_cnt + 1);
            LAUNCHCHK();
            if (pl.nd_ws == 2) {
                dim3 gs((unsigned)maxZ, nb);
                k_dt_slice_stats<<<gs, 256, 0, h->stream>>>(w.desc, w.stat, w.dt, w.smin, w.smax);
                LAUNCHCHK();
            }
        }
    }
    if (h->trace && !real_edt) {
        uint32_t c[2];
        HIPCHK(hipMemcpy(c, h->edt_fh.p, sizeof(c), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[ctws] edt lower-envelope columns: y %u z %u\n", c[0], c[1]);
    }
    if (pl.pass2 && pl.nd_ws == 2) {
        // two_pass_watershed.py:139: no maxima on initial seeds; per-slice dt stats again
        k_p2_zero_dt<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.dt);
        HIPCHK(hipMemsetD32Async((hipDeviceptr_t)w.smin, 0xFFFFFFFFu, (size_t)TS, h->stream));
        HIPCHK(hipMemsetAsync(w.smax, 0, sizeof(uint32_t) * TS, h->stream));
        dim3 gs((unsigned)maxZ, nb);
        k_dt_slice_stats<<<gs, 256, 0, h->stream>>>(w.desc, w.stat, w.dt, w.smin, w.smax);
        LAUNCHCHK();
    }
    mark("edt_yz");

    // ---- seed map smoothing, hmap -----------------------------------------------------------
    HmapParams hp{(float)cfg->alpha, (float)(1.0 - cfg->alpha), pl.nd_ws == 2 ? 1 : 0};
    const float* seedmap = w.dt;
    if (pl.seeds_smooth) {
        bool any = false;
        for (int a = (pl.nd_ws == 3 ? 0 : 1); a < 3; ++a) any |= pl.sig_seeds[a] > 0.0;
        if (any) {
            if ((r = run_gauss(h, pl, pl.sig_seeds, false, w.dt, w.sm, nb, maxZ, maxY, maxX, hp, 0)) != CTWS_OK)
                return r;
            seedmap = w.sm;
        }
    }
    mark("smooth_seeds");
    {
        const double sw[3] = {pl.weights_smooth ? pl.sig_weights[0] : 0.0, pl.weights_smooth ? pl.sig_weights[1] : 0.0,
                              pl.weights_smooth ? pl.sig_weights[2] : 0.0};
        if ((r = run_gauss(h, pl, sw, true, w.fin, w.hm, nb, maxZ, maxY, maxX, hp, 1)) != CTWS_OK) return r;
    }
    mark("hmap");

    // ---- seeds: local maxima, plateaus, CC, vigra scan-order ids -----------------------------
    {
        HIPCHK(hipMemsetAsync(h->ptile.p, 0, sizeof(uint32_t) * (size_t)std::max<int64_t>(TPT, 1), h->stream));
        k_localmax<<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, seedmap, w.cls, w.smax, (uint32_t*)h->ptile.p);
        LAUNCHCHK();
        // plateaus (equal-valued maxima candidates) and the seed CC: LDS tile union-find
        // (k_tilecc.hip); blocks without plateau voxels skip the plateau kernels on the device
        // the seed CC's member bitmap (CcArgs::troot for SEED): its parents are members-only
        HIPCHK(hipMemsetAsync(w.fseed, 0, sizeof(uint64_t) * (size_t)TF, h->stream));
        CcArgs ca{seedmap, w.cls, w.P, nullptr, nullptr, 0, w.fseed, nullptr, (const uint32_t*)h->ptile.p};
        if (pl.nd_ws == 3) {
            using T = CcTileM<3, CC_SEED>;  // (= the plateau tile)
            const dim3 tg(tiles8(cdiv(maxZ, T::TZ) * cdiv(maxY, T::TY) * cdiv(maxX, T::TX)), nb);
            k_tile_cc<3, CC_PLATEAU><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.P);
            k_tile_merge<3, CC_PLATEAU><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.P);
            k_plateau_flag<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.cls, w.P);
            if (h->seed_tilecc) {
                k_tile_cc<3, CC_SEED><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
                k_tile_merge<3, CC_SEED><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
            } else {
                // the seed components are the maximal plateaus and the isolated maxima (k_cc.hip)
                k_seed_members<3><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.cls, w.P, w.PF, w.fseed, nullptr);
            }
        } else {
            using T = CcTile<2>;
            const dim3 tg(tiles8(cdiv(maxZ, T::TZ) * cdiv(maxY, T::TY) * cdiv(maxX, T::TX)), nb);
            k_tile_cc<2, CC_PLATEAU><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.P);
            k_tile_merge<2, CC_PLATEAU><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.P);
            k_plateau_flag<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.cls, w.P);
            if (h->seed_tilecc) {
                k_tile_cc<2, CC_SEED><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
                k_tile_merge<2, CC_SEED><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
            } else {
                // every maximum its own root; the plateau maxima listed (in w.A, free until the size
                // filter) and united with their 4-adjacent maxima (k_cc.hip)
                k_seed_members<2><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.cls, w.P, w.PF, w.fseed,
                                                             (uint32_t*)w.A);
                k_seed_union2<<<dim3(64, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.cls, w.P, (const uint32_t*)w.A,
                                                                   w.PF);
            }
        }
        LAUNCHCHK();
    }
    HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
    k_flatten_seeds<<<dim3((unsigned)std::min<int64_t>((TF / nb + 255) / 256 + 1, 4096), nb), 256, 0, h->stream>>>(
        w.desc, w.stat, w.PF, w.fseed, w.W);
    k_bitmap_csum<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum);
    k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.csum, 0);
    k_word_prefix<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum, w.Wp);
    // (pass 1: the roots' positions per label for the sparse size filter, in w.Bf -- free after
    // the hmap; pass 2 relabels the seeds and records its ids' first positions below)
    k_root_label<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.PF, w.W, w.Wp, pl.pass2 ? nullptr : (uint32_t*)w.Bf);
    if (pl.pass2) {
        // _apply_watershed_with_seeds: shifted seeds + initial seeds, relabelConsecutive
        // the slices' seed bases of the seed CC into w.soff (free until k_slice_offsets): the
        // relabel keys of 2-D blocks need them after w.sb is rewritten for the new ids
        k_slice_seed_base<<<gsb, 256, 0, h->stream>>>(w.desc, w.stat, w.W, w.Wp, w.soff);
        HIPCHK(hipMemsetAsync(w.hkey, 0xFF, sizeof(uint64_t) * (size_t)TH, h->stream));
        HIPCHK(hipMemsetAsync(w.hpos, 0xFF, sizeof(uint32_t) * (size_t)TH, h->stream));
        // the relabel key of a voxel is computed where it is read (p2_value), no key array in HBM
        k_p2_insert<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, w.hpos, w.PF, w.fseed, w.soff,
                                               (const uint32_t*)h->p2_hint_dev.p);
        HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
        const dim3 hg((unsigned)std::min<int64_t>((maxH + 255) / 256, 4096), nb);
        k_p2_roots<<<hg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, w.hpos, w.W);
        k_bitmap_csum<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum);
        k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.csum, 0);
        k_word_prefix<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum, w.Wp);
        // the first position of each new id (a seed: it keeps the id) for the sparse size
        // filter, in w.dt (free after the seed CC)
        k_root_label<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, nullptr, w.W, w.Wp, (uint32_t*)w.dt);
        LAUNCHCHK();
    }
    }  // !from_seeds
    // packed flood keys need labels < 2^20 in every block of the batch
    {
        HIPCHK(hipMemcpyAsync(s2.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        for (auto& s : s2) {
            // (WatershedFromSeeds: a seedless block's seeds are its n_auto strict minima)
            const uint32_t ns = std::max(s.n_seeds, pl.from_seeds ? s.n_auto : 0u);
            if (ns >= (1u << 20) - 1u) packed = false;
            max_seeds = std::max(max_seeds, ns);
        }
        if (h->force_wide || h->wide_rerun) packed = false;
        if (!packed) {
            set_tiles(false);
            HIPCHK(hipMemcpyAsync(w.desc, desc.data(), sizeof(BlockDesc) * nb, hipMemcpyHostToDevice, h->stream));
            h->last_desc = desc;
        }
    }
    uint8_t* excl = nullptr;
    const bool descent = packed && !h->no_descent;
    const bool cc_seeds = descent && !pl.pass2 && !pl.from_seeds && h->stop_after != CTWS_STOP_SEEDS;
    const uint32_t* cc = cc_seeds ? w.PF : nullptr;
    if (pl.pass2) {
        k_slice_seed_base<<<gsb, 256, 0, h->stream>>>(w.desc, w.stat, w.W, w.Wp, w.sb);
        excl = (uint8_t*)w.fin;  // free after the hmap
        k_p2_excl_zero<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, excl);
        // 3-D: k_p2_label marks the exclusions from the initial values it reads anyway
        const int fused3 = pl.nd_ws == 3 ? 1 : 0;
        k_p2_label<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, w.hpos, w.W, w.Wp, w.hm, w.lab, w.key, w.cls,
                                              (uint32_t*)w.Bf, (uint32_t*)w.sm, packed ? 1 : 0, descent ? 0 : 1, w.PF,
                                              w.fseed, w.soff, (const uint32_t*)h->p2_hint_dev.p,
                                              fused3 ? excl : nullptr);
        if (!fused3) k_p2_excl<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.sb, excl);
    } else if (pl.from_seeds) {
        // labels, keys and seed flags in the packed / wide key form (fs_seeds counted them)
        k_fs_label<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, w.hpos, w.hm, w.lab, w.key, w.cls, packed ? 1 : 0);
        k_fs_auto_label<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.surv, w.W, w.Wp, w.hm, w.lab, w.key, w.cls,
                                                   packed ? 1 : 0);
    } else {
        // the descent flood reads the seeds from the CC parents directly (cc_seeds)
        if (!cc_seeds)
            k_seed_label<<<rg, 256, 0, h->stream>>>(w.desc, w.stat, w.PF, w.fseed, w.hm, w.lab, w.key, w.cls,
                                                    packed ? 1 : 0);
        k_slice_seed_base<<<gsb, 256, 0, h->stream>>>(w.desc, w.stat, w.W, w.Wp, w.sb);
    }
    LAUNCHCHK();
    mark("seeds");
    if (h->stop_after == CTWS_STOP_SEEDS) {
        HIPCHK(hipStreamSynchronize(h->stream));
        return CTWS_OK;
    }

    // ---- flood ------------------------------------------------------------------------------
    int rounds1 = 0, rounds2 = 0;
    h->flood_tiles = h->flood_iters = h->flood_lines = 0;
    float fk1 = 0.f, fk2 = 0.f;
    int fallback = 0, fiters = 0, fiters2 = 0;
    // statistics (CTWS_TRACE only): open voxels and frontier visits per block
    uint32_t* fst = h->trace ? w.fstat : nullptr;
    if (descent) {
        // descent pre-pass (k_flood.hip): voxels whose steepest descent reaches a seed are final
        // tile-local descent + pointer jumping (16^3 / 1 x 64 x 64 tiles)
        const int dz = pl.nd_ws == 3 ? 16 : 1, dy = pl.nd_ws == 3 ? 16 : 64, dx = pl.nd_ws == 3 ? 16 : 64;  // DTile
        const dim3 dg(tiles8(((maxZ + dz - 1) / dz) * ((maxY + dy - 1) / dy) * ((maxX + dx - 1) / dx)), nb);
        {
            if (pl.nd_ws == 3) k_descent_tile<3><<<dg, 512, 0, h->stream>>>(w.desc, w.stat, w.hm, w.lab, cc, w.fseed, w.P);
            else k_descent_tile<2><<<dg, 512, 0, h->stream>>>(w.desc, w.stat, w.hm, w.lab, cc, w.fseed, w.P);
            LAUNCHCHK();
        }
        mark("descent_tile");
        if (fst) HIPCHK(hipMemsetAsync(fst, 0, sizeof(uint32_t) * 2 * (size_t)nb, h->stream));
        // masked blocks: their plateau leaves the open set until the rest is flooded (k_plateau.hip);
        // the plateau level comes out of the descent pass
        bool any_mask = false;
        for (int i = 0; i < nb; ++i) any_mask |= desc[i].mask != nullptr;
        const bool plat_fill = h->plateau_fill && packed && any_mask;
        if (plat_fill) HIPCHK(hipMemsetAsync(w.plev, 0, sizeof(uint32_t) * (size_t)nb, h->stream));
        // 8 words in flight per wave step (4: +0.1 ms on config 3, +0.6 ms on config 4)
        k_descent_init<8><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.P, w.key, w.cls, w.fopen,
                                                     w.front0, fst, plat_fill ? w.plev : nullptr);
        LAUNCHCHK();
        if (plat_fill) {
            HIPCHK(hipMemsetAsync(w.fplat, 0, sizeof(uint64_t) * (size_t)TF, h->stream));
            k_plat_mark<<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.plev, w.fopen, w.fplat);
            LAUNCHCHK();
        }
        mark("flood_descent");
        // the remaining voxels: the frontier relaxation (k_frontier, one voxel per lane)
        if ((r = run_frontier(h, pl, nb, TF, max_tiles, TT, packed, fst, &fiters, &rounds1, &fk1)) != CTWS_OK)
            return r;
        if (plat_fill) {
            // the plateau: entries, min-plus runs along x, y (, z), then the frontier from there
            if (pl.nd_ws == 3) k_plat_entry<3><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fplat, w.plev);
            else k_plat_entry<2><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fplat, w.plev);
            const unsigned rows_g = (unsigned)std::min<int64_t>(((int64_t)maxZ * maxY + 3) / 4, 4096);
            const unsigned cols_g = (unsigned)std::min<int64_t>(((int64_t)std::max(maxZ, maxY) * ((maxX + 63) / 64) + 3) / 4, 4096);
            k_plat_scan_x<<<dim3(rows_g, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.key, w.fplat, w.plev);
            k_plat_scan_col<1><<<dim3(cols_g, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.key, w.fplat, w.plev);
            if (pl.nd_ws == 3)
                k_plat_scan_col<2><<<dim3(cols_g, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.key, w.fplat, w.plev);
            k_plat_restore<<<dim3((unsigned)std::min<int64_t>(((int64_t)maxZ * maxY * ((maxX + 63) / 64) + 255) / 256, 4096), nb), 256, 0, h->stream>>>(w.desc, w.stat, w.fopen, w.fplat,
                                                                                  w.front0);
            LAUNCHCHK();
            if ((r = run_frontier(h, pl, nb, TF, max_tiles, TT, packed, fst, &fiters, &rounds1, &fk1)) != CTWS_OK)
                return r;
        }
        mark("flood_relax");
        if (fst) {
            std::vector<uint32_t> hs(2 * (size_t)nb);
            HIPCHK(hipMemcpyAsync(hs.data(), fst, sizeof(uint32_t) * 2 * (size_t)nb, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            double no = 0, nv = 0;
            for (int i = 0; i < nb; ++i) {
                no += hs[i];
                nv += hs[nb + i];
            }
            add_timing(h, "open_voxels", (float)no);
            add_timing(h, "frontier_visits", (float)nv);
        }
        // fixpoint check of every voxel the relaxation solved (a guard: the descent argument and
        // the frontier's convergence make a violation impossible; on a violation the batch is
        // flooded again from the seeds alone) and the d-saturation detector (a solved key with d
        // at kDMax sets BlockStat::dsat: the block runs again on the wide keys).  The kernel
        // always runs; CTWS_VERIFY=0 drops only the violation handling.
        HIPCHK(hipMemsetAsync(w.counter, 0, 40, h->stream));
        if (pl.nd_ws == 3)
            k_flood_verify<3><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fopen, w.counter);
        else
            k_flood_verify<2><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fopen, w.counter);
        LAUNCHCHK();
        if (h->verify) {
            HIPCHK(hipMemcpyAsync(h->h_counter, w.counter, 40, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            if (h->trace && h->h_counter[0]) {
                fprintf(stderr, "[ctws] flood verify: violations at");
                for (uint32_t k = 0; k < std::min(8u, h->h_counter[1]); ++k) fprintf(stderr, " %u", h->h_counter[2 + k]);
                fprintf(stderr, "\n");
            }
            if (h->h_counter[0] && h->verify >= 2) {
                h->err = "flood fixpoint check failed (CTWS_VERIFY=2)";
                return CTWS_EHIP;
            }
            if (h->h_counter[0] && !h->no_fallback) {
                fallback = 1;
                k_flood_reset<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.lab, cc, w.fseed, w.key, w.cls);
                LAUNCHCHK();
                if ((r = run_flood(h, pl.nd_ws, packed, nb, max_tiles, TT, w.hm, false, &rounds1, &fk1)) != CTWS_OK)
                    return r;
            }
        }
        mark("flood_verify");
    } else {
        mark("flood_descent");
        if ((r = run_flood(h, pl.nd_ws, packed, nb, max_tiles, TT, w.hm, false, &rounds1, &fk1)) != CTWS_OK) return r;
    }
    // test hooks that stop after the flood read the workspace: a batch with a saturated packed
    // key (note_dsat) is run again whole on the wide keys, so they see the unbounded fixpoint too
    bool rerun_done = false;
    auto stop_dsat = [&]() -> int {
        if (!packed) return CTWS_OK;
        std::vector<BlockStat> sd(nb);
        HIPCHK(hipMemcpyAsync(sd.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        bool any = false;
        for (auto& x : sd) any |= x.active && x.dsat;
        if (!any) return CTWS_OK;
        ++h->wide_rerun;
        const int rr = run_batch(h, cfg, pl, blocks, io, nb);
        --h->wide_rerun;
        rerun_done = true;
        return rr;
    };
    if (h->stop_after == CTWS_STOP_FLOOD) {
        if ((r = stop_dsat()) != CTWS_OK || rerun_done) return r;
    }
    // the histogram, the filter and (pass 1) the final labels read the packed keys directly
    // (pass 2 reads its final labels from the packed keys too: k_slice_max, k_p2_output)
    if (packed && h->stop_after == CTWS_STOP_FLOOD)
        k_unpack_labels<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.key, w.lab);
    mark("flood");
    if (h->stop_after == CTWS_STOP_FLOOD) {
        HIPCHK(hipStreamSynchronize(h->stream));
        return CTWS_OK;
    }

    // ---- size filter + regrow ---------------------------------------------------------------
    std::vector<uint32_t> surv(TS, 1u);
    int n_auto_blocks = 0;
    bool regrow_bad = false;  // the regrow's fixpoint check failed: the batch's blocks fail
    if (cfg->size_filter > 0) {
        uint32_t* counts = (uint32_t*)w.A;
        auto histogram = [&]() -> int {
            k_hist_zero<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, counts);
            if (pl.nd_ws == 2) {
                // one LDS histogram per slice quarter over the slice's label range
                const dim3 g2((unsigned)maxZ * 4, nb);
                if (packed) k_hist2d<1><<<g2, 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key, w.sb, counts, 4);
                else k_hist2d<0><<<g2, 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key, w.sb, counts, 4);
            } else {
                // 32K voxels per workgroup: the LDS histogram is cleared / flushed once per 128 voxels
                dim3 hg((unsigned)std::min<int64_t>((maxN + 32767) / 32768, 2048), nb);
                const int bins = (int64_t)max_seeds + 1 <= kHistBins ? (int)max_seeds + 1 : 0;
                const size_t lds = sizeof(uint32_t) * (size_t)bins;
                if (packed) k_hist<1><<<hg, 256, lds, h->stream>>>(w.desc, w.stat, w.lab, w.key, counts, bins);
                else k_hist<0><<<hg, 256, lds, h->stream>>>(w.desc, w.stat, w.lab, w.key, counts, bins);
            }
            LAUNCHCHK();
            return CTWS_OK;
        };
        if ((r = histogram()) != CTWS_OK) return r;
        if (packed) {
            // survivors -> regrow seeds, removed voxels -> open; then the frontier relaxation
            std::vector<BlockStat> s3(nb);
            // a small size filter: the removed segments walked from their seeds (k_sf_plan decides
            // per block; CTWS_SF_SPARSE=0 scans every block).  WatershedFromSeeds numbers its
            // labels by seed value, without first positions: it scans
            const bool sparse_ok = h->sf_sparse && !pl.from_seeds && cfg->size_filter <= 64;
            const uint32_t* rootpos = pl.pass2 ? (const uint32_t*)w.dt : (const uint32_t*)w.Bf;
            auto regrow_init = [&]() -> int {
                HIPCHK(hipMemsetAsync(w.surv, 0, sizeof(uint32_t) * TS, h->stream));
                if (sparse_ok) {
                    k_sf_plan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, (uint32_t)cfg->size_filter, counts, excl,
                                                         w.sb, w.surv);
                    HIPCHK(hipMemsetAsync(w.fopen, 0, sizeof(uint64_t) * (size_t)TF, h->stream));
                    HIPCHK(hipMemsetAsync(w.front0, 0, sizeof(uint64_t) * (size_t)TF, h->stream));
                    k_sf_sparse<<<dim3((unsigned)std::max<uint32_t>((max_seeds + 255) / 256, 1u), nb), 256, 0,
                                   h->stream>>>(w.desc, w.stat, (uint32_t)cfg->size_filter, counts, excl,
                                                rootpos, w.hm, w.key, w.cls, w.fopen, w.front0);
                    LAUNCHCHK();
                }
                // 4 words per wave step (8: +1.2 ms on config 3, +2.2 ms on config 4)
                k_regrow_init<4><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, (uint32_t)cfg->size_filter, counts,
                                                            excl, w.hm, w.key, w.cls, w.fopen, w.front0, w.surv);
                LAUNCHCHK();
                HIPCHK(hipMemcpyAsync(surv.data(), w.surv, sizeof(uint32_t) * TS, hipMemcpyDeviceToHost, h->stream));
                HIPCHK(hipMemcpyAsync(s3.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
                HIPCHK(hipStreamSynchronize(h->stream));
                return CTWS_OK;
            };
            if ((r = regrow_init()) != CTWS_OK) return r;
            for (int i = 0; i < nb; ++i) {
                if (!s3[i].active) continue;
                const int ns = pl.nd_ws == 2 ? desc[i].Z : 1;
                bool need = false;
                for (int z = 0; z < ns; ++z) need |= !surv[desc[i].sbase + z];
                n_auto_blocks += need;
            }
            if (n_auto_blocks) {
                // every segment of a slice / block removed: vigra seeds the regrow from the strict
                // local minima of the hmap (watershedsNew with an all-zero seed image)
                HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
                const dim3 ag((unsigned)std::min<int64_t>(maxRows, 65535), nb);
                k_auto_minima<<<ag, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.surv, w.W);
                k_bitmap_csum<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum);
                k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.csum, 2);
                k_word_prefix<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum, w.Wp);
                k_auto_seed_set<<<ag, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.surv, w.W, w.Wp, w.sb, w.key,
                                                           w.cls, w.fopen, w.front0, nullptr);
                LAUNCHCHK();
            }
            if ((r = run_frontier(h, pl, nb, TF, max_tiles, TT, packed, nullptr, &fiters2, &rounds2, &fk2, true)) !=
                CTWS_OK)
                return r;
            // the regrow's fixpoint at the voxels it solved (the removed ones), and its d
            // saturation (as after the first flood: the kernel always runs)
            HIPCHK(hipMemsetAsync(w.counter, 0, 40, h->stream));
            if (pl.nd_ws == 3)
                k_flood_verify<3><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fopen, w.counter);
            else
                k_flood_verify<2><<<wtg, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.key, w.fopen, w.counter);
            LAUNCHCHK();
            if (h->verify) {
                HIPCHK(hipMemcpyAsync(h->h_counter, w.counter, 40, hipMemcpyDeviceToHost, h->stream));
                HIPCHK(hipStreamSynchronize(h->stream));
                if (h->h_counter[0] && h->verify >= 2) {
                    h->err = "regrow fixpoint check failed (CTWS_VERIFY=2)";
                    return CTWS_EHIP;
                }
                regrow_bad = h->h_counter[0] != 0;
            }
        } else {
            FilterParams fp{(uint32_t)cfg->size_filter, 0, 0, 0, w.act0};
            flood_tile_dims(pl.nd_ws, packed, &fp.tz, &fp.ty, &fp.tx);
            HIPCHK(hipMemsetAsync(w.act0, 0, sizeof(uint32_t) * (size_t)TT, h->stream));
            HIPCHK(hipMemsetAsync(w.surv, 0, sizeof(uint32_t) * TS, h->stream));
            k_size_filter<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, fp, counts, excl, w.hm, w.lab, w.key, w.cls,
                                                     w.surv, packed ? 1 : 0);
            LAUNCHCHK();
            HIPCHK(hipMemcpyAsync(surv.data(), w.surv, sizeof(uint32_t) * TS, hipMemcpyDeviceToHost, h->stream));
            std::vector<BlockStat> s3(nb);
            HIPCHK(hipMemcpyAsync(s3.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            for (int i = 0; i < nb; ++i) {
                if (!s3[i].active) continue;
                const int ns = pl.nd_ws == 2 ? desc[i].Z : 1;
                bool need = false;
                for (int z = 0; z < ns; ++z) need |= !surv[desc[i].sbase + z];
                n_auto_blocks += need;
            }
            if (n_auto_blocks) {
                // vigra's auto-seeding (above) on the wide keys: the strict minima as fixed seeds
                // with their labels in lab (any width); their tiles were freed, so they are active
                HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
                const dim3 ag((unsigned)std::min<int64_t>(maxRows, 65535), nb);
                k_auto_minima<<<ag, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.surv, w.W);
                k_bitmap_csum<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum);
                k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.csum, 2);
                k_word_prefix<<<wg, 256, 0, h->stream>>>(w.desc, w.stat, 0, w.W, w.csum, w.Wp);
                k_auto_seed_set<<<ag, 256, 0, h->stream>>>(w.desc, w.stat, w.hm, w.surv, w.W, w.Wp, w.sb, w.key,
                                                           w.cls, nullptr, nullptr, w.lab);
                LAUNCHCHK();
            }
            if ((r = run_flood(h, pl.nd_ws, packed, nb, max_tiles, TT, w.hm, true, &rounds2, &fk2)) != CTWS_OK)
                return r;
        }
    }
    mark("size_filter");
    const int keys_final = packed ? 1 : 0;  // final labels still in the keys

    // ---- pass 2: per-slice offsets, takeDict, uncropped inner write --------------------------
    const int ssplit = 4;  // workgroups per slice of the per-slice reductions
    if (pl.pass2) {
        if (pl.nd_ws == 2) {
            k_slice_max<<<dim3((unsigned)maxZ * ssplit, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key,
                                                                                  keys_final, w.sb, w.slmax, ssplit, 1);
            k_slice_offsets<<<nb, 64, 0, h->stream>>>(w.desc, w.stat, w.slmax, w.soff);
            k_p2_check<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.hkey, w.soff);
        }
        // per slice: an in-mask voxel (2-D only: a seedless 3-D block fails whatever its mask)
        HIPCHK(hipMemsetAsync(w.smin, 0, sizeof(uint32_t) * TS, h->stream));  // free after the hmap
        if (pl.nd_ws == 2) k_slice_inmask<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.smin);
        mark("finalize");
        mark("crop_cc");
        k_p2_output<<<ig, 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key, keys_final, (const uint32_t*)w.Bf,
                                               (const uint32_t*)w.sm, w.soff);
        LAUNCHCHK();
        mark("output");
    } else if (pl.from_seeds) {
        // WatershedFromSeeds: labels -> seed values (uint64), masked voxels 0; no crop / offset
        mark("finalize");
        mark("crop_cc");
        k_fs_output<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key, keys_final, (const uint32_t*)h->fs_sorted.p,
                                               w.surv, cfg->size_filter > 0 ? 1 : 0);
        LAUNCHCHK();
        mark("output");
    } else {
        // ---- 2-D offsets (uncropped blocks only: a cropped block is renumbered by its CC) ----
        bool any_crop = false, any_plain2d = false;
        for (int i = 0; i < nb; ++i) {
            any_crop |= desc[i].crop != 0;
            any_plain2d |= desc[i].crop == 0 && pl.nd_ws == 2;
        }
        const bool stop_ws = h->stop_after == CTWS_STOP_WS;
        if (pl.nd_ws == 2 && (any_plain2d || stop_ws)) {
            k_slice_max<<<dim3((unsigned)maxZ * ssplit, nb), 256, 0, h->stream>>>(
                w.desc, w.stat, w.lab, w.key, keys_final, w.sb, w.slmax, ssplit, stop_ws ? 1 : 0);
            k_slice_offsets<<<nb, 64, 0, h->stream>>>(w.desc, w.stat, w.slmax, w.soff);
        }
        if (stop_ws) {
            if ((r = stop_dsat()) != CTWS_OK || rerun_done) return r;
            // test hook: the final uint32 ws of the outer block in `lab`
            k_finalize_ws<<<vg, 256, 0, h->stream>>>(w.desc, w.stat, w.sb, w.soff, w.key, keys_final, w.lab);
            LAUNCHCHK();
            HIPCHK(hipStreamSynchronize(h->stream));
            return CTWS_OK;
        }
        LAUNCHCHK();
        mark("finalize");

        // ---- halo crop CC (labelVolumeWithBackground) + uint64 output --------------------------
        if (any_crop) {
            // tile roots of the crop CC marked in the (free) frontier bitmap front0
            HIPCHK(hipMemsetAsync(w.front0, 0, sizeof(uint64_t) * (size_t)TF, h->stream));
            CcArgs ca{nullptr, nullptr, nullptr, w.lab, w.key, keys_final, w.front0, (uint64_t*)h->xface.p, nullptr};
            const dim3 wgi((unsigned)((words_of(maxNI) + 255) / 256), nb);
            if (pl.nd_ws == 3) {
                using T = CcTile<3>;
                const dim3 tg(tiles8(cdiv(maxIZ, T::TZ) * cdiv(maxIY, T::TY) * cdiv(maxIX, T::TX)), nb);
                k_tile_cc<3, CC_CROP><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
                k_tile_merge<3, CC_CROP><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
            } else {
                using T = CcTile<2>;
                const dim3 tg(tiles8(cdiv(maxIZ, T::TZ) * cdiv(maxIY, T::TY) * cdiv(maxIX, T::TX)), nb);
                k_tile_cc<2, CC_CROP><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
                k_tile_merge<2, CC_CROP><<<dim3(std::min(tg.x, 2048u), tg.y), 256, 0, h->stream>>>(w.desc, w.stat, ca, w.PF);
            }
            HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
            k_flatten_tile_roots<<<wgi, 256, 0, h->stream>>>(w.desc, w.stat, w.PF, w.front0, w.W);
            k_bitmap_csum<<<wgi, 256, 0, h->stream>>>(w.desc, w.stat, 1, w.W, w.csum);
            k_chunk_scan<<<nb, 256, 0, h->stream>>>(w.desc, w.stat, 1, w.csum, 1);
            k_word_prefix<<<wgi, 256, 0, h->stream>>>(w.desc, w.stat, 1, w.W, w.csum, w.Wp);
            k_root_label<<<wgi, 256, 0, h->stream>>>(w.desc, w.stat, 1, w.PF, w.W, w.Wp, nullptr);
            LAUNCHCHK();
        }
        mark("crop_cc");
        bool any_plain = false;
        for (int i = 0; i < nb; ++i) any_plain |= desc[i].crop == 0;
        // uncropped blocks count their distinct ids in W (cropped blocks: n_cc of the crop CC)
        if (any_plain) HIPCHK(hipMemsetAsync(w.W, 0, sizeof(uint64_t) * (size_t)TW, h->stream));
        // cropped blocks: one workgroup per crop-CC tile, labels through LDS (k_output_crop)
        const bool crop_tiles = any_crop && h->output_tile;
        // (k_output still writes the uncropped blocks and the empty ones: constant offset)
        k_output<<<wtig, 256, 0, h->stream>>>(w.desc, w.stat, w.lab, w.key, keys_final, w.PF, w.sb, w.soff,
                                             (unsigned long long*)w.W, crop_tiles ? 1 : 0);
        if (crop_tiles) {
            if (pl.nd_ws == 3) {
                using T = CcTile<3>;
                const dim3 tg(tiles8(cdiv(maxIZ, T::TZ) * cdiv(maxIY, T::TY) * cdiv(maxIX, T::TX)), nb);
                k_output_crop<3><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, w.PF, w.front0);
            } else {
                using T = CcTile<2>;
                const dim3 tg(tiles8(cdiv(maxIZ, T::TZ) * cdiv(maxIY, T::TY) * cdiv(maxIX, T::TX)), nb);
                k_output_crop<2><<<tg, 256, 0, h->stream>>>(w.desc, w.stat, w.PF, w.front0);
            }
        }
        if (any_plain) k_count_ids<<<dim3(64, nb), 256, 0, h->stream>>>(w.desc, w.stat, w.W);
        LAUNCHCHK();
        mark("output");
    }

    HIPCHK(hipMemcpyAsync(st.data(), w.stat, sizeof(BlockStat) * nb, hipMemcpyDeviceToHost, h->stream));
    std::vector<uint32_t> sbh, inmask, soffh;
    if (pl.pass2) {
        sbh.resize(TS);
        inmask.resize(TS);
        HIPCHK(hipMemcpyAsync(sbh.data(), w.sb, sizeof(uint32_t) * TS, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipMemcpyAsync(inmask.data(), w.smin, sizeof(uint32_t) * TS, hipMemcpyDeviceToHost, h->stream));
        if (pl.nd_ws == 2) {
            soffh.resize(TS);
            HIPCHK(hipMemcpyAsync(soffh.data(), w.soff, sizeof(uint32_t) * TS, hipMemcpyDeviceToHost, h->stream));
        }
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    for (size_t i = 1; i < ev; ++i) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, h->events[i - 1], h->events[i]);
        add_timing(h, names[i], ms);
    }
    add_timing(h, "flood_rounds", (float)rounds1);
    add_timing(h, "frontier_iters", (float)fiters);
    add_timing(h, "regrow_iters", (float)fiters2);
    add_timing(h, "flood_fallback", (float)fallback);
    add_timing(h, "regrow_rounds", (float)rounds2);
    add_timing(h, "auto_seeded_blocks", (float)n_auto_blocks);
    add_timing(h, "flood_kernel_ms", fk1);
    add_timing(h, "flood_packed", packed ? 1.f : 0.f);
    add_timing(h, "flood_tiles_solved", (float)h->flood_tiles);
    add_timing(h, "flood_local_iters", (float)h->flood_iters);
    add_timing(h, "flood_lines_swept", (float)h->flood_lines);
    add_timing(h, "size_filter_kernel_ms", fk2);
    // blocks whose packed flood ended with a key with d at kDMax (note_dsat): the 12-bit hop distance
    // may have saturated, so they are flooded again on the wide keys (32-bit d) below, never
    // returned with a possibly different fixpoint
    std::vector<int> wide;
    if (packed)
        for (int i = 0; i < nb; ++i)
            if (st[i].active && st[i].dsat) wide.push_back(i);
    auto in_wide = [&](int i) { return std::find(wide.begin(), wide.end(), i) != wide.end(); };
    // pass 2 (2-D): blocks whose relabel needs the wrapped-id merge (k_p2_check) or whose offsets
    // differ from the hint they ran with run again with their offsets as the hint
    std::vector<int> redo;
    std::vector<std::vector<uint32_t>> redo_hint;
    if (pl.pass2 && pl.nd_ws == 2) {
        for (int i = 0; i < nb; ++i) {
            if (!st[i].active || in_wide(i)) continue;
            std::vector<uint32_t> so(soffh.begin() + desc[i].sbase, soffh.begin() + desc[i].sbase + desc[i].Z);
            const bool again = desc[i].p2hint < 0 ? (st[i].err & kErrCollision) != 0 : so != h->p2_hints[i];
            if (!again || (st[i].err & ~kErrCollision)) continue;  // (other failures stay failures)
            if (h->p2_depth > desc[i].Z + 1) continue;  // not converging: reported as a collision
            redo.push_back(i);
            redo_hint.push_back(std::move(so));
        }
    }
    for (int i = 0; i < nb; ++i) {
        blocks[i].status = st[i].active ? CTWS_BLOCK_WRITTEN : (pl.pass2 ? CTWS_BLOCK_EMPTY_PASS2 : CTWS_BLOCK_EMPTY);
        blocks[i].max_label = st[i].active ? st[i].max_label : 0;
        if (pl.from_seeds) {
            uint64_t mx;
            std::memcpy(&mx, &st[i]._p[2], sizeof(mx));
            blocks[i].max_label = mx;
        }
        // distinct nonzero output ids: the labels, plus the bare offset of unlabelled in-mask
        // voxels (empty block: only that one, watershed.py:310-321); block 0's offset is 0
        const uint32_t bare = (st[i].active ? st[i]._p[0] : 1u) && desc[i].id_offset != 0;
        blocks[i].n_ids = (pl.pass2 || pl.from_seeds) ? -1 : (int32_t)((st[i].active ? st[i].n_cc : 0u) + bare);
        if (!st[i].active) continue;
        if (std::find(redo.begin(), redo.end(), i) != redo.end()) continue;  // filled by the re-run below
        if (in_wide(i)) continue;  // filled by the wide re-run below
        uint32_t err = st[i].err | (regrow_bad ? kErrVerify : 0u);
        if (desc[i].p2hint >= 0 && !soffh.empty() &&
            !std::equal(h->p2_hints[i].begin(), h->p2_hints[i].end(), soffh.begin() + desc[i].sbase))
            err |= kErrCollision;  // the re-runs did not converge
        const int ns = pl.nd_ws == 2 ? desc[i].Z : 1;
        if (pl.pass2) {
            // a slice/block without any seed: watershedsNew seeds from the hmap minima and the
            // result has no new_to_old entry (takeDict, two_pass_watershed.py:173/204) where it
            // is not masked before the lookup (2-D: in-mask voxels; 3-D: every voxel)
            for (int z = 0; z < ns; ++z) {
                const int64_t s0 = desc[i].sbase + z;
                const uint32_t nl = pl.nd_ws == 2 ? ((z + 1 < ns ? sbh[s0 + 1] : st[i].n_seeds) - sbh[s0]) : st[i].n_seeds;
                if (!nl && (pl.nd_ws == 3 || inmask[s0])) err |= kErrTakeDict;
            }
        }
        if (err) {
            blocks[i].status = CTWS_BLOCK_FAILED;
            char msg[256];
            std::snprintf(msg, sizeof msg, "block %lld failed (%s%s%s%s%s%s%s); ", (long long)blocks[i].block_id,
                          (err & kErrHashFull) ? "pass-2 relabel hash table full " : "",
                          (err & kErrCollision) ? "pass-2 2-D wrapped-id merge did not converge " : "",
                          (err & kErrLabelBits) ? "auto-seed labels beyond 2^20 " : "",
                          (err & kErrTakeDict) ? "takeDict: no new_to_old entry, as in the reference " : "",
                          (err & kErrUnsupported) ? "auto-seeded regrow with >= 2^20 seeds " : "",
                          (err & kErrOverflow) ? "seed id >= 2^32 - 1: Overflow detected, as in the reference " : "",
                          (err & kErrVerify) ? "size-filter regrow fixpoint check failed " : "");
            h->err += msg;
        }
    }
    // per block: an in-mask voxel without a label (its output is the bare id offset), for the
    // host path's widening of the uint32 codes (empty blocks: every in-mask voxel)
    std::vector<uint8_t> bare(nb);
    for (int i = 0; i < nb; ++i) bare[i] = st[i].active ? (st[i]._p[0] != 0) : 1;
    if (!redo.empty()) {
        std::vector<ctws_block> rb;
        std::vector<BlockIO> rio;
        for (int i : redo) {
            rb.push_back(blocks[i]);
            rio.push_back(io[i]);
        }
        auto saved = std::move(h->p2_hints);
        h->p2_hints = std::move(redo_hint);
        ++h->p2_depth;
        const int rr = run_batch(h, cfg, pl, rb.data(), rio.data(), (int)rb.size());
        --h->p2_depth;
        h->p2_hints = std::move(saved);
        if (rr != CTWS_OK) return rr;
        for (size_t k = 0; k < redo.size(); ++k) {
            blocks[redo[k]].status = rb[k].status;
            blocks[redo[k]].max_label = rb[k].max_label;
            blocks[redo[k]].n_ids = rb[k].n_ids;
            if (k < h->last_bare.size()) bare[redo[k]] = h->last_bare[k];  // the re-run's result
        }
        // the device workspace now holds the re-run's blocks only: no block of this call can be
        // read back consistently (ctws_debug_read answers EINVAL)
        h->last_desc.clear();
        add_timing(h, "p2_merge_reruns", (float)redo.size());
    }
    if (!wide.empty()) {
        std::vector<ctws_block> rb;
        std::vector<BlockIO> rio;
        std::vector<std::vector<uint32_t>> rh;
        const bool hints = h->p2_hints.size() == (size_t)nb;
        for (int i : wide) {
            rb.push_back(blocks[i]);
            rio.push_back(io[i]);
            if (hints) rh.push_back(h->p2_hints[i]);
        }
        auto saved = std::move(h->p2_hints);
        h->p2_hints = std::move(rh);
        ++h->wide_rerun;
        const int rr = run_batch(h, cfg, pl, rb.data(), rio.data(), (int)rb.size());
        --h->wide_rerun;
        h->p2_hints = std::move(saved);
        if (rr != CTWS_OK) return rr;
        for (size_t k = 0; k < wide.size(); ++k) {
            blocks[wide[k]].status = rb[k].status;
            blocks[wide[k]].max_label = rb[k].max_label;
            blocks[wide[k]].n_ids = rb[k].n_ids;
            if (k < h->last_bare.size()) bare[wide[k]] = h->last_bare[k];
        }
        h->last_desc.clear();
        add_timing(h, "flood_wide_reruns", (float)wide.size());
    }
    h->last_bare = std::move(bare);
    return CTWS_OK;
}

// Why a block cannot run, or nullptr.  These blocks get CTWS_BLOCK_FAILED with the reason (the
// reference job would raise at that block, or the block is outside what the kernels support)
// while the other blocks of the call run.
const char* block_refusal(const Plan& pl, const ctws_block& b) {
    const int64_t Z = b.outer_shape[0], Y = b.outer_shape[1], X = b.outer_shape[2];
    if (X > kMaxRowX || Y > kMaxColLen || Z > kMaxColLen || Z * Y * X >= (1ll << 31))
        return "outer block too large for the kernels (X <= 10176, Y, Z <= 5088, fewer than 2^31 voxels)";
    // vigra's convolveLine: "kernel longer than line" (the reference raises at this block)
    auto too_short = [&](const double* sg, bool en) -> bool {
        if (!en) return false;
        const int64_t lens[3] = {Z, Y, X};
        for (int a = (pl.nd_ws == 3 ? 0 : 1); a < 3; ++a) {
            if (sg[a] <= 0) continue;
            int r = (int)(3.0 * sg[a] + 0.5);
            if (r == 0) r = 1;
            if (lens[a] < r + 1) return true;
        }
        return false;
    };
    if (!pl.from_seeds && (too_short(pl.sig_seeds, pl.seeds_smooth) || too_short(pl.sig_weights, pl.weights_smooth)))
        return "convolveLine(): kernel longer than line (vigra raises, as the reference job would)";
    return nullptr;
}

int64_t batch_voxels_budget() {
    const char* e = std::getenv("CTWS_BATCH_VOXELS");
    if (e) return std::max<int64_t>(1, std::atoll(e));
    return 512ll << 20;  // ~26 GB of workspace at ~50 B per voxel
}

// ---- host-pointer path: pinned staging, copies overlapped with the compute -----------------
// Batch j uses slot j & 1.  A worker thread packs batch j + 1's inputs into the slot's pinned
// buffer and starts its host-to-device copy on s_in while the calling thread runs batch j on
// the library stream; batch j's outputs go device-to-host on s_out and another worker unpacks
// them into the callers' arrays while batch j + 1 computes.  Events order every reuse of a slot.
// Host copies run on two persistent worker pools of the handle (ctws_host::WorkerPool): one for
// packing, one for widening.  Their sizes (CTWS_PACK_THREADS, CTWS_UNPACK_THREADS) leave a core
// to the calling thread, whose host round trips inside run_batch must not wait for one.
constexpr size_t kCopyChunk = (size_t)4 << 20;  // bytes per pool task

// the copies (dst, src, bytes) in 4 MiB tasks over the pool, streaming stores
void pool_copy(ctws_host::WorkerPool& pool, const std::vector<std::pair<void*, const void*>>& dst_src,
               const std::vector<size_t>& sizes) {
    std::vector<std::pair<size_t, size_t>> tasks;  // (copy index, byte offset)
    for (size_t i = 0; i < sizes.size(); ++i)
        for (size_t o = 0; o < sizes[i]; o += kCopyChunk) tasks.push_back({i, o});
    pool.parallel_for((int64_t)tasks.size(), [&](int64_t t) {
        const size_t i = tasks[t].first, o = tasks[t].second;
        ctws_host::stream_copy((char*)dst_src[i].first + o, (const char*)dst_src[i].second + o,
                               std::min(kCopyChunk, sizes[i] - o));
    });
}

// host <-> device copy in pieces of at most 1 GiB: larger copies are not given to the SDMA
// engines but run as a blit kernel that competes with the compute kernels for the CUs
hipError_t copy_pieces(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
    constexpr size_t kPiece = (size_t)1 << 30;
    for (size_t o = 0; o < bytes; o += kPiece) {
        const hipError_t e = hipMemcpyAsync((char*)dst + o, (const char*)src + o, std::min(kPiece, bytes - o), kind, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int grow_pinned(ctws_handle* h, void*& p, size_t& have, size_t bytes) {
    if (have >= bytes) return CTWS_OK;
    if (p) hipHostFree(p);
    p = nullptr;
    have = 0;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 256), hipHostMallocDefault) != hipSuccess) {
        h->err = "hipHostMalloc staging failed (" + std::to_string(bytes) + " bytes)";
        return CTWS_ENOMEM;
    }
    have = bytes;
    return CTWS_OK;
}

// uint32 codes of a block's inner region (k_output: the local label) -> the caller's uint64
// output: code + off, except for masked voxels (0).  A zero code is a masked voxel, or -- when
// the block has `bare` voxels (in-mask without a label) -- looked up in the caller's mask.
// Row ranges are the pool's tasks; stores stream past the caches.
void widen_codes(ctws_host::WorkerPool& pool, const ctws_block& b, const uint32_t* codes, uint64_t off, bool bare) {
    const int64_t IY = b.inner_shape[1], IX = b.inner_shape[2];
    const int64_t rows = b.inner_shape[0] * IY;
    const uint8_t* mask = (b.mask && off != 0 && bare) ? b.mask : nullptr;
    const bool masked = b.mask != nullptr && off != 0;
    const int64_t per = std::max<int64_t>(1, (int64_t)(kCopyChunk / 12) / std::max<int64_t>(IX, 1));  // rows per task
    pool.parallel_for((rows + per - 1) / per, [&](int64_t t) {
        const int64_t r0 = t * per, r1 = std::min(rows, r0 + per);
        if (!masked) {
            ctws_host::widen_add(b.output + r0 * IX, codes + r0 * IX, (r1 - r0) * IX, off);
        } else if (!mask) {
            ctws_host::widen_add_nz(b.output + r0 * IX, codes + r0 * IX, (r1 - r0) * IX, off);
        } else {
            for (int64_t r = r0; r < r1; ++r) {
                const uint32_t* c = codes + r * IX;
                uint64_t* o = b.output + r * IX;
                const int64_t z = r / IY, y = r - z * IY;
                const uint8_t* m = mask + ((z + b.inner_begin[0]) * b.outer_shape[1] + (y + b.inner_begin[1])) *
                                              b.outer_shape[2] + b.inner_begin[2];
                for (int64_t x = 0; x < IX; ++x) o[x] = (c[x] || m[x]) ? (uint64_t)c[x] + off : 0ull;
            }
        }
        _mm_sfence();
    });
}

struct HostBatch {
    int k, nb;  // blocks todo[k .. k + nb)
    std::vector<size_t> in_off, in_sz, m_off, i_off, o_off, o_sz;
    size_t in_bytes = 0, out_bytes = 0;
};

int run_blocks_host(ctws_handle* h, const ctws_cfg* cfg, const Plan& pl, ctws_block* blocks,
                    const std::vector<int>& todo) {
    int r;
    // (r02: 8-12 blocks of config 3 per batch, 4.3 Gvoxel/s, against 4.0 at the device budget)
    const int64_t budget = std::min(batch_voxels_budget(), h->host_batch_voxels);
    // batches and their packed layouts (inputs, masks and initial seeds in one buffer)
    std::vector<HostBatch> hb;
    size_t max_in = 0, max_out = 0;
    int64_t rem_vox = 0;
    for (int i : todo) rem_vox += blocks[i].outer_shape[0] * blocks[i].outer_shape[1] * blocks[i].outer_shape[2];
    for (size_t k = 0; k < todo.size();) {
        size_t e = k;
        int64_t vox = 0;
        // ramped batches: the first upload and the last download + widening are not overlapped
        // with compute, so the first two and the last batches are smaller (1/4, 1/2 of the budget)
        int64_t bud = budget;
        if (h->host_ramp) {
            if (hb.size() == 0) bud = budget / 4;
            else if (hb.size() == 1) bud = budget / 2;
            if (rem_vox < 2 * budget) bud = std::min(bud, std::max(budget / 4, rem_vox / 2));
        }
        while (e < todo.size()) {
            const ctws_block& b = blocks[todo[e]];
            const int64_t nv = b.outer_shape[0] * b.outer_shape[1] * b.outer_shape[2];
            if (e > k && (vox + nv > bud || e - k >= 4096 || (h->host_batch_blocks > 0 &&
                                                               (int)(e - k) >= h->host_batch_blocks)))
                break;
            vox += nv;
            ++e;
        }
        rem_vox -= vox;
        HostBatch B;
        B.k = (int)k;
        B.nb = (int)(e - k);
        auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
        for (int i = 0; i < B.nb; ++i) {
            const ctws_block& b = blocks[todo[k + i]];
            const int64_t nv = b.outer_shape[0] * b.outer_shape[1] * b.outer_shape[2];
            const size_t es = b.input_dtype == CTWS_U8 ? 1 : (b.input_dtype == CTWS_U16 ? 2 : (b.input_dtype == CTWS_F32 ? 4 : 8));
            B.in_sz.push_back((size_t)nv * es * (size_t)std::max(1, b.n_channels));
            B.in_off.push_back(B.in_bytes);
            B.in_bytes += al(B.in_sz.back());
            B.m_off.push_back(b.mask ? B.in_bytes : 0);
            if (b.mask) B.in_bytes += al((size_t)nv);
            B.i_off.push_back(b.initial_seeds ? B.in_bytes : 0);
            if (b.initial_seeds) B.in_bytes += al((size_t)nv * 8);
            B.o_sz.push_back((size_t)(b.inner_shape[0] * b.inner_shape[1] * b.inner_shape[2]) * 4);  // uint32 codes
            B.o_off.push_back(B.out_bytes);
            B.out_bytes += al(B.o_sz.back());
        }
        max_in = std::max(max_in, B.in_bytes);
        max_out = std::max(max_out, B.out_bytes);
        hb.push_back(std::move(B));
        k = e;
    }
    if (hb.empty()) return CTWS_OK;
    if (!h->pack_pool) h->pack_pool.reset(new ctws_host::WorkerPool(h->pack_threads));
    if (!h->unpack_pool) h->unpack_pool.reset(new ctws_host::WorkerPool(h->unpack_threads));
    if (!h->s_in) {
        HIPCHK(hipStreamCreateWithFlags(&h->s_in, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&h->s_out, hipStreamNonBlocking));
        for (auto& sl : h->hslot) {
            HIPCHK(hipEventCreateWithFlags(&sl.ev_h2d, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&sl.ev_comp, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&sl.ev_d2h, hipEventDisableTiming));
            HIPCHK(hipEventCreate(&sl.ev_t0));
            HIPCHK(hipEventCreate(&sl.ev_t1));
        }
    }
    const int nslots = hb.size() > 1 ? 2 : 1;
    for (int s = 0; s < nslots; ++s) {
        auto& sl = h->hslot[s];
        if ((r = grow_pinned(h, sl.pin_in, sl.pin_in_bytes, max_in)) != CTWS_OK) return r;
        if ((r = grow_pinned(h, sl.pin_out, sl.pin_out_bytes, max_out)) != CTWS_OK) return r;
        if ((r = grow(h, sl.d_in, max_in)) != CTWS_OK) return r;
        if ((r = grow(h, sl.d_out, max_out)) != CTWS_OK) return r;
        // a fresh handle's events have never been recorded: mark the slots free
        HIPCHK(hipEventRecord(sl.ev_d2h, h->s_out));
        HIPCHK(hipEventRecord(sl.ev_comp, h->stream));
    }
    // wall times (summed over batches) of the packing, widening and compute phases; the first
    // two run on worker threads, so they are only added to the timings at the end
    double pack_ms = 0.0, unpack_ms = 0.0, compute_ms = 0.0;
    const auto tcall = std::chrono::steady_clock::now();
    auto since = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - tcall).count() * 1e3; };
    // pack batch j's inputs into its slot and start the upload (worker thread)
    // pack batch j's inputs block by block into its slot, each block's upload starting as soon
    // as it is packed (worker thread)
    auto stage_in = [&](int j) -> int {
        const HostBatch& B = hb[j];
        auto& sl = h->hslot[j % nslots];
        // the slot's previous upload is complete (and its batch computed: run_batch returns
        // after its stream drained).  Copies wait on the host, never on another queue's event.
        if (hipEventSynchronize(sl.ev_h2d) != hipSuccess) return CTWS_EHIP;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < B.nb; ++i) {
            const ctws_block& b = blocks[todo[B.k + i]];
            const int64_t nv = b.outer_shape[0] * b.outer_shape[1] * b.outer_shape[2];
            std::vector<std::pair<void*, const void*>> ds{{(char*)sl.pin_in + B.in_off[i], b.input}};
            std::vector<size_t> sz{B.in_sz[i]};
            if (b.mask) {
                ds.push_back({(char*)sl.pin_in + B.m_off[i], b.mask});
                sz.push_back((size_t)nv);
            }
            if (b.initial_seeds) {
                ds.push_back({(char*)sl.pin_in + B.i_off[i], b.initial_seeds});
                sz.push_back((size_t)nv * 8);
            }
            pool_copy(*h->pack_pool, ds, sz);
            if (h->h2d_mode == 1 && i + 1 < B.nb) continue;  // one copy for the whole batch
            const size_t beg = h->h2d_mode == 1 ? 0 : B.in_off[i];
            const size_t end = i + 1 < B.nb ? B.in_off[i + 1] : B.in_bytes;
            if (i == 0 || h->h2d_mode == 1) {
                if (h->trace) hipEventRecord(sl.ev_t0, h->s_in);
            }
            if (h->h2d_mode == 2) {
                // pull kernel: a few workgroups read the pinned buffer over PCIe
                void* hsrc = nullptr;
                if (hipHostGetDevicePointer(&hsrc, sl.pin_in, 0) != hipSuccess) return CTWS_EHIP;
                k_copy_to_host<<<h->h2d_wgs, 256, 0, h->s_in>>>((const uint4*)((char*)hsrc + beg),
                                                                 (uint4*)((char*)sl.d_in.p + beg), (end - beg + 15) / 16);
                if (hipGetLastError() != hipSuccess) return CTWS_EHIP;
            } else if (copy_pieces((char*)sl.d_in.p + beg, (char*)sl.pin_in + beg, end - beg, hipMemcpyHostToDevice,
                                   h->s_in) != hipSuccess) {
                return CTWS_EHIP;
            }
        }
        if (h->trace) hipEventRecord(sl.ev_t1, h->s_in);
        const double ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
        pack_ms += ms;
        if (h->trace) std::fprintf(stderr, "[ctws] t=%.1f host batch %d: packed+queued in %.1f ms (%zu B)\n", since(), j, ms, B.in_bytes);
        return hipEventRecord(sl.ev_h2d, h->s_in) == hipSuccess ? CTWS_OK : CTWS_EHIP;
    };
    // widen batch j's uint32 codes into the callers' uint64 outputs block by block as their
    // downloads complete (worker thread)
    const uint64_t bvol = (uint64_t)(cfg->block_shape[0] * cfg->block_shape[1] * cfg->block_shape[2]);
    std::vector<std::vector<uint8_t>> bare_of(hb.size());
    auto drain_out = [&](int j, std::vector<ctws_block>* bbp) -> int {
        const HostBatch& B = hb[j];
        auto& sl = h->hslot[j % nslots];
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < B.nb; ++i) {
            const int st = (*bbp)[i].status;
            // nothing written: pass-2 empty (:240-242) or a failed block
            if (st == CTWS_BLOCK_EMPTY_PASS2 || st == CTWS_BLOCK_FAILED) continue;
            if (hipEventSynchronize(sl.ev_blk[i]) != hipSuccess) return CTWS_EHIP;
            const ctws_block& b = blocks[todo[B.k + i]];
            // pass 1: in-mask voxels get + block_id * prod(block_shape); pass 2 / from-seeds
            // outputs are the uint32 values themselves
            const uint64_t off = (pl.pass2 || pl.from_seeds) ? 0ull : (uint64_t)b.block_id * bvol;
            const bool bare = i < (int)bare_of[j].size() ? bare_of[j][i] != 0 : true;
            widen_codes(*h->unpack_pool, b, (const uint32_t*)((char*)sl.pin_out + B.o_off[i]), off, bare);
        }
        const double ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
        unpack_ms += ms;
        if (h->trace) std::fprintf(stderr, "[ctws] t=%.1f host batch %d: widened in %.1f ms (%zu B)\n", since(), j, ms, B.out_bytes);
        return CTWS_OK;
    };
    for (auto& sl : h->hslot) HIPCHK(hipEventRecord(sl.ev_h2d, h->s_in));
    int rin = stage_in(0);
    if (rin != CTWS_OK) return rin;
    std::vector<std::vector<ctws_block>> bbs(hb.size());
    std::thread t_in, t_out;
    int r_in = CTWS_OK, r_out = CTWS_OK;
    auto join_all = [&]() {
        if (t_in.joinable()) t_in.join();
        if (t_out.joinable()) t_out.join();
    };
    for (size_t j = 0; j < hb.size(); ++j) {
        const HostBatch& B = hb[j];
        auto& sl = h->hslot[j % nslots];
        if (j + 1 < hb.size()) t_in = std::thread([&, j]() { r_in = stage_in((int)j + 1); });
        std::vector<ctws_block>& bb = bbs[j];
        bb.resize(B.nb);
        std::vector<BlockIO> io(B.nb);
        for (int i = 0; i < B.nb; ++i) {
            bb[i] = blocks[todo[B.k + i]];
            const ctws_block& b = bb[i];
            io[i].in = (char*)sl.d_in.p + B.in_off[i];
            io[i].mask = b.mask ? (const uint8_t*)((char*)sl.d_in.p + B.m_off[i]) : nullptr;
            io[i].init = b.initial_seeds ? (const uint64_t*)((char*)sl.d_in.p + B.i_off[i]) : nullptr;
            io[i].out = nullptr;
            io[i].out32 = (uint32_t*)((char*)sl.d_out.p + B.o_off[i]);
        }
        // inputs uploaded; the slot's previous outputs downloaded
        if (hipEventSynchronize(sl.ev_h2d) != hipSuccess || hipEventSynchronize(sl.ev_d2h) != hipSuccess) {
            join_all();
            return CTWS_EHIP;
        }
        if (h->trace) {
            float up = 0.f;
            hipEventElapsedTime(&up, sl.ev_t0, sl.ev_t1);
            std::fprintf(stderr, "[ctws] t=%.1f host batch %zu: inputs on the device (first copy -> last: %.1f ms)\n",
                         since(), j, up);
        }
        const auto tb = std::chrono::steady_clock::now();
        if ((r = run_batch(h, cfg, pl, bb.data(), io.data(), B.nb)) != CTWS_OK) {
            join_all();
            return r;
        }
        {
            const double ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - tb).count() * 1e3;
            compute_ms += ms;
            if (h->trace) std::fprintf(stderr, "[ctws] t=%.1f host batch %zu (%d blocks): computed in %.1f ms\n", since(), j, B.nb, ms);
        }
        HIPCHK(hipEventRecord(sl.ev_comp, h->stream));
        bare_of[j] = h->last_bare;
        // the slot's pinned outputs are free once the drain of batch j - 2 finished
        if (t_out.joinable()) t_out.join();
        if (r_out != CTWS_OK) {
            join_all();
            return r_out;
        }
        // download block by block, an event after each
        while ((int)sl.ev_blk.size() < B.nb) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            sl.ev_blk.push_back(e);
        }
        hipError_t ce = hipSuccess;
        void* hdst = nullptr;
        if (h->d2h_wgs > 0) ce = hipHostGetDevicePointer(&hdst, sl.pin_out, 0);
        for (int i = 0; i < B.nb && ce == hipSuccess; ++i) {
            const size_t o = B.o_off[i], nbytes = (B.o_sz[i] + 15) & ~(size_t)15;
            if (h->d2h_wgs > 0) {
                k_copy_to_host<<<h->d2h_wgs, 256, 0, h->s_out>>>((const uint4*)((char*)sl.d_out.p + o),
                                                                  (uint4*)((char*)hdst + o), nbytes / 16);
                ce = hipGetLastError();
            } else {
                ce = copy_pieces((char*)sl.pin_out + o, (char*)sl.d_out.p + o, B.o_sz[i], hipMemcpyDeviceToHost,
                                 h->s_out);
            }
            if (ce == hipSuccess) ce = hipEventRecord(sl.ev_blk[i], h->s_out);
        }
        if (ce != hipSuccess ||
            hipEventRecord(sl.ev_d2h, h->s_out) != hipSuccess) {
            join_all();
            return CTWS_EHIP;
        }
        t_out = std::thread([&, j]() { r_out = drain_out((int)j, &bbs[j]); });
        if (t_in.joinable()) t_in.join();
        if (r_in != CTWS_OK) {
            join_all();
            return r_in;
        }
        for (int i = 0; i < B.nb; ++i) {
            blocks[todo[B.k + i]].status = bb[i].status;
            blocks[todo[B.k + i]].n_ids = bb[i].n_ids;
            blocks[todo[B.k + i]].max_label = bb[i].max_label;
        }
    }
    join_all();
    add_timing(h, "host_pack_ms", (float)pack_ms);
    add_timing(h, "host_unpack_ms", (float)unpack_ms);
    add_timing(h, "host_compute_ms", (float)compute_ms);
    add_timing(h, "host_batches", (float)hb.size());
    return r_out;
}

int run_blocks(ctws_handle* h, const ctws_cfg* cfg_in, ctws_block* blocks, int n, bool device_ptrs,
               bool from_seeds = false) {
    if (!h || !cfg_in || (!blocks && n > 0) || n < 0) return CTWS_EINVAL;
    h->err.clear();
    h->timings.clear();
    HIPCHK(hipSetDevice(h->device));
    ctws_cfg fcfg = *cfg_in;
    if (from_seeds) {
        // watershed_from_seeds.py: 3-D watershedsNew on the normalized input, no dt / smoothing
        fcfg.apply_ws_2d = fcfg.apply_dt_2d = 0;
        fcfg.has_pixel_pitch = 0;
        fcfg.sigma_seeds_is_list = fcfg.sigma_weights_is_list = 0;
        fcfg.sigma_seeds[0] = fcfg.sigma_weights[0] = 0.0;
        fcfg.invert_inputs = 0;
        fcfg.pass_id = 0;
        for (int i = 0; i < n; ++i) {
            ctws_block& b = blocks[i];
            for (int k = 0; k < 3; ++k) {
                if (b.inner_begin[k] != 0 || b.inner_shape[k] != b.outer_shape[k]) {
                    h->err = "WatershedFromSeeds blocks have no halo: inner block == block";
                    return CTWS_EINVAL;
                }
            }
            if (!b.initial_seeds) {
                h->err = "WatershedFromSeeds needs the seeds (ds_seeds[bb]) of every block";
                return CTWS_EINVAL;
            }
        }
    }
    const ctws_cfg* cfg = &fcfg;
    Plan pl;
    int r = make_plan(h, cfg, pl);
    if (r != CTWS_OK) return r;
    pl.from_seeds = from_seeds ? 1 : 0;
    // blocks whose inner mask is empty are skipped entirely (watershed.py:290-297); the
    // host-pointer path checks this on the host, the device path on the caller's side
    std::vector<int> todo;
    for (int i = 0; i < n; ++i) {
        ctws_block& b = blocks[i];
        b.status = CTWS_BLOCK_WRITTEN;
        b.n_ids = 0;
        b.max_label = 0;
        if (const char* why = block_refusal(pl, b)) {
            b.status = CTWS_BLOCK_FAILED;
            h->err += "block " + std::to_string((long long)b.block_id) + " failed (" + why + "); ";
            continue;
        }
        if (!device_ptrs && b.mask) {
            const int64_t* sh = b.outer_shape;
            bool any = false;
            for (int64_t z = 0; z < b.inner_shape[0] && !any; ++z)
                for (int64_t y = 0; y < b.inner_shape[1] && !any; ++y) {
                    const uint8_t* row = b.mask + ((z + b.inner_begin[0]) * sh[1] + (y + b.inner_begin[1])) * sh[2] +
                                         b.inner_begin[2];
                    for (int64_t x = 0; x < b.inner_shape[2]; ++x)
                        if (row[x]) {
                            any = true;
                            break;
                        }
                }
            if (!any) {
                b.status = CTWS_BLOCK_SKIPPED_MASK;
                continue;
            }
        }
        todo.push_back(i);
    }
    if (!device_ptrs) return run_blocks_host(h, cfg, pl, blocks, todo);
    const int64_t budget = batch_voxels_budget();
    size_t k = 0;
    while (k < todo.size()) {
        // batch [k, e)
        size_t e = k;
        int64_t vox = 0;
        while (e < todo.size()) {
            const ctws_block& b = blocks[todo[e]];
            const int64_t nv = b.outer_shape[0] * b.outer_shape[1] * b.outer_shape[2];
            if (e > k && (vox + nv > budget || e - k >= 4096)) break;  // <= 4096 blocks (worklist entries)
            vox += nv;
            ++e;
        }
        const int nb = (int)(e - k);
        std::vector<ctws_block> bb(nb);
        std::vector<BlockIO> io(nb);
        for (int i = 0; i < nb; ++i) bb[i] = blocks[todo[k + i]];
        if (device_ptrs) {
            for (int i = 0; i < nb; ++i)
                io[i] = {bb[i].input, bb[i].mask, bb[i].initial_seeds, bb[i].output};
            if ((r = run_batch(h, cfg, pl, bb.data(), io.data(), nb)) != CTWS_OK) return r;
        } else {
            if ((r = run_batch(h, cfg, pl, bb.data(), io.data(), nb)) != CTWS_OK) return r;
        }
        for (int i = 0; i < nb; ++i) {
            blocks[todo[k + i]].status = bb[i].status;
            blocks[todo[k + i]].n_ids = bb[i].n_ids;
            blocks[todo[k + i]].max_label = bb[i].max_label;
        }
        k = e;
    }
    return CTWS_OK;
}

}  // namespace

// =========================================================================================
extern "C" {

int ctws_abi_version(void) { return CTWS_ABI_VERSION; }

int ctws_open(int device, ctws_handle** out) {
    if (!out) return CTWS_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CTWS_EHIP;
    if (device < 0 || device >= n) return CTWS_EINVAL;
    ctws_handle* h = new ctws_handle();
    h->device = device;
    if (const char* t = std::getenv("CTWS_TRACE")) h->trace = std::atoi(t);
    if (const char* t = std::getenv("CTWS_NO_DESCENT")) h->no_descent = std::atoi(t);
    if (const char* t = std::getenv("CTWS_SEED_TILECC")) h->seed_tilecc = std::atoi(t);
    if (const char* t = std::getenv("CTWS_NO_FALLBACK")) h->no_fallback = std::atoi(t);
    if (const char* t = std::getenv("CTWS_FORCE_WIDE")) h->force_wide = std::atoi(t);
    if (const char* t = std::getenv("CTWS_SF_SPARSE")) h->sf_sparse = std::atoi(t);
    if (const char* t = std::getenv("CTWS_VERIFY")) h->verify = std::atoi(t);
    if (const char* t = std::getenv("CTWS_PREP_LDS")) h->prep_lds = std::atoi(t);
    if (const char* t = std::getenv("CTWS_FRONTIER_ITERS"))
        h->frontier_max_iters = std::max(0, std::min(kFrontierMaxItersCap, std::atoi(t)));
    if (const char* t = std::getenv("CTWS_GAUSS_YX")) h->gauss_yx = std::atoi(t);
    if (const char* t = std::getenv("CTWS_HOST_BATCH_VOXELS")) h->host_batch_voxels = std::max<int64_t>(1, std::atoll(t));
    if (const char* t = std::getenv("CTWS_HOST_RAMP")) h->host_ramp = std::atoi(t);
    if (const char* t = std::getenv("CTWS_PLATEAU_FILL")) h->plateau_fill = std::atoi(t);
    if (const char* t = std::getenv("CTWS_OUTPUT_TILE")) h->output_tile = std::atoi(t);
    if (const char* t = std::getenv("CTWS_H2D_MODE")) h->h2d_mode = std::atoi(t);
    if (const char* t = std::getenv("CTWS_H2D_WGS")) h->h2d_wgs = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_HOST_BATCH_BLOCKS")) h->host_batch_blocks = std::max(0, std::atoi(t));
    if (const char* t = std::getenv("CTWS_PACK_THREADS")) h->pack_threads = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_UNPACK_THREADS")) h->unpack_threads = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_D2H_WGS")) h->d2h_wgs = std::max(0, std::atoi(t));
    if (const char* t = std::getenv("CTWS_WORDS_PER_WAVE")) h->words_per_wave = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_GAUSS_W")) {
        const int v = std::atoi(t);
        h->gauss_w = (v == 8 || v == 16 || v == 32) ? v : 0;
    }
    if (const char* t = std::getenv("CTWS_EDT_W")) {
        const int v = std::atoi(t);
        h->edt_w = (v == 8 || v == 16 || v == 32 || v == 64) ? v : 0;
    }
    if (const char* t = std::getenv("CTWS_EDT_WZ")) {
        const int v = std::atoi(t);
        h->edt_wz = (v == 8 || v == 16 || v == 32 || v == 64) ? v : 0;
    }
    auto parse_chunk = [](const char* t, int* c, bool three_d) {
        int a = 0, b = 0, d = 0;
        if (std::sscanf(t, "%dx%dx%d", &a, &b, &d) == 3 && frontier_chunk_ok(three_d ? 3 : 2, a, b, d)) {
            c[0] = a;
            c[1] = b;
            c[2] = d;
        }
    };
    if (const char* t = std::getenv("CTWS_FRONTIER_CHUNK2D")) parse_chunk(t, h->fchunk2, false);
    if (const char* t = std::getenv("CTWS_FRONTIER_CHUNK3D")) {
        parse_chunk(t, h->fchunk3, true);
        h->fchunk3_env = 1;
    }
    if (const char* t = std::getenv("CTWS_FRONTIER_GRID")) h->frontier_grid = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_FRONTIER_REPS")) h->frontier_reps = std::max(1, std::atoi(t));
    if (const char* t = std::getenv("CTWS_FRONTIER_DIR")) h->frontier_dir = std::atoi(t) ? 1 : 0;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&h->h_counter, kCounterBytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&h->h_taps, 6 * kTapSlot * sizeof(double), hipHostMallocDefault) != hipSuccess) {
        delete h;
        return CTWS_EHIP;
    }
    *out = h;
    return CTWS_OK;
}

void ctws_close(ctws_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    Workspace& w = h->ws;
    void* ptrs[] = {w.fin, w.dt, w.A, w.Bf, w.sm, w.hm, w.cls, w.P, w.PF, w.lab, w.key, w.W, w.Wp, w.csum,
                    w.smin, w.smax, w.sb, w.slmax, w.soff, w.surv, w.act0, w.act1, w.lines0, w.lines1, w.desc, w.stat, w.counter,
                    w.taps, w.hkey, w.hpos, w.p2err, w.front0, w.front1, w.fopen, w.fflags, w.fchunk0, w.fchunk1, w.wl0, w.wl1, w.qgen, w.wlcnt,
                    w.fstat, h->st_in.p, h->st_mask.p, h->st_init.p, h->st_out.p, h->rl_lab.p, h->rl_bits.p,
                    h->rl_cnt.p, h->rl_offs.p, h->rl_out.p, h->rl_keys.p, h->rl_vals.p, h->rl_red.p,
                    h->edt_fh.p, h->edt_scratch.p, h->p2_hint_dev.p, h->rl_sorted.p, h->rl_uniq.p, h->rl_counts.p, h->rl_tmp.p,
                    h->fs_vals.p, h->fs_sorted.p, h->fs_off.p, h->fs_tmp.p, h->ev_ka.p, h->ev_ca.p, h->ev_kb.p,
                    h->ev_cb.p, h->ev_kp.p, h->ev_cp.p, h->ev_state.p, h->ev_out.p, h->ev_stage.p,
                    w.fplat, w.plev, w.fseed, h->tc_P.p, h->tc_bits.p, h->tc_cnt.p, h->tc_offs.p, h->tc_woff.p,
                    h->tc_red.p, h->tc_in.p, h->tc_mask.p, h->tc_out.p, h->tc_raw.p, h->tc_tmp.p, h->tc_taps.p};
    for (void* p : ptrs)
        if (p) hipFree(p);
    for (auto e : h->events) hipEventDestroy(e);
    for (auto e : h->fev)
        if (e) hipEventDestroy(e);
    if (h->h_counter) hipHostFree(h->h_counter);
    if (h->h_taps) hipHostFree(h->h_taps);
    for (auto& sl : h->hslot) {
        if (sl.pin_in) hipHostFree(sl.pin_in);
        if (sl.pin_out) hipHostFree(sl.pin_out);
        if (sl.d_in.p) hipFree(sl.d_in.p);
        if (sl.d_out.p) hipFree(sl.d_out.p);
        for (hipEvent_t e : {sl.ev_h2d, sl.ev_comp, sl.ev_d2h, sl.ev_t0, sl.ev_t1})
            if (e) hipEventDestroy(e);
        for (hipEvent_t e : sl.ev_blk) hipEventDestroy(e);
    }
    if (h->s_in) hipStreamDestroy(h->s_in);
    if (h->s_out) hipStreamDestroy(h->s_out);
    hipStreamDestroy(h->stream);
    delete h;
}

const char* ctws_last_error(const ctws_handle* h) { return h ? h->err.c_str() : "null handle"; }

int ctws_ws_blocks(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks) {
    return run_blocks(h, cfg, blocks, n_blocks, false);
}

int ctws_ws_blocks_device(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks) {
    return run_blocks(h, cfg, blocks, n_blocks, true);
}

// ---- evaluation: contingency table in HBM (k_eval.hip) ----------------------------------
static int64_t pow2_at_least(int64_t v) {
    int64_t c = 1024;
    while (c < v) c <<= 1;
    return c;
}

int ctws_eval_begin(ctws_handle* h, int64_t cap_labels, int64_t cap_pairs) {
    if (!h || cap_labels < 0 || cap_pairs < 0) return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    const int64_t ca = pow2_at_least(2 * std::max<int64_t>(cap_labels, 1));
    const int64_t cp = pow2_at_least(2 * std::max<int64_t>(cap_pairs, 1));
    if (ca > (1ll << 31) || cp > (1ll << 33)) {  // slots + the 2^64 - 1 slot fit the pair key's 32-bit halves
        h->err = "ctws_eval_begin: capacity too large";
        return CTWS_EINVAL;
    }
    int r;
    if ((r = grow(h, h->ev_ka, 8 * (size_t)(ca + 1))) != CTWS_OK || (r = grow(h, h->ev_ca, 8 * (size_t)(ca + 1))) != CTWS_OK ||
        (r = grow(h, h->ev_kb, 8 * (size_t)(ca + 1))) != CTWS_OK || (r = grow(h, h->ev_cb, 8 * (size_t)(ca + 1))) != CTWS_OK ||
        (r = grow(h, h->ev_kp, 8 * (size_t)cp)) != CTWS_OK || (r = grow(h, h->ev_cp, 8 * (size_t)cp)) != CTWS_OK ||
        (r = grow(h, h->ev_state, 16)) != CTWS_OK || (r = grow(h, h->ev_out, 6 * sizeof(double))) != CTWS_OK)
        return r;
    h->ev_cap_a = h->ev_cap_b = ca;
    h->ev_cap_p = cp;
    HIPCHK(hipMemsetAsync(h->ev_ka.p, 0xFF, 8 * (size_t)(ca + 1), h->stream));
    HIPCHK(hipMemsetAsync(h->ev_kb.p, 0xFF, 8 * (size_t)(ca + 1), h->stream));
    HIPCHK(hipMemsetAsync(h->ev_kp.p, 0xFF, 8 * (size_t)cp, h->stream));
    HIPCHK(hipMemsetAsync(h->ev_ca.p, 0, 8 * (size_t)(ca + 1), h->stream));
    HIPCHK(hipMemsetAsync(h->ev_cb.p, 0, 8 * (size_t)(ca + 1), h->stream));
    HIPCHK(hipMemsetAsync(h->ev_cp.p, 0, 8 * (size_t)cp, h->stream));
    HIPCHK(hipMemsetAsync(h->ev_state.p, 0, 16, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return CTWS_OK;
}

int ctws_eval_add(ctws_handle* h, const uint64_t* seg, const uint64_t* gt, int64_t n, int on_device, int ignore_gt_zero) {
    if (!h || n < 0 || (n > 0 && (!seg || !gt))) return CTWS_EINVAL;
    if (!h->ev_cap_a) {
        h->err = "ctws_eval_add before ctws_eval_begin";
        return CTWS_EINVAL;
    }
    HIPCHK(hipSetDevice(h->device));
    auto launch = [&](const uint64_t* s, const uint64_t* g, int64_t m) -> int {
        const unsigned grid = (unsigned)std::min<int64_t>((m + 255) / 256, 8192);
        k_eval_add<<<grid, 256, 0, h->stream>>>(s, g, m, ignore_gt_zero, (uint64_t*)h->ev_ka.p,
                                                 (unsigned long long*)h->ev_ca.p, h->ev_cap_a, (uint64_t*)h->ev_kb.p,
                                                 (unsigned long long*)h->ev_cb.p, h->ev_cap_b, (uint64_t*)h->ev_kp.p,
                                                 (unsigned long long*)h->ev_cp.p, h->ev_cap_p,
                                                 (unsigned long long*)h->ev_state.p);
        LAUNCHCHK();
        return CTWS_OK;
    };
    int r;
    if (on_device) {
        if ((r = launch(seg, gt, n)) != CTWS_OK) return r;
    } else {
        const int64_t chunk = (int64_t)1 << 25;  // voxels per staged piece (2 x 256 MiB)
        if ((r = grow(h, h->ev_stage, 16 * (size_t)std::min(chunk, std::max<int64_t>(n, 1)))) != CTWS_OK) return r;
        uint64_t* ds = (uint64_t*)h->ev_stage.p;
        for (int64_t o = 0; o < n; o += chunk) {
            const int64_t m = std::min(chunk, n - o);
            uint64_t* dg = ds + std::min(chunk, std::max<int64_t>(n, 1));
            HIPCHK(hipMemcpyAsync(ds, seg + o, 8 * (size_t)m, hipMemcpyHostToDevice, h->stream));
            HIPCHK(hipMemcpyAsync(dg, gt + o, 8 * (size_t)m, hipMemcpyHostToDevice, h->stream));
            if ((r = launch(ds, dg, m)) != CTWS_OK) return r;
        }
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    return CTWS_OK;
}

int ctws_eval_end(ctws_handle* h, double* scores, int64_t* n_points) {
    if (!h || !scores) return CTWS_EINVAL;
    if (!h->ev_cap_a) {
        h->err = "ctws_eval_end before ctws_eval_begin";
        return CTWS_EINVAL;
    }
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemsetAsync(h->ev_out.p, 0, 6 * sizeof(double), h->stream));
    const unsigned grid = (unsigned)std::min<int64_t>((std::max(h->ev_cap_a, h->ev_cap_p) + 255) / 256, 4096);
    k_eval_reduce<<<grid, 256, 0, h->stream>>>((const uint64_t*)h->ev_ka.p, (const unsigned long long*)h->ev_ca.p,
                                               h->ev_cap_a, (const uint64_t*)h->ev_kb.p,
                                               (const unsigned long long*)h->ev_cb.p, h->ev_cap_b,
                                               (const uint64_t*)h->ev_kp.p, (const unsigned long long*)h->ev_cp.p,
                                               h->ev_cap_p, (const unsigned long long*)h->ev_state.p,
                                               (double*)h->ev_out.p);
    LAUNCHCHK();
    double v[6];
    unsigned long long st[2];
    HIPCHK(hipMemcpyAsync(v, h->ev_out.p, sizeof(v), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(st, h->ev_state.p, sizeof(st), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (st[1]) {
        h->err = "contingency hash table full: call ctws_eval_begin with larger capacities";
        return CTWS_EUNSUPPORTED;
    }
    const double n = (double)st[0];
    if (n_points) *n_points = (int64_t)st[0];
    // validation_utils.py:60-76 (a = gt, b = seg) and :178-198
    scores[0] = v[1] - v[2];  // vi split
    scores[1] = v[0] - v[2];  // vi merge
    const double prec = v[4] > 0 ? v[5] / v[4] : 0.0, rec = v[3] > 0 ? v[5] / v[3] : 0.0;
    const double ari = (prec + rec) > 0 ? 2 * prec * rec / (prec + rec) : 0.0;
    scores[2] = 1.0 - ari;
    scores[3] = n > 0 ? 1.0 - (v[3] + v[4] - 2 * v[5]) / (n * n) : 1.0;
    return CTWS_OK;
}

int ctws_ws_from_seeds(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks) {
    return run_blocks(h, cfg, blocks, n_blocks, false, true);
}

int ctws_ws_from_seeds_device(ctws_handle* h, const ctws_cfg* cfg, ctws_block* blocks, int n_blocks) {
    return run_blocks(h, cfg, blocks, n_blocks, true, true);
}

int ctws_last_timings(const ctws_handle* h, const char** names, float* ms, int max_entries) {
    if (!h) return 0;
    const int n = (int)std::min<size_t>(h->timings.size(), (size_t)std::max(0, max_entries));
    for (int i = 0; i < n; ++i) {
        if (names) names[i] = h->timings[i].first;
        if (ms) ms[i] = h->timings[i].second;
    }
    return (int)h->timings.size();
}

int ctws_debug_set_stop(ctws_handle* h, int stage) {
    if (!h || stage < 0 || stage > 3) return CTWS_EINVAL;
    h->stop_after = stage;
    return CTWS_OK;
}

int ctws_debug_sqrt_int(ctws_handle* h, uint32_t n0, uint32_t count, float* dst) {
    if (!h || !dst || count == 0u || (uint64_t)n0 + count > (1ull << 24)) return CTWS_EINVAL;
    HIPCHK(hipSetDevice(h->device));
    float* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(float) * (size_t)count));
    k_sqrt_int_check<<<(count + 255u) / 256u, 256, 0, h->stream>>>(n0, count, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(dst, d, sizeof(float) * (size_t)count, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    hipFree(d);
    if (e != hipSuccess) {
        h->err = hipGetErrorString(e);
        return CTWS_EHIP;
    }
    return CTWS_OK;
}

int ctws_debug_read(ctws_handle* h, const char* array, int block, void* dst, int64_t nbytes) {
    if (!h || !array || !dst || block < 0 || block >= (int)h->last_desc.size()) return CTWS_EINVAL;
    const BlockDesc& d = h->last_desc[block];
    const Workspace& w = h->ws;
    const std::string a(array);
    const void* src = nullptr;
    size_t es = 4;
    if (a == "fin") src = w.fin;
    else if (a == "dt") src = w.dt;
    else if (a == "seedmap") src = w.sm;
    else if (a == "hmap") src = w.hm;
    else if (a == "labels") src = w.lab;
    else if (a == "cls") { src = w.cls; es = 1; }
    else return CTWS_EINVAL;
    if (nbytes != (int64_t)(d.N * es)) {
        h->err = "ctws_debug_read: nbytes must be N * itemsize";
        return CTWS_EINVAL;
    }
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipMemcpy(dst, (const char*)src + d.base * es, (size_t)nbytes, hipMemcpyDeviceToHost));
    return CTWS_OK;
}

}  // extern "C"

namespace {
// np.unique(labels[, return_counts]) by radix sort + run-length encoding (k_relabel.hip): any
// value range.  dl: device labels; out / counts: caller buffers (device or host), cap entries.
int unique_sorted(ctws_handle* h, const uint64_t* dl, int64_t n, int on_device, uint64_t* out, uint64_t* counts,
                  int64_t cap, int64_t* n_unique) {
    if (n >= (1ll << 31)) {
        h->err = "unique: more than 2^31 - 1 labels in one call";
        return CTWS_EUNSUPPORTED;
    }
    int r;
    size_t tb_sort = 0, tb_rle = 0;
    HIPCHK(u64_sort(nullptr, tb_sort, dl, nullptr, n, h->stream));
    HIPCHK(u64_runs(nullptr, tb_rle, nullptr, nullptr, nullptr, nullptr, n, h->stream));
    if ((r = grow(h, h->rl_sorted, sizeof(uint64_t) * (size_t)n)) != CTWS_OK) return r;
    if ((r = grow(h, h->rl_uniq, sizeof(uint64_t) * (size_t)n)) != CTWS_OK) return r;
    if ((r = grow(h, h->rl_counts, sizeof(uint64_t) * (size_t)n + 64)) != CTWS_OK) return r;
    if ((r = grow(h, h->rl_tmp, std::max(tb_sort, tb_rle))) != CTWS_OK) return r;
    uint64_t* sorted = (uint64_t*)h->rl_sorted.p;
    uint64_t* uniq = (uint64_t*)h->rl_uniq.p;
    uint64_t* cnt = (uint64_t*)h->rl_counts.p;
    uint64_t* nruns = cnt + n;  // (the counts buffer has 64 spare bytes)
    HIPCHK(u64_sort(h->rl_tmp.p, tb_sort, dl, sorted, n, h->stream));
    HIPCHK(u64_runs(h->rl_tmp.p, tb_rle, sorted, uniq, cnt, nruns, n, h->stream));
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, nruns, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    *n_unique = (int64_t)total;
    if ((int64_t)total > cap) {
        h->err = "unique: output capacity too small";
        return CTWS_EINVAL;
    }
    const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (total) {
        HIPCHK(hipMemcpyAsync(out, uniq, sizeof(uint64_t) * total, k, h->stream));
        if (counts) HIPCHK(hipMemcpyAsync(counts, cnt, sizeof(uint64_t) * total, k, h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    return CTWS_OK;
}

const uint64_t* stage_labels(ctws_handle* h, const uint64_t* labels, int64_t n, int on_device, int* r) {
    *r = CTWS_OK;
    if (on_device) return labels;
    if ((*r = grow(h, h->rl_lab, sizeof(uint64_t) * (size_t)n)) != CTWS_OK) return nullptr;
    if (hipMemcpyAsync(h->rl_lab.p, labels, sizeof(uint64_t) * (size_t)n, hipMemcpyHostToDevice, h->stream) !=
        hipSuccess) {
        h->err = "unique: label upload failed";
        *r = CTWS_EHIP;
        return nullptr;
    }
    return (const uint64_t*)h->rl_lab.p;
}
}  // namespace

extern "C" {

// ---- RelabelWorkflow kernels (k_relabel.hip) ----------------------------------------------
int ctws_unique_counts_u64(ctws_handle* h, const uint64_t* labels, int64_t n, int on_device, uint64_t* out,
                           uint64_t* counts, int64_t cap, int64_t* n_unique) {
    if (!h || (!labels && n > 0) || n < 0 || !n_unique || cap < 0 || ((!out || !counts) && cap > 0))
        return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    *n_unique = 0;
    if (n == 0) return CTWS_OK;
    int r;
    const uint64_t* dl = stage_labels(h, labels, n, on_device, &r);
    if (r != CTWS_OK) return r;
    return unique_sorted(h, dl, n, on_device, out, counts, cap, n_unique);
}

int ctws_unique_u64(ctws_handle* h, const uint64_t* labels, int64_t n, int on_device, uint64_t* out, int64_t cap,
                    int64_t* n_unique) {
    if (!h || (!labels && n > 0) || n < 0 || !n_unique || cap < 0 || (!out && cap > 0)) return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    *n_unique = 0;
    if (n == 0) return CTWS_OK;
    int r;
    const uint64_t* dl = stage_labels(h, labels, n, on_device, &r);
    if (r != CTWS_OK) return r;
    if ((r = grow(h, h->rl_red, 4 * sizeof(uint64_t))) != CTWS_OK) return r;
    unsigned long long* red = (unsigned long long*)h->rl_red.p;
    const unsigned long long init[3] = {~0ull, 0ull, 0ull};
    HIPCHK(hipMemcpyAsync(red, init, sizeof(init), hipMemcpyHostToDevice, h->stream));
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    k_u64_range<<<g, 256, 0, h->stream>>>(dl, n, red);
    LAUNCHCHK();
    unsigned long long hr[3];
    HIPCHK(hipMemcpyAsync(hr, red, sizeof(hr), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    const bool has_nz = hr[1] != 0ull;  // (the min stays ~0 when every nonzero label is 2^64 - 1)
    const int64_t first = hr[2] ? 1 : 0;
    int64_t total = first;
    if (has_nz) {
        const uint64_t lo = hr[0], span = hr[1] - hr[0];  // (+ 1 below; 0 .. 2^64 - 1 would wrap)
        // the bitmap (span / 8 bytes) only while it is no larger than sorting the labels would
        // need (~16 bytes each) or small anyway; otherwise sort (any value range)
        if (span >= (1ull << 35) || span / 64 + 1 > (uint64_t)std::max<int64_t>(2 * n, 1 << 20))
            return unique_sorted(h, dl, n, on_device, out, nullptr, cap, n_unique);
        const int64_t nw = (int64_t)(span / 64 + 1), nc = (nw + 255) / 256;
        if ((r = grow(h, h->rl_bits, sizeof(uint64_t) * (size_t)nw)) != CTWS_OK) return r;
        if ((r = grow(h, h->rl_cnt, sizeof(uint32_t) * (size_t)nc)) != CTWS_OK) return r;
        if ((r = grow(h, h->rl_offs, sizeof(uint64_t) * (size_t)(nc + 1))) != CTWS_OK) return r;
        HIPCHK(hipMemsetAsync(h->rl_bits.p, 0, sizeof(uint64_t) * (size_t)nw, h->stream));
        k_u64_bits<<<g, 256, 0, h->stream>>>(dl, n, lo, (unsigned long long*)h->rl_bits.p);
        k_bits_chunk_count<<<(unsigned)nc, 256, 0, h->stream>>>((const uint64_t*)h->rl_bits.p, nw,
                                                               (uint32_t*)h->rl_cnt.p);
        k_scan_chunks<<<1, 256, 0, h->stream>>>((const uint32_t*)h->rl_cnt.p, nc, (uint64_t*)h->rl_offs.p);
        LAUNCHCHK();
        uint64_t cnt = 0;
        HIPCHK(hipMemcpyAsync(&cnt, (uint64_t*)h->rl_offs.p + nc, sizeof(uint64_t), hipMemcpyDeviceToHost,
                              h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        total += (int64_t)cnt;
        *n_unique = total;
        if (total > cap) {
            h->err = "ctws_unique_u64: output capacity too small";
            return CTWS_EINVAL;
        }
        uint64_t* dout = out;
        if (!on_device) {
            if ((r = grow(h, h->rl_out, sizeof(uint64_t) * (size_t)total)) != CTWS_OK) return r;
            dout = (uint64_t*)h->rl_out.p;
        }
        k_bits_compact<<<(unsigned)nc, 256, 0, h->stream>>>((const uint64_t*)h->rl_bits.p, nw,
                                                           (const uint64_t*)h->rl_offs.p, lo, (uint64_t)first, dout);
        LAUNCHCHK();
        if (first) HIPCHK(hipMemsetAsync(dout, 0, sizeof(uint64_t), h->stream));
        if (!on_device)
            HIPCHK(hipMemcpyAsync(out, dout, sizeof(uint64_t) * (size_t)total, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        return CTWS_OK;
    }
    *n_unique = total;  // only zeros
    if (total > cap) {
        h->err = "ctws_unique_u64: output capacity too small";
        return CTWS_EINVAL;
    }
    if (on_device) HIPCHK(hipMemsetAsync(out, 0, sizeof(uint64_t), h->stream));
    else out[0] = 0;
    HIPCHK(hipStreamSynchronize(h->stream));
    return CTWS_OK;
}

int ctws_set_table_u64(ctws_handle* h, const uint64_t* keys, const uint64_t* values, int64_t n_table) {
    if (!h || n_table < 0 || ((!keys || !values) && n_table > 0)) return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    int r;
    if ((r = grow(h, h->rl_keys, sizeof(uint64_t) * (size_t)std::max<int64_t>(1, n_table))) != CTWS_OK) return r;
    if ((r = grow(h, h->rl_vals, sizeof(uint64_t) * (size_t)std::max<int64_t>(1, n_table))) != CTWS_OK) return r;
    if (n_table) {
        HIPCHK(hipMemcpyAsync(h->rl_keys.p, keys, sizeof(uint64_t) * (size_t)n_table, hipMemcpyHostToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->rl_vals.p, values, sizeof(uint64_t) * (size_t)n_table, hipMemcpyHostToDevice,
                              h->stream));
    }
    HIPCHK(hipStreamSynchronize(h->stream));
    h->rl_ntable = n_table;
    return CTWS_OK;
}

int ctws_lookup_u64(ctws_handle* h, uint64_t* labels, int64_t n, int on_device, const uint64_t* keys,
                    const uint64_t* values, int64_t n_table, int64_t* n_missing) {
    if (!h || (!labels && n > 0) || n < 0) return CTWS_EINVAL;
    const bool resident = !keys && !values;
    if (!resident && (n_table < 0 || ((!keys || !values) && n_table > 0))) return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    if (n_missing) *n_missing = 0;
    if (n == 0) return CTWS_OK;
    int r;
    if (resident) {
        n_table = h->rl_ntable;
    } else if (!on_device) {
        // host table: upload it as the resident one
        if ((r = ctws_set_table_u64(h, keys, values, n_table)) != CTWS_OK) return r;
    }
    const uint64_t* dk = (resident || !on_device) ? (const uint64_t*)h->rl_keys.p : keys;
    const uint64_t* dv = (resident || !on_device) ? (const uint64_t*)h->rl_vals.p : values;
    uint64_t* dl = labels;
    if (!on_device) {
        if ((r = grow(h, h->rl_lab, sizeof(uint64_t) * (size_t)n)) != CTWS_OK) return r;
        dl = (uint64_t*)h->rl_lab.p;
        HIPCHK(hipMemcpyAsync(dl, labels, sizeof(uint64_t) * (size_t)n, hipMemcpyHostToDevice, h->stream));
    }
    if ((r = grow(h, h->rl_red, 4 * sizeof(uint64_t))) != CTWS_OK) return r;
    unsigned long long* miss = (unsigned long long*)h->rl_red.p + 3;
    HIPCHK(hipMemsetAsync(miss, 0, sizeof(uint64_t), h->stream));
    const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);
    k_u64_lookup<<<g, 256, 0, h->stream>>>(dl, n, dk, dv, n_table, miss);
    LAUNCHCHK();
    unsigned long long hm = 0;
    HIPCHK(hipMemcpyAsync(&hm, miss, sizeof(hm), hipMemcpyDeviceToHost, h->stream));
    if (!on_device) HIPCHK(hipMemcpyAsync(labels, dl, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (n_missing) *n_missing = (int64_t)hm;
    return CTWS_OK;
}


// ---- ThresholdedComponentsWorkflow: BlockComponents (k_threshcc.hip) -----------------------
extern "C++" {
namespace {
size_t tc_dtype_size(int dt) {
    switch (dt) {
        case CTWS_U8: case CTWS_I8: return 1;
        case CTWS_U16: case CTWS_I16: return 2;
        case CTWS_F32: case CTWS_I32: case CTWS_U32: return 4;
        case CTWS_F64: case CTWS_I64: case CTWS_U64: return 8;
        default: return 0;
    }
}
// dispatch a k_tc_* template over the dataset dtype (float32 is the caller's own case)
template <class F>
void tc_dispatch(int dt, F f) {
    switch (dt) {
        case CTWS_U8: f((const uint8_t*)nullptr); break;
        case CTWS_I8: f((const int8_t*)nullptr); break;
        case CTWS_U16: f((const uint16_t*)nullptr); break;
        case CTWS_I16: f((const int16_t*)nullptr); break;
        case CTWS_U32: f((const uint32_t*)nullptr); break;
        case CTWS_I32: f((const int32_t*)nullptr); break;
        case CTWS_U64: f((const uint64_t*)nullptr); break;
        case CTWS_I64: f((const int64_t*)nullptr); break;
        case CTWS_F64: f((const double*)nullptr); break;
        default: break;
    }
}
}  // namespace
}  // extern "C++"

int ctws_threshold_components(ctws_handle* h, const float* input, const uint8_t* mask, int64_t nz, int64_t ny,
                              int64_t nx, int on_device, int mode, double threshold, int normalize, uint64_t* out,
                              int64_t* n_labels) {
    return ctws_threshold_components_ex(h, input, CTWS_F32, mask, nz, ny, nx, on_device, mode, threshold, normalize,
                                        0.0, out, n_labels);
}

int ctws_threshold_components_ex(ctws_handle* h, const void* input, int dtype, const uint8_t* mask, int64_t nz,
                                 int64_t ny, int64_t nx, int on_device, int mode, double threshold, int normalize,
                                 double sigma, uint64_t* out, int64_t* n_labels) {
    if (!h || !n_labels || nz < 0 || ny < 0 || nx < 0 || mode < 0 || mode > 2 || !(sigma >= 0.0)) return CTWS_EINVAL;
    const size_t esz = tc_dtype_size(dtype);
    if (!esz) {
        h->err = "ctws_threshold_components_ex: unsupported dtype";
        return CTWS_EINVAL;
    }
    const int64_t n = nz * ny * nx;
    if ((!input || !out) && n > 0) return CTWS_EINVAL;
    h->err.clear();
    HIPCHK(hipSetDevice(h->device));
    *n_labels = 0;
    if (n == 0) return CTWS_OK;
    if (n >= (int64_t)kNoParent || nz > INT32_MAX || ny > INT32_MAX || nx > INT32_MAX) {
        h->err = "ctws_threshold_components: block too large (needs < 2^32 - 1 voxels)";
        return CTWS_EINVAL;
    }
    std::vector<double> taps;
    if (sigma > 0.0) {
        taps = gaussian_taps(sigma);
        const int64_t rad = (int64_t)taps.size() / 2;
        if (nz < rad + 1 || ny < rad + 1 || nx < rad + 1) {  // vigra: "kernel longer than line"
            h->err = "ctws_threshold_components_ex: block shorter than the Gaussian radius + 1 along an axis";
            return CTWS_EINVAL;
        }
    }
    int r;
    const void* dsrc = input;
    const uint8_t* dmask = mask;
    uint64_t* dout = out;
    if (!on_device) {
        if ((r = grow(h, h->tc_raw, esz * (size_t)n)) != CTWS_OK) return r;
        if ((r = grow(h, h->tc_out, sizeof(uint64_t) * (size_t)n)) != CTWS_OK) return r;
        HIPCHK(hipMemcpyAsync(h->tc_raw.p, input, esz * (size_t)n, hipMemcpyHostToDevice, h->stream));
        dsrc = h->tc_raw.p;
        dout = (uint64_t*)h->tc_out.p;
        if (mask) {
            if ((r = grow(h, h->tc_mask, (size_t)n)) != CTWS_OK) return r;
            HIPCHK(hipMemcpyAsync(h->tc_mask.p, mask, (size_t)n, hipMemcpyHostToDevice, h->stream));
            dmask = (const uint8_t*)h->tc_mask.p;
        }
    }
    const int64_t nw = (n + 63) / 64, nc = (nw + 255) / 256;
    if ((r = grow(h, h->tc_P, sizeof(uint32_t) * (size_t)n)) != CTWS_OK) return r;
    if ((r = grow(h, h->tc_bits, sizeof(uint64_t) * (size_t)nw)) != CTWS_OK) return r;
    if ((r = grow(h, h->tc_cnt, sizeof(uint32_t) * (size_t)nc)) != CTWS_OK) return r;
    if ((r = grow(h, h->tc_offs, sizeof(uint64_t) * (size_t)(nc + 1))) != CTWS_OK) return r;
    if ((r = grow(h, h->tc_woff, sizeof(uint32_t) * (size_t)nw)) != CTWS_OK) return r;
    if ((r = grow(h, h->tc_red, 4 * sizeof(uint32_t))) != CTWS_OK) return r;
    uint32_t* red = (uint32_t*)h->tc_red.p;  // [0] min, [1] max (ordered float bits), [2] any member
    const uint32_t init[3] = {0xFFFFFFFFu, 0u, 0u};
    HIPCHK(hipMemcpyAsync(red, init, sizeof(init), hipMemcpyHostToDevice, h->stream));
    const unsigned gs = (unsigned)std::min<int64_t>((n + 255) / 256, 8192);  // grid of the streaming passes
    const unsigned gm = (unsigned)std::min<int64_t>((n + 4095) / 4096, 256);  // k_tc_minmax
    TcParams p;
    p.nz = (int)nz;
    p.ny = (int)ny;
    p.nx = (int)nx;
    p.mode = mode;
    p.normalize = normalize ? 1 : 0;
    p.thr = (float)threshold;
    const float* din = (const float*)dsrc;  // the float32 values k_tc_tile thresholds
    const bool raw_cmp = !normalize && sigma == 0.0 && dtype != CTWS_F32;
    if (raw_cmp || dtype != CTWS_F32) {
        if ((r = grow(h, h->tc_in, sizeof(float) * (size_t)n)) != CTWS_OK) return r;
        float* f = (float*)h->tc_in.p;
        if (raw_cmp) {
            // numpy's float64 comparison of the raw values; k_tc_tile tests the 0 / 1 result
            tc_dispatch(dtype, [&](auto tp) {
                using T = std::remove_cv_t<std::remove_pointer_t<decltype(tp)>>;
                k_tc_raw_members<T><<<gs, 256, 0, h->stream>>>((const T*)dsrc, n, mode, threshold, f);
            });
            p.mode = 0;
            p.thr = 0.5f;
        } else {
            tc_dispatch(dtype, [&](auto tp) {
                using T = std::remove_cv_t<std::remove_pointer_t<decltype(tp)>>;
                k_tc_to_f32<T><<<gs, 256, 0, h->stream>>>((const T*)dsrc, n, f);
            });
        }
        LAUNCHCHK();
        din = f;
    }
    if (sigma > 0.0) {
        // x (float32) -> [normalize] -> Gaussian z, y, x -> normalized by k_tc_tile
        if ((r = grow(h, h->tc_tmp, sizeof(float) * (size_t)n)) != CTWS_OK) return r;
        if ((r = grow(h, h->tc_taps, sizeof(double) * taps.size())) != CTWS_OK) return r;
        if (din == (const float*)dsrc) {  // float32 input: work on a copy, the caller's buffer is const
            if ((r = grow(h, h->tc_in, sizeof(float) * (size_t)n)) != CTWS_OK) return r;
            HIPCHK(hipMemcpyAsync(h->tc_in.p, din, sizeof(float) * (size_t)n, hipMemcpyDeviceToDevice, h->stream));
            din = (const float*)h->tc_in.p;
        }
        float* a = (float*)h->tc_in.p;
        float* b = (float*)h->tc_tmp.p;
        if (normalize) {
            k_tc_minmax<<<gm, 256, 0, h->stream>>>(a, n, red);
            k_tc_normalize<<<gs, 256, 0, h->stream>>>(a, n, red);
            HIPCHK(hipMemcpyAsync(red, init, sizeof(init), hipMemcpyHostToDevice, h->stream));
        }
        // (pageable upload: the host vector is gone after this call returns, the copy is not)
        HIPCHK(hipMemcpy(h->tc_taps.p, taps.data(), sizeof(double) * taps.size(), hipMemcpyHostToDevice));
        const int rad = (int)taps.size() / 2;
        for (int axis = 0; axis < 3; ++axis) {
            k_tc_gauss<<<gs, 256, 0, h->stream>>>(a, b, (int)nz, (int)ny, (int)nx, axis,
                                                  (const double*)h->tc_taps.p, rad);
            std::swap(a, b);
        }
        LAUNCHCHK();
        din = a;
        p.normalize = 1;  // vu.normalize of the smoothed block
    }
    if (p.normalize) {
        if (reinterpret_cast<uintptr_t>(din) % 16 != 0) {
            h->err = "ctws_threshold_components: input not 16-byte aligned";
            return CTWS_EINVAL;
        }
        k_tc_minmax<<<gm, 256, 0, h->stream>>>(din, n, red);
    }
    const int64_t tiles = ((nx + 63) / 64) * ((ny + 7) / 8) * ((nz + 7) / 8);
    uint32_t* P = (uint32_t*)h->tc_P.p;
    k_tc_tile<<<(unsigned)tiles, 256, 0, h->stream>>>(din, dmask, p, red, P, red + 2);
    LAUNCHCHK();
    uint32_t any = 0;
    HIPCHK(hipMemcpyAsync(&any, red + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    if (!any) return CTWS_OK;  // an empty block: no labels, the output is not written
    k_tc_merge<<<(unsigned)std::min<int64_t>(tiles, 4096), 256, 0, h->stream>>>(p, P);
    const unsigned gv = (unsigned)((n + 255) / 256);
    k_tc_roots<<<gv, 256, 0, h->stream>>>(P, n, (uint64_t*)h->tc_bits.p);
    k_bits_chunk_count<<<(unsigned)nc, 256, 0, h->stream>>>((const uint64_t*)h->tc_bits.p, nw,
                                                           (uint32_t*)h->tc_cnt.p);
    k_scan_chunks<<<1, 256, 0, h->stream>>>((const uint32_t*)h->tc_cnt.p, nc, (uint64_t*)h->tc_offs.p);
    k_tc_wordoff<<<(unsigned)nc, 256, 0, h->stream>>>((const uint64_t*)h->tc_bits.p, nw,
                                                     (const uint64_t*)h->tc_offs.p, (uint32_t*)h->tc_woff.p);
    k_tc_label<<<gv, 256, 0, h->stream>>>(P, n, (const uint64_t*)h->tc_bits.p, (const uint32_t*)h->tc_woff.p, dout);
    LAUNCHCHK();
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, (uint64_t*)h->tc_offs.p + nc, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    if (!on_device) HIPCHK(hipMemcpyAsync(out, dout, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    *n_labels = (int64_t)total;
    return CTWS_OK;
}


// ---- ThresholdedComponentsWorkflow: MergeAssignments (host) --------------------------------
// nifty.ufd.boost_ufd(n).merge(pairs); find(arange(n)) (merge_assignments.py:125-130): boost's
// disjoint_sets with union by rank -- link(find(a), find(b)) puts the root of lower rank under
// the other and, at equal ranks, the first root under the second (whose rank grows).  The
// representatives depend on the merge order, so this stays a sequential pass over the pairs.
int ctws_ufd_find(int64_t n, const uint64_t* pairs, int64_t n_pairs, uint64_t* out) {
    if (n < 0 || n_pairs < 0 || (!out && n > 0) || (!pairs && n_pairs > 0)) return CTWS_EINVAL;
    std::vector<uint64_t> parent((size_t)n);
    std::vector<uint8_t> rank((size_t)n, 0);
    for (int64_t i = 0; i < n; ++i) parent[(size_t)i] = (uint64_t)i;
    auto find = [&](uint64_t a) {
        uint64_t r = a;
        while (parent[r] != r) r = parent[r];
        while (parent[a] != r) {  // full path compression (boost's default find)
            const uint64_t nx = parent[a];
            parent[a] = r;
            a = nx;
        }
        return r;
    };
    for (int64_t k = 0; k < n_pairs; ++k) {
        const uint64_t a = pairs[2 * k], b = pairs[2 * k + 1];
        if (a >= (uint64_t)n || b >= (uint64_t)n) return CTWS_EINVAL;
        const uint64_t i = find(a), j = find(b);
        if (i == j) continue;
        if (rank[i] > rank[j]) {
            parent[j] = i;
        } else {
            parent[i] = j;
            if (rank[i] == rank[j]) ++rank[j];
        }
    }
    for (int64_t i = 0; i < n; ++i) out[i] = find((uint64_t)i);
    return CTWS_OK;
}

}  // extern "C"
