// k_post.hip — size filter, per-slice offsets and masking of the watershed labels.
//
// Reference: utils/volume_utils.py:131-139 (apply_size_filter: np.unique counts, ids with
// count < size_filter are zeroed, then a watershedsNew regrow seeded by the survivors),
// watershed.py:211-249 (_apply_watershed: 2-D per-slice offsets `offset += max_id`, mask
// zeroing), two_pass_watershed.py:160-161,199-202 (`exclude` ids, mismatched id space).
//
// Labels during the pipeline are unique within the block: in 2-D ws mode the seeds of
// slice z are numbered after those of slices < z (global rank in the slice-major key
// space), so one histogram serves all slices; `slice_seed_base[z]` converts back to the
// reference's per-slice numbering.
#include "ctws_kernels.h"

namespace ctws {

#define BLOCK_LOOP(i, B)                                                                      \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).N;              \
         i += (int64_t)gridDim.x * blockDim.x)

// seeds numbered before slice z: rank of key z*Y*X in the seed-root bitmap (2-D ws)
__global__ void __launch_bounds__(256) k_slice_seed_base(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                         const uint64_t* __restrict__ W,
                                                         const uint32_t* __restrict__ Wp, uint32_t* sb) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int z = blockIdx.x * blockDim.x + threadIdx.x;
    if (z >= B.Z) return;
    const uint32_t f = (uint32_t)((int64_t)z * B.Y * B.X);
    sb[B.sbase + z] = (B.nd_ws == 2) ? bitmap_rank(W + B.wbase, Wp + B.wbase, f) : 0u;
}

__global__ void __launch_bounds__(256) k_hist_zero(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   uint32_t* __restrict__ counts) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t n = (int64_t)S[blockIdx.y].n_seeds + 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        counts[B.base + i] = 0;
}

// count a wave's labels: one add per run of equal labels in consecutive lanes (voxels along x
// mostly share their label, so a mixed wave is a few runs, not 64 atomics on the same bins).
// ok: the lane holds a label to count (the invalid lanes are a tail of the wave)
template <class Add>
__device__ __forceinline__ void count_label_runs(uint32_t l, bool ok, int lane, Add add) {
    const uint32_t prev = (uint32_t)__shfl_up((int)l, 1);
    const uint64_t act = __ballot(ok);
    const uint64_t starts = __ballot(ok && (lane == 0 || prev != l));
    if (!((starts >> lane) & 1ull)) return;
    const uint64_t ends = (starts | ~act) & ~((2ull << lane) - 1ull);  // run boundaries above the lane
    const int next = ends ? __builtin_ctzll(ends) : 64;
    add(l, (uint32_t)(next - lane));
}

// label counts over the whole outer block (3-D) / slice (2-D: labels are slice-unique).
// Each workgroup counts a contiguous range in an LDS histogram of `bins` entries (dynamic
// LDS, sized by the host to the batch's largest seed count so that a few thousand labels do
// not cap the occupancy) and flushes its non-zero bins with one global atomic each; a block
// with more labels than bins counts with global atomics.
template <int PACKED>
__global__ void __launch_bounds__(256) k_hist(const BlockDesc* __restrict__ D, const BlockStat* S,
                                              const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                              uint32_t* __restrict__ counts, int bins) {
    extern __shared__ uint32_t sh[];
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    uint32_t* c = counts + B.base;
    const int64_t nb = (int64_t)S[blockIdx.y].n_seeds + 1;
    const bool use_lds = nb <= bins;
    if (use_lds)
        for (int j = threadIdx.x; j < nb; j += 256) sh[j] = 0;
    __syncthreads();
    const int64_t chunk = ((B.N + gridDim.x - 1) / gridDim.x + 255) & ~(int64_t)255;
    const int64_t i0 = (int64_t)blockIdx.x * chunk, i1 = min(B.N, i0 + chunk);
    const int lane = threadIdx.x & 63;
    constexpr int U = 8;  // loads in flight per thread
    for (int64_t ib = i0; ib < i1; ib += 256 * U) {
        uint32_t lv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * 256 + threadIdx.x;
            const int64_t ic = B.base + min(i, i1 - 1);  // unconditional loads: all in flight
            if (PACKED) {
                const uint64_t kv = key[ic];
                lv[u] = (uint32_t)(kv & ((1ull << 20) - 1ull)) | (kv == kInfKey ? 0x80000000u : 0u);
            } else {
                lv[u] = lab[ic] & ~kFixedBit;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * 256 + threadIdx.x;
            lv[u] = i >= i1 ? 0xFFFFFFFFu : ((lv[u] & 0x80000000u) ? 0u : lv[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t l = lv[u];
            count_label_runs(l, l != 0xFFFFFFFFu, lane, [&](uint32_t lb, uint32_t n) {
                if (use_lds) atomicAdd(&sh[lb], n);
                else atomicAdd(&c[lb], n);
            });
        }
    }
    if (!use_lds) return;
    __syncthreads();
    for (int j = threadIdx.x; j < nb; j += 256)
        if (sh[j]) atomicAdd(&c[j], sh[j]);
}

// 2-D ws: the labels of slice z are the block labels (sb[z], sb[z + 1]] (seeds are numbered
// slice-major), so each workgroup counts a quarter of one slice into a small LDS histogram of
// that range — no contention on a block-wide table of tens of thousands of labels.
constexpr int kHist2dBins = 8192;
template <int PACKED>
__global__ void __launch_bounds__(256) k_hist2d(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                                const uint32_t* __restrict__ sb, uint32_t* __restrict__ counts,
                                                int splits) {
    __shared__ uint32_t sh[kHist2dBins];
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int z = blockIdx.x / splits, s = blockIdx.x % splits;
    if (z >= B.Z) return;
    const uint32_t b0 = sb[B.sbase + z];
    const uint32_t b1 = z + 1 < B.Z ? sb[B.sbase + z + 1] : S[blockIdx.y].n_seeds;
    const uint32_t nb = b1 - b0;  // labels b0 + 1 .. b1 -> bins 0 .. nb - 1
    const bool use_lds = nb <= (uint32_t)kHist2dBins;
    if (use_lds)
        for (uint32_t j = threadIdx.x; j < nb; j += 256) sh[j] = 0;
    __syncthreads();
    const int64_t YX = (int64_t)B.Y * B.X;
    const int64_t i0 = (int64_t)z * YX + YX * s / splits, i1 = (int64_t)z * YX + YX * (s + 1) / splits;
    uint32_t* c = counts + B.base + b0 + 1;
    const int lane = threadIdx.x & 63;
    constexpr int U = 8;
    for (int64_t ib = i0; ib < i1; ib += 256 * U) {
        uint32_t lv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * 256 + threadIdx.x;
            const int64_t ic = B.base + min(i, i1 - 1);  // unconditional loads: all in flight
            if (PACKED) {
                const uint64_t kv = key[ic];
                lv[u] = (uint32_t)(kv & ((1ull << 20) - 1ull)) | (kv == kInfKey ? 0x80000000u : 0u);
            } else {
                lv[u] = lab[ic] & ~kFixedBit;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * 256 + threadIdx.x;
            lv[u] = i < i1 ? ((lv[u] & 0x80000000u) ? 0u : lv[u]) : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t l = lv[u];
            // (0, unreached, is not counted: k_sf_plan derives it from the counts)
            count_label_runs(l, l != 0xFFFFFFFFu, lane, [&](uint32_t lb, uint32_t n) {
                if (lb <= b0 || lb > b1) return;
                if (use_lds) atomicAdd(&sh[lb - b0 - 1], n);
                else atomicAdd(&c[lb - b0 - 1], n);
            });
        }
    }
    if (!use_lds) return;
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nb; j += 256)
        if (sh[j]) atomicAdd(&c[j], sh[j]);
}

// ---- sparse size-filter initialisation ---------------------------------------------------
// With a small size filter the removed segments are a few voxels each, yet k_regrow_init reads
// every voxel's key and seed flag.  A watershed segment is connected and contains its seed (the
// seed CC root of its label keeps it), so each removed segment can be walked from its seed
// instead: k_sf_plan decides per block (pass 1, packed keys: labels are seed CC ranks whose roots
// k_root_label recorded), k_sf_sparse walks each removed segment, and k_regrow_init skips the
// sparse blocks.  The walk writes what k_regrow_init would write where the regrow reads it: the
// removed voxels' keys (INF), seed flags and open bits, and the surviving neighbours' changed bits
// and seed keys (h, 0, label) -- survivors elsewhere are never read by the regrow.
constexpr uint32_t kSfSparseMax = 64;  // the largest size filter walked (a segment below it fits the queue)

// a label survives the size filter: count >= size_filter, or (pass 2) an excluded initial id
__device__ __forceinline__ bool sf_keeps(const uint32_t* c, const uint8_t* ex, uint32_t l, uint32_t size_filter) {
    return c[l] >= size_filter || (ex && ex[l]);
}

__global__ void __launch_bounds__(256) k_sf_plan(const BlockDesc* __restrict__ D, BlockStat* S, uint32_t size_filter,
                                                 const uint32_t* __restrict__ counts, const uint8_t* __restrict__ excl,
                                                 const uint32_t* __restrict__ sb, uint32_t* __restrict__ survivors) {
    const BlockDesc& B = D[blockIdx.x];
    BlockStat& st = S[blockIdx.x];
    if (!st.active) return;
    const uint32_t ns = st.n_seeds;
    const uint32_t* c = counts + B.base;
    const uint8_t* ex = excl ? excl + B.base : nullptr;
    uint32_t nsmall = 0, tot = 0;
    for (uint32_t l = 1 + threadIdx.x; l <= ns; l += 256) {
        nsmall += sf_keeps(c, ex, l, size_filter) ? 0u : 1u;
        tot += c[l];
    }
    nsmall = wg_reduce_u32(nsmall, OpAdd());
    // the voxels without a label (unreached by the flood): the block's voxels the labels' counts
    // leave over (every labelled voxel is counted once, 2-D slices in their own label ranges)
    tot = wg_reduce_u32(tot, OpAdd());
    // every slice (2-D) / the block (3-D) keeps a segment: no auto-seeded regrow
    uint32_t bare = 0;
    if (B.nd_ws == 2) {
        for (int z = threadIdx.x; z < B.Z; z += 256) {
            const uint32_t l0 = sb[B.sbase + z], l1 = z + 1 < B.Z ? sb[B.sbase + z + 1] : ns;
            bool any = false;
            for (uint32_t l = l0 + 1; l <= l1 && !any; ++l) any = sf_keeps(c, ex, l, size_filter);
            bare += any ? 0u : 1u;
        }
    } else {
        bare = threadIdx.x == 0 && nsmall == ns ? 1u : 0u;
    }
    bare = wg_reduce_u32(bare, OpAdd());
    const uint32_t unreached = (uint32_t)B.N - tot;
    const bool sparse = size_filter <= kSfSparseMax && !unreached && !bare &&
                        (uint64_t)nsmall * size_filter <= (uint64_t)B.N / 8;
    if (threadIdx.x == 0) st.sf_sparse = sparse ? 1u : 0u;
    if (sparse)
        for (int z = threadIdx.x; z < (B.nd_ws == 2 ? B.Z : 1); z += 256) survivors[B.sbase + z] = 1u;
}

// one thread per label of the block: a removed segment (count < size_filter) is walked from its
// seed (breadth first, in-plane 4-neighbourhood in 2-D ws mode, 6 in 3-D)
__global__ void __launch_bounds__(256) k_sf_sparse(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   uint32_t size_filter, const uint32_t* __restrict__ counts,
                                                   const uint8_t* __restrict__ excl,
                                                   const uint32_t* __restrict__ rootpos, const float* __restrict__ h,
                                                   uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv,
                                                   uint64_t* __restrict__ open, uint64_t* __restrict__ chg) {
    const BlockDesc& B = D[blockIdx.y];
    const BlockStat& st = S[blockIdx.y];
    if (!st.active || !st.sf_sparse) return;
    const uint32_t l = 1u + blockIdx.x * blockDim.x + threadIdx.x;
    if (l > st.n_seeds) return;
    const uint32_t* c = counts + B.base;
    const uint8_t* ex = excl ? excl + B.base : nullptr;
    if (sf_keeps(c, ex, l, size_filter)) return;
    uint64_t* kb = key + B.base;
    const int wpr = (B.X + 63) >> 6;
    const int64_t YX = (int64_t)B.Y * B.X;
    auto setbit = [&](uint64_t* bm, int64_t i) {
        const int64_t row = i / B.X;
        const int x = (int)(i - row * B.X);
        atomicOr((unsigned long long*)&bm[B.fbase + row * wpr + (x >> 6)], 1ull << (x & 63));
    };
    uint32_t q[kSfSparseMax];
    int qh = 0, qt = 0;
    auto claim = [&](int64_t i) {
        kb[i] = kPackInf;
        fixedv[B.base + i] = 0;
        setbit(open, i);
        q[qt++] = (uint32_t)i;
    };
    claim((int64_t)rootpos[B.base + l]);
    while (qh < qt) {
        const int64_t v = q[qh++];
        // (32-bit divisions: a block holds fewer than 2^31 voxels)
        const int z = (int)((uint32_t)v / (uint32_t)YX);
        const uint32_t r = (uint32_t)v - (uint32_t)z * (uint32_t)YX;
        const int y = (int)(r / (uint32_t)B.X), x = (int)(r - (uint32_t)y * (uint32_t)B.X);
        int64_t nbr[6];
        int nn = 0;
        if (x > 0) nbr[nn++] = v - 1;
        if (x + 1 < B.X) nbr[nn++] = v + 1;
        if (y > 0) nbr[nn++] = v - B.X;
        if (y + 1 < B.Y) nbr[nn++] = v + B.X;
        if (B.nd_ws == 3) {
            if (z > 0) nbr[nn++] = v - YX;
            if (z + 1 < B.Z) nbr[nn++] = v + YX;
        }
        for (int k = 0; k < nn; ++k) {
            const int64_t u = nbr[k];
            const uint64_t ku = kb[u];
            if (ku == kPackInf) continue;  // removed already (this segment or another)
            const uint32_t lu = (uint32_t)(ku & kLabelMask);
            if (lu == l) {
                if (qt < (int)kSfSparseMax) claim(u);
                continue;
            }
            if (!sf_keeps(c, ex, lu, size_filter)) continue;  // another removed segment (its own thread)
            // a survivor next to the removed segment: a regrow seed, read by the frontier
            setbit(chg, u);
            if (ku & kDMask) {
                kb[u] = ((uint64_t)ordf(h[B.base + u]) << 32) | (uint64_t)lu;
                fixedv[B.base + u] = 1;
            }
        }
    }
}

// seed flags from the open bitmap (the fallback tile flood of a sparse regrow: every voxel that
// is not open is a survivor, a seed of the regrow)
__global__ void __launch_bounds__(256) k_fixed_from_open(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                         const uint64_t* __restrict__ open, uint8_t* __restrict__ fixedv) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !S[blockIdx.y].sf_sparse) return;
    WORD_TILES(B.Z, B.Y, B.X, {
        if (valid) fixedv[B.base + i] = ((open[B.fbase + w_] >> lane) & 1ull) ? 0 : 1;
    })
}

// Size filter + regrow initialisation for the frontier relaxation (packed keys).  The regrow
// is watershedsNew(hmap, seeds=seg) on the filtered labels (volume_utils.py:131-139): every
// surviving voxel is a seed pushed with priority h (key (h, 0, label)), every removed voxel is
// reset.  The open bitmap gets the removed voxels and the changed bitmap the survivors, so
// the first frontier is exactly the removed voxels next to a survivor (k_frontier, k_flood.hip).
// survivors[slice (2-D) / 0 (3-D)] = 1 if any label survives there.
template <int U>
__global__ void __launch_bounds__(256) k_regrow_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     uint32_t size_filter, const uint32_t* __restrict__ counts,
                                                     const uint8_t* __restrict__ excl, const float* __restrict__ h,
                                                     uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv,
                                                     uint64_t* __restrict__ open, uint64_t* __restrict__ chg,
                                                     uint32_t* __restrict__ survivors) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || S[blockIdx.y].sf_sparse) return;  // (walked by k_sf_sparse)
    constexpr uint64_t kLab = (1ull << 20) - 1ull;
    // word tiles (a wave's ballot is exactly one word of the open / changed bitmaps), U words per
    // step: the loads of the U words, then their dependent count loads, in flight together
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nwords + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t wbeg = wid * per, wend = min(nwords, wbeg + per);
    // (row, word in the row) of the wave's next word, advanced word by word: no 64-bit division
    // per word (the emulated scalar divisions cost more issue time than the loads)
    int row_n = (int)(wbeg / wpr), xw_n = (int)(wbeg - (int64_t)row_n * wpr);
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
        int64_t gi[U];
        bool valid[U];
        int rows[U];
        uint64_t kv[U];
        uint8_t fx[U];
        float hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            rows[u] = row_n;
            const int x = xw_n * 64 + lane;
            if (++xw_n == wpr) {
                xw_n = 0;
                ++row_n;
            }
            valid[u] = w0 + u < wend && x < B.X;
            // loads unconditional (clamped index): key and seed flag together
            gi[u] = B.base + (valid[u] ? (int64_t)rows[u] * B.X + x : 0);
            kv[u] = key[gi[u]];
            fx[u] = fixedv[gi[u]];
        }
        uint32_t lb[U], cnt[U];
        bool ex[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!valid[u]) {
                kv[u] = kInfKey;
                fx[u] = 0;
            }
            lb[u] = kv[u] == kInfKey ? 0u : (uint32_t)(kv[u] & kLab);
            cnt[u] = counts[B.base + lb[u]];
            ex[u] = excl ? excl[B.base + lb[u]] != 0 : false;
            // the height only where a relaxed voxel's key is not (h, 0, label) already: a key
            // with d = 0 is (h, 0, label) (f resets to the voxel's own height), so only the
            // voxels flooded over an equal-C plateau (d > 0: a few per cent of the relaxed ones)
            // need it; words without one skip the load
            hv[u] = __ballot(valid[u] && !fx[u] && lb[u] != 0 && (kv[u] & kDMask) != 0ull) ? h[gi[u]] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool keep = lb[u] != 0 && (cnt[u] >= size_filter || ex[u]);
            if (valid[u]) {
                if (keep) {
                    if (!fx[u]) {
                        if (kv[u] & kDMask) key[gi[u]] = ((uint64_t)ordf(hv[u]) << 32) | (uint64_t)lb[u];
                        fixedv[gi[u]] = 1;
                    }
                } else {
                    if (kv[u] != kInfKey) key[gi[u]] = kInfKey;
                    if (fx[u]) fixedv[gi[u]] = 0;
                }
            }
            const uint64_t op = __ballot(valid[u] && !keep);
            const uint64_t kp = __ballot(valid[u] && keep);
            if (lane == 0 && w0 + u < wend) {
                open[B.fbase + w0 + u] = op;
                chg[B.fbase + w0 + u] = kp;
                if (kp) {
                    uint32_t* sv = survivors + B.sbase + (B.nd_ws == 2 ? rows[u] / B.Y : 0);
                    if (!*sv) *sv = 1;
                }
            }
        }
    }
}
template __global__ void k_regrow_init<4>(const BlockDesc*, const BlockStat*, uint32_t, const uint32_t*,
                                          const uint8_t*, const float*, uint64_t*, uint8_t*, uint64_t*, uint64_t*,
                                          uint32_t*);

// Auto-seeded regrow: a slice (2-D) / block (3-D) whose every segment was removed leaves
// watershedsNew an all-zero seed image, and vigra then seeds from the strict local minima of
// the hmap (direct nbhd, labelled in scan order; oracle/ctws_oracle.cpp:local_minima_strict).
// Strict minima are never adjacent, so each one is its own seed: its bit is set at its scan
// key in W, and its label is 1 + its rank among the slice's / block's minima.
__global__ void __launch_bounds__(256) k_auto_minima(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const float* __restrict__ h,
                                                     const uint32_t* __restrict__ survivors,
                                                     uint64_t* __restrict__ W) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const float* p = h + B.base;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int64_t nrows = (int64_t)B.Z * B.Y;
    for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
        const int z = (int)(row / B.Y), y = (int)(row - (int64_t)z * B.Y);
        if (survivors[B.sbase + (B.nd_ws == 2 ? z : 0)]) continue;
        for (int x = threadIdx.x; x < B.X; x += blockDim.x) {
            const int64_t i = row * B.X + x;
            const float c = p[i];
            bool mn = c < 3.402823466e+38f;
            if (B.nd_ws == 3) {
                if (z > 0) mn &= c < p[i - YX];
                if (z + 1 < B.Z) mn &= c < p[i + YX];
            }
            if (y > 0) mn &= c < p[i - B.X];
            if (y + 1 < B.Y) mn &= c < p[i + B.X];
            if (x > 0) mn &= c < p[i - 1];
            if (x + 1 < B.X) mn &= c < p[i + 1];
            if (mn) {
                const uint32_t f = scan_key_of(B, z, y, x);
                atomicOr((unsigned long long*)&W[B.wbase + (f >> 6)], 1ull << (f & 63));
            }
        }
    }
}

// the minima become fixed seeds of the regrow (after k_bitmap_csum / k_chunk_scan /
// k_word_prefix over W).  2-D: label = sb[z] + per-slice rank (the slice's own labels are all
// gone; label ranges of different slices may overlap, which is harmless because slices never
// meet in 2-D).  Pass 2: the reference maps the result through new_to_old (takeDict,
// two_pass_watershed.py:173/204), which has no entry beyond the slice's / block's relabelled
// seed count: such a block fails like the reference (kErrTakeDict).
__global__ void __launch_bounds__(256) k_auto_seed_set(const BlockDesc* __restrict__ D, BlockStat* S,
                                                       const float* __restrict__ h,
                                                       const uint32_t* __restrict__ survivors,
                                                       const uint64_t* __restrict__ W, const uint32_t* __restrict__ Wp,
                                                       const uint32_t* __restrict__ sb, uint64_t* __restrict__ key,
                                                       uint8_t* __restrict__ fixedv, uint64_t* __restrict__ open,
                                                       uint64_t* __restrict__ chg, uint32_t* __restrict__ lab) {
    const BlockDesc& B = D[blockIdx.y];
    BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    const int64_t nrows = (int64_t)B.Z * B.Y;
    const int wpr = (B.X + 63) >> 6;
    const uint64_t* Wb = W + B.wbase;
    const uint32_t* Wpb = Wp + B.wbase;
    uint32_t err = 0;
    for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
        const int z = (int)(row / B.Y), y = (int)(row - (int64_t)z * B.Y);
        if (survivors[B.sbase + (B.nd_ws == 2 ? z : 0)]) continue;
        for (int x = threadIdx.x; x < B.X; x += blockDim.x) {
            const uint32_t f = scan_key_of(B, z, y, x);
            if (!((Wb[f >> 6] >> (f & 63)) & 1ull)) continue;
            uint32_t l = bitmap_rank(Wb, Wpb, f) + 1u;
            if (B.nd_ws == 2) {
                const uint32_t ls = l - bitmap_rank(Wb, Wpb, (uint32_t)((int64_t)z * B.Y * B.X));
                const uint32_t m = (z + 1 < B.Z ? sb[B.sbase + z + 1] : st.n_seeds) - sb[B.sbase + z];
                if (B.pass2 && ls > m) err |= kErrTakeDict;
                l = sb[B.sbase + z] + ls;
            } else if (B.pass2 && l > st.n_seeds) {
                err |= kErrTakeDict;
            }
            const int64_t gi = B.base + row * B.X + x;
            if (lab) {
                // wide keys (k_flood): the label apart, any width; the minimum's tile is active
                // already (every voxel of the slice / block was freed by k_size_filter)
                lab[gi] = l | kFixedBit;
                key[gi] = (uint64_t)ordf(h[gi]) << 32;
                fixedv[gi] = 1;
                continue;
            }
            if (l >= (1u << 20) - 1u) {
                err |= kErrLabelBits;
                continue;
            }
            key[gi] = ((uint64_t)ordf(h[gi]) << 32) | (uint64_t)l;
            fixedv[gi] = 1;
            const int64_t wi = B.fbase + row * wpr + (x >> 6);
            const uint64_t bit = 1ull << (x & 63);
            atomicAnd((unsigned long long*)&open[wi], ~bit);
            atomicOr((unsigned long long*)&chg[wi], bit);
        }
    }
    if (err) atomicOr(&st.err, err);
}

template __global__ void k_hist<0>(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, uint32_t*,
                                   int);
template __global__ void k_hist<1>(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*, uint32_t*,
                                   int);
template __global__ void k_hist2d<0>(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*,
                                     const uint32_t*, uint32_t*, int);
template __global__ void k_hist2d<1>(const BlockDesc*, const BlockStat*, const uint32_t*, const uint64_t*,
                                     const uint32_t*, uint32_t*, int);

// zero small segments; survivors become the regrow seeds (fixed, key (h, 0, label)).
// Packed keys: a voxel that is already fixed (seed or steepest-descent voxel of the first
// flood) holds exactly that key, so only voxels the relaxation reached (a minority) and
// removed voxels are written; the heights are read for the former only.
__global__ void __launch_bounds__(256) k_size_filter(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     FilterParams fp, const uint32_t* __restrict__ counts,
                                                     const uint8_t* __restrict__ excl, const float* __restrict__ h,
                                                     uint32_t* __restrict__ lab, uint64_t* __restrict__ key,
                                                     uint8_t* __restrict__ fixedv, uint32_t* __restrict__ survivors,
                                                     int packed) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    auto freed = [&](int64_t i) {
        // only tiles with a free voxel can change in the regrow flood
        const int x = (int)(i % B.X), y = (int)((i / B.X) % B.Y), z = (int)(i / YX);
        uint32_t* a = fp.act + B.tbase + ((z / fp.tz) * B.ty + y / fp.ty) * B.tx + x / fp.tx;
        if (!*a) atomicOr(a, 8u);
    };
    auto survive = [&](int64_t i) {
        const int z = (B.nd_ws == 2) ? (int)(i / YX) : 0;
        if (!survivors[B.sbase + z]) survivors[B.sbase + z] = 1;
    };
    if (packed) {
        constexpr int U = 4;  // voxels per thread in flight
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < B.N; i0 += stride * U) {
            uint64_t kv[U];
            uint8_t fx[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * stride;
                kv[u] = kInfKey;
                fx[u] = 0;
                if (i < B.N) {
                    kv[u] = key[B.base + i];
                    fx[u] = fixedv[B.base + i];
                }
            }
            bool keep[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t l = kv[u] == kInfKey ? 0u : (uint32_t)(kv[u] & ((1ull << 20) - 1ull));
                keep[u] = l != 0 && (counts[B.base + l] >= fp.size_filter || (excl && excl[B.base + l]));
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + u * stride;
                if (i >= B.N) continue;
                if (keep[u]) {
                    if (!fx[u]) {
                        const uint32_t l = (uint32_t)(kv[u] & ((1ull << 20) - 1ull));
                        key[B.base + i] = ((uint64_t)ordf(h[B.base + i]) << 32) | (uint64_t)l;
                        fixedv[B.base + i] = 1;
                    }
                    survive(i);
                } else {
                    if (kv[u] != kInfKey) key[B.base + i] = kInfKey;
                    if (fx[u]) fixedv[B.base + i] = 0;
                    freed(i);
                }
            }
        }
        return;
    }
    BLOCK_LOOP(i, B) {
        const uint32_t l = lab[B.base + i] & ~kFixedBit;
        bool keep = l != 0 && (counts[B.base + l] >= fp.size_filter || (excl && excl[B.base + l]));
        if (keep) {
            lab[B.base + i] = l | kFixedBit;
            key[B.base + i] = (uint64_t)ordf(h[B.base + i]) << 32;
            fixedv[B.base + i] = 1;
            survive(i);
        } else {
            lab[B.base + i] = 0;
            key[B.base + i] = kInfKey;
            fixedv[B.base + i] = 0;
            freed(i);
        }
    }
}

// per-slice max_id (2-D ws): max per-slice label over in-mask voxels (all voxels without a
// mask).  Equals watershedsNew's maxRegionLabel of the (regrow) flood when unmasked.
// Grid (Z * splits, blocks): a workgroup reduces a quarter of one slice and issues one atomic.
// all == 0 skips cropped blocks (their output is the crop CC numbering, which needs no offsets).
__global__ void __launch_bounds__(256) k_slice_max(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                                   int packed, const uint32_t* __restrict__ sb,
                                                   uint32_t* __restrict__ smax, int splits, int all) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || B.nd_ws != 2 || (B.crop && !all)) return;
    const int z = blockIdx.x / splits, s = blockIdx.x % splits;
    if (z >= B.Z) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int64_t i0 = (int64_t)z * YX + YX * s / splits, i1 = (int64_t)z * YX + YX * (s + 1) / splits;
    const uint32_t base = sb[B.sbase + z];
    uint32_t v = 0;
    constexpr int U = 8;
    for (int64_t ib = i0; ib < i1; ib += 256 * U) {
        uint32_t lv[U];
        bool in[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = ib + u * 256 + threadIdx.x;
            lv[u] = i < i1 ? flood_label(lab, key, packed, B.base + i) : 0u;
            in[u] = i < i1 && (!B.mask || gbl(B.mask)[i]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (lv[u] && in[u]) v = max(v, lv[u] - base);
    }
    v = wg_reduce_u32(v, OpMax());
    if (threadIdx.x == 0 && v) atomicMax(&smax[B.sbase + z], v);
}

// exclusive scan over slices of max_id (uint32 arithmetic, as `wsz += offset` on uint32)
__global__ void k_slice_offsets(const BlockDesc* __restrict__ D, const BlockStat* S, const uint32_t* __restrict__ smax,
                                uint32_t* __restrict__ soff) {
    const BlockDesc& B = D[blockIdx.x];
    if (threadIdx.x != 0 || !S[blockIdx.x].active || B.nd_ws != 2) return;
    uint32_t off = 0;
    for (int z = 0; z < B.Z; ++z) {
        soff[B.sbase + z] = off;
        off += smax[B.sbase + z];
    }
}

// final uint32 ws of the outer block: 3-D: label, masked -> 0 (watershed.py:245-248);
// 2-D: per-slice label + slice offset, masked -> 0 (:220-237)
__global__ void __launch_bounds__(256) k_finalize_ws(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const uint32_t* __restrict__ sb, const uint32_t* __restrict__ soff,
                                                     const uint64_t* __restrict__ key, int packed,
                                                     uint32_t* __restrict__ lab) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    BLOCK_LOOP(i, B) {
        uint32_t l = flood_label(lab, key, packed, B.base + i);
        const bool inm = !B.mask || gbl(B.mask)[i];
        if (B.nd_ws == 2) {
            const int z = (int)(i / YX);
            l = inm ? (l - sb[B.sbase + z]) + soff[B.sbase + z] : 0u;
        } else if (!inm) {
            l = 0;
        }
        lab[B.base + i] = l;
    }
}

}  // namespace ctws
