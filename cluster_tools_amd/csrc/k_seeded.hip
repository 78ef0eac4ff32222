// k_seeded.hip — WatershedFromSeeds on gfx950: the given seeds become the flood's labels.
//
// Reference: watershed/watershed_from_seeds.py:143-199 (`_ws_block`, `_ws_block_masked`):
//     input = normalize(ds_in[bb]) (4-D: joint normalize + channel agglomeration); masked
//     voxels -> 1;  seeds = ds_seeds[bb].astype(uint32) after `max_id < uint32 max`;
//     ws = vu.watershed(input, seeds, size_filter)  (vigra watershedsNew, 3-D direct nbhd);
//     ws[~mask] = 0;  ds_out[bb] = ws.astype(uint64)
// There is no halo, id offset or CC relabel.  The packed flood key carries a 20-bit label, so
// the block's distinct seed values are compacted ORDER-PRESERVINGLY: label = 1 + rank of the
// value among the block's sorted distinct values (a per-block hash of the values, a segmented
// radix sort of the distinct values, a binary search per hash slot).  Equal-key ties of the
// flood are broken by label, and the rank order is the value order, so the flood computes the
// same (C, d, value) fixpoint as on the raw values; the output maps labels back to values.
// A block without any seed is seeded by vigra from the strict hmap minima (labels 1..n in
// scan order, k_auto_minima + k_fs_auto_label); its labels are output as they are.
#include <hipcub/hipcub.hpp>

#include "ctws_kernels.h"

namespace ctws {

constexpr uint64_t kFsEmpty = ~0ull;

__device__ __forceinline__ uint64_t fs_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__device__ __forceinline__ int64_t fs_find(const uint64_t* hk, int64_t cap, uint64_t k) {
    int64_t s = (int64_t)(fs_mix(k) & (uint64_t)(cap - 1));
    for (int64_t p = 0; p < cap; ++p) {
        const uint64_t v = hk[s];
        if (v == k) return s;
        if (v == kFsEmpty) return -1;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

#define FS_LOOP(i, B)                                                                         \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).N;              \
         i += (int64_t)gridDim.x * blockDim.x)

// every block takes part (no threshold / empty-block branch in WatershedFromSeeds)
__global__ void k_fs_active(const BlockDesc* __restrict__ D, BlockStat* S, int n) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n) S[b].active = 1u;
}

// distinct nonzero seed values (uint32 after the overflow assert) -> the block's hash table.
// A voxel whose scan predecessor along x holds the same value is skipped (runs insert once).
__global__ void __launch_bounds__(256) k_fs_insert(const BlockDesc* __restrict__ D, BlockStat* S,
                                                   uint64_t* __restrict__ hkey) {
    const BlockDesc& B = D[blockIdx.y];
    uint64_t* hk = hkey + B.hbase;
    const int64_t cap = B.hcap;
    uint32_t err = 0;
    FS_LOOP(i, B) {
        const uint64_t s64 = gbl(B.init)[i];
        if (s64 >= 0xFFFFFFFFull) err |= kErrOverflow;  // "Overflow detected" (:160-163)
        const uint32_t s = (uint32_t)s64;
        if (!s) continue;
        if (i % B.X && (uint32_t)gbl(B.init)[i - 1] == s) continue;
        int64_t p0 = (int64_t)(fs_mix(s) & (uint64_t)(cap - 1));
        bool done = false;
        for (int64_t p = 0; p < cap; ++p) {
            uint64_t v = hk[p0];
            if (v == kFsEmpty) v = atomicCAS((unsigned long long*)&hk[p0], (unsigned long long)kFsEmpty, (unsigned long long)s);
            if (v == kFsEmpty || v == s) {
                done = true;
                break;
            }
            p0 = (p0 + 1) & (cap - 1);
        }
        if (!done) err |= kErrHashFull;
    }
    if (err) atomicOr(&S[blockIdx.y].err, err);
}

// the table's values -> a dense list per block (vals[hbase .. hbase + n_seeds)); n_seeds counts
__global__ void __launch_bounds__(256) k_fs_collect(const BlockDesc* __restrict__ D, BlockStat* S,
                                                    const uint64_t* __restrict__ hkey, uint32_t* __restrict__ vals) {
    const BlockDesc& B = D[blockIdx.y];
    const int lane = threadIdx.x & 63;
    for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); s0 < B.hcap;
         s0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = s0 + lane;
        const bool has = s < B.hcap && hkey[B.hbase + s] != kFsEmpty;
        const uint64_t m = __ballot(has);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&S[blockIdx.y].n_seeds, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, 0);
        if (has) vals[B.hbase + base + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)hkey[B.hbase + s];
    }
}

// segment offsets of the segmented sort: block b's distinct values [hbase, hbase + n_seeds)
__global__ void k_fs_offsets(const BlockDesc* __restrict__ D, const BlockStat* S, int n, int* __restrict__ beg,
                             int* __restrict__ end) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n) return;
    beg[b] = (int)D[b].hbase;
    end[b] = (int)(D[b].hbase + S[b].n_seeds);
}

// hash slot -> label = 1 + rank of its value among the sorted distinct values (in hpos)
__global__ void __launch_bounds__(256) k_fs_rank(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                 const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ sorted,
                                                 uint32_t* __restrict__ hpos) {
    const BlockDesc& B = D[blockIdx.y];
    const int n = (int)S[blockIdx.y].n_seeds;
    const uint32_t* sv = sorted + B.hbase;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B.hcap; s += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = hkey[B.hbase + s];
        if (k == kFsEmpty) continue;
        const uint32_t v = (uint32_t)k;
        int lo = 0, hi = n;  // first index with sv[idx] >= v
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sv[mid] < v) lo = mid + 1;
            else hi = mid;
        }
        hpos[B.hbase + s] = (uint32_t)lo + 1u;
    }
}

// seeds -> flood labels, keys and fixed flags (the pass-2 convention of k_p2_label: a seed's
// lab carries kFixedBit, its key (h, 0, label))
__global__ void __launch_bounds__(256) k_fs_label(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                  const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ hpos,
                                                  const float* __restrict__ h, uint32_t* __restrict__ lab,
                                                  uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv, int packed) {
    const BlockDesc& B = D[blockIdx.y];
    FS_LOOP(i, B) {
        const uint32_t s = (uint32_t)gbl(B.init)[i];
        const int64_t gi = B.base + i;
        if (!s) {
            lab[gi] = 0u;
            key[gi] = kInfKey;
            fixedv[gi] = 0;
            continue;
        }
        const int64_t p = fs_find(hkey + B.hbase, B.hcap, s);
        const uint32_t l = p >= 0 ? hpos[B.hbase + p] : 0u;  // p < 0 cannot happen after insert
        lab[gi] = l | kFixedBit;
        key[gi] = ((uint64_t)ordf(h[gi]) << 32) | (packed ? (uint64_t)l : 0ull);
        fixedv[gi] = 1;
    }
}

// seedless blocks (survivors[sbase] == 0): the strict minima found by k_auto_minima (bits in W,
// ranked by k_bitmap_csum / k_chunk_scan(counter 2) / k_word_prefix) become seeds 1..n in scan
// order; the block is flagged auto (_p[1]) so that its labels are output as they are
__global__ void __launch_bounds__(256) k_fs_auto_label(const BlockDesc* __restrict__ D, BlockStat* S,
                                                       const uint32_t* __restrict__ survivors,
                                                       const uint64_t* __restrict__ W, const uint32_t* __restrict__ Wp,
                                                       const float* __restrict__ h, uint32_t* __restrict__ lab,
                                                       uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv,
                                                       int packed) {
    const BlockDesc& B = D[blockIdx.y];
    BlockStat& st = S[blockIdx.y];
    if (survivors[B.sbase]) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st.n_seeds = st.n_auto;
        st._p[1] = 1u;
    }
    const int64_t YX = (int64_t)B.Y * B.X;
    FS_LOOP(i, B) {
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / B.X, x = rem - (rem / B.X) * B.X;
        const uint32_t f = scan_key_of(B, z, y, x);
        if (!((W[B.wbase + (f >> 6)] >> (f & 63)) & 1ull)) continue;
        const uint32_t l = bitmap_rank(W + B.wbase, Wp + B.wbase, f) + 1u;
        const int64_t gi = B.base + i;
        lab[gi] = l | kFixedBit;
        key[gi] = ((uint64_t)ordf(h[gi]) << 32) | (packed ? (uint64_t)l : 0ull);
        fixedv[gi] = 1;
    }
}

// final labels -> uint64 seed values (auto-seeded blocks: the labels), masked voxels 0; the
// largest output id in _p[2..3]
__global__ void __launch_bounds__(256) k_fs_output(const BlockDesc* __restrict__ D, BlockStat* S,
                                                   const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                                   int keys_final, const uint32_t* __restrict__ sorted,
                                                   const uint32_t* __restrict__ survivors, int use_surv) {
    const BlockDesc& B = D[blockIdx.y];
    BlockStat& st = S[blockIdx.y];
    if (st.err) return;  // a failed block writes nothing
    const bool raw = st._p[1] != 0u || (use_surv && !survivors[B.sbase]);
    const uint32_t* sv = sorted + B.hbase;
    uint64_t mx = 0;
    FS_LOOP(i, B) {
        const uint32_t l = flood_label(lab, key, keys_final, B.base + i);
        uint64_t v = l == 0u ? 0ull : (raw ? (uint64_t)l : (uint64_t)sv[l - 1]);
        if (B.mask && !gbl(B.mask)[i]) v = 0ull;
        if (B.out32) B.out32[i] = (uint32_t)v;  // seed ids < 2^32 - 1 (the overflow assert)
        else B.out[i] = v;
        mx = v > mx ? v : mx;
    }
    for (int s = 32; s > 0; s >>= 1) {
        const uint64_t o = (uint64_t)__shfl_xor((long long)mx, s);
        mx = o > mx ? o : mx;
    }
    if ((threadIdx.x & 63) == 0 && mx) atomicMax((unsigned long long*)&st._p[2], (unsigned long long)mx);
}

// per-block ascending sort of the distinct values (segments [beg[b], end[b]) of `in`)
hipError_t fs_segmented_sort(void* tmp, size_t& bytes, const uint32_t* in, uint32_t* out, int n, int nseg,
                             const int* beg, const int* end, hipStream_t stream) {
    return hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, bytes, in, out, n, nseg, beg, end, 0, 32, stream);
}

}  // namespace ctws
