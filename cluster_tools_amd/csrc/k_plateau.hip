// k_plateau.hip — the flood across a block's masked plateau without hop-by-hop relaxation.
//
// Reference: watershed.py:299-303 (a masked block's input is set to 1 outside the mask, so
// the whole masked region is flooded), :245-248 (masked voxels are zeroed only after the
// watershed and its size filter, volume_utils.py:123-139: the masked region's labels count
// towards the segment sizes, so its keys have to be the fixpoint's).
//
// Away from the mask boundary the hmap of the masked region is one exact plateau (fin = 1,
// dt = 0, and the Gaussian of a constant).  A plateau voxel q has h(q) = H, and every key that
// can reach it has C >= H, so inside the plateau f_q is "+1 hop" and the fixpoint keys are
//     K(q) = min over entries e of K(e) + (geodesic hop distance e -> q inside the plateau),
// a multi-source BFS.  The frontier relaxation crosses it one hop per local sweep (a plateau
// hundreds of voxels wide costs tens of launches).  Here instead:
//   1. P = the open voxels (not resolved by the descent) of height H = the largest height of an
//      open masked voxel of the block (k_descent_init's plev, k_plat_mark); P is taken out of the open
//      set and the frontier floods the rest of the block first.
//   2. entries: every P voxel gets f(min of its neighbours' keys) (k_plat_entry);
//   3. min-plus scans along x, then y, then z restricted to runs of P voxels (k_plat_scan_x,
//      k_plat_scan_col): every key written is f applied along a path of P voxels from an entry
//      (an entry, then a run along x, y and z), so each is an upper bound of the fixpoint key;
//      for a plateau whose shortest paths are such staircases it is the fixpoint itself;
//   4. P is open again with every P voxel marked changed, and the frontier relaxation runs to
//      its fixpoint from there (correcting whatever the staircases missed);
// k_flood_verify then checks the fixpoint as for every flood.  Only the schedule changes: the
// fixpoint is unique, so the result is bit-identical to the hop-by-hop flood.
#include "ctws_kernels.h"

namespace ctws {

// n more hops inside the plateau: d + n, saturating at kDMax as f_packed does (the plateau voxels
// rejoin the open set, k_plat_restore, so a saturated final key is reported by k_flood_verify);
// INF stays INF
__device__ __forceinline__ uint64_t key_hops(uint64_t k, uint32_t n) {
    if (k == kPackInf) return k;
    const uint32_t d = (uint32_t)((k & kDMask) >> kLabelBits);
    const uint32_t d2 = min(d + n, kDMax);
    return (k & ~kDMask) | ((uint64_t)d2 << kLabelBits);
}

// P bitmap (zeroed beforehand) and open &= ~P
__global__ void __launch_bounds__(256) k_plat_mark(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   const float* __restrict__ h, const uint32_t* __restrict__ plev,
                                                   uint64_t* __restrict__ open, uint64_t* __restrict__ plat) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const uint32_t lv = plev[blockIdx.y];
    if (!lv) return;
    WORD_TILES(B.Z, B.Y, B.X, {
        const uint64_t ow = open[B.fbase + w_];
        bool p = false;
        if (ow) p = valid && ((ow >> lane) & 1ull) && ordf(h[B.base + i]) == lv;
        const uint64_t pm = __ballot(p);
        if (lane == 0 && pm) {
            open[B.fbase + w_] = ow & ~pm;
            plat[B.fbase + w_] = pm;
        }
    })
}

// entries: K(q) = f(min of the neighbours' keys) at every P voxel (plateau neighbours are still
// unreached, or already entries: either way a key reached along a path)
template <int ND>
__global__ void __launch_bounds__(256) k_plat_entry(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const float* __restrict__ h, uint64_t* __restrict__ key,
                                                    const uint64_t* __restrict__ plat, const uint32_t* __restrict__ plev) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !plev[blockIdx.y]) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    uint64_t* kb = key + B.base;
    WORD_TILES(B.Z, B.Y, B.X, {
        const uint64_t pw = plat[B.fbase + w_];
        if (pw && valid && ((pw >> lane) & 1ull)) {
            uint64_t m = kPackInf;
            if (ND == 3) {
                if (z > 0) m = min(m, kb[i - YX]);
                if (z + 1 < B.Z) m = min(m, kb[i + YX]);
            }
            if (y > 0) m = min(m, kb[i - B.X]);
            if (y + 1 < B.Y) m = min(m, kb[i + B.X]);
            if (x > 0) m = min(m, kb[i - 1]);
            if (x + 1 < B.X) m = min(m, kb[i + 1]);
            if (m != kPackInf) {
                const uint64_t k = f_packed(ordf(h[B.base + i]), m);
                kb[i] = k;
            }
        }
    })
}

// one word of a row: segmented min-plus inclusive scan over the lanes in increasing lane order,
// runs = consecutive P bits of pw; carry = the key of the voxel just before lane 0 (kPackInf
// when it is not in P).  Returns the lane's new key.
__device__ __forceinline__ uint64_t plat_word_scan(uint64_t v, uint64_t pw, uint64_t carry, int lane) {
    // start of the lane's run: one past the last non-P position before the lane (0: none)
    const uint64_t below = lane ? (~pw & ((1ull << lane) - 1ull)) : 0ull;
    const int rs = below ? 64 - __builtin_clzll(below) : 0;
    if (rs == 0) v = min(v, key_hops(carry, (uint32_t)lane + 1u));
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t o = shfl_up_u64(v, off);
        if (lane - off >= rs) v = min(v, key_hops(o, (uint32_t)off));
    }
    return v;
}

// x runs: one wave per row, words left to right then right to left (the backward pass mirrors
// the lanes and the bits, so it is the same forward scan)
__global__ void __launch_bounds__(256) k_plat_scan_x(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     uint64_t* __restrict__ key, const uint64_t* __restrict__ plat,
                                                     const uint32_t* __restrict__ plev) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !plev[blockIdx.y]) return;
    const int lane = threadIdx.x & 63;
    const int wpr = (B.X + 63) >> 6;
    const int64_t rows = (int64_t)B.Z * B.Y;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t* kb = key + B.base;
    const uint64_t* pb = plat + B.fbase;
    for (int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < rows; row += nwaves) {
        for (int dir = 0; dir < 2; ++dir) {
            uint64_t carry = kPackInf;
            for (int k = 0; k < wpr; ++k) {
                const int xw = dir == 0 ? k : wpr - 1 - k;
                uint64_t pw = pb[row * wpr + xw];
                if (!pw) {
                    carry = kPackInf;
                    continue;
                }
                // lane l handles position p = l (forward) or 63 - l (backward)
                const int p = dir == 0 ? lane : 63 - lane;
                if (dir == 1) pw = __builtin_bitreverse64(pw);
                const bool inp = (pw >> lane) & 1ull;
                const int64_t i = row * B.X + (int64_t)xw * 64 + p;
                const uint64_t v0 = inp ? kb[i] : kPackInf;
                uint64_t v = plat_word_scan(v0, pw, carry, lane);
                if (!inp) v = kPackInf;
                if (inp && v != v0) {
                    kb[i] = v;
                }
                carry = shfl_u64(v, 63);  // kPackInf when the run does not reach the word's end
            }
        }
    }
}

// y (AX = 1) or z (AX = 2) runs: a wave takes 64 consecutive x of one (z, x-word) / (y, x-word)
// column and walks it forward then backward; U positions per step with their loads in flight
template <int AX>
__global__ void __launch_bounds__(256) k_plat_scan_col(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                       uint64_t* __restrict__ key, const uint64_t* __restrict__ plat,
                                                       const uint32_t* __restrict__ plev) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !plev[blockIdx.y]) return;
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
    const int wpr = (B.X + 63) >> 6;
    const int len = AX == 1 ? B.Y : B.Z;
    const int64_t ngroups = (int64_t)(AX == 1 ? B.Z : B.Y) * wpr;
    const int64_t wstride = AX == 1 ? wpr : (int64_t)B.Y * wpr;   // bitmap words per step
    const int64_t vstride = AX == 1 ? B.X : (int64_t)B.Y * B.X;   // voxels per step
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t* kb = key + B.base;
    const uint64_t* pb = plat + B.fbase;
    for (int64_t g = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < ngroups; g += nwaves) {
        const int64_t outer = g / wpr;
        const int xw = (int)(g - outer * wpr);
        const int x = xw * 64 + lane;
        const bool xok = x < B.X;
        // first word / voxel of the column
        const int64_t w0 = AX == 1 ? outer * B.Y * wpr + xw : outer * wpr + xw;
        const int64_t v0 = AX == 1 ? outer * B.Y * B.X + (xok ? x : 0) : outer * B.X + (xok ? x : 0);
        for (int dir = 0; dir < 2; ++dir) {
            uint64_t run = kPackInf;
            for (int s0 = 0; s0 < len; s0 += U) {
                uint64_t pw[U], kv[U];
                int64_t vi[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int s = s0 + u < len ? s0 + u : len - 1;
                    const int t = dir == 0 ? s : len - 1 - s;
                    pw[u] = s0 + u < len ? pb[w0 + t * wstride] : 0ull;
                    vi[u] = v0 + t * vstride;
                    kv[u] = kb[vi[u]];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool inp = xok && ((pw[u] >> lane) & 1ull);
                    if (!inp) {
                        run = kPackInf;
                        continue;
                    }
                    const uint64_t nv = min(kv[u], key_hops(run, 1u));
                    if (nv != kv[u]) {
                        kb[vi[u]] = nv;
                    }
                    run = nv;
                }
            }
        }
    }
}

// P open again; the changed bitmap (every word of the batch) = P, for the frontier that follows
__global__ void __launch_bounds__(256) k_plat_restore(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      uint64_t* __restrict__ open, const uint64_t* __restrict__ plat,
                                                      uint64_t* __restrict__ chg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nw = (int64_t)B.Z * B.Y * wpr;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t p = plat[B.fbase + w];
        if (p) open[B.fbase + w] |= p;
        chg[B.fbase + w] = p;
    }
}

template __global__ void k_plat_entry<2>(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint64_t*,
                                         const uint32_t*);
template __global__ void k_plat_entry<3>(const BlockDesc*, const BlockStat*, const float*, uint64_t*, const uint64_t*,
                                         const uint32_t*);
template __global__ void k_plat_scan_col<1>(const BlockDesc*, const BlockStat*, uint64_t*, const uint64_t*,
                                            const uint32_t*);
template __global__ void k_plat_scan_col<2>(const BlockDesc*, const BlockStat*, uint64_t*, const uint64_t*,
                                            const uint32_t*);

}  // namespace ctws
