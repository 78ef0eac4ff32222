// k_cc.hip — local maxima seeds, connected components and vigra-scan-order numbering.
//
// Reference: watershed.py:179-207 (_make_seeds: localMaxima[3D](allowPlateaus,
// allowAtBorder) -> labelMultiArrayWithBackground), watershed.py:326-341 (halo crop,
// labelVolumeWithBackground, uint64 id offset), :310-321 (empty block).
//
// Numbering.  vigra numbers components 1..k by their first voxel in vigra scan order,
// which for a plain numpy array is the F-order index (axis 0 fastest), the *scan key*
//     3-D: f = z + Z*(y + Y*x)        2-D (per slice): f = z*Y*X + (y + Y*x).
// Union-find parents are indexed by the C-order voxel index (so every pass is coalesced),
// and a union links the root with the larger scan key under the one with the smaller, so
// every root is its component's first voxel in scan order.  Roots set their scan-key bit in
// a per-block bitmap; the label of a root is 1 + (number of roots with a smaller key), from
// the bitmap's per-word exclusive prefix.  After k_root_label every root slot holds
// (label | kRootBit) and every other member points straight at its root.
//
// Voxel passes walk row tiles: a workgroup iteration covers kRows consecutive rows (z, y)
// and each thread an x column, so coordinates need no divisions and the loads of the rows
// are independent (issued together).
#include "ctws_kernels.h"

namespace ctws {

#define BLOCK_LOOP(i, B)                                                                      \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).N;              \
         i += (int64_t)gridDim.x * blockDim.x)

// row-tile traversal of an (nz, ny, nx) C-order volume; BODY sees z, y, x, i (local index)
#define ROW_TILES(nz, ny, nx, ...)                                                           \
    {                                                                                         \
        const int64_t nrows_ = (int64_t)(nz) * (ny);                                          \
        for (int64_t r0_ = (int64_t)blockIdx.x * kRows; r0_ < nrows_; r0_ += (int64_t)gridDim.x * kRows) \
            for (int x = threadIdx.x; x < (nx); x += blockDim.x) {                           \
                _Pragma("unroll") for (int rr_ = 0; rr_ < kRows; ++rr_) {                      \
                    const int64_t row_ = r0_ + rr_;                                           \
                    if (row_ >= nrows_) break;                                                \
                    const int z = (int)(row_ / (ny));                                         \
                    const int y = (int)(row_ - (int64_t)z * (ny));                            \
                    const int64_t i = row_ * (nx) + x;                                        \
                    (void)z;                                                                  \
                    (void)y;                                                                  \
                    __VA_ARGS__                                                               \
                }                                                                             \
            }                                                                                 \
    }

// ---- local maxima classification ---------------------------------------------------------
// cls bit0: a neighbour is strictly greater; bit1: a neighbour is equal (plateau voxel).
// Neighbourhood: 6 (3-D ws) or 8 in-plane (2-D ws), as localMaxima3D / localMaxima.
// Word columns (wtg grid): the unit of work is U vertically adjacent words (rows y0 .. y0+U-1
// of one 64-voxel column of a slice); a wave takes a contiguous range of units and loads the
// U + 2 rows y0-1 .. y0+U once (every load of the unit in flight together, clamped positions),
// so each row serves as centre, upper and lower row from registers.  The x neighbours come
// from the neighbouring lanes; lane 0 / 63 fetch the voxel left / right of the word with one
// extra load per row (3-D: z neighbours are one load each).  U = 8 rows per unit (U = 4: 1.5x
// the rows loaded; 2.90 -> 2.39 ms on config 3, 4.35 -> 3.92 ms on config 4).
//
// Zero short cut: the seed map is >= 0 (a distance transform, Gaussian-smoothed with positive
// taps), so 0 is its minimum, and a slice (2-D ws) / block (3-D ws) whose dt has a positive
// value has a positive seed-map voxel (at the same position).  On the connected grid every
// zero component then touches a strictly greater voxel: no zero voxel is a maximum, whatever
// its neighbours.  Those voxels are classified "greater neighbour" outright and stay out of
// the plateau union-find (the masked region of a masked block — fin = 1, dt = 0 — is one
// huge zero plateau otherwise).  pos: the slice's / block's dt maximum > 0.
template <int ND>
__device__ __forceinline__ void localmax_words(const BlockDesc& B, const BlockStat& st, const uint32_t* __restrict__ smax,
                                               const float* __restrict__ p, uint8_t* __restrict__ cl, uint32_t& nplat,
                                               uint32_t* __restrict__ ptile) {
    const uint32_t ord0 = 0x80000000u;  // ordf(+0.0f)
    constexpr int U = 8, R = U + 2;
    const int Y = B.Y, X = B.X, Z = B.Z;
    const int64_t YX = (int64_t)Y * X;
    const int wpr = (X + 63) >> 6;
    const int ngy = (Y + U - 1) / U;
    const int64_t nunits = (int64_t)Z * wpr * ngy;  // unit = (z, xw, y group), y group fastest
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nunits + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t ubeg = wid * per, uend = min(nunits, ubeg + per);
    const float NEG = -__builtin_huge_valf();
    const gptr_t<float> gp = gbl(p);
    for (int64_t un = ubeg; un < uend; ++un) {
        // (32-bit unsigned division: a block has < 2^31 units; the emulated 64-bit one is long)
        const uint32_t un32 = (uint32_t)un;
        const int gy = (int)(un32 % (uint32_t)ngy);
        const uint32_t strip = un32 / (uint32_t)ngy;
        const int xw = (int)(strip % (uint32_t)wpr), z = (int)(strip / (uint32_t)wpr);
        const int y0 = gy * U;
        bool ueq = false;  // a plateau voxel in the unit (this lane)
        const int x = xw * 64 + lane;
        const int xc = min(x, X - 1);
        const int xe = lane == 0 ? max(xc - 1, 0) : min(xc + 1, X - 1);  // lane 0: left, others: right
        const int64_t zb = (int64_t)z * YX;
        float rc[R], re[R];  // rows y0-1 .. y0+U (clamped): centre word and edge voxel
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int yy = min(max(y0 - 1 + k, 0), Y - 1);
            rc[k] = gp[zb + (int64_t)yy * X + xc];
            re[k] = gp[zb + (int64_t)yy * X + xe];
        }
        float zm[U], zp[U];
        if (ND == 3) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int yy = min(y0 + u, Y - 1);
                const int64_t i = zb + (int64_t)yy * X + xc;
                zm[u] = gp[i - (z > 0 ? YX : 0)];
                zp[u] = gp[i + (z + 1 < Z ? YX : 0)];
            }
        }
        const bool xl = x > 0, xh = x + 1 < X;
        const bool pos = (ND == 2 ? smax[B.sbase + z] : st.dt_max) > ord0;
        auto left = [&](float v, float ev) {
            const float t = __shfl(v, (lane + 63) & 63);
            return lane == 0 ? ev : t;
        };
        auto right = [&](float v, float ev) {
            const float t = __shfl(v, (lane + 1) & 63);
            const float e63 = __shfl(ev, 63);
            return lane == 63 ? e63 : t;
        };
        float lft[R], rgt[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            if (ND == 2 || (k >= 1 && k <= U)) {
                lft[k] = left(rc[k], re[k]);
                rgt[k] = right(rc[k], re[k]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u;
            const int k = u + 1;  // row y in the window
            const bool yl = y > 0, yh = y + 1 < Y;
            const float cc = rc[k];
            float w[8];
            if (ND == 3) {
                w[0] = z > 0 ? zm[u] : NEG;
                w[1] = z + 1 < Z ? zp[u] : NEG;
                w[2] = yl ? rc[k - 1] : NEG;
                w[3] = yh ? rc[k + 1] : NEG;
                w[4] = xl ? lft[k] : NEG;
                w[5] = xh ? rgt[k] : NEG;
                w[6] = w[7] = NEG;
            } else {
                w[0] = yl && xl ? lft[k - 1] : NEG;
                w[1] = yl ? rc[k - 1] : NEG;
                w[2] = yl && xh ? rgt[k - 1] : NEG;
                w[3] = xl ? lft[k] : NEG;
                w[4] = xh ? rgt[k] : NEG;
                w[5] = yh && xl ? lft[k + 1] : NEG;
                w[6] = yh ? rc[k + 1] : NEG;
                w[7] = yh && xh ? rgt[k + 1] : NEG;
            }
            bool gt = false, eq = false;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                gt |= w[q] > cc;
                eq |= w[q] == cc;
            }
            if (cc == 0.0f && pos) {
                gt = true;
                eq = false;
            }
            const bool valid = y < Y && x < X;
            if (valid) cl[zb + (int64_t)y * X + x] = (uint8_t)((gt ? 1 : 0) | (eq ? 2 : 0));
            nplat += valid && eq;  // plateau parents: k_tile_cc<.., CC_PLATEAU> (k_tilecc.hip)
            ueq |= valid && eq;
        }
        // the plateau CC's tiles that hold a plateau voxel (CcTileM<ND, CC_PLATEAU>: 2-D
        // 1 x 32 x 64, one word column; 3-D 8 x 16 x 32, two tiles per word): the others are
        // skipped by k_tile_cc / k_tile_merge without reading cls
        const uint64_t em = __ballot(ueq);
        if (em && lane < (ND == 3 ? 2 : 1)) {
            using PT = CcTileM<ND, CC_PLATEAU>;
            const int ntx = (X + PT::TX - 1) / PT::TX, nty = (Y + PT::TY - 1) / PT::TY;
            const uint64_t half = ND == 3 ? ((em >> (32 * lane)) & 0xFFFFFFFFull) : em;
            const int txi = ND == 3 ? 2 * xw + lane : xw;
            if (half && txi < ntx) {
                uint32_t* f = ptile + B.ptbase + ((int64_t)(z / PT::TZ) * nty + y0 / PT::TY) * ntx + txi;
                if (!*f) *f = 1u;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_localmax(const BlockDesc* __restrict__ D, BlockStat* S,
                                                  const float* __restrict__ v, uint8_t* __restrict__ cls,
                                                  const uint32_t* __restrict__ smax, uint32_t* __restrict__ ptile) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    uint32_t nplat = 0;
    if (B.nd_ws == 3) localmax_words<3>(B, S[blockIdx.y], smax, v + B.base, cls + B.base, nplat, ptile);
    else localmax_words<2>(B, S[blockIdx.y], smax, v + B.base, cls + B.base, nplat, ptile);
    nplat = wg_reduce_u32(nplat, OpAdd());
    if (threadIdx.x == 0 && nplat) atomicAdd(&S[blockIdx.y].plateau, nplat);
}

// Seed components without a seed tile CC.  Two adjacent local maxima have equal values (else
// the smaller has a strictly greater neighbour), so they lie on one plateau, and every voxel of
// a maximal plateau is a maximum.  3-D: the seed components (direct 6-nbhd, as the plateau CC's)
// are the maximal plateau components and the isolated maxima; the 3-D plateau CC roots each
// component at its first voxel in scan order (k_tile_cc / k_tile_merge<3, CC_PLATEAU>), so
// member i's parent is its plateau's root or i itself -- the same seed forest (members' parents
// at their roots) and member bitmap as k_tile_cc + k_tile_merge<3, CC_SEED>.  2-D: the plateau
// CC is 8-connected in-plane and the seed CC 4-connected, so every maximum starts as its own
// root and the plateau maxima (rare) go to a list for k_seed_union2.  One pass over the classes,
// 8 words in flight per wave (the plateau voxels follow their plateau parents).
template <int ND>
__global__ void __launch_bounds__(256) k_seed_members(const BlockDesc* __restrict__ D, BlockStat* S,
                                                      const uint8_t* __restrict__ cls, const uint32_t* __restrict__ Pp,
                                                      uint32_t* __restrict__ PFg, uint64_t* __restrict__ fseed,
                                                      uint32_t* __restrict__ plist) {
    const BlockDesc& B = D[blockIdx.y];
    BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    const bool plat = st.plateau != 0;
    const uint8_t* cl = cls + B.base;
    const uint32_t* PP = Pp + B.base;
    uint32_t* PF = PFg + B.base;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nwords + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t wbeg = wid * per, wend = min(nwords, wbeg + per);
    // (row, word in the row) of the wave's next word, advanced word by word
    int row_n = (int)((uint32_t)wbeg / (uint32_t)wpr), xw_n = (int)(wbeg - (int64_t)row_n * wpr);
    constexpr int U = 8;
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
        int64_t gi[U];
        bool valid[U];
        uint8_t c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = row_n;
            const int x = xw_n * 64 + lane;
            if (++xw_n == wpr) {
                xw_n = 0;
                ++row_n;
            }
            valid[u] = w0 + u < wend && x < B.X;
            gi[u] = valid[u] ? row * B.X + x : 0;
            c[u] = gbl(cl)[gi[u]];  // unconditional (clamped): all U loads in flight
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            bool mx = valid[u] && !(c[u] & 1);
            uint32_t par = (uint32_t)gi[u];
            bool listed = false;
            if (mx && (c[u] & 2) && plat) {  // cc_is_max of a plateau voxel
                const uint32_t r = uf_find(PP, par);
                if (cl[r] & 4) mx = false;
                else if (ND == 3) par = r;
                else listed = true;
            }
            const uint64_t m = __ballot(mx);
            if (lane == 0 && w0 + u < wend) fseed[B.fbase + w0 + u] = m;
            if (mx) PF[gi[u]] = par;
            if (ND == 2) {
                const uint64_t lm = __ballot(listed);
                if (lm) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&st._u, (uint32_t)__popcll(lm));
                    base = (uint32_t)__shfl((int)base, 0);
                    if (listed) plist[B.base + base + __popcll(lm & ((1ull << lane) - 1ull))] = par;
                }
            }
        }
    }
}
template __global__ void k_seed_members<2>(const BlockDesc*, BlockStat*, const uint8_t*, const uint32_t*, uint32_t*,
                                           uint64_t*, uint32_t*);
template __global__ void k_seed_members<3>(const BlockDesc*, BlockStat*, const uint8_t*, const uint32_t*, uint32_t*,
                                           uint64_t*, uint32_t*);

// 2-D: the listed plateau maxima united with their 4-adjacent backward maxima (x - 1, y - 1 in
// the slice) by scan key, so each seed component is rooted at its first voxel in scan order as by
// the tile CC.  The parents are read with device-scope loads and the finds do not halve paths:
// with uf_union_scan (plain loads, path-halving stores) a whole-slice plateau of maxima -- every
// voxel listed, some 16K threads uniting at once across the XCDs -- left a few members on a root
// that k_flatten_seeds never saw in about one run in 24 (tests/test_gpu_parity.py::
// test_seeds_repeatable); this form passed 120 runs of every case.
__global__ void __launch_bounds__(256) k_seed_union2(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const uint8_t* __restrict__ cls, const uint32_t* __restrict__ Pp,
                                                     const uint32_t* __restrict__ plist, uint32_t* __restrict__ PFg) {
    const BlockDesc& B = D[blockIdx.y];
    const BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    const uint8_t* cl = cls + B.base;
    const uint32_t* PP = Pp + B.base;
    uint32_t* PF = PFg + B.base;
    auto plat_max = [&](uint32_t i) {
        const uint8_t c = cl[i];
        return !(c & 1) && (c & 2) && !(cl[uf_find(PP, i)] & 4);
    };
    // device-scope loads and no path halving: the parents are read coherently across XCDs
    auto ld = [](const uint32_t* q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto find = [&](uint32_t a) {
        uint32_t p = ld(&PF[a]);
        while (p != a) {
            a = p;
            p = ld(&PF[a]);
        }
        return a;
    };
    auto unite = [&](uint32_t a, uint32_t b) {
        while (true) {
            a = find(a);
            b = find(b);
            if (a == b) return;
            if (scan_key_idx(B, 0, a) > scan_key_idx(B, 0, b)) {
                const uint32_t t = a;
                a = b;
                b = t;
            }
            const uint32_t old = atomicCAS(&PF[b], b, a);
            if (old == b) return;
            b = old;
        }
    };
    const uint32_t n = st._u;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const uint32_t i = plist[B.base + e];
        const uint32_t x = i % (uint32_t)B.X, y = (i / (uint32_t)B.X) % (uint32_t)B.Y;
        if (x > 0 && plat_max(i - 1)) unite(i, i - 1);
        if (y > 0 && plat_max(i - (uint32_t)B.X)) unite(i, i - (uint32_t)B.X);
    }
}

// mark roots of plateaus that touch a strictly greater value (cls bit2 on the root)
__global__ void __launch_bounds__(256) k_plateau_flag(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      uint8_t* __restrict__ cls, uint32_t* __restrict__ Pg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !S[blockIdx.y].plateau) return;
    uint8_t* cl = cls + B.base;
    uint32_t* P = Pg + B.base;
    // 16 classes per thread: aligned 16-byte loads over the block's byte range (plateau voxels
    // are rare, so nearly every load is the whole work)
    const int64_t a0 = B.base >> 4, a1 = (B.base + B.N + 15) >> 4;
    const uint4* c16 = reinterpret_cast<const uint4*>(cls);
    for (int64_t a = a0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; a < a1; a += (int64_t)gridDim.x * blockDim.x) {
        const uint4 q = c16[a];
        const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // bytes with both bit 0 and bit 1 set
            uint32_t m = wv[k] & (wv[k] >> 1) & 0x01010101u;
            while (m) {
                const int b = __builtin_ctz(m) >> 3;
                m &= m - 1u;
                const int64_t i = a * 16 + k * 4 + b - B.base;
                if (i < 0 || i >= B.N) continue;
                const uint32_t r = uf_find_compress(P, (uint32_t)i);
                cl[r] |= 4;  // benign race: every writer sets the same bit
            }
        }
    }
}

// ---- root bitmap + exclusive prefix -----------------------------------------------------
// keys per block: n = N (seeds, outer) or NI (crop, inner); words = n/64 + 1, chunks of 256
// words.  inner != 0 selects NI and the inner-sized parent array offset (ibase).  W must be
// zeroed beforehand.
// popcount sums of 256-word chunks
__global__ void __launch_bounds__(256) k_bitmap_csum(const BlockDesc* __restrict__ D, const BlockStat* S, int inner,
                                                     const uint64_t* __restrict__ Wg, uint32_t* __restrict__ csum) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || (inner && !B.crop)) return;
    const int64_t n = inner ? B.NI : B.N;
    const int64_t nw = n / 64 + 1;
    if ((int64_t)blockIdx.x * 256 >= nw) return;
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t c = w < nw ? (uint32_t)__popcll(Wg[B.wbase + w]) : 0u;
    for (int s = 32; s > 0; s >>= 1) c += (uint32_t)__shfl_xor((int)c, s);
    __shared__ uint32_t red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) csum[B.cbase + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// one workgroup per block: exclusive scan of chunk sums in place; total -> counter
__global__ void __launch_bounds__(256) k_chunk_scan(const BlockDesc* __restrict__ D, BlockStat* S, int inner,
                                                    uint32_t* __restrict__ csum, int which_counter) {
    const BlockDesc& B = D[blockIdx.x];
    if (!S[blockIdx.x].active || (inner && !B.crop)) return;
    const int64_t n = inner ? B.NI : B.N;
    const int64_t nw = n / 64 + 1;
    const int64_t nc = (nw + 255) / 256;
    __shared__ uint32_t tmp[256];
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < nc; c0 += 256) {
        const int64_t c = c0 + threadIdx.x;
        uint32_t v = c < nc ? csum[B.cbase + c] : 0u;
        tmp[threadIdx.x] = v;
        __syncthreads();
        for (int s = 1; s < 256; s <<= 1) {
            uint32_t a = threadIdx.x >= (unsigned)s ? tmp[threadIdx.x - s] : 0u;
            __syncthreads();
            tmp[threadIdx.x] += a;
            __syncthreads();
        }
        const uint32_t incl = tmp[threadIdx.x];
        if (c < nc) csum[B.cbase + c] = carry + incl - v;
        carry += tmp[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (which_counter == 0) S[blockIdx.x].n_seeds = carry;
        else if (which_counter == 1) S[blockIdx.x].n_cc = carry;
        else S[blockIdx.x].n_auto = carry;
    }
}

__global__ void __launch_bounds__(256) k_word_prefix(const BlockDesc* __restrict__ D, const BlockStat* S, int inner,
                                                     const uint64_t* __restrict__ Wg, const uint32_t* __restrict__ csum,
                                                     uint32_t* __restrict__ Wp) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || (inner && !B.crop)) return;
    const int64_t n = inner ? B.NI : B.N;
    const int64_t nw = n / 64 + 1;
    if ((int64_t)blockIdx.x * 256 >= nw) return;
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t v = w < nw ? (uint32_t)__popcll(Wg[B.wbase + w]) : 0u;
    // workgroup exclusive scan (wave scan + wave totals)
    uint32_t x = v;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int s = 1; s < 64; s <<= 1) {
        uint32_t a = __shfl_up((int)x, s);
        if (lane >= s) x += a;
    }
    __shared__ uint32_t wt[4];
    if (lane == 63) wt[wv] = x;
    __syncthreads();
    uint32_t woff = 0;
    for (int k = 0; k < wv; ++k) woff += wt[k];
    if (w < nw) Wp[B.wbase + w] = csum[B.cbase + blockIdx.x] + woff + x - v;
}

// roots: slot <- (1 + rank of the root's scan key) | kRootBit, walking the set bits of the
// root bitmap (roots are few: no pass over the voxels)
// rootpos (seed CC, nullable): rootpos[base + label] = the root's block C index (the sparse
// size-filter initialisation starts its walk over a small segment there: a seed keeps its label)
__global__ void __launch_bounds__(256) k_root_label(const BlockDesc* __restrict__ D, const BlockStat* S, int inner,
                                                    uint32_t* __restrict__ PFg, const uint64_t* __restrict__ Wg,
                                                    const uint32_t* __restrict__ Wpg, uint32_t* __restrict__ rootpos) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || (inner && !B.crop)) return;
    uint32_t* P = PFg ? PFg + (inner ? B.ibase : B.base) : nullptr;  // null: rootpos only (pass 2)
    const int64_t n = inner ? B.NI : B.N;
    const int64_t nw = n / 64 + 1;
    const int nz = inner ? B.IZ : B.Z, ny = inner ? B.IY : B.Y, nx = inner ? B.IX : B.X;
    const int64_t yx = (int64_t)ny * nx;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t bits = Wg[B.wbase + w];
        uint32_t rank = Wpg[B.wbase + w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            const int64_t f = w * 64 + b;
            int z, y, x;
            if (inner || B.nd_ws == 3) {  // f = z + nz * (y + ny * x)
                z = (int)(f % nz);
                const int64_t t = f / nz;
                y = (int)(t % ny);
                x = (int)(t / ny);
            } else {  // f = z * Y * X + y + Y * x
                z = (int)(f / yx);
                const int64_t rem = f - (int64_t)z * yx;
                y = (int)(rem % ny);
                x = (int)(rem / ny);
            }
            const int64_t ci = ((int64_t)z * ny + y) * nx + x;
            ++rank;
            if (P) P[ci] = rank | kRootBit;
            if (rootpos) rootpos[B.base + rank] = (uint32_t)ci;
        }
    }
}

// ---- seed labels + flood initialisation --------------------------------------------------
// labels = vigra label (| kFixedBit: seed), keys = (ordf(h) << 32) for seeds, INF otherwise.
__global__ void __launch_bounds__(256) k_seed_label(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const uint32_t* __restrict__ PFg, const uint64_t* __restrict__ sbits,
                                                    const float* __restrict__ h, uint32_t* __restrict__ lab,
                                                    uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv, int packed) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const uint32_t* P = PFg + B.base;
    ROW_TILES(B.Z, B.Y, B.X, {
        const int64_t gi = B.base + i;
        const uint32_t l = bit_of(sbits, B, i) ? cc_label(P, P[i]) : 0u;
        uint64_t k = kInfKey;
        if (l) k = ((uint64_t)ordf(h[gi]) << 32) | (packed ? (uint64_t)l : 0ull);
        lab[gi] = l ? (l | kFixedBit) : 0u;
        key[gi] = k;
        fixedv[gi] = l ? 1 : 0;
    })
}

// ---- halo crop CC (labelVolumeWithBackground, 6-nbhd, equal values, bg 0) -----------------
__device__ __forceinline__ int64_t outer_of_inner(const BlockDesc& B, int z, int y, int x) {
    return ((int64_t)(z + B.iz0) * B.Y + (y + B.iy0)) * B.X + (x + B.ix0);
}

// ---- uint64 output: crop CC label (cropped blocks) or final ws label, + id offset ----------
// Cropped blocks (watershed.py:327-330): the label is the labelVolumeWithBackground number of
// the voxel's component (k_tile_cc<.., CC_CROP> + k_root_label; kNoParent = background).
// Otherwise the final ws label is computed from the flood result as _apply_watershed leaves
// it: 3-D: masked -> 0 (:245-248); 2-D: per-slice label + slice offset, masked -> 0 (:220-237).
// Uncropped blocks also mark their final labels in the (zeroed) bitmap W, so that
// k_count_ids can count the distinct output ids (the label sets have gaps after the size
// filter).
__global__ void __launch_bounds__(256) k_output(const BlockDesc* __restrict__ D, BlockStat* S,
                                                const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                                int packed, const uint32_t* __restrict__ PFg,
                                                const uint32_t* __restrict__ sb, const uint32_t* __restrict__ soff,
                                                unsigned long long* W, int skip_crop) {
    const BlockDesc& B = D[blockIdx.y];
    const bool active = S[blockIdx.y].active;
    if (skip_crop && active && B.crop) return;  // k_output_crop writes it
    const uint32_t* P = PFg + B.ibase;
    const gwptr_t<uint64_t> out = gblw(B.out);
    uint32_t mx = 0;
    bool zero_in = false;  // an in-mask voxel without a label: its output is the bare id offset
    // word tiles over the inner block: lanes past the row end read a clamped position and
    // store nothing
    WORD_TILES(B.IZ, B.IY, B.IX, {
        const int xq = valid ? x : B.IX - 1;
        const int64_t iq = row * B.IX + xq;
        const int64_t o = outer_of_inner(B, z, y, xq);
        const bool inm = !B.mask || gbl(B.mask)[o];
        uint64_t v = 0;  // empty block: constant offset (watershed.py:310-321)
        if (active) {
            uint32_t l;
            if (B.crop) {
                // member -> its tile root -> (the tile root's global root, k_flatten_tile_roots)
                const uint32_t p = gbl(P)[iq];
                l = 0u;
                if (p != kNoParent) {
                    if (p & kRootBit) {
                        l = p & ~kRootBit;
                    } else {
                        const uint32_t q = P[p];
                        l = (q & kRootBit) ? (q & ~kRootBit) : (P[q] & ~kRootBit);
                    }
                }
            } else {
                l = packed ? (uint32_t)(gbl(key)[B.base + o] & kLabelMask) : (gbl(lab)[B.base + o] & ~kFixedBit);
                if (packed && gbl(key)[B.base + o] == kInfKey) l = 0u;
                if (!inm) l = 0;
                else if (B.nd_ws == 2) l = (l - sb[B.sbase + z + B.iz0]) + soff[B.sbase + z + B.iz0];
            }
            if (valid) mx = max(mx, l);
            v = l;
        }
        // out32 (host path): the uint32 local label; the host adds the block's id offset to every
        // in-mask voxel, so half the bytes cross PCIe (the offset is a per-block constant)
        if (valid) {
            if (B.out32) gblw(B.out32)[i] = (uint32_t)v;
            else out[i] = inm ? v + B.id_offset : v;
        }
        zero_in |= valid && active && inm && v == 0;
        if (active && !B.crop) {
            const uint32_t l = valid ? (uint32_t)v : 0u;
            // only the first lane of each run of equal labels along the wave marks it, and it
            // reads the bit before the atomic: the few words of a block's labels are read by
            // every wave of the block, so same-address traffic is kept to a few lanes per wave
            const uint32_t lp = (uint32_t)__shfl_up((int)l, 1);
            const bool first = l != 0u && ((threadIdx.x & 63) == 0 || lp != l);
            if (first && !((W[B.wbase + (l >> 6)] >> (l & 63)) & 1ull)) atomicOr(&W[B.wbase + (l >> 6)], 1ull << (l & 63));
        }
    })
    mx = wg_reduce_u32(mx, OpMax());
    if (threadIdx.x == 0 && mx) atomic_max_if(&S[blockIdx.y].max_label, mx);
    if (__ballot(zero_in) && (threadIdx.x & 63) == 0 && !S[blockIdx.y]._p[0]) atomicOr(&S[blockIdx.y]._p[0], 1u);
}

// k_output for the cropped blocks, one workgroup per crop-CC tile (CcTile): a member of a tile
// component points at its tile root (k_tile_cc<.., CC_CROP>), the tile roots (bits of TR) at
// their global root or carry the label (k_flatten_tile_roots, k_root_label).  The tile roots'
// labels are resolved first (one dependent load each) into LDS, then every member reads its
// root's label from LDS: no dependent global load per member (k_output: two).
template <int ND>
__global__ void __launch_bounds__(256) k_output_crop(const BlockDesc* __restrict__ D, BlockStat* S,
                                                     const uint32_t* __restrict__ PFg, const uint64_t* __restrict__ TR) {
    using T = CcTile<ND>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX, TN = TZ * TY * TX, PER = TN / 256;
    __shared__ uint32_t sl[TN];
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !B.crop) return;
    const int nz = B.IZ, ny = B.IY, nx = B.IX;
    const int ntx = (nx + TX - 1) / TX, nty = (ny + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    // XCD-contiguous tiles (gridDim.x is a multiple of 8): the uint64 rows of neighbouring tiles
    // share lines in one L2 (config 3 output 3.1 -> 2.8 ms)
    const int t = xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
    if (t >= ntx * nty * ntz) return;
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    const gptr_t<uint32_t> P = gbl(PFg + B.ibase);
    uint32_t e[PER];
    int64_t gi[PER];
    bool in[PER], root[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
        in[j] = z < nz && y < ny && x < nx;
        gi[j] = ((int64_t)min(z, nz - 1) * ny + min(y, ny - 1)) * nx + min(x, nx - 1);
        e[j] = P[gi[j]];
        root[j] = (gbl(TR)[B.fbase + (gi[j] >> 6)] >> (gi[j] & 63)) & 1ull;
    }
    // tile roots: their label (a global root carries it; the others point at their global root)
    uint32_t rl[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const bool need = in[j] && root[j] && e[j] != kNoParent && !(e[j] & kRootBit);
        rl[j] = P[need ? e[j] : 0u];  // unconditional: all in flight
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!(in[j] && root[j])) continue;
        const uint32_t l = (e[j] & kRootBit) ? (e[j] & ~kRootBit) : (rl[j] & ~kRootBit);
        sl[threadIdx.x + j * 256] = l;
    }
    __syncthreads();
    const gwptr_t<uint64_t> out = gblw(B.out);
    uint32_t mx = 0;
    bool zero_in = false;
    // a member's tile root r lies in this tile: its offset from the tile's first voxel is
    // (lz * ny + ly) * nx + lx with lz < TZ, ly < TY, lx < TX, split by div_small
    const uint32_t tb = (uint32_t)(((int64_t)z0 * ny + y0) * nx + x0);
    const int plane = ny * nx;
    const float inv_nx = 1.0f / (float)nx, inv_plane = 1.0f / (float)plane;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!in[j]) continue;
        uint32_t l = 0u;
        if (e[j] != kNoParent) {
            if (root[j]) {
                l = sl[threadIdx.x + j * 256];
            } else {
                const int d = (int)(e[j] - tb);
                const int lz = TZ > 1 ? div_small(d, plane, inv_plane) : 0;
                const int rem = d - lz * plane;
                const int ly = div_small(rem, nx, inv_nx);
                l = sl[(lz * TY + ly) * TX + (rem - ly * nx)];
            }
        }
        const int c = threadIdx.x + j * 256;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int64_t o = outer_of_inner(B, z0 + lz, y0 + ly, x0 + lx);
        const bool inm = !B.mask || gbl(B.mask)[o];
        mx = max(mx, l);
        if (B.out32) gblw(B.out32)[gi[j]] = l;
        else out[gi[j]] = inm ? (uint64_t)l + B.id_offset : (uint64_t)l;
        zero_in |= inm && l == 0u;
    }
    mx = wg_reduce_u32(mx, OpMax());
    if (threadIdx.x == 0 && mx) atomic_max_if(&S[blockIdx.y].max_label, mx);
    if (__ballot(zero_in) && (threadIdx.x & 63) == 0 && !S[blockIdx.y]._p[0]) atomicOr(&S[blockIdx.y]._p[0], 1u);
}
template __global__ void k_output_crop<2>(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*);
template __global__ void k_output_crop<3>(const BlockDesc*, BlockStat*, const uint32_t*, const uint64_t*);

// distinct ids of an uncropped block: popcount of its label bitmap (k_output) -> n_cc
__global__ void __launch_bounds__(256) k_count_ids(const BlockDesc* __restrict__ D, BlockStat* S,
                                                   const uint64_t* __restrict__ W) {
    const BlockDesc& B = D[blockIdx.y];
    BlockStat& st = S[blockIdx.y];
    if (!st.active || B.crop) return;
    const int64_t nw = (int64_t)(st.max_label >> 6) + 1;
    uint32_t c = 0;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x)
        c += (uint32_t)__popcll(W[B.wbase + w]);
    c = wg_reduce_u32(c, OpAdd());
    if (threadIdx.x == 0 && c) atomicAdd(&st.n_cc, c);
}

// Crop CC: only the tile roots (bits of the tile-root bitmap TR, set by k_tile_cc<.., CC_CROP>)
// are pointed at their global root; members keep pointing at their tile root, and k_output
// follows member -> tile root -> root.  Global roots set their scan-key bit in W (zeroed).
// One thread per bitmap word: the roots are few (a handful per tile), the voxels are not read.
__global__ void __launch_bounds__(256) k_flatten_tile_roots(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                            uint32_t* __restrict__ PFg, const uint64_t* __restrict__ TR,
                                                            uint64_t* __restrict__ Wg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !B.crop) return;
    uint32_t* P = PFg + B.ibase;
    uint64_t* W = Wg + B.wbase;
    const int64_t nw = B.NI / 64 + 1;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t bits = TR[B.fbase + w];
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            const uint32_t i = (uint32_t)(w * 64 + b);
            const uint32_t r = uf_find(P, i);
            if (r != i) {
                P[i] = r;
            } else {
                const int x = (int)(i % (uint32_t)B.IX);
                const uint32_t t = i / (uint32_t)B.IX;
                const int y = (int)(t % (uint32_t)B.IY), z = (int)(t / (uint32_t)B.IY);
                const uint32_t f = (uint32_t)(z + B.IZ * (y + B.IY * x));
                atomicOr((unsigned long long*)&W[f >> 6], 1ull << (f & 63));
            }
        }
    }
}

// The seed forest (k_tile_cc<.., CC_SEED> writes its members only): every member is pointed at
// its root, roots set their scan-key bit in W (zeroed).  One thread per member-bitmap word: the
// seeds are ~1 % of the voxels, the non-members are not read at all.
__global__ void __launch_bounds__(256) k_flatten_seeds(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                       uint32_t* __restrict__ PFg, const uint64_t* __restrict__ bits,
                                                       uint64_t* __restrict__ Wg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    uint32_t* P = PFg + B.base;
    uint64_t* W = Wg + B.wbase;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nw = (int64_t)B.Z * B.Y * wpr;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t m = bits[B.fbase + w];
        if (!m) continue;
        const int64_t row = w / wpr;
        const int xw = (int)(w - row * wpr);
        const int z = (int)(row / B.Y), y = (int)(row - (int64_t)z * B.Y);
        while (m) {
            const int b = __builtin_ctzll(m);
            m &= m - 1;
            const int x = xw * 64 + b;
            const uint32_t i = (uint32_t)(row * B.X + x);
            const uint32_t p = P[i];
            if (p == i) {
                const uint32_t f = scan_key_of(B, z, y, x);
                atomicOr((unsigned long long*)&W[f >> 6], 1ull << (f & 63));
            } else {
                const uint32_t r = uf_find(P, p);
                if (r != p) P[i] = r;
            }
        }
    }
}

}  // namespace ctws
