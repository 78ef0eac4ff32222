// k_tilecc.hip — block-based union-find connected components in LDS on gfx950.
//
// Three CC problems of the path share this machinery:
//   PLATEAU  equal-valued neighbours of the seed map (localMaxima's plateau handling,
//            watershed.py:187-192; 6-nbhd in 3-D, 8-nbhd in-plane in 2-D)
//   SEED     the maxima voxels (labelMultiArrayWithBackground, watershed.py:205; direct nbhd)
//   CROP     equal final labels of the cropped inner block (labelVolumeWithBackground,
//            watershed.py:329; 6-nbhd in 3-D; in 2-D ws mode labels of different slices are
//            never equal — per-slice offsets make their ranges disjoint — so in-plane only)
//
// A global union-find over every voxel (one atomicCAS chain per neighbour pair through HBM)
// costs ~100x a streaming pass on large components.  Here a workgroup first solves its tile
// (CcTileM: 3-D 8x16x32, crop 4x16x32; 2-D 1x32x64) completely in LDS: parents are tile-local positions and a
// union links the root with the larger *order key* under the smaller (atomicCAS in LDS), so
// every tile component is rooted at its smallest key.  For SEED/CROP (and 3-D PLATEAU) the order key is the local F-order index
// (x most significant, then y, then z — vigra scan order, A.0), so the tile root is the
// component's first voxel in scan order within the tile; for 2-D PLATEAU the C-order index.
// The tile writes each member's global parent = its tile root (C-order block index), non-
// members get kNoParent.  k_tile_merge then unions the tile roots across the tile faces with
// the global (scan-key ordered) union-find; only face pairs whose local roots differ from the
// previous lane's pair reach the atomics.  k_flatten_seeds / k_flatten_tile_roots (k_cc.hip) finish.
#include "ctws_kernels.h"

namespace ctws {

constexpr uint32_t kLNone = 0xFFFFFFFFu;

// local scan key (vigra order) of tile position (lz, ly, lx)
template <int TZ, int TY>
__device__ __forceinline__ uint32_t fkey_local(int lz, int ly, int lx) {
    return (uint32_t)(lz + TZ * (ly + TY * lx));
}

// ---- per-mode domain, membership and connectivity ---------------------------------------

// is voxel i (outer index) a local maximum? (k_cc.hip's is_max with the plateau flag)
__device__ __forceinline__ bool cc_is_max(const uint8_t* cl, const uint32_t* P, int64_t i, bool plat) {
    const uint8_t c = cl[i];
    if (c & 1) return false;
    if (!(c & 2) || !plat) return true;
    return !(cl[uf_find(P, (uint32_t)i)] & 4);
}

// value of voxel (z, y, x) of the mode's domain; kLNone = not a member
template <int MODE>
__device__ __forceinline__ uint32_t cc_value(const BlockDesc& B, const CcArgs& a, bool plat, int z, int y, int x) {
    if (MODE == CC_CROP) {
        const int64_t o = ((int64_t)(z + B.iz0) * B.Y + (y + B.iy0)) * B.X + (x + B.ix0);
        if (B.mask && !gbl(B.mask)[o]) return kLNone;
        const uint32_t l = flood_label(a.lab, a.key, a.packed, B.base + o);
        return l ? l : kLNone;
    } else {
        const int64_t i = ((int64_t)z * B.Y + y) * B.X + x;
        if (MODE == CC_PLATEAU) {
            if (!(a.cls[B.base + i] & 2)) return kLNone;
            const uint32_t u = __float_as_uint(a.v[B.base + i]);
            return u == 0x80000000u ? 0u : u;  // -0.0 == +0.0
        }
        return cc_is_max(a.cls + B.base, a.Pp + B.base, i, plat) ? 1u : kLNone;
    }
}

// backward neighbours (dz, dy, dx) of the mode: 3-D 6-nbhd; 2-D 4-nbhd (8 for PLATEAU)
template <int ND, int MODE>
struct CcNbrs;
template <int MODE>
struct CcNbrs<3, MODE> {
    static constexpr int N = 3;
    __device__ static constexpr int dz(int k) { return k == 0 ? -1 : 0; }
    __device__ static constexpr int dy(int k) { return k == 1 ? -1 : 0; }
    __device__ static constexpr int dx(int k) { return k == 2 ? -1 : 0; }
};
template <int MODE>
struct CcNbrs<2, MODE> {
    static constexpr int N = MODE == CC_PLATEAU ? 4 : 2;
    __device__ static constexpr int dz(int) { return 0; }
    __device__ static constexpr int dy(int k) { return k == 1 ? 0 : -1; }            // k: 0 (-1,0) 1 (0,-1)
    __device__ static constexpr int dx(int k) { return k == 0 ? 0 : (k == 1 ? -1 : (k == 2 ? -1 : 1)); }
};

template <int MODE>
__device__ __forceinline__ void domain_dims(const BlockDesc& B, int& nz, int& ny, int& nx) {
    if (MODE == CC_CROP) {
        nz = B.IZ;
        ny = B.IY;
        nx = B.IX;
    } else {
        nz = B.Z;
        ny = B.Y;
        nx = B.X;
    }
}

template <int ND, int MODE>
__global__ void __launch_bounds__(256) k_tile_cc(const BlockDesc* __restrict__ D, const BlockStat* S, CcArgs a,
                                                 uint32_t* __restrict__ Pg) {
    using T = CcTileM<ND, MODE>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX, TN = TZ * TY * TX, PER = TN / 256;
    static_assert(TN % 256 == 0, "");
    __shared__ uint32_t sv[TN];  // values, C-layout c = (lz * TY + ly) * TX + lx
    __shared__ uint32_t sp[TN];  // parents, C-layout like sv
    const BlockDesc& B = D[blockIdx.y];
    const BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    if (MODE == CC_PLATEAU && !st.plateau) return;
    if (MODE == CC_CROP && !B.crop) return;
    const bool plat = st.plateau != 0;
    int nz, ny, nx;
    domain_dims<MODE>(B, nz, ny, nx);
    const int ntx = (nx + TX - 1) / TX, nty = (ny + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    // (dispatch order, not xcd_swizzle: XCD-contiguous tiles measured slower for the seed CC;
    // gridDim.x may be rounded up to a multiple of 8)
    const int t = blockIdx.x;
    if (t >= ntx * nty * ntz) return;
    if (MODE == CC_PLATEAU && !a.ptile[B.ptbase + t]) return;  // no plateau voxel (k_localmax)
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    // order key of tile position c: the C index (PLATEAU) or the vigra scan key (SEED, CROP)
    auto ordk = [&](uint32_t c) -> uint32_t {
        const int lx = (int)(c % TX), ly = (int)((c / TX) % TY), lz = (int)(c / (TX * TY));
        // (3-D plateaus are rooted at their first voxel in scan order too: k_seed_members
        // takes the maximal plateaus' roots as seed-component roots)
        return (MODE == CC_PLATEAU && ND == 2) ? c : fkey_local<TZ, TY>(lz, ly, lx);
    };
    // load values: every load unconditional (position clamped into the domain, global address
    // space) so that all of a thread's loads are in flight together; non-members and positions
    // outside the domain are selected away afterwards.  Same values as cc_value.
    uint32_t vv[PER];
    {
        uint64_t l0[PER];
        uint32_t l1[PER];
        uint32_t inm = 0;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int c = threadIdx.x + j * 256;
            const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
            const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
            inm |= ((z < nz && y < ny && x < nx) ? 1u : 0u) << j;
            const int cz = min(z, nz - 1), cy = min(y, ny - 1), cx = min(x, nx - 1);
            if (MODE == CC_CROP) {
                const int64_t o = ((int64_t)(cz + B.iz0) * B.Y + (cy + B.iy0)) * B.X + (cx + B.ix0);
                l0[j] = a.packed ? gbl(a.key)[B.base + o] : (uint64_t)gbl(a.lab)[B.base + o];
                l1[j] = B.mask ? (uint32_t)gbl(B.mask)[o] : 1u;
            } else {
                const int64_t i = B.base + ((int64_t)cz * B.Y + cy) * B.X + cx;
                l0[j] = gbl(a.cls)[i];
                l1[j] = 0u;
            }
        }
        if (MODE == CC_PLATEAU) {
            // a tile without plateau voxels writes nothing (P is read only at plateau voxels:
            // cc_is_max, k_plateau_flag, k_tile_merge check cls first) and skips the value loads
            bool any = false;
#pragma unroll
            for (int j = 0; j < PER; ++j) any |= ((inm >> j) & 1u) && (l0[j] & 2);
            if (!__syncthreads_or(any)) return;
#pragma unroll
            for (int j = 0; j < PER; ++j) {
                const int c = threadIdx.x + j * 256;
                const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
                const int cz = min(z0 + lz, nz - 1), cy = min(y0 + ly, ny - 1), cx = min(x0 + lx, nx - 1);
                l1[j] = (l0[j] & 2) ? __float_as_uint(gbl(a.v)[B.base + ((int64_t)cz * B.Y + cy) * B.X + cx]) : 0u;
            }
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            uint32_t v = kLNone;
            if (MODE == CC_CROP) {
                uint32_t l = a.packed ? (l0[j] == kInfKey ? 0u : (uint32_t)(l0[j] & kLabelMask))
                                      : ((uint32_t)l0[j] & ~kFixedBit);
                if (!l1[j]) l = 0u;  // masked
                v = l ? l : kLNone;
            } else if (MODE == CC_PLATEAU) {
                v = (l0[j] & 2) ? (l1[j] == 0x80000000u ? 0u : l1[j]) : kLNone;
            } else {
                const uint32_t cl = (uint32_t)l0[j];
                v = (cl & 1) ? kLNone : 1u;
                if (!(cl & 1) && (cl & 2) && plat && ((inm >> j) & 1u)) {
                    // a plateau voxel: maximum iff its plateau is (k_plateau_flag's bit 4)
                    const int c = threadIdx.x + j * 256;
                    const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
                    const int64_t i = ((int64_t)(z0 + lz) * B.Y + (y0 + ly)) * B.X + (x0 + lx);
                    v = cc_is_max(a.cls + B.base, a.Pp + B.base, i, plat) ? 1u : kLNone;
                }
            }
            vv[j] = ((inm >> j) & 1u) ? v : kLNone;
        }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) sv[threadIdx.x + j * 256] = vv[j];
    __syncthreads();
    // Runs along x: a wave holds 64 consecutive voxels (64 / TX whole tile rows), so every
    // member links straight to the first voxel of its run (found by ballot) — the x
    // connectivity needs no union at all.
    const int lane = threadIdx.x & 63;
    auto conn = [&](uint32_t u, uint32_t w) { return u != kLNone && w != kLNone && (MODE == CC_SEED || u == w); };
    uint32_t contm = 0;  // bit j: voxel j continues the run of its x predecessor
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c % TX;
        const bool cont = lx > 0 && conn(sv[c - 1], vv[j]);
        contm |= (cont ? 1u : 0u) << j;
        const uint64_t starts = __ballot(!cont);
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const int s0 = 63 - __builtin_clzll(starts & upto);
        // (the run start has the smallest x, so the smallest scan key of the run)
        sp[c] = vv[j] == kLNone ? kLNone : (uint32_t)(c - (lane - s0));
    }
    __syncthreads();
    // unions with the other backward neighbours; a y / z pair is redundant when both voxels
    // continue their x runs (the pair of their x predecessors covers it)
    using NB = CcNbrs<ND, MODE>;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (vv[j] == kLNone) continue;
        const int c = threadIdx.x + j * 256;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
#pragma unroll
        for (int k = 0; k < NB::N; ++k) {
            const int dz = NB::dz(k), dy = NB::dy(k), dx = NB::dx(k);
            if (dz == 0 && dy == 0) continue;  // the x neighbour: runs
            const int qz = lz + dz, qy = ly + dy, qx = lx + dx;
            if (qz < 0 || qy < 0 || qx < 0 || qx >= TX) continue;
            const int cq = (qz * TY + qy) * TX + qx;
            if (!conn(sv[cq], vv[j])) continue;
            if (dx == 0 && ((contm >> j) & 1u) && conn(sv[cq - 1], sv[cq])) continue;
            lds_union(sp, (uint32_t)c, (uint32_t)cq, ordk);
        }
    }
    __syncthreads();
    // members -> global parent = C-order block index of the tile root.  SEED: members only (the
    // seed voxels are ~1 %), plus their bits in the member bitmap (a.troot): the readers of the
    // seed forest test the bitmap first, and the stores of kNoParent (4 B per voxel) go away
    uint32_t* P = Pg + (MODE == CC_CROP ? B.ibase : B.base);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
        if (MODE == CC_SEED) {
            // a wave's 64 positions are whole tile rows (TX = 64, or two rows of 32): one word
            // (or two halves) of the member bitmap
            const bool mem = z < nz && y < ny && x < nx && vv[j] != kLNone;
            const uint64_t bm = __ballot(mem);
            if ((lane == 0 || lane == TX) && bm) {
                const uint64_t part = TX == 64 ? bm : ((lane == 0 ? bm : bm >> 32) & 0xFFFFFFFFull);
                const int wpr = (nx + 63) >> 6;
                if (part && z < nz && y < ny)
                    atomicOr((unsigned long long*)&a.troot[B.fbase + ((int64_t)z * ny + y) * wpr + (x0 >> 6)],
                             (unsigned long long)(part << (x0 & 63)));
            }
            if (!mem) continue;
        }
        const bool ind = z < nz && y < ny && x < nx;
        uint32_t g = kNoParent;
        const int64_t gi = ((int64_t)z * ny + y) * nx + x;
        if (ind && vv[j] != kLNone) {
            const uint32_t r = lds_find(sp, (uint32_t)c);
            const int rx = (int)(r % TX), ry = (int)((r / TX) % TY), rz = (int)(r / (TX * TY));
            g = (uint32_t)(((int64_t)(z0 + rz) * ny + (y0 + ry)) * nx + (x0 + rx));
            // CROP: the tile roots, so that only they are flattened (k_flatten_tile_roots)
            if (MODE == CC_CROP && r == (uint32_t)c)
                atomicOr((unsigned long long*)&a.troot[B.fbase + (gi >> 6)], 1ull << (gi & 63));
        }
        if (MODE == CC_CROP && (lx == 0 || lx == TX - 1)) {
            // the x columns for k_tile_merge: its x face reads them contiguously instead of one
            // cache line per voxel for each of P, key and mask on both sides
            const int64_t xb = B.xcbase + (int64_t)t * 2 * TZ * TY + (lx == 0 ? 0 : TZ * TY) + lz * TY + ly;
            a.xface[xb] = ((uint64_t)g << 32) | (uint64_t)(ind ? vv[j] : kLNone);
        }
        if (!ind) continue;
        P[gi] = g;
    }
}

// union the tile roots across the tiles' backward faces (global union-find: by C index for
// 2-D PLATEAU, by scan key otherwise so that roots stay the first voxel in scan order)
template <int ND, int MODE>
__global__ void __launch_bounds__(256) k_tile_merge(const BlockDesc* __restrict__ D, const BlockStat* S, CcArgs a,
                                                    uint32_t* __restrict__ Pg) {
    using T = CcTileM<ND, MODE>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX;
    const BlockDesc& B = D[blockIdx.y];
    const BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    if (MODE == CC_PLATEAU && !st.plateau) return;
    if (MODE == CC_CROP && !B.crop) return;
    int nz, ny, nx;
    domain_dims<MODE>(B, nz, ny, nx);
    const int ntx = (nx + TX - 1) / TX, nty = (ny + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    // a workgroup walks several tiles (a face is only a few hundred voxels: one workgroup per
    // tile would make the dispatch of ~10^5 workgroups the cost)
    for (int t = blockIdx.x; t < ntx * nty * ntz; t += gridDim.x) {
    // a face pair needs a plateau voxel on this tile's side: tiles without one are skipped
    if (MODE == CC_PLATEAU && !a.ptile[B.ptbase + t]) continue;
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    uint32_t* P = Pg + (MODE == CC_CROP ? B.ibase : B.base);
    const int inner = MODE == CC_CROP ? 1 : 0;
    using NB = CcNbrs<ND, MODE>;
    // face voxels: the low z / y / x planes (and, for 2-D plateaus, the high x plane below),
    // enumerated per face so that consecutive lanes walk consecutive face voxels
    const int fsz[3] = {TY * TX, TZ * TX, TZ * TY};  // z-face (y, x), y-face (z, x), x-face (z, y)
    for (int f = (ND == 3 ? 0 : 1); f < 3; ++f) {
        const int n = fsz[f];
        for (int e0 = 0; e0 < n; e0 += 256) {
            const int e = e0 + (int)threadIdx.x;
            uint32_t ra = kNoParent, rb = kNoParent;
            if (MODE == CC_CROP && f == 2) {
                // x face from the tiles' x columns (k_tile_cc): this tile's low column against
                // the high column of the tile before it in x, (root << 32 | label) each
                if (e < n && txi > 0) {
                    const int64_t tb = B.xcbase + (int64_t)t * 2 * TZ * TY;
                    const uint64_t own = a.xface[tb + e];
                    const uint64_t prv = a.xface[tb - 2 * TZ * TY + TZ * TY + e];
                    const uint32_t lo = (uint32_t)own, lp = (uint32_t)prv;
                    if (lo != kLNone && lo == lp) {
                        ra = (uint32_t)(own >> 32);
                        rb = (uint32_t)(prv >> 32);
                    }
                }
            } else if (MODE == CC_CROP) {
                // z / y face: one backward neighbour q across it.  Members are exactly the voxels
                // with a parent (k_tile_cc), so two members connect iff their flood labels match:
                // both parents and both labels are loaded together (clamped, unconditional), one
                // round trip instead of parent -> neighbour's parent -> mask and label
                const int lz = f == 0 ? 0 : e / TX, ly = f == 0 ? e / TX : 0, lx = e % TX;
                const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
                const bool ok = e < n && z < nz && y < ny && x < nx && (f == 0 ? z > 0 : y > 0);
                const int64_t i = ok ? ((int64_t)z * ny + y) * nx + x : 0;
                const int64_t q = ok ? i - (f == 0 ? (int64_t)ny * nx : (int64_t)nx) : 0;
                const int64_t o = ok ? ((int64_t)(z + B.iz0) * B.Y + (y + B.iy0)) * B.X + (x + B.ix0) : 0;
                const int64_t oq = ok ? o - (f == 0 ? (int64_t)B.Y * B.X : (int64_t)B.X) : 0;
                const uint32_t pi = gbl(P)[i], pq = gbl(P)[q];
                const uint32_t li = flood_label(a.lab, a.key, a.packed, B.base + o);
                const uint32_t lq = flood_label(a.lab, a.key, a.packed, B.base + oq);
                if (ok && pi != kNoParent && pq != kNoParent && li == lq) {
                    ra = pi;
                    rb = pq;
                }
            } else if (e < n) {
                int lz, ly, lx;
                if (f == 0) { lz = 0; ly = e / TX; lx = e % TX; }
                else if (f == 1) { lz = e / TX; ly = 0; lx = e % TX; }
                else { lz = e / TY; ly = e % TY; lx = 0; }
                const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
                if (z < nz && y < ny && x < nx) {
                    const int64_t i = ((int64_t)z * ny + y) * nx + x;
                    // PLATEAU: tiles without plateau voxels leave P unwritten; SEED: P holds
                    // the members only (the member bitmap a.troot says which)
                    const bool mi = MODE == CC_SEED ? bit_of(a.troot, B, i)
                                                    : (MODE != CC_PLATEAU || (a.cls[B.base + i] & 2));
                    const uint32_t pi = mi ? P[i] : kNoParent;
                    if (pi != kNoParent) {
                        // the backward neighbours of (z, y, x) that leave the tile through face f
                        // (a diagonal through the tile corner belongs to the y face)
#pragma unroll
                        for (int k = 0; k < NB::N; ++k) {
                            const int dz = NB::dz(k), dy = NB::dy(k), dx = NB::dx(k);
                            const bool out = (f == 0 && dz < 0) || (f == 1 && dy < 0) ||
                                             (f == 2 && dx < 0 && (dy == 0 || ly > 0));
                            const int qz = z + dz, qy = y + dy, qx = x + dx;
                            if (!out || qz < 0 || qy < 0 || qx < 0 || qx >= nx) continue;
                            const int64_t q = ((int64_t)qz * ny + qy) * nx + qx;
                            if (MODE == CC_PLATEAU && !(a.cls[B.base + q] & 2)) continue;
                            if (MODE == CC_SEED && !bit_of(a.troot, B, q)) continue;
                            const uint32_t pq = P[q];
                            if (pq == kNoParent) continue;
                            if (MODE != CC_SEED &&
                                cc_value<MODE>(B, a, true, z, y, x) != cc_value<MODE>(B, a, true, qz, qy, qx))
                                continue;
                            const bool axial = (dz != 0) + (dy != 0) + (dx != 0) == 1;
                            if (axial) {
                                ra = pi;
                                rb = pq;
                            } else {
                                uf_union(P, pi, pq);  // 2-D plateau diagonal (rare)
                            }
                        }
                    }
                }
            }
            // skip the pair of the previous lane (runs along a face share their tile roots)
            const uint32_t pa = (uint32_t)__shfl_up((int)ra, 1), pb = (uint32_t)__shfl_up((int)rb, 1);
            const bool dup = ((threadIdx.x & 63) != 0) && pa == ra && pb == rb;
            if (ra != kNoParent && !dup) {
                if (MODE == CC_PLATEAU && ND == 2) uf_union(P, ra, rb);
                else uf_union_scan(P, ra, rb, B, inner);
            }
        }
    }
    if (ND == 2 && MODE == CC_PLATEAU) {
        // diagonal (-1, +1) across the high x face (voxels lx == TX - 1, ly > 0; ly == 0 is
        // covered by the y face above)
        for (int e = threadIdx.x; e < TZ * TY; e += 256) {
            const int lz = e / TY, ly = e % TY;
            const int z = z0 + lz, y = y0 + ly, x = x0 + TX - 1;
            if (ly == 0 || z >= nz || y >= ny || x + 1 >= nx) continue;
            const int64_t i = ((int64_t)z * ny + y) * nx + x;
            const int64_t q = i - nx + 1;
            if (!(a.cls[B.base + i] & 2) || !(a.cls[B.base + q] & 2)) continue;
            const uint32_t pi = P[i], pq = P[q];
            if (pi == kNoParent || pq == kNoParent) continue;
            if (cc_value<MODE>(B, a, true, z, y, x) != cc_value<MODE>(B, a, true, z, y - 1, x + 1)) continue;
            uf_union(P, pi, pq);
        }
    }
    }  // tiles
}

#define CTWS_TILECC_INST(ND, MODE)                                                                   \
    template __global__ void k_tile_cc<ND, MODE>(const BlockDesc*, const BlockStat*, CcArgs, uint32_t*); \
    template __global__ void k_tile_merge<ND, MODE>(const BlockDesc*, const BlockStat*, CcArgs, uint32_t*);
CTWS_TILECC_INST(3, CC_PLATEAU)
CTWS_TILECC_INST(2, CC_PLATEAU)
CTWS_TILECC_INST(3, CC_SEED)
CTWS_TILECC_INST(2, CC_SEED)
CTWS_TILECC_INST(3, CC_CROP)
CTWS_TILECC_INST(2, CC_CROP)
#undef CTWS_TILECC_INST

}  // namespace ctws
