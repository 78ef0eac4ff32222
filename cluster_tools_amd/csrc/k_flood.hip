// k_flood.hip — seeded watershed (vigra watershedsNew, region growing) on gfx950.
//
// Reference: utils/volume_utils.py:123-139 (vu.watershed, apply_size_filter) calling
// vigra.analysis.watershedsNew -> seededWatersheds: a min-priority queue, label-on-push,
// priority(q) = max(h(q), priority(parent)).  Popped priorities are non-decreasing, so every
// voxel q gets
//     C(q) = minimax path height from the seeds (the priority it is pushed with), and
//     label(q) = label of the neighbour popped first, i.e. the neighbour with the smallest C.
// Equal C values (plateaus) are ordered by the heap in vigra; here the order inside a
// plateau is the hop distance d from where the plateau level was entered, so the key
//     K(q) = (C(q), d(q)),   K(q) = f_q(min_p K(p)),
//     f_q(C, d) = h(q) > C ? (h(q), 0) : (C, d + 1)
// is strictly increasing along parent edges, and the fixpoint (K, label) with
// label(q) = label(argmin_p (K(p), label(p))) is unique and independent of the schedule.
// Seeds are fixed at K = (h, 0).  The parity bar for this stage is VI <= 0.01 / ARand <= 1e-3
// against the oracle (which reproduces the heap order), not bit-exactness.
//
// Schedule: tiles of TZxTYxTX voxels with a 1-voxel halo in LDS relax to the local fixpoint
// (each thread owns a run of 8 voxels along x and sweeps it forward and backward, so a
// change crosses the run in one sweep); changed face voxels activate the face-neighbour
// tiles for the next round; rounds repeat until no tile is active.
//
// Keys are uint64 (ordf(C) << 32 | d); labels carry kFixedBit for seeds.
#include <type_traits>

#include "ctws_kernels.h"

namespace ctws {

template <int ND>
struct FloodTile;
template <>
struct FloodTile<3> {
    static constexpr int TZ = 4, TY = 8, TX = 64, HZ = TZ + 2;
};
template <>
struct FloodTile<2> {
    static constexpr int TZ = 1, TY = 32, TX = 64, HZ = 1;
};

__device__ __forceinline__ void take_min(uint64_t nk, uint32_t nl, uint64_t& bk, uint32_t& bl) {
    if (nk < bk || (nk == bk && nl < bl)) {
        bk = nk;
        bl = nl;
    }
}

// (C, d + 1): d is 32 bits here and never saturates (a hop distance is < N < 2^31), so this
// kernel computes the unbounded (C, d, label) fixpoint -- the one the packed flood equals when
// none of its keys reached kDMax, and the one run_batch falls back to when one did (dsat)
__device__ __forceinline__ uint64_t f_key(uint32_t hb, uint64_t bk) {
    const uint32_t c = (uint32_t)(bk >> 32);
    if (hb > c) return (uint64_t)hb << 32;
    return bk + 1ull;
}

template <int ND>
__global__ void __launch_bounds__(256) k_flood(const BlockDesc* __restrict__ D, const BlockStat* S,
                                               const float* __restrict__ h, uint64_t* __restrict__ key,
                                               uint32_t* __restrict__ lab, const uint32_t* __restrict__ act_cur,
                                               uint32_t* __restrict__ act_next, uint32_t* __restrict__ counter) {
    using T = FloodTile<ND>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX;
    constexpr int HZ = T::HZ, HY = TY + 2, HX = TX + 2;
    constexpr int HN = HZ * HY * HX;
    constexpr int RUN = 8;
    __shared__ uint64_t sk[HN];
    __shared__ uint32_t sl[HN];
    __shared__ int sface[6];

    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int ntile = B.tz * B.ty * B.tx;
    const int t = blockIdx.x;
    if (t >= ntile) return;
    if (!act_cur[B.tbase + t]) return;
    const int txi = t % B.tx, tyi = (t / B.tx) % B.ty, tzi = t / (B.tx * B.ty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int64_t gb = B.base;

    if (threadIdx.x < 6) sface[threadIdx.x] = 0;
    // ---- load tile + halo
    for (int c = threadIdx.x; c < HN; c += 256) {
        const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
        const int gz = (ND == 3) ? z0 + hz - 1 : z0;
        const int gy = y0 + hy - 1, gx = x0 + hx - 1;
        uint64_t k = kInfKey;
        uint32_t l = 0;
        if (gz >= 0 && gz < B.Z && gy >= 0 && gy < B.Y && gx >= 0 && gx < B.X) {
            const int64_t gi = gb + gz * YX + (int64_t)gy * B.X + gx;
            k = key[gi];
            l = lab[gi] & ~kFixedBit;
        }
        sk[c] = k;
        sl[c] = l;
    }
    // ---- owned run
    const int run = threadIdx.x % (TX / RUN);
    const int row = threadIdx.x / (TX / RUN);  // 0 .. TZ*TY-1
    const int lz = (ND == 3) ? row / TY : 0, ly = row % TY;
    const int lx0 = run * RUN;
    const int gz = z0 + lz, gy = y0 + ly;
    const int hz = (ND == 3) ? lz + 1 : 0, hy = ly + 1;
    const int hrow = (hz * HY + hy) * HX;
    uint64_t k[RUN], k0[RUN];
    uint32_t l[RUN], l0[RUN], hb[RUN];
    uint32_t fixed = 0, valid = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RUN; ++j) {
        const int gx = x0 + lx0 + j;
        const bool in = gz < B.Z && gy < B.Y && gx < B.X;
        hb[j] = 0;
        if (in) {
            const int64_t gi = gb + gz * YX + (int64_t)gy * B.X + gx;
            hb[j] = ordf(h[gi]);
            if (lab[gi] & kFixedBit) fixed |= 1u << j;
            valid |= 1u << j;
        }
        k[j] = k0[j] = sk[hrow + lx0 + j + 1];
        l[j] = l0[j] = sl[hrow + lx0 + j + 1];
    }
    const uint32_t upd = valid & ~fixed;

    // ---- local relaxation to the fixpoint
    for (int it = 0; it < 4096; ++it) {
        bool ch = false;
        auto relax = [&](int j) {
            const int c = hrow + lx0 + j + 1;
            uint64_t bk = kInfKey;
            uint32_t bl = 0xFFFFFFFFu;
            // x-neighbours: own registers inside the run, LDS at the run ends
            if (j > 0) take_min(k[j - 1], l[j - 1], bk, bl);
            else take_min(sk[c - 1], sl[c - 1], bk, bl);
            if (j < RUN - 1) take_min(k[j + 1], l[j + 1], bk, bl);
            else take_min(sk[c + 1], sl[c + 1], bk, bl);
            take_min(sk[c - HX], sl[c - HX], bk, bl);
            take_min(sk[c + HX], sl[c + HX], bk, bl);
            if (ND == 3) {
                take_min(sk[c - HX * HY], sl[c - HX * HY], bk, bl);
                take_min(sk[c + HX * HY], sl[c + HX * HY], bk, bl);
            }
            if (bk == kInfKey) return;
            const uint64_t nk = f_key(hb[j], bk);
            if (nk != k[j] || bl != l[j]) {
                k[j] = nk;
                l[j] = bl;
                ch = true;
            }
        };
#pragma unroll
        for (int j = 0; j < RUN; ++j)
            if (upd & (1u << j)) relax(j);
#pragma unroll
        for (int j = RUN - 1; j >= 0; --j)
            if (upd & (1u << j)) relax(j);
        __syncthreads();
        if (ch) {
#pragma unroll
            for (int j = 0; j < RUN; ++j) {
                sk[hrow + lx0 + j + 1] = k[j];
                sl[hrow + lx0 + j + 1] = l[j];
            }
        }
        if (!__syncthreads_or(ch)) break;
    }

    // ---- write back, activate face neighbours whose halo changed
#pragma unroll
    for (int j = 0; j < RUN; ++j) {
        if (!(upd & (1u << j))) continue;
        if (k[j] == k0[j] && l[j] == l0[j]) continue;
        const int gx = x0 + lx0 + j;
        const int64_t gi = gb + gz * YX + (int64_t)gy * B.X + gx;
        key[gi] = k[j];
        lab[gi] = l[j];
        const int lx = lx0 + j;
        if (ND == 3) {
            if (lz == 0) sface[0] = 1;
            if (lz == TZ - 1) sface[1] = 1;
        }
        if (ly == 0) sface[2] = 1;
        if (ly == TY - 1) sface[3] = 1;
        if (lx == 0) sface[4] = 1;
        if (lx == TX - 1) sface[5] = 1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int n = 0;
        auto act = [&](int zz, int yy, int xx) {
            if (zz < 0 || zz >= B.tz || yy < 0 || yy >= B.ty || xx < 0 || xx >= B.tx) return;
            atomicOr(&act_next[B.tbase + (zz * B.ty + yy) * B.tx + xx], 8u);
            ++n;
        };
        if (sface[0]) act(tzi - 1, tyi, txi);
        if (sface[1]) act(tzi + 1, tyi, txi);
        if (sface[2]) act(tzi, tyi - 1, txi);
        if (sface[3]) act(tzi, tyi + 1, txi);
        if (sface[4]) act(tzi, tyi, txi - 1);
        if (sface[5]) act(tzi, tyi, txi + 1);
        if (n && !*(volatile uint32_t*)counter) atomicOr(counter, 1u);
    }
}

template __global__ void k_flood<3>(const BlockDesc*, const BlockStat*, const float*, uint64_t*, uint32_t*,
                                    const uint32_t*, uint32_t*, uint32_t*);
template __global__ void k_flood<2>(const BlockDesc*, const BlockStat*, const float*, uint64_t*, uint32_t*,
                                    const uint32_t*, uint32_t*, uint32_t*);

}  // namespace ctws

namespace ctws {

// =========================================================================================
// Packed flood: one uint64 per voxel, key = C (32) | d (12, saturating) | label (20), so the
// min over neighbours of the packed word IS the (C, d, label) order.  Used when every block of
// the batch has fewer than 2^20 seeds (the wide kernel above handles the rest).
//
// Tile: 16^3 (3-D) or 4 slices x 32 x 32 (2-D, no coupling between slices), 1-voxel halo in
// LDS.  Each local iteration sweeps every axis: a thread owns one line along the axis and
// relaxes it forward then backward in place (a change travels the whole line in one sweep),
// then all threads switch to lines along the next axis.  LDS words are 64-bit and written
// whole, so concurrent readers never see a torn key.
// =========================================================================================
// packed key helpers (kPackInf, f_packed): ctws_dev.h

template <int ND>
struct PTile;
template <>
struct PTile<3> {
    static constexpr int TZ = 16, TY = 16, TX = 16, THREADS = 256;
    static constexpr int HZ = TZ + 2, HY = TY + 2, HX = TX + 3;  // x padded (odd row length)
};
template <>
struct PTile<2> {
    static constexpr int TZ = 4, TY = 32, TX = 32, THREADS = 128;
    static constexpr int HZ = TZ, HY = TY + 2, HX = TX + 3;
};

// act[] per tile: bit3 = solve the whole tile (first round), bit0 = halo voxels changed; the
// lines through the changed halo voxels are in lines[tile * kLineWords]: 8 words per axis
// (x-lines, y-lines, z-lines), one bit per line, indexed as the dirty bitmaps below.
constexpr uint32_t kActFull = 8u;

template <int ND>
__global__ void __launch_bounds__(PTile<ND>::THREADS, 2) k_flood_packed(const BlockDesc* __restrict__ D,
                                                                        const BlockStat* S,
                                                                        const float* __restrict__ h,
                                                                        uint64_t* __restrict__ key,
                                                                        const uint8_t* __restrict__ fixedv,
                                                                        const uint32_t* __restrict__ act_cur,
                                                                        uint32_t* __restrict__ act_next,
                                                                        uint32_t* __restrict__ lines_cur,
                                                                        uint32_t* __restrict__ lines_next,
                                                                        uint32_t* __restrict__ counter) {
    using T = PTile<ND>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX, NT = T::THREADS;
    constexpr int HZ = T::HZ, HY = T::HY, HX = T::HX;
    constexpr int HN = HZ * HY * HX;
    constexpr int TN = TZ * TY * TX;
    constexpr int ZOFF = (ND == 3) ? 1 : 0;
    constexpr int NW = NT / 32;  // dirty-bitmap words per axis (one bit per line, NT lines)
    static_assert(TZ * TY == NT && TZ * TX == NT && (ND == 2 || TY * TX == NT), "one line per thread");
    __shared__ uint64_t sk[HN];
    __shared__ uint32_t sh[TN];
    __shared__ uint8_t sf[TN];  // bit0: fixed (seed), bit1: changed, bit2: outside the block
    __shared__ uint32_t dirty[3][NW];
    __shared__ uint32_t sfl[6][NW];  // lines of the face neighbours whose halo voxel changed

    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int t = blockIdx.x;
    if (t >= B.tz * B.ty * B.tx) return;
    const uint32_t am = act_cur[B.tbase + t];
    if (!am) return;
    const int txi = t % B.tx, tyi = (t / B.tx) % B.ty, tzi = t / (B.tx * B.ty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int64_t gb = B.base;
    const int tid = threadIdx.x;

    if (tid < 6 * NW) sfl[tid / NW][tid % NW] = 0;
    if (tid < kLineWords) {
        uint32_t* lin = lines_cur + (int64_t)(B.tbase + t) * kLineWords;
        const uint32_t v = lin[tid];
        lin[tid] = 0;  // consumed: the array is next round's lines_next
        if ((tid & 7) < NW) dirty[tid >> 3][tid & 7] = (am & kActFull) ? 0xFFFFFFFFu : v;
    }
    // All global loads of a phase are issued before the first LDS store so that their
    // latencies overlap (a load/store loop serialises them at this occupancy).
    // Phase 1: keys of the tile and its halo.
    constexpr int NLK = (HN + NT - 1) / NT;
    uint64_t kk[NLK];
#pragma unroll
    for (int i = 0; i < NLK; ++i) {
        const int c = tid + i * NT;
        const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
        const int gz = z0 + hz - ZOFF, gy = y0 + hy - 1, gx = x0 + hx - 1;
        kk[i] = kPackInf;
        if (c < HN && hx <= TX + 1 && gz >= 0 && gz < B.Z && gy >= 0 && gy < B.Y && gx >= 0 && gx < B.X)
            kk[i] = key[gb + gz * YX + (int64_t)gy * B.X + gx];
    }
    int any_key = 0;
#pragma unroll
    for (int i = 0; i < NLK; ++i) {
        const int c = tid + i * NT;
        if (c < HN) sk[c] = kk[i];
        any_key |= kk[i] != kPackInf;
    }
    // nothing reached in the tile or its halo yet: nothing can change
    if (!__syncthreads_or(any_key)) return;
    // Phase 2: heights and seed flags.
    constexpr int NLT = TN / NT;
    static_assert(TN % NT == 0, "");
    float hv[NLT];
    uint8_t fv[NLT];
#pragma unroll
    for (int i = 0; i < NLT; ++i) {
        const int c = tid + i * NT;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int gz = z0 + lz, gy = y0 + ly, gx = x0 + lx;
        fv[i] = 4;
        hv[i] = 0.f;
        if (gz < B.Z && gy < B.Y && gx < B.X) {
            const int64_t gi = gb + gz * YX + (int64_t)gy * B.X + gx;
            hv[i] = h[gi];
            fv[i] = fixedv[gi] ? 1 : 0;
        }
    }
#pragma unroll
    for (int i = 0; i < NLT; ++i) {
        sh[tid + i * NT] = fv[i] == 4 ? 0u : ordf(hv[i]);
        sf[tid + i * NT] = fv[i];
    }
    __syncthreads();

    // Line indices: x-lines (z, y) -> z*TY + y; y-lines (z, x) -> z*TX + x; z-lines (y, x) ->
    // y*TX + x.  A thread owns line `tid` of the axis being swept.
    auto mark = [&](int ax, int line) { atomicOr(&dirty[ax][line >> 5], 1u << (line & 31)); };
    uint32_t nlines = 0;

    // One sweep of the thread's line along `axis` (if dirty): the line lives in registers;
    // the off-axis neighbour minimum is read once per voxel, then the line is relaxed forward
    // and backward.  Changed voxels dirty the lines of the other axes through them.
    auto sweep = [&](auto axis_c, bool& ch) {
        constexpr int axis = decltype(axis_c)::value;
        constexpr int len = axis == 0 ? TX : (axis == 1 ? TY : TZ);
        constexpr int cstride = axis == 0 ? 1 : (axis == 1 ? HX : HX * HY);
        constexpr int tstride = axis == 0 ? 1 : (axis == 1 ? TX : TX * TY);
        constexpr int o1 = axis == 0 ? HX : 1;          // off-axis neighbour strides
        constexpr int o2 = axis == 2 ? HX : HX * HY;
        const uint32_t bit = 1u << (tid & 31);
        const uint32_t old = atomicAnd(&dirty[axis][tid >> 5], ~bit);
        if (!(old & bit)) return;
        ++nlines;
        int lz = 0, ly = 0, lx = 0;
        if (axis == 0) { lz = tid / TY; ly = tid % TY; }
        else if (axis == 1) { lz = tid / TX; lx = tid % TX; }
        else { ly = tid / TX; lx = tid % TX; }
        const int c0 = ((lz + ZOFF) * HY + (ly + 1)) * HX + (lx + 1);
        const int t0 = (lz * TY + ly) * TX + lx;
        uint64_t v[len], off[len];
        uint32_t hb[len];
        uint32_t upd = 0;
#pragma unroll
        for (int p = 0; p < len; ++p) {
            const int c = c0 + p * cstride;
            v[p] = sk[c];
            uint64_t m = min(sk[c - o1], sk[c + o1]);
            if (ND == 3) m = min(m, min(sk[c - o2], sk[c + o2]));
            off[p] = m;
            hb[p] = sh[t0 + p * tstride];
            if (!(sf[t0 + p * tstride] & 5)) upd |= 1u << p;
        }
        const uint64_t before_lo = sk[c0 - cstride];
        const uint64_t after_hi = sk[c0 + len * cstride];
        uint32_t chg = 0;
        // Branch-free relaxation K(p) = f(min over the 6 neighbours): new C = max(h, C); d
        // reset or incremented (saturating); label of the argmin neighbour.  f(INF) = INF;
        // seeds and voxels outside the block keep their key.  (The label makes f
        // non-monotone, so this is a replacement, not a min with the old key.)
        auto step = [&](int p) {
            uint64_t b = min(off[p], p > 0 ? v[p - 1] : before_lo);
            b = min(b, p + 1 < len ? v[p + 1] : after_hi);
            const uint32_t bh = (uint32_t)(b >> 32), bl = (uint32_t)b;
            const bool above = hb[p] > bh;
            const uint32_t nh = max(hb[p], bh);
            // d + 1 saturating at kDMax, as f_packed
            const bool sat = (bl >> kLabelBits) >= kDMax;
            const uint32_t nl = above ? (bl & (uint32_t)kLabelMask) : (sat ? bl : bl + (1u << kLabelBits));
            uint64_t nk = ((uint64_t)nh << 32) | nl;
            nk = (upd & (1u << p)) ? nk : v[p];
            chg |= (nk != v[p]) ? (1u << p) : 0u;
            v[p] = nk;
        };
#pragma unroll
        for (int p = 0; p < len; ++p) step(p);
#pragma unroll
        for (int p = len - 1; p >= 0; --p) step(p);
        if (!chg) return;
        ch = true;
#pragma unroll
        for (int p = 0; p < len; ++p)
            if (chg & (1u << p)) {
                sk[c0 + p * cstride] = v[p];
                sf[t0 + p * tstride] |= 2;
            }
        // dirty the other axes' lines through the changed voxels
        if (axis == 0) {
            // y-lines (z, x = p): bits z*TX + p, contiguous
            const int yb = lz * TX;
            atomicOr(&dirty[1][yb >> 5], chg << (yb & 31));
            if (ND == 3) {  // z-lines (y, x = p)
                const int zb = ly * TX;
                atomicOr(&dirty[2][zb >> 5], chg << (zb & 31));
            }
        } else if (axis == 1) {
            // x-lines (z, y = p): bits z*TY + p, contiguous
            const int xb = lz * TY;
            atomicOr(&dirty[0][xb >> 5], chg << (xb & 31));
            if (ND == 3) {  // z-lines (y = p, x)
                uint32_t m = chg;
                while (m) {
                    const int p = __builtin_ctz(m);
                    m &= m - 1;
                    mark(2, p * TX + lx);
                }
            }
        } else {
            // x-lines (z = p, y) and y-lines (z = p, x)
            uint32_t m = chg;
            while (m) {
                const int p = __builtin_ctz(m);
                m &= m - 1;
                mark(0, p * TY + ly);
                mark(1, p * TX + lx);
            }
        }
    };

    // Sweep the axes in turn while any line is dirty.
    int iters = 0;
    for (int k = 0; k < 3 * 4096; ++k) {
        bool ch = false;
        const int axis = k % ND;
        if (axis == 0) sweep(std::integral_constant<int, 0>(), ch);
        else if (axis == 1) sweep(std::integral_constant<int, 1>(), ch);
        else if constexpr (ND == 3) sweep(std::integral_constant<int, 2>(), ch);
        ++iters;
        __syncthreads();
        uint32_t any = 0;
#pragma unroll
        for (int ax = 0; ax < ND; ++ax)
#pragma unroll
            for (int w = 0; w < NW; ++w) any |= dirty[ax][w];
        if (!any) break;
        __syncthreads();
    }

    // write back changed voxels; collect the lines of the face neighbours whose halo changed
    for (int c = tid; c < TN; c += NT) {
        if (!(sf[c] & 2)) continue;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int gz = z0 + lz, gy = y0 + ly, gx = x0 + lx;
        const uint64_t kw = sk[((lz + ZOFF) * HY + (ly + 1)) * HX + (lx + 1)];
        key[gb + gz * YX + (int64_t)gy * B.X + gx] = kw;
        if (key_dsat(kw)) note_dsat(S, blockIdx.y);
        auto fl = [&](int f, int line) { atomicOr(&sfl[f][line >> 5], 1u << (line & 31)); };
        if (ND == 3) {
            if (lz == 0) fl(0, ly * TX + lx);
            if (lz == TZ - 1) fl(1, ly * TX + lx);
        }
        if (ly == 0) fl(2, lz * TX + lx);
        if (ly == TY - 1) fl(3, lz * TX + lx);
        if (lx == 0) fl(4, lz * TY + ly);
        if (lx == TX - 1) fl(5, lz * TY + ly);
    }
    __syncthreads();
    if (tid < 6 * NW) {
        const int f = tid / NW, wd = tid % NW;
        const uint32_t bits = sfl[f][wd];
        const int zz = tzi + (f == 0 ? -1 : f == 1 ? 1 : 0);
        const int yy = tyi + (f == 2 ? -1 : f == 3 ? 1 : 0);
        const int xx = txi + (f == 4 ? -1 : f == 5 ? 1 : 0);
        if (bits && zz >= 0 && zz < B.tz && yy >= 0 && yy < B.ty && xx >= 0 && xx < B.tx) {
            const int64_t nt = B.tbase + (zz * B.ty + yy) * B.tx + xx;
            const int axis = f < 2 ? 2 : (f < 4 ? 1 : 0);
            atomicOr(&lines_next[nt * kLineWords + axis * 8 + wd], bits);
            if (!act_next[nt]) atomicOr(&act_next[nt], 1u);
            if (!*(volatile uint32_t*)counter) atomicOr(counter, 1u);  // another round is needed
        }
    }
    // statistics, spread over kStatSlots slots (same-address atomics serialise)
    nlines = wg_reduce_u32(nlines, OpAdd());
    if (tid == 0) {
        uint32_t* st = counter + 4 + (blockIdx.x % kStatSlots) * 4;
        atomicAdd(st + 1, 1u);              // tiles solved
        atomicAdd(st + 2, (uint32_t)iters);  // sweeps
        atomicAdd(st + 3, nlines);           // lines swept
    }
}

template __global__ void k_flood_packed<3>(const BlockDesc*, const BlockStat*, const float*, uint64_t*,
                                           const uint8_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                           uint32_t*);
template __global__ void k_flood_packed<2>(const BlockDesc*, const BlockStat*, const float*, uint64_t*,
                                           const uint8_t*, const uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                           uint32_t*);


// packed keys -> labels (keeps the seed bit of `lab`)
__global__ void __launch_bounds__(256) k_unpack_labels(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                       const uint64_t* __restrict__ key, uint32_t* __restrict__ lab) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.N; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = key[B.base + i];
        lab[B.base + i] = (k == kPackInf) ? 0u : (uint32_t)(k & kLabelMask);
    }
}

}  // namespace ctws

namespace ctws {

// =========================================================================================
// Descent pre-pass of the packed flood.
//
// Let sd(q) be the neighbour with the smallest height strictly below h(q) (6-nbhd; 4-nbhd in
// plane for 2-D ws), defined only when that smallest height is attained by ONE neighbour.  If
// the chain q -> sd(q) -> ... ends in a seed s, the reversed chain is a path from s on which
// the height rises to h(q), so C(q) = h(q); every other neighbour p has C(p) >= h(p) >
// h(sd(q)) = C(sd(q)), so sd(q) is q's unique argmin neighbour, d(q) = 0 (h(q) > C(sd(q))),
// and by induction along the chain the fixpoint key of q is (h(q), 0, label(s)).  Such voxels
// are final before any relaxation: they are written as fixed keys and only the remaining
// voxels (catchments of local minima of h that hold no seed, and of tie voxels) are flooded.
// k_flood_verify re-checks K(q) = f(min_p K(p)) everywhere; on a violation the batch is
// flooded again from the seeds alone.
// =========================================================================================

// Descent inside a tile: tile (3-D 16^3, 2-D 1 x 64 x 64) + 1-voxel halo of heights in LDS;
// every tile voxel gets its steepest-descent parent (itself for seeds, local minima and ties),
// then pointer jumping in LDS runs each chain to its end inside the tile: a root of the tile
// or the first voxel outside it.  exit[q] = kDescRes | label for a chain ending at a tile root
// (the seed's label, 0 for a root without a seed), else the block C-order index of the first
// voxel outside the tile; k_descent_init follows those across tiles (a hop per tile crossed).
// One pass over the volume instead of a global pointer-jumping pass per doubling.
// seed test / seed label: from the seed CC parents (pass 1: `cc` = PF after k_root_label) or,
// when cc is null, from lab (kFixedBit; pass 2 and the fallbacks)
__device__ __forceinline__ uint32_t seed_label(const uint32_t* lab, const uint32_t* cc, int64_t base, uint32_t r) {
    if (cc) return cc_label(cc + base, cc[base + r]);  // (a member: the caller tested the member bitmap)
    const uint32_t l = lab[base + r];
    return (l & kFixedBit) ? (l & ~kFixedBit) : 0u;
}

// threads per descent tile (4096 voxels): 512 keeps the per-thread arrays at 8 voxels
constexpr int kDescThreads = 512;

template <int ND>
struct DTile;
template <>
struct DTile<3> {
    // (8 x 8 x 64 tiles, whose 66-height halo rows are 3 contiguous lines instead of 1-2 lines
    // per 18-height row, measured slower in round 6: config 4 descent tile 12.1 -> 12.9 ms and
    // the cross-tile hops of k_descent_init 8.9 -> 9.6 ms, more chains leave a flat tile)
    static constexpr int TZ = 16, TY = 16, TX = 16, HZ = 18;
};
template <>
struct DTile<2> {
    static constexpr int TZ = 1, TY = 64, TX = 64, HZ = 1;
};

template <int ND>
__global__ void __launch_bounds__(kDescThreads) __attribute__((amdgpu_waves_per_eu(ND == 2 ? 8 : 6, 8))) k_descent_tile(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      const float* __restrict__ h, const uint32_t* __restrict__ lab,
                                                      const uint32_t* __restrict__ cc, const uint64_t* __restrict__ sbits,
                                                      uint32_t* __restrict__ exitp) {
    using T = DTile<ND>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX, HZ = T::HZ, HY = TY + 2, HX = TX + 2;
    constexpr int HN = HZ * HY * HX, TN = TZ * TY * TX;
    constexpr int ZOFF = ND == 3 ? 1 : 0;
    __shared__ uint32_t sh[HN];  // ordered heights (0xFFFFFFFF outside the block)
    // pointer: < TN interior voxel, >= TN halo voxel (TN + halo index); 16 bits (TN + HN < 2^15)
    // so that 5 tiles fit a CU's LDS
    __shared__ int16_t sp[TN];
    static_assert(TN + HN < 32768, "");
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int ntx = (B.X + TX - 1) / TX, nty = (B.Y + TY - 1) / TY, ntz = (B.Z + TZ - 1) / TZ;
    // (dispatch order, not xcd_swizzle: XCD-contiguous tiles measured slower, config 4 12.1 ->
    // 13.4 ms; gridDim.x may be rounded up to a multiple of 8)
    const int t = blockIdx.x;
    if (t >= ntx * nty * ntz) return;
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    const int64_t YX = (int64_t)B.Y * B.X;
    const float* hb = h + B.base;
    constexpr int NT = kDescThreads, PER = TN / NT;  // voxels per thread: c = threadIdx.x + k * NT
    static_assert(TN % NT == 0 && PER <= 32, "");
    // seed entries of the thread's voxels, then the halo heights: loads unconditional (clamped
    // index, global address space) so that all of them are in flight together; out-of-block
    // values are selected away afterwards.
    // lab (pass 2, fallbacks): every voxel's entry (kFixedBit = seed).  cc (the seed forest,
    // pass 1): members only, their bits in sbits; the tile's bitmap rows (a 32-bit half word per
    // TX <= 32 voxels of a row) go to LDS with the halo heights, and only the members' entries
    // (~1 % of the voxels) are loaded after that, a second round trip instead of 4 B per voxel
    constexpr int WPR32 = (TX + 31) / 32, NW32 = TZ * TY * WPR32;
    __shared__ uint32_t sbm[NW32];
    uint32_t inm = 0, seedm = 0;
    uint32_t sv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int c = threadIdx.x + k * NT;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int gz = min(z0 + lz, B.Z - 1), gy = min(y0 + ly, B.Y - 1), gx = min(x0 + lx, B.X - 1);
        inm |= ((z0 + lz < B.Z && y0 + ly < B.Y && x0 + lx < B.X) ? 1u : 0u) << k;
        sv[k] = cc ? kNoParent : gbl(lab)[B.base + gz * YX + (int64_t)gy * B.X + gx];
    }
    static_assert(NW32 <= NT, "");
    uint32_t bwv = ~0u;
    if (cc && (int)threadIdx.x < NW32) {
        const int r = threadIdx.x / WPR32, hw = threadIdx.x % WPR32;
        const int gz = min(z0 + r / TY, B.Z - 1), gy = min(y0 + r % TY, B.Y - 1);
        const int64_t row = B.fbase + ((int64_t)gz * B.Y + gy) * ((B.X + 63) >> 6);
        bwv = gbl((const uint32_t*)sbits)[2 * row + (x0 >> 5) + hw];
    }
    {
        constexpr int NH = (HN + NT - 1) / NT;
        uint32_t hv[NH];
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int c = min((int)threadIdx.x + k * NT, HN - 1);
            const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
            const int gz = z0 + hz - ZOFF, gy = y0 + hy - 1, gx = x0 + hx - 1;
            const int cz = min(max(gz, 0), B.Z - 1), cy = min(max(gy, 0), B.Y - 1), cx = min(max(gx, 0), B.X - 1);
            hv[k] = __float_as_uint(gbl(hb)[cz * YX + (int64_t)cy * B.X + cx]);
        }
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int c = (int)threadIdx.x + k * NT;
            if (c < HN) {
                const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
                const int gz = z0 + hz - ZOFF, gy = y0 + hy - 1, gx = x0 + hx - 1;
                const bool out = gz < 0 || gz >= B.Z || gy < 0 || gy >= B.Y || gx < 0 || gx >= B.X;
                sh[c] = out ? 0xFFFFFFFFu : ordf(__uint_as_float(hv[k]));
            }
        }
    }
    if (cc && (int)threadIdx.x < NW32) sbm[threadIdx.x] = bwv;
    __syncthreads();
    if (cc) {
        // the members' seed-forest entries
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * NT;
            const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY), r = c / TX;
            const int gx = x0 + lx;
            if (((inm >> k) & 1u) && ((sbm[r * WPR32 + (lx >> 5)] >> (gx & 31)) & 1u))
                sv[k] = gbl(cc)[B.base + (z0 + lz) * YX + (int64_t)(y0 + ly) * B.X + gx];
        }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const bool sd = cc ? sv[k] != kNoParent : (sv[k] & kFixedBit) != 0u;
        seedm |= (((inm >> k) & 1u) && sd ? 1u : 0u) << k;
    }
    // parents
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int c = threadIdx.x + k * NT;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        int p = c;
        if (((inm & ~seedm) >> k) & 1u) {
            const int hc = ((lz + ZOFF) * HY + ly + 1) * HX + lx + 1;
            uint32_t best = sh[hc];
            int bh = -1;
            bool tie = false;
            auto cand = [&](int o) {
                const uint32_t v = sh[hc + o];
                tie = (v == best) || (tie && v > best);
                if (v < best) {
                    best = v;
                    bh = hc + o;
                }
            };
            if (ND == 3) {
                cand(-HX * HY);
                cand(HX * HY);
            }
            cand(-HX);
            cand(HX);
            cand(-1);
            cand(1);
            // an exact tie at the lowest neighbour height: left to the flood (see above)
            if (bh >= 0 && !tie) {
                const int hx = bh % HX, hy = (bh / HX) % HY, hz = bh / (HX * HY);
                const bool inside = hx >= 1 && hx <= TX && hy >= 1 && hy <= TY && (ND == 2 || (hz >= 1 && hz <= TZ));
                p = inside ? ((hz - ZOFF) * TY + (hy - 1)) * TX + (hx - 1) : TN + bh;
            }
        }
        sp[c] = (int16_t)p;
    }
    __syncthreads();
    // pointer jumping inside the tile
    for (int it = 0; it < 16; ++it) {
        bool moved = false;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * NT;
            const int p = sp[c];
            if (p < TN) {
                const int pp = sp[p];
                if (pp != p) {
                    sp[c] = (int16_t)pp;
                    moved = true;
                }
            }
        }
        if (!__syncthreads_or(moved)) break;
    }
    // tile roots: seed label (seeds) or 0 (local minima without a seed, ties), kept in sh[]
    // (the heights are no longer read).  The label comes from the seed entry loaded above: a
    // cc root carries it, a non-root cc entry needs its root's (one more load, seeds only: a
    // wave without such a seed voxel skips the load instruction)
    {
        uint32_t rl[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const uint32_t v = sv[k];
            const bool need = cc && v != kNoParent && !(v & kRootBit) && ((seedm >> k) & 1u);
            rl[k] = need ? gbl(cc)[B.base + v] : 0u;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int c = threadIdx.x + k * NT;
            const uint32_t v = sv[k];
            uint32_t l = 0u;
            if ((seedm >> k) & 1u) {
                if (!cc) l = v & ~kFixedBit;
                else l = (v & kRootBit) ? (v & ~kRootBit) : (rl[k] & ~kRootBit);
            }
            if (sp[c] == c) sh[c] = l;
        }
    }
    __syncthreads();
    // exit entry: kDescRes | label when the chain ends at a seed root of this tile; the block
    // index of the root when it ends at a root without a seed (the root itself: kDescRes | 0);
    // else the block index of the first voxel outside the tile (k_descent_init follows it)
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int c = threadIdx.x + k * NT;
        if (!((inm >> k) & 1u)) continue;
        const int lx = c % TX, ly = (c / TX) % TY, lz = c / (TX * TY);
        const int gz = z0 + lz, gy = y0 + ly, gx = x0 + lx;
        const int p = sp[c];
        uint32_t e;
        if (p < TN) {
            const uint32_t l = sh[p];
            if (l != 0u || p == c) {
                e = kDescRes | l;
            } else {
                const int rx = p % TX, ry = (p / TX) % TY, rz = p / (TX * TY);
                e = (uint32_t)((z0 + rz) * YX + (int64_t)(y0 + ry) * B.X + (x0 + rx));
            }
        } else {
            const int q = p - TN;
            const int ex = x0 + q % HX - 1;
            const int ey = y0 + (q / HX) % HY - 1;
            const int ez = z0 + q / (HX * HY) - ZOFF;
            e = (uint32_t)(ez * YX + (int64_t)ey * B.X + ex);
        }
        exitp[B.base + gz * YX + (int64_t)gy * B.X + gx] = e;
    }
}
template __global__ void k_descent_tile<3>(const BlockDesc*, const BlockStat*, const float*, const uint32_t*,
                                           const uint32_t*, const uint64_t*, uint32_t*);
template __global__ void k_descent_tile<2>(const BlockDesc*, const BlockStat*, const float*, const uint32_t*,
                                           const uint32_t*, const uint64_t*, uint32_t*);

// voxels whose descent ends in a seed get their final key, fixed; the others wait for the
// flood (INF key).  Bitmaps, one word per 64 voxels of a row (the 64 lanes of a wave cover
// exactly one word): open = not final yet, chg = final (the first "changed" set, whose
// neighbours form the first frontier).
template <int U>
__global__ void __launch_bounds__(256) k_descent_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      const float* __restrict__ h, const uint32_t* __restrict__ par,
                                                      uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv,
                                                      uint64_t* __restrict__ open, uint64_t* __restrict__ chg,
                                                      uint32_t* __restrict__ nopen, uint32_t* __restrict__ plev) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    uint32_t cnt_open = 0;  // statistics (CTWS_TRACE): voxels left to the relaxation
    // masked blocks (k_plateau.hip): the largest height of an open masked-out voxel (the plateau
    // level, plev[block]; the plateau fill's k_plat_level folded into this pass)
    const bool want_lev = plev && B.mask;
    uint32_t lev = 0;
    // word tiles (a wave's ballot is exactly one word of the open / changed bitmaps), U words
    // per step: the U chains of a lane hop together, so U dependent-load latencies overlap
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nwords + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t wbeg = wid * per, wend = min(nwords, wbeg + per);
    // (row, word in the row) of the wave's next word, advanced word by word (no 64-bit division)
    int row_n = (int)(wbeg / wpr), xw_n = (int)(wbeg - (int64_t)row_n * wpr);
    for (int64_t w0 = wbeg; w0 < wend; w0 += U) {
        int64_t gi[U];
        bool valid[U];
        uint32_t e[U];
        float hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t wu = w0 + u;
            const int64_t row = row_n;
            const int x = xw_n * 64 + lane;
            if (++xw_n == wpr) {
                xw_n = 0;
                ++row_n;
            }
            valid[u] = wu < wend && x < B.X;
            gi[u] = B.base + (valid[u] ? row * B.X + x : 0);
            e[u] = gbl(par)[gi[u]];
            hv[u] = gbl(h)[gi[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (!valid[u]) e[u] = kDescRes;
        for (int hop = 0; hop < 1 << 16; ++hop) {  // one hop per tile crossed
            bool more = false;
#pragma unroll
            for (int u = 0; u < U; ++u) more |= !(e[u] & kDescRes);
            if (!more) break;
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (!(e[u] & kDescRes)) e[u] = gbl(par)[B.base + e[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t lr = e[u] & ~kDescRes;
            const bool res = lr != 0;
            if (valid[u]) {
                key[gi[u]] = res ? (((uint64_t)ordf(hv[u]) << 32) | (uint64_t)lr) : kPackInf;
                fixedv[gi[u]] = res ? 1 : 0;
                if (want_lev && !res && !gbl(B.mask)[gi[u] - B.base]) lev = max(lev, ordf(hv[u]));
            }
            const uint64_t op = __ballot(valid[u] && !res);
            const uint64_t fi = __ballot(valid[u] && res);
            if (lane == 0 && w0 + u < wend) {
                open[B.fbase + w0 + u] = op;
                chg[B.fbase + w0 + u] = fi;
            }
            cnt_open += lane == 0 ? (uint32_t)__popcll(op) : 0u;
        }
    }
    if (nopen) {
        cnt_open = wg_reduce_u32(cnt_open, OpAdd());
        if (threadIdx.x == 0 && cnt_open) atomicAdd(&nopen[blockIdx.y], cnt_open);
    }
    if (want_lev) {
        lev = wg_reduce_u32(lev, OpMax());
        if (threadIdx.x == 0 && lev) atomic_max_if(&plev[blockIdx.y], lev);
    }
}
template __global__ void k_descent_init<8>(const BlockDesc*, const BlockStat*, const float*, const uint32_t*,
                                           uint64_t*, uint8_t*, uint64_t*, uint64_t*, uint32_t*, uint32_t*);

// One iteration of the frontier relaxation.  frontier = (neighbours of the voxels changed in
// the previous iteration) & open; every frontier voxel recomputes K = f(min of its
// neighbours' keys) in place (a stale read is repaired by the next iteration, as the
// neighbour's change is recorded).
//
// Work unit: a *chunk*, a brick of 64 bitmap words (one per lane) — CW words along x, CY rows
// along y, CZ slices along z (FChunk; 2-D ws: CZ = 1) — so that a front crosses up to 64
// voxels in x and CY / CZ in y / z inside one launch.  The list holds the chunks that contain
// open voxels in iteration 0, afterwards the chunks next to a chunk change, so a late
// iteration with a handful of active chunks costs a handful of waves.  A wave builds its
// chunk's frontier from the previous changed bitmap, expands the set bits into an LDS list and
// relaxes 64 voxels per step, one per lane; then it sweeps locally (the in-chunk neighbours of
// this sweep's changes) until nothing changes or `reps` sweeps are done.  Its changed bits
// collect in LDS and are stored whole.
//
// Chunk generations instead of cleared flags: gen[it & 1][ch] = (it + 1) | kGenConv? when
// chunk ch changed in iteration it, so a word of the previous changed bitmap is valid iff its
// chunk's generation is it.  kGenConv marks a chunk whose local sweeps converged: every
// in-chunk neighbour of each of its changes was re-evaluated after that change by the same
// wave, so the chunk neither queues itself nor rebuilds its own frontier from its own words
// (its words still feed the neighbouring chunks).  qgen[ch] = it + 1 when ch is queued for
// iteration it + 1.  Neighbour chunks are queued only when a change lies on the shared face.
constexpr int kFrontierWaves = 4;
constexpr uint32_t kWlChunkBits = 20;  // list entry = block << 20 | chunk
constexpr uint32_t kGenConv = 0x80000000u;

// chunk grid of a block (words along x, rows, slices) for brick CW x CY x CZ
template <int CW, int CY, int CZ>
struct FChunk {
    static_assert(CW * CY * CZ <= 64 && 64 % (CW * CY * CZ) == 0, "a chunk is at most 64 words, one per lane");
    int wpr, ncx, ncy, ncz;
    __device__ FChunk(const BlockDesc& B) {
        wpr = (B.X + 63) >> 6;
        ncx = (wpr + CW - 1) / CW;
        ncy = (B.Y + CY - 1) / CY;
        ncz = (B.Z + CZ - 1) / CZ;
    }
    __device__ int64_t count() const { return (int64_t)ncx * ncy * ncz; }
};

// position of the k-th (0-based) set bit of w (k < popcount(w))
__device__ __forceinline__ int kth_set_bit(uint64_t w, int k) {
    int pos = 0;
#pragma unroll
    for (int half = 32; half > 0; half >>= 1) {
        const uint64_t lo = w & ((1ull << half) - 1ull);
        const int c = __popcll(lo);
        if (k >= c) {
            k -= c;
            w >>= half;
            pos += half;
        } else {
            w = lo;
        }
    }
    return pos;
}

// iteration-0 list: every chunk holding an open voxel.  A wave takes 64 consecutive chunks,
// reads each one's 64 words (one word per lane) and appends the non-empty ones with one atomic.
template <int CW, int CY, int CZ>
__global__ void __launch_bounds__(256) k_frontier_list0(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                        const uint64_t* __restrict__ open, uint32_t* __restrict__ list,
                                                        uint32_t* __restrict__ cnt) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int lane = threadIdx.x & 63;
    const int lx = lane % CW, ly = (lane / CW) % CY, lz = lane / (CW * CY);
    const FChunk<CW, CY, CZ> G(B);
    const int64_t nch = G.count();
    const uint64_t* op = open + B.fbase;
    for (int64_t c0 = ((int64_t)blockIdx.x * kFrontierWaves + (threadIdx.x >> 6)) * 64; c0 < nch;
         c0 += (int64_t)gridDim.x * kFrontierWaves * 64) {
        uint64_t m = 0ull;  // bit k: chunk c0 + k holds an open voxel
        int cx = (int)(c0 % G.ncx), cy = (int)((c0 / G.ncx) % G.ncy), cz = (int)(c0 / ((int64_t)G.ncx * G.ncy));
        for (int k = 0; k < 64 && c0 + k < nch; ++k) {
            const int xw = cx * CW + lx, y = cy * CY + ly, z = cz * CZ + lz;
            const bool ok = lane < CW * CY * CZ && xw < G.wpr && y < B.Y && z < B.Z;
            const bool any = __ballot(ok && op[((int64_t)z * B.Y + y) * G.wpr + xw] != 0ull) != 0ull;
            m |= (any ? 1ull : 0ull) << k;
            if (++cx == G.ncx) {
                cx = 0;
                if (++cy == G.ncy) {
                    cy = 0;
                    ++cz;
                }
            }
        }
        if (!m) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(cnt, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, 0);
        if ((m >> lane) & 1ull)
            list[base + __popcll(m & ((1ull << lane) - 1ull))] = (blockIdx.y << kWlChunkBits) | (uint32_t)(c0 + lane);
    }
}

template <int ND, int CW, int CY, int CZ>
__global__ void __launch_bounds__(256) k_frontier(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                  const float* __restrict__ h, uint64_t* __restrict__ key,
                                                  const uint64_t* __restrict__ open, const uint64_t* __restrict__ cprev,
                                                  uint64_t* __restrict__ cnext, const uint32_t* __restrict__ gprev,
                                                  uint32_t* __restrict__ gnext, int it, const uint32_t* __restrict__ list,
                                                  const uint32_t* __restrict__ cnt, uint32_t* __restrict__ list_next,
                                                  uint32_t* __restrict__ cnt_next, uint32_t* __restrict__ qgen,
                                                  uint32_t* __restrict__ nvisit, int reps, int dirf) {
    static_assert(ND == 3 || CZ == 1, "2-D ws: slices are independent, chunks are one slice deep");
    __shared__ uint64_t schg[kFrontierWaves][64];
    // dirf: the local sweeps queue only the neighbours a change of p can affect, by the (C, d)
    // part of the keys (the label ignored).  (C, d) never increases during the relaxation (from
    // INF: C = max(h, min C), d from the lexicographic minimum), while a key's label may change
    // either way.  f_q(K) >= K in (C, d), so a neighbour q whose (C, d) is below p's new (C, d)
    // can neither take a lower key through p nor have had p as its argmin (that needs (C, d)_q
    // > (C, d)_p); q's read may be stale, and a stale (C, d) is only larger.  (Comparing whole
    // keys would not do: a label change can raise p's key, and the voxels that took their label
    // from p must see it.)  Equal (C, d) is queued too (only d's saturation at kDMax makes it
    // possible).  sdir[d]: changed voxels whose neighbour in direction d (-z, +z, -y, +y, -x,
    // +x) must be re-evaluated
    constexpr int NDIR = ND == 3 ? 6 : 4;
    __shared__ uint64_t sdir[kFrontierWaves][6][64];
    __shared__ uint64_t sfw[kFrontierWaves][64];
    __shared__ int spre[kFrontierWaves][64];
    // per word of the chunk (lane): its first voxel's block index, (z << 16 | y), its first x
    __shared__ uint32_t sbase[kFrontierWaves][64];
    __shared__ uint32_t szy[kFrontierWaves][64];
    __shared__ int sx0[kFrontierWaves][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int lx = lane % CW, ly = (lane / CW) % CY, lz = lane / (CW * CY);
    const uint32_t n_entries = *cnt;
    const uint32_t prev_gen = (uint32_t)it;  // gprev[ch] & ~kGenConv == it: changed in iteration it - 1
    // XCD-contiguous entries: the workgroups of one XCD take neighbouring chunks, so the lines
    // two adjacent chunks share stay in one L2
    const uint32_t wg = (uint32_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x);
    for (uint32_t e0 = wg * kFrontierWaves + wv; e0 < n_entries; e0 += gridDim.x * kFrontierWaves) {
        const uint32_t ent = list[e0];
        const int bi = (int)(ent >> kWlChunkBits);
        // word and chunk indices fit 32 bits (Z * Y * wpr < 2^27, chunks < 2^20)
        const int ch0 = (int)(ent & ((1u << kWlChunkBits) - 1u));
        const BlockDesc& B = D[bi];
        const FChunk<CW, CY, CZ> G(B);
        const int wpr = G.wpr;
        const int ws = B.Y * wpr;
        const int64_t YX = (int64_t)B.Y * B.X;
        const int cplane = G.ncx * G.ncy;
        const uint64_t* cp = cprev + B.fbase;
        const uint64_t* op = open + B.fbase;
        uint64_t* cn = cnext + B.fbase;
        uint64_t* kb = key + B.base;
        const float* hb = h + B.base;
        const uint32_t* gp = gprev + (B.fbase >> kChunkShift);
        uint32_t* gn = gnext + (B.fbase >> kChunkShift);
        uint32_t* qg = qgen + (B.fbase >> kChunkShift);
        const int cx = (int)(ch0 % G.ncx), cy = (int)((ch0 / G.ncx) % G.ncy), cz = (int)(ch0 / cplane);
        const int xw = cx * CW + lx, yy = cy * CY + ly, zz = cz * CZ + lz;
        const bool wok = xw < wpr && yy < B.Y && zz < B.Z;
        const int wc = wok ? (zz * B.Y + yy) * wpr + xw : 0;
        const int row = zz * B.Y + yy;
        // word k of the lane's neighbourhood and the chunk holding it; previous changed words
        // count only when their chunk changed in iteration it - 1 (own chunk: and did not
        // converge).  All generation and word loads are unconditional (clamped, global address
        // space) and issued together; the neighbours outside the block are selected away.
        constexpr int NW = ND == 3 ? 7 : 5;
        int wi[NW], ci[NW];
        bool ok[NW];
        wi[0] = wc;
        ci[0] = ch0;
        ok[0] = wok;
        wi[1] = wc - 1;
        ci[1] = lx == 0 ? ch0 - 1 : ch0;
        ok[1] = wok && xw > 0;
        wi[2] = wc + 1;
        ci[2] = lx == CW - 1 ? ch0 + 1 : ch0;
        ok[2] = wok && xw + 1 < wpr;
        wi[3] = wc - wpr;
        ci[3] = ly == 0 ? ch0 - G.ncx : ch0;
        ok[3] = wok && yy > 0;
        wi[4] = wc + wpr;
        ci[4] = ly == CY - 1 ? ch0 + G.ncx : ch0;
        ok[4] = wok && yy + 1 < B.Y;
        if (ND == 3) {
            wi[5] = wc - ws;
            ci[5] = lz == 0 ? ch0 - cplane : ch0;
            ok[5] = wok && zz > 0;
            wi[6] = wc + ws;
            ci[6] = lz == CZ - 1 ? ch0 + cplane : ch0;
            ok[6] = wok && zz + 1 < B.Z;
        }
        uint32_t gv[NW];
        uint64_t cv[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            gv[k] = gbl(gp)[ok[k] ? ci[k] : ch0];
            cv[k] = gbl(cp)[ok[k] ? wi[k] : wc];
        }
        const uint64_t opw = wok ? gbl(op)[wc] : 0ull;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const bool own = ci[k] == ch0;
            const bool valid = own ? gv[k] == prev_gen : (gv[k] & ~kGenConv) == prev_gen;
            cv[k] = (ok[k] && valid) ? cv[k] : 0ull;
        }
        uint64_t f = (cv[0] << 1) | (cv[0] >> 1) | (cv[1] >> 63) | (cv[2] << 63) | cv[3] | cv[4];
        if (ND == 3) f |= cv[5] | cv[6];
        f &= opw;  // open voxels only (their x < X)
        uint64_t acc = 0ull;  // changed bits of this word over all local sweeps
        bool conv = true;     // the local sweeps ended without a pending change
        uint32_t vis = 0;     // statistics (CTWS_TRACE): voxels visited
        for (int rep = 0;; ++rep) {
            // exclusive prefix of the per-word bit counts: entry e of the chunk's frontier list
            // is bit (e - pre[j]) of word j, the last j with pre[j] <= e
            const int cnt_bits = __popcll(f);
            int incl = cnt_bits;
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            const int total = __shfl(incl, 63);
            if (total == 0) break;
            vis += (uint32_t)total;
            schg[wv][lane] = 0ull;
            if (dirf) {
#pragma unroll
                for (int d = 0; d < NDIR; ++d) sdir[wv][d][lane] = 0ull;
            }
            sfw[wv][lane] = f;
            spre[wv][lane] = incl - cnt_bits;
            // (constant over the chunk's sweeps; z, y < 2^16, block indices < 2^32)
            sbase[wv][lane] = (uint32_t)((int64_t)row * B.X + xw * 64);
            szy[wv][lane] = ((uint32_t)zz << 16) | (uint32_t)yy;
            sx0[wv][lane] = xw * 64;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // entries per lane and step: index, loads, update as three unrolled phases (the loop
            // in this form relaxes faster than one guarded body: config 4 relax 32.3 -> 28.3 ms);
            // ILP = 2 (two entries' loads in flight together) measured no faster
            constexpr int ILP = 1;
            for (int t0 = 0; t0 < total; t0 += 64 * ILP) {
                int jv[ILP], bv[ILP], zv[ILP], yv[ILP], xv[ILP];
                int64_t iv[ILP];
                bool av[ILP];
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    // odd sweeps walk the list backwards: a later step reads what an earlier
                    // step of the same sweep wrote, so alternating the order carries changes
                    // both ways along the list (symmetric Gauss-Seidel over the steps)
                    const int eo = t0 + u * 64 + lane;
                    av[u] = eo < total;
                    const int e = ((rep & 1) && av[u]) ? total - 1 - eo : eo;
                    int j = 0;
#pragma unroll
                    for (int step = 32; step > 0; step >>= 1)
                        if (spre[wv][j + step] <= e) j += step;
                    const int b = av[u] ? kth_set_bit(sfw[wv][j], e - spre[wv][j]) : 0;
                    const uint32_t zy = szy[wv][j];
                    zv[u] = (int)(zy >> 16);
                    yv[u] = (int)(zy & 0xFFFFu);
                    xv[u] = sx0[wv][j] + b;
                    iv[u] = (int64_t)sbase[wv][j] + b;
                    jv[u] = j;
                    bv[u] = b;
                }
                uint64_t nb[ILP][6], own[ILP];
                float hv[ILP];
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
#pragma unroll
                    for (int k = 0; k < 6; ++k) nb[u][k] = kPackInf;
                    own[u] = kPackInf;
                    hv[u] = 0.f;
                    if (!av[u]) continue;
                    const int64_t i = iv[u];
                    if (ND == 3) {
                        if (zv[u] > 0) nb[u][0] = kb[i - YX];
                        if (zv[u] + 1 < B.Z) nb[u][1] = kb[i + YX];
                    }
                    if (yv[u] > 0) nb[u][2] = kb[i - B.X];
                    if (yv[u] + 1 < B.Y) nb[u][3] = kb[i + B.X];
                    if (xv[u] > 0) nb[u][4] = kb[i - 1];
                    if (xv[u] + 1 < B.X) nb[u][5] = kb[i + 1];
                    own[u] = kb[i];
                    hv[u] = hb[i];
                }
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    if (!av[u]) continue;
                    const uint64_t m = min(min(min(nb[u][0], nb[u][1]), min(nb[u][2], nb[u][3])), min(nb[u][4], nb[u][5]));
                    if (m == kPackInf) continue;
                    const uint64_t k = f_packed(ordf(hv[u]), m);
                    if (k == own[u]) continue;
                    // (a saturated d is detected on the final keys, k_flood_verify; no statistics
                    // either: each extra live value here costs a wave per SIMD, 3-D 125 -> 137
                    // VGPRs with a write counter and the saturation test, config 4 relax +5 ms)
                    kb[iv[u]] = k;
                    atomicOr((unsigned long long*)&schg[wv][jv[u]], 1ull << bv[u]);
                    if (dirf) {
                        // nb[] order: -z, +z, -y, +y, -x, +x (outside the block: INF, its bit is
                        // shifted out of the chunk or masked by open)
#pragma unroll
                        for (int d = 0; d < 6; ++d)
                            if ((ND == 3 || d >= 2) && (nb[u][d] >> kLabelBits) >= (k >> kLabelBits))
                                atomicOr((unsigned long long*)&sdir[wv][ND == 3 ? d : d - 2][jv[u]], 1ull << bv[u]);
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uint64_t c = schg[wv][lane];
            acc |= c;
            if (__ballot(c != 0ull) == 0ull) break;
            if (rep + 1 >= reps) {
                conv = false;
                break;
            }
            // local sweep: the neighbours of this sweep's changes inside the chunk; changes are
            // also in acc, so the neighbours outside the chunk see them in the next launch.
            // dirf: per direction, only the neighbours the change may lower (sdir)
            uint64_t dzm = c, dzp = c, dym = c, dyp = c, dxm = c, dxp = c;
            if (dirf) {
                constexpr int o = ND == 3 ? 2 : 0;
                if (ND == 3) {
                    dzm = sdir[wv][0][lane];
                    dzp = sdir[wv][1][lane];
                }
                dym = sdir[wv][o][lane];
                dyp = sdir[wv][o + 1][lane];
                dxm = sdir[wv][o + 2][lane];
                dxp = sdir[wv][o + 3][lane];
            }
            f = (dxp << 1) | (dxm >> 1);
            const uint64_t cxm = __shfl(dxp, lx > 0 ? lane - 1 : lane);
            const uint64_t cxp = __shfl(dxm, lx < CW - 1 ? lane + 1 : lane);
            if (lx > 0) f |= cxm >> 63;
            if (lx < CW - 1 && xw + 1 < wpr) f |= cxp << 63;
            const uint64_t cym = __shfl(dyp, ly > 0 ? lane - CW : lane);
            const uint64_t cyp = __shfl(dym, ly < CY - 1 ? lane + CW : lane);
            if (ly > 0) f |= cym;
            if (ly < CY - 1 && yy + 1 < B.Y) f |= cyp;
            if (ND == 3 && CZ > 1) {
                const uint64_t czm = __shfl(dzp, lz > 0 ? lane - CW * CY : lane);
                const uint64_t czp = __shfl(dzm, lz < CZ - 1 ? lane + CW * CY : lane);
                if (lz > 0) f |= czm;
                if (lz < CZ - 1 && zz + 1 < B.Z) f |= czp;
            }
            f &= opw;
        }
        if (nvisit && lane == 0 && vis) atomicAdd(&nvisit[bi], vis);
        if (__ballot(acc != 0ull) == 0ull) continue;
        // the chunk changed: publish its changed words and queue the chunks that hold a
        // neighbour of a change (faces), and itself unless its local sweeps converged
        if (wok) cn[wc] = acc;
        if (lane == 0) gn[ch0] = ((uint32_t)it + 1u) | (conv ? kGenConv : 0u);
        const bool fxm = __ballot(lx == 0 && (acc & 1ull)) != 0ull;
        const bool fxp = __ballot(lx == CW - 1 && (acc >> 63)) != 0ull;
        const bool fym = __ballot(ly == 0 && acc != 0ull) != 0ull;
        const bool fyp = __ballot(ly == CY - 1 && acc != 0ull) != 0ull;
        const bool fzm = ND == 3 && __ballot(lz == 0 && acc != 0ull) != 0ull;
        const bool fzp = ND == 3 && __ballot(lz == CZ - 1 && acc != 0ull) != 0ull;
        int cand = -1;
        if (lane == 0 && !conv) cand = ch0;
        else if (lane == 1 && fxm && cx > 0) cand = ch0 - 1;
        else if (lane == 2 && fxp && cx + 1 < G.ncx) cand = ch0 + 1;
        else if (lane == 3 && fym && cy > 0) cand = ch0 - G.ncx;
        else if (lane == 4 && fyp && cy + 1 < G.ncy) cand = ch0 + G.ncx;
        else if (lane == 5 && fzm && cz > 0) cand = ch0 - cplane;
        else if (lane == 6 && fzp && cz + 1 < G.ncz) cand = ch0 + cplane;
        bool push = false;
        if (cand >= 0) push = atomicMax(&qg[cand], (uint32_t)it + 1u) < (uint32_t)it + 1u;
        const uint64_t pm = __ballot(push);
        uint32_t base = 0;
        if (lane == 0 && pm) base = atomicAdd(cnt_next, (uint32_t)__popcll(pm));
        base = (uint32_t)__shfl((int)base, 0);
        if (push)
            list_next[base + __popcll(pm & ((1ull << lane) - 1ull))] = ((uint32_t)bi << kWlChunkBits) | (uint32_t)cand;
    }
}
// chunk bricks: 2-D ws (CZ = 1) and 3-D; CTWS_FRONTIER_CHUNK2D / _3D select one (frontier_chunk_kind)
#define CTWS_FRONTIER_INST(ND, CW, CY, CZ)                                                                           \
    template __global__ void k_frontier<ND, CW, CY, CZ>(const BlockDesc*, const BlockStat*, const float*, uint64_t*, \
                                                        const uint64_t*, const uint64_t*, uint64_t*, const uint32_t*,  \
                                                        uint32_t*, int, const uint32_t*, const uint32_t*, uint32_t*,   \
                                                        uint32_t*, uint32_t*, uint32_t*, int, int);
#define CTWS_LIST0_INST(CW, CY, CZ)                                                                             \
    template __global__ void k_frontier_list0<CW, CY, CZ>(const BlockDesc*, const BlockStat*, const uint64_t*, \
                                                          uint32_t*, uint32_t*);
CTWS_FRONTIER_INST(2, 1, 64, 1)
CTWS_FRONTIER_INST(2, 4, 16, 1)
CTWS_FRONTIER_INST(3, 1, 8, 8)
CTWS_FRONTIER_INST(3, 8, 8, 1)
CTWS_FRONTIER_INST(3, 1, 32, 2)
CTWS_LIST0_INST(1, 64, 1)
CTWS_LIST0_INST(4, 16, 1)
CTWS_LIST0_INST(1, 8, 8)
CTWS_LIST0_INST(8, 8, 1)
CTWS_LIST0_INST(1, 32, 2)
#undef CTWS_FRONTIER_INST
#undef CTWS_LIST0_INST

// tiles still holding open voxels -> full solve in the tile flood (when the frontier loop stops)
__global__ void __launch_bounds__(256) k_frontier_tiles(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                        const uint64_t* __restrict__ open, uint32_t* __restrict__ act,
                                                        int tz, int ty, int tx) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wpr = (B.X + 63) >> 6;
    const int64_t nwords = (int64_t)B.Z * B.Y * wpr;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t bits = open[B.fbase + w];
        if (!bits) continue;
        const int64_t row = w / wpr;
        const int xw = (int)(w - row * wpr);
        const int z = (int)(row / B.Y), y = (int)(row - (int64_t)z * B.Y);
        while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            const int x = xw * 64 + b;
            uint32_t* a = act + B.tbase + ((z / tz) * B.ty + y / ty) * B.tx + x / tx;
            if (!*a) atomicOr(a, kActFull);
        }
    }
}

// fixpoint check of the packed flood: K(q) == f(min_p K(p)) at every voxel the relaxation
// solved (the open bitmap of k_descent_init / k_regrow_init).  The descent-resolved voxels are
// final by construction (the unique-argmin argument above) and are never written by the
// relaxation, so a unit without an open voxel is skipped after its bitmap loads.  Word columns
// as k_localmax: a unit is U vertically adjacent words of one 64-voxel column, whose U + 2 key
// rows are loaded once (all loads of the unit in flight together) and serve as centre, upper
// and lower rows; x-neighbours come from the neighbouring lanes, lane 0 / 63 fetch the key
// left / right of the word.
template <int ND>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 8))) k_flood_verify(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      const float* __restrict__ h, const uint64_t* __restrict__ key,
                                                      const uint64_t* __restrict__ open, uint32_t* __restrict__ flag) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    constexpr int U = 4, R = U + 2;
    const gptr_t<uint64_t> k = gbl(key + B.base);
    const gptr_t<float> hb = gbl(h + B.base);
    const int64_t YX = (int64_t)B.Y * B.X;
    const int wpr = (B.X + 63) >> 6;
    const int ngy = (B.Y + U - 1) / U;
    const int64_t nunits = (int64_t)B.Z * wpr * ngy;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t per = (nunits + nwaves - 1) / nwaves;
    const int64_t wid = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t ubeg = wid * per, uend = min(nunits, ubeg + per);
    bool bad = false, dsat = false;
    // 64 units at a time: lane l loads the open words of unit un0 + l, and only the units with an
    // open voxel are visited (the regrow's open set is a few removed segments: most units skip)
    for (int64_t un0 = ubeg; un0 < uend; un0 += 64) {
      uint64_t lw[U];
      {
        // (32-bit unsigned division: a block has < 2^31 units; the emulated 64-bit one is long)
        const int64_t ul = un0 + lane;
        const uint32_t ul32 = (uint32_t)ul;
        const int gyl = (int)(ul32 % (uint32_t)ngy);
        const uint32_t sl = ul32 / (uint32_t)ngy;
        const int xwl = (int)(sl % (uint32_t)wpr), zl = (int)(sl / (uint32_t)wpr);
#pragma unroll
        for (int u = 0; u < U; ++u)
            lw[u] = (ul < uend && gyl * U + u < B.Y) ? gbl(open)[B.fbase + ((int64_t)zl * B.Y + gyl * U + u) * wpr + xwl]
                                                     : 0ull;
      }
      uint64_t todo = __ballot((lw[0] | lw[1] | lw[2] | lw[3]) != 0ull);
      while (todo) {
        const int src = __builtin_ctzll(todo);
        todo &= todo - 1;
        const int64_t un = un0 + src;
        const uint32_t un32 = (uint32_t)un;
        const int gy = (int)(un32 % (uint32_t)ngy);
        const uint32_t strip = un32 / (uint32_t)ngy;
        const int xw = (int)(strip % (uint32_t)wpr), z = (int)(strip / (uint32_t)wpr);
        const int y0 = gy * U;
        // open words of the unit's rows
        uint64_t ow[U];
#pragma unroll
        for (int u = 0; u < U; ++u) ow[u] = shfl_u64(lw[u], src);
        const int x = xw * 64 + lane;
        const int xc = min(x, B.X - 1);
        const int xe = lane == 0 ? max(xc - 1, 0) : min(xc + 1, B.X - 1);
        const int64_t zb = (int64_t)z * YX;
        uint64_t rk[R];
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int yy = min(max(y0 - 1 + q, 0), B.Y - 1);
            rk[q] = k[zb + (int64_t)yy * B.X + xc];
        }
        uint64_t ke[U], kzm[U], kzp[U];
        float hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int yy = min(y0 + u, B.Y - 1);
            const int64_t ic = zb + (int64_t)yy * B.X + xc;
            ke[u] = k[zb + (int64_t)yy * B.X + xe];
            hv[u] = hb[ic];
            if (ND == 3) {
                kzm[u] = k[z > 0 ? ic - YX : ic];
                kzp[u] = k[z + 1 < B.Z ? ic + YX : ic];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int y = y0 + u;
            const bool valid = y < B.Y && x < B.X;
            const uint64_t o = valid ? rk[u + 1] : kPackInf;
            uint64_t l = shfl_up_u64(o, 1), r = shfl_down_u64(o, 1);
            const uint64_t ker = shfl_u64(ke[u], 63);
            if (lane == 0) l = (x > 0) ? ke[u] : kPackInf;
            if (lane == 63) r = ker;
            if (x + 1 >= B.X) r = kPackInf;
            uint64_t m = min(l, r);
            if (y > 0) m = min(m, rk[u]);
            if (y + 1 < B.Y) m = min(m, rk[u + 2]);
            if (ND == 3) {
                if (z > 0) m = min(m, kzm[u]);
                if (z + 1 < B.Z) m = min(m, kzp[u]);
            }
            // an open voxel is never a seed (descent: seeds resolve to themselves; regrow: the
            // survivors and auto seeds are taken out of the open set)
            const uint64_t e = (m == kPackInf) ? kPackInf : f_packed(ordf(hv[u]), m);
            const bool b1 = valid && ((ow[u] >> lane) & 1ull) && e != o;
            // a solved key with d at kDMax: the 12-bit hop distance may have saturated (with every
            // final d below kDMax the keys are a fixpoint of the exact f, which is unique)
            dsat |= valid && ((ow[u] >> lane) & 1ull) && key_dsat(o);
            if (b1 && flag[1] < 8u) {  // diagnostics: the first few violations
                const uint32_t slot = atomicAdd(&flag[1], 1u);
                if (slot < 8u) flag[2 + slot] = (uint32_t)(B.base + zb + (int64_t)y * B.X + x);
            }
            bad |= b1;
        }
      }
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
    if (__ballot(dsat) && (threadIdx.x & 63) == 0) note_dsat(S, blockIdx.y);
}
template __global__ void k_flood_verify<3>(const BlockDesc*, const BlockStat*, const float*, const uint64_t*,
                                           const uint64_t*, uint32_t*);
template __global__ void k_flood_verify<2>(const BlockDesc*, const BlockStat*, const float*, const uint64_t*,
                                           const uint64_t*, uint32_t*);

// seeds only (fallback after a failed verification)
__global__ void __launch_bounds__(256) k_flood_reset(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const float* __restrict__ h, const uint32_t* __restrict__ lab,
                                                     const uint32_t* __restrict__ cc, const uint64_t* __restrict__ sbits,
                                                     uint64_t* __restrict__ key, uint8_t* __restrict__ fixedv) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.N; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t l = (!cc || bit_of(sbits, B, i)) ? seed_label(lab, cc, B.base, (uint32_t)i) : 0u;
        key[B.base + i] = l ? (((uint64_t)ordf(h[B.base + i]) << 32) | (uint64_t)l) : kPackInf;
        fixedv[B.base + i] = l ? 1 : 0;
    }
}

}  // namespace ctws
