// k_relax.hip — the flood's relaxation of the open voxels in LDS-resident tiles.
//
// Reference: utils/volume_utils.py:123-139 (vu.watershed -> vigra watershedsNew, region
// growing).  After the descent pre-pass (k_flood.hip) every voxel whose steepest descent ends
// in a seed holds its final packed key; the remaining "open" voxels (the catchments of hmap
// minima without a seed, and tie voxels) need the fixpoint
//     K(q) = f_q(min over the neighbours p of K(p))      (f_packed, ctws_dev.h)
// The same fixpoint is reached by the size-filter regrow from the surviving segments.
//
// Schedule.  A tile (2-D ws: one slice x 32 x 32; 3-D: 8 x 8 x 16) is staged in LDS by ONE
// wave with a 1-voxel key halo: keys 8 B per voxel, heights 4 B per tile voxel, the tile's
// open bits (16 words of 64 bits, one per lane).  Inside the tile the open voxels relax with a
// worklist: round r visits the frontier (a tile's first round: all its open voxels; afterwards
// the open neighbours of the voxels changed in round r-1), expanded from the frontier bitmap
// into a list the wave's 64 lanes share.  Rounds are wave-synchronous (no workgroup barrier):
// four tiles per workgroup progress independently.  Every visit reads six (four) LDS neighbours — no global memory traffic per
// visit, which is what bounds the global-memory frontier (k_frontier: one scattered 128-B line
// per neighbour gather, TA-bound).  When the tile has converged, its changed keys are written
// back and the face-neighbour tiles whose halo changed are queued for the next launch; a tile
// re-reads its halo from global memory then.  Keys never need a global atomic: a tile owns its
// voxels during a launch, and a halo read that races with the neighbour's write-back is
// repaired in the next launch (the neighbour queues this tile whenever a shared face voxel
// changes).  The host loops launches until no tile is queued.
#include "ctws_kernels.h"

namespace ctws {

template <int ND>
struct RTile;
template <>
struct RTile<2> {
    static constexpr int TZ = 1, TY = 32, TX = 32, HZ = 1, HY = 34, HX = 34, ZO = 0;
};
template <>
struct RTile<3> {
    static constexpr int TZ = 8, TY = 8, TX = 16, HZ = 10, HY = 10, HX = 18, ZO = 1;
};
constexpr int kRTN = 1024;  // voxels per tile
constexpr int kRNW = 16;    // 64-bit bitmap words per tile
constexpr int kRWaves = 4;  // waves (tiles in flight) per workgroup
constexpr int kRMaxRounds = 1 << 14;

__device__ __forceinline__ int rt_kth_bit(uint64_t w, int k) {
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

// open bits of tile word w: tile rows w * RPW .. + RPW - 1 (row r = lz * TY + ly), TX bits each
template <int ND>
__device__ __forceinline__ uint64_t rt_open_word(const BlockDesc& B, const uint64_t* open, int w, int z0, int y0,
                                                 int x0) {
    using T = RTile<ND>;
    constexpr int RPW = 64 / T::TX;
    constexpr uint64_t RM = T::TX == 64 ? ~0ull : ((1ull << T::TX) - 1ull);
    const int wpr = (B.X + 63) >> 6;
    const uint64_t* op = open + B.fbase;
    uint64_t v = 0ull;
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int r = w * RPW + k;
        const int z = z0 + r / T::TY, y = y0 + r % T::TY;
        if (z < B.Z && y < B.Y) v |= ((op[((int64_t)z * B.Y + y) * wpr + (x0 >> 6)] >> (x0 & 63)) & RM) << (k * T::TX);
    }
    return v;
}

// iteration-0 list: every tile holding an open voxel; a thread per tile, one append per wave
template <int ND>
__global__ void __launch_bounds__(256) k_relax_list0(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     const uint64_t* __restrict__ open, uint64_t* __restrict__ list,
                                                     uint32_t* __restrict__ cnt) {
    using T = RTile<ND>;
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int ntx = (B.X + T::TX - 1) / T::TX, nty = (B.Y + T::TY - 1) / T::TY, ntz = (B.Z + T::TZ - 1) / T::TZ;
    const int ntiles = ntx * nty * ntz;
    const int lane = threadIdx.x & 63;
    for (int t0 = blockIdx.x * 256 + (threadIdx.x & ~63); t0 < ntiles; t0 += gridDim.x * 256) {
        const int t = t0 + lane;
        bool any = false;
        if (t < ntiles) {
            const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
            const int z0 = tzi * T::TZ, y0 = tyi * T::TY, x0 = txi * T::TX;
            for (int w = 0; w < kRNW && !any; ++w) any = rt_open_word<ND>(B, open, w, z0, y0, x0) != 0ull;
        }
        const uint64_t m = __ballot(any);
        if (!m) continue;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(cnt, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, 0);
        if (any) list[base + __popcll(m & ((1ull << lane) - 1ull))] = ((uint64_t)blockIdx.y << 32) | (uint32_t)t;
    }
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One tile per wave: the tile's rounds are wave-synchronous (no workgroup barrier), the
// frontier words live in lanes 0..15, the list is expanded by a 16-lane prefix.
template <int ND>
__global__ void __launch_bounds__(256) k_tile_relax(const BlockDesc* __restrict__ D, const float* __restrict__ h,
                                                    uint64_t* __restrict__ key, const uint64_t* __restrict__ open,
                                                    const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                    uint64_t* __restrict__ list_next, uint32_t* __restrict__ cnt_next,
                                                    uint32_t* __restrict__ tgen, int it, uint32_t* __restrict__ stats) {
    using T = RTile<ND>;
    constexpr int TZ = T::TZ, TY = T::TY, TX = T::TX, HY = T::HY, HX = T::HX, ZO = T::ZO;
    constexpr int HN = T::HZ * HY * HX;
    __shared__ uint64_t sk_[kRWaves][HN];
    __shared__ uint32_t sh_[kRWaves][kRTN];
    __shared__ uint64_t sfb_[kRWaves][kRNW], schg_[kRWaves][kRNW], sfa_[kRWaves][kRNW];
    __shared__ int spre_[kRWaves][kRNW + 1];
    __shared__ uint32_t sface_[kRWaves];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t* sk = sk_[wv];
    uint32_t* sh = sh_[wv];
    uint64_t* sfb = sfb_[wv];
    uint64_t* schg = schg_[wv];
    uint64_t* sfa = sfa_[wv];
    int* spre = spre_[wv];
    const uint32_t n = *cnt;
    uint32_t visits = 0, rounds_total = 0;
    for (uint32_t e = blockIdx.x * kRWaves + wv; e < n; e += gridDim.x * kRWaves) {
        const uint64_t ent = list[e];
        const int bi = (int)(ent >> 32);
        const int t = (int)(uint32_t)ent;
        const BlockDesc& B = D[bi];
        const int ntx = (B.X + TX - 1) / TX, nty = (B.Y + TY - 1) / TY;
        const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
        const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
        const int64_t YX = (int64_t)B.Y * B.X;
        const uint64_t* kb = key + B.base;
        const float* hb = h + B.base;
        // ---- stage: open words (lanes 0..15), keys + halo, heights; loads of a batch together
        const uint64_t opw = lane < kRNW ? rt_open_word<ND>(B, open, lane, z0, y0, x0) : 0ull;
        if (__ballot(opw != 0ull) == 0ull) continue;
        if (lane < kRNW) schg[lane] = 0ull;
        if (lane == 0) sface_[wv] = 0u;
        constexpr int NK = (HN + 63) / 64;
        constexpr int KB = 10;  // keys per lane in flight
        for (int k0 = 0; k0 < NK; k0 += KB) {
            uint64_t kv[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const int c = min(lane + (k0 + k) * 64, HN - 1);
                const int hx = c % HX, hy = (c / HX) % HY, hz = c / (HX * HY);
                const int gz = z0 + hz - ZO, gy = y0 + hy - 1, gx = x0 + hx - 1;
                const bool in = gz >= 0 && gz < B.Z && gy >= 0 && gy < B.Y && gx >= 0 && gx < B.X;
                kv[k] = gbl(kb)[in ? (gz * YX + (int64_t)gy * B.X + gx) : 0];
                if (!in) kv[k] = kPackInf;
            }
#pragma unroll
            for (int k = 0; k < KB; ++k)
                if (k0 + k < NK && lane + (k0 + k) * 64 < HN) sk[lane + (k0 + k) * 64] = kv[k];
        }
        {
            constexpr int NH = kRTN / 64;
            float hv[NH];
#pragma unroll
            for (int k = 0; k < NH; ++k) {
                const int tl = lane + k * 64;
                const int lx = tl % TX, ly = (tl / TX) % TY, lz = tl / (TX * TY);
                const int gz = min(z0 + lz, B.Z - 1), gy = min(y0 + ly, B.Y - 1), gx = min(x0 + lx, B.X - 1);
                hv[k] = gbl(hb)[gz * YX + (int64_t)gy * B.X + gx];
            }
#pragma unroll
            for (int k = 0; k < NH; ++k) sh[lane + k * 64] = ordf(hv[k]);
        }
        // ---- wave-synchronous worklist rounds; frontier word j in lane j
        uint64_t fa = opw;
        int rounds = 0;
        for (; rounds < kRMaxRounds; ++rounds) {
            const int c = __popcll(fa);
            int incl = c;
#pragma unroll
            for (int o = 1; o < kRNW; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const int total = __shfl(incl, kRNW - 1);
            if (total == 0) break;
            visits += (uint32_t)total;
            if (lane < kRNW) {
                spre[lane] = incl - c;
                sfa[lane] = fa;
                sfb[lane] = 0ull;
            }
            wave_sync_lds();
            for (int q = lane; q < total; q += 64) {
                int j = 0;
#pragma unroll
                for (int step = kRNW / 2; step > 0; step >>= 1)
                    if (j + step < kRNW && spre[j + step] <= q) j += step;
                const int b = rt_kth_bit(sfa[j], q - spre[j]);
                const int tl = j * 64 + b;
                const int lx = tl % TX, ly = (tl / TX) % TY, lz = tl / (TX * TY);
                const int cc = ((lz + ZO) * HY + ly + 1) * HX + lx + 1;
                uint64_t m = min(min(sk[cc - 1], sk[cc + 1]), min(sk[cc - HX], sk[cc + HX]));
                if (ND == 3) m = min(m, min(sk[cc - HX * HY], sk[cc + HX * HY]));
                if (m == kPackInf) continue;
                const uint64_t nk = f_packed(sh[tl], m);
                if (nk == sk[cc]) continue;
                sk[cc] = nk;
                atomicOr((unsigned long long*)&schg[j], 1ull << b);
                uint32_t face = 0;
                auto q_nb = [&](int t2) { atomicOr((unsigned long long*)&sfb[t2 >> 6], 1ull << (t2 & 63)); };
                if (lx > 0) q_nb(tl - 1);
                else face |= 16u;
                if (lx + 1 < TX) q_nb(tl + 1);
                else face |= 32u;
                if (ly > 0) q_nb(tl - TX);
                else face |= 4u;
                if (ly + 1 < TY) q_nb(tl + TX);
                else face |= 8u;
                if (ND == 3) {
                    if (lz > 0) q_nb(tl - TX * TY);
                    else face |= 1u;
                    if (lz + 1 < TZ) q_nb(tl + TX * TY);
                    else face |= 2u;
                }
                if (face) atomicOr(&sface_[wv], face);
            }
            wave_sync_lds();
            fa = lane < kRNW ? (sfb[lane] & opw) : 0ull;
        }
        rounds_total += (uint32_t)rounds;
        // ---- write back the changed keys (lane-strided over the tile)
#pragma unroll 4
        for (int k = 0; k < kRTN / 64; ++k) {
            const int tl = lane + k * 64;
            if (!((schg[tl >> 6] >> (tl & 63)) & 1ull)) continue;
            const int lx = tl % TX, ly = (tl / TX) % TY, lz = tl / (TX * TY);
            const int cc = ((lz + ZO) * HY + ly + 1) * HX + lx + 1;
            key[B.base + (z0 + lz) * YX + (int64_t)(y0 + ly) * B.X + (x0 + lx)] = sk[cc];
        }
        // ---- queue the face neighbours whose halo changed (and this tile if it hit the cap)
        if (lane < 7) {
            const uint32_t f = sface_[wv];
            bool go;
            int zz = tzi, yy = tyi, xx = txi;
            if (lane < 6) {
                go = (f >> lane) & 1u;
                zz += lane == 0 ? -1 : (lane == 1 ? 1 : 0);
                yy += lane == 2 ? -1 : (lane == 3 ? 1 : 0);
                xx += lane == 4 ? -1 : (lane == 5 ? 1 : 0);
            } else {
                go = rounds >= kRMaxRounds;
            }
            const int ntz = (B.Z + TZ - 1) / TZ;
            if (go && zz >= 0 && zz < ntz && yy >= 0 && yy < nty && xx >= 0 && xx < ntx) {
                const uint32_t nt = (uint32_t)((zz * nty + yy) * ntx + xx);
                if (atomicMax(&tgen[B.rbase + nt], (uint32_t)it + 1u) < (uint32_t)it + 1u) {
                    const uint32_t slot = atomicAdd(cnt_next, 1u);
                    list_next[slot] = ((uint64_t)bi << 32) | nt;
                }
            }
        }
        wave_sync_lds();
    }
    if (stats && lane == 0 && visits) {
        atomicAdd(&stats[(blockIdx.x & 63) * 2], visits);
        atomicAdd(&stats[(blockIdx.x & 63) * 2 + 1], rounds_total);
    }
}

template __global__ void k_relax_list0<2>(const BlockDesc*, const BlockStat*, const uint64_t*, uint64_t*, uint32_t*);
template __global__ void k_relax_list0<3>(const BlockDesc*, const BlockStat*, const uint64_t*, uint64_t*, uint32_t*);
template __global__ void k_tile_relax<2>(const BlockDesc*, const float*, uint64_t*, const uint64_t*, const uint64_t*,
                                         const uint32_t*, uint64_t*, uint32_t*, uint32_t*, int, uint32_t*);
template __global__ void k_tile_relax<3>(const BlockDesc*, const float*, uint64_t*, const uint64_t*, const uint64_t*,
                                         const uint32_t*, uint64_t*, uint32_t*, uint32_t*, int, uint32_t*);

}  // namespace ctws
