// k_threshcc.hip — BlockComponents of ThresholdedComponentsWorkflow on gfx950: threshold a
// block and label its 26-connected components the way skimage.morphology.label numbers them
// (cluster_tools/thresholded_components/block_components.py:143-230).
//
//   k_tc_minmax   min / max of the block (vu.normalize, volume_utils.py:113-120)
//   k_tc_tile     member = threshold(normalized value) & mask; an 8x8x64 tile is labelled in LDS
//                 (x runs by ballot, then unions with the 12 other backward neighbours); every
//                 member's parent = its tile root, non-members kNoParent
//   k_tc_merge    unions across the tile faces (global union-find, by C index)
//   k_tc_roots    root bitmap (P[i] == i), one 64-bit word per wave
//   k_tc_wordoff  exclusive word offsets of the roots (chunk offsets from k_scan_chunks)
//   k_tc_label    out[i] = rank of its root in C order + 1 (0 for the background)
//
// Every union links the root with the larger C index under the smaller, so a component's root
// is its first voxel in C order and the ranks of the roots are skimage's numbering (labels in
// order of first appearance in a C-order scan; pinned by tests/golden/threshcc_*.npz).
#include "ctws_kernels.h"

namespace ctws {

namespace {
constexpr int kTcTZ = 8, kTcTY = 8, kTcTX = 64, kTcTN = kTcTZ * kTcTY * kTcTX, kTcPer = kTcTN / 256;
constexpr int kTcPairs = 2048;  // LDS union-pair list; beyond it a thread unites in place
static_assert(kTcTN <= 4096, "pairs pack two 12-bit tile positions");

__device__ __forceinline__ bool tc_member(float v, const TcParams& p, float vmin, float range) {
    // numpy in float32: v - min, divided by max(v - min) = fl(max - min) when that is positive
    // (normalize), then the comparison with the threshold as float32 (a Python float is weak)
    float t = v;
    if (p.normalize) {
        t = v - vmin;
        if (range > 0.0f) t = t / range;
    }
    return p.mode == 0 ? t > p.thr : (p.mode == 1 ? t < p.thr : t == p.thr);
}

// find without compression (the label pass reads the forest only)
__device__ __forceinline__ uint32_t tc_find(const uint32_t* P, uint32_t a) {
    uint32_t p = P[a];
    while (p != a) {
        a = p;
        p = P[a];
    }
    return a;
}
}  // namespace

// one workgroup per CU at most (the two atomics per workgroup on one address are what a wide
// grid pays for: 4096 of them cost ~45 us); float4 loads, the tail scalar
__global__ void __launch_bounds__(256) k_tc_minmax(const float* __restrict__ v, int64_t n, uint32_t* __restrict__ mm) {
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * 256;
    const float4* v4 = reinterpret_cast<const float4*>(v);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
        const float4 f = v4[i];
        const uint32_t a = ordf(f.x), b = ordf(f.y), c = ordf(f.z), d = ordf(f.w);
        lo = min(lo, min(min(a, b), min(c, d)));
        hi = max(hi, max(max(a, b), max(c, d)));
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint32_t u = ordf(v[i]);
        lo = min(lo, u);
        hi = max(hi, u);
    }
    lo = wg_reduce_u32(lo, OpMin());
    hi = wg_reduce_u32(hi, OpMax());
    if (threadIdx.x == 0) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
}

// ---- inputs other than a raw float32 block (ctws_threshold_components_ex) ---------------------
// astype('float32') of the dataset's values (numpy rounds to nearest, as the conversions here)
template <class T>
__global__ void __launch_bounds__(256) k_tc_to_f32(const T* __restrict__ in, int64_t n, float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        out[i] = (float)in[i];
}
// the raw comparison of `_cc_block_with_mask` / the channel sum (block_components.py:199-220) for
// a float64 or integer dataset: numpy compares `x > python float` in float64 there (NEP 50; every
// integer converts to the nearest double, as numpy's cast); members become 1.0f, the others 0.0f
// (k_tc_tile then tests > 0.5)
template <class T>
__global__ void __launch_bounds__(256) k_tc_raw_members(const T* __restrict__ in, int64_t n, int mode, double thr,
                                                        float* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const double v = (double)in[i];
        const bool m = mode == 0 ? v > thr : (mode == 1 ? v < thr : v == thr);
        out[i] = m ? 1.0f : 0.0f;
    }
}
#define CTWS_TC_DT(T)                                                                              \
    template __global__ void k_tc_to_f32<T>(const T*, int64_t, float*);                            \
    template __global__ void k_tc_raw_members<T>(const T*, int64_t, int, double, float*);
CTWS_TC_DT(uint8_t)
CTWS_TC_DT(int8_t)
CTWS_TC_DT(uint16_t)
CTWS_TC_DT(int16_t)
CTWS_TC_DT(uint32_t)
CTWS_TC_DT(int32_t)
CTWS_TC_DT(uint64_t)
CTWS_TC_DT(int64_t)
CTWS_TC_DT(double)
#undef CTWS_TC_DT

// vu.normalize in place (the normalize before the prefilter of a masked block): v - min, divided
// by fl(max - min) when positive, in float32 (min / max from k_tc_minmax)
__global__ void __launch_bounds__(256) k_tc_normalize(float* __restrict__ v, int64_t n, const uint32_t* __restrict__ mm) {
    const float vmin = unordf(mm[0]), range = unordf(mm[1]) - vmin;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float t = v[i] - vmin;
        if (range > 0.0f) t = t / range;
        v[i] = t;
    }
}

// the prefilter's vigra gaussianSmoothing along one axis (vu.apply_filter, block_components.py:161
// / :210): out[x] = float(sum over p = x - r .. x + r ascending of taps[r + x - p] * in[reflect(p)])
// in double without FMA contraction (the Makefile's -ffp-contract=off), as the oracle's
// convolve_line_reflect and k_gauss.hip.  One thread per output voxel: the prefilter is an
// option of a small workflow, not a hot path (lanes along x keep the loads coalesced).
__global__ void __launch_bounds__(256) k_tc_gauss(const float* __restrict__ in, float* __restrict__ out, int nz,
                                                  int ny, int nx, int axis, const double* __restrict__ taps, int r) {
    const int64_t n = (int64_t)nz * ny * nx;
    const int64_t st = axis == 0 ? (int64_t)ny * nx : (axis == 1 ? nx : 1);
    const int L = axis == 0 ? nz : (axis == 1 ? ny : nx);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int64_t rest = i % (int64_t)nx, row = i / nx;
        const int c = axis == 2 ? (int)rest : (axis == 1 ? (int)(row % ny) : (int)(row / ny));
        const int64_t base = i - (int64_t)c * st;
        double sum = 0.0;
        for (int p = c - r; p <= c + r; ++p) {
            const int q = p < 0 ? -p : (p >= L ? 2 * (L - 1) - p : p);
            sum += taps[r + c - p] * (double)in[base + (int64_t)q * st];
        }
        out[i] = (float)sum;
    }
}

__global__ void __launch_bounds__(256) k_tc_tile(const float* __restrict__ v, const uint8_t* __restrict__ mask,
                                                 TcParams p, const uint32_t* __restrict__ mm,
                                                 uint32_t* __restrict__ P, uint32_t* __restrict__ any) {
    constexpr int TZ = kTcTZ, TY = kTcTY, TX = kTcTX, TN = kTcTN, PER = kTcPer;
    __shared__ uint8_t sm[TN];   // members, C layout c = (lz * TY + ly) * TX + lx
    __shared__ uint32_t sp[TN];  // tile-local parents
    __shared__ uint32_t pbuf[kTcPairs];  // union pairs (source << 12 | target), tile positions
    __shared__ uint32_t pcnt;
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const int ntx = (nx + TX - 1) / TX, nty = (ny + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    const int t = blockIdx.x;
    if (t >= ntx * nty * ntz) return;
    const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
    const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
    float vmin = 0.0f, range = 0.0f;
    if (p.normalize) {
        vmin = unordf(mm[0]);
        range = unordf(mm[1]) - vmin;
    }
    // loads: every one unconditional (clamped into the block) so that all are in flight together
    float lv[PER];
    uint8_t lm[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c & (TX - 1), ly = (c / TX) % TY, lz = c / (TX * TY);
        const int cz = min(z0 + lz, nz - 1), cy = min(y0 + ly, ny - 1), cx = min(x0 + lx, nx - 1);
        const int64_t i = ((int64_t)cz * ny + cy) * nx + cx;
        lv[j] = gbl(v)[i];
        lm[j] = mask ? gbl(mask)[i] : (uint8_t)1;
    }
    uint32_t memb = 0;  // bit j: position j is a member
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c & (TX - 1), ly = (c / TX) % TY, lz = c / (TX * TY);
        const bool in = z0 + lz < nz && y0 + ly < ny && x0 + lx < nx;
        const bool m = in && lm[j] && tc_member(lv[j], p, vmin, range);
        memb |= (m ? 1u : 0u) << j;
        sm[c] = m ? 1 : 0;
    }
    if (threadIdx.x == 0) pcnt = 0u;
    if (__syncthreads_or(memb != 0) && threadIdx.x == 0) any[0] = 1u;
    // x runs: a wave holds one tile row (TX = 64); members link to the first voxel of their run
    const int lane = threadIdx.x & 63;
    uint32_t contm = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const bool m = (memb >> j) & 1u;
        const bool cont = m && lane > 0 && sm[c - 1];
        contm |= (cont ? 1u : 0u) << j;
        const uint64_t starts = __ballot(!cont);
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const int s0 = 63 - __builtin_clzll(starts & upto);
        sp[c] = m ? (uint32_t)(c - (lane - s0)) : kNoParent;
    }
    __syncthreads();
    // the four backward rows (dz, dy) = (-1, -1), (-1, 0), (-1, 1), (0, -1), each with dx in
    // {-1, 0, 1}: one union per run of members among the three (adjacent ones share an x run);
    // a voxel that continues its run needs only q + 1 when q is no member (its x predecessor
    // covered q - 1 and q); with a member right below (dz = -1), the rows (-1, -1) and (-1, +1)
    // are its in-plane neighbours, connected through its own unions.
    // The pairs are first collected into an LDS list (one atomic per wave and row) and then
    // united by all 256 threads at once: done in place, a wave's few active lanes per row
    // walked 64 dependent union chains one after the other (tile kernel 365 -> see DESIGN §3.2).
    auto ordk = [](uint32_t c) { return c; };
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const bool mem = (memb >> j) & 1u;
        const int c = threadIdx.x + j * 256;
        const int lx = c & (TX - 1), ly = (c / TX) % TY, lz = c / (TX * TY);
        const bool cont = (contm >> j) & 1u;
        const bool below = mem && lz > 0 && sm[c - TY * TX];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int dz = r < 3 ? -1 : 0, dy = r < 3 ? r - 1 : -1;
            const int qz = lz + dz, qy = ly + dy;
            const bool valid = mem && qz >= 0 && qy >= 0 && qy < TY && !((r == 0 || r == 2) && below);
            const int cq = valid ? (qz * TY + qy) * TX + lx : 0;
            const bool m0 = valid && sm[cq] != 0;
            const bool mr = valid && !m0 && lx + 1 < TX && sm[cq + 1];
            const bool ml = valid && !m0 && !cont && lx > 0 && sm[cq - 1];
            // first pair: q (m0, not cont) or q - 1 (ml); second pair: q + 1 (mr)
            const bool has1 = (m0 && !cont) || ml, has2 = mr;
            const uint32_t v1 = ((uint32_t)c << 12) | (uint32_t)(m0 ? cq : cq - 1);
            const uint32_t v2 = ((uint32_t)c << 12) | (uint32_t)(cq + 1);
            const uint64_t b1 = __ballot(has1), b2 = __ballot(has2);
            if (b1 | b2) {
                const int leader = __builtin_ctzll(b1 | b2);
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(&pcnt, (uint32_t)(__popcll(b1) + __popcll(b2)));
                base = (uint32_t)__shfl((int)base, leader);
                const uint64_t lt = (1ull << lane) - 1ull;
                const uint32_t i1 = base + (uint32_t)__popcll(b1 & lt);
                const uint32_t i2 = base + (uint32_t)__popcll(b1) + (uint32_t)__popcll(b2 & lt);
                if (has1) {
                    if (i1 < kTcPairs) pbuf[i1] = v1;
                    else lds_union(sp, v1 >> 12, v1 & 0xFFFu, ordk);
                }
                if (has2) {
                    if (i2 < kTcPairs) pbuf[i2] = v2;
                    else lds_union(sp, v2 >> 12, v2 & 0xFFFu, ordk);
                }
            }
        }
    }
    __syncthreads();
    {
        const uint32_t np = min(pcnt, (uint32_t)kTcPairs);
        for (uint32_t e = threadIdx.x; e < np; e += 256) {
            const uint32_t v = pbuf[e];
            lds_union(sp, v >> 12, v & 0xFFFu, ordk);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int c = threadIdx.x + j * 256;
        const int lx = c & (TX - 1), ly = (c / TX) % TY, lz = c / (TX * TY);
        const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
        if (z >= nz || y >= ny || x >= nx) continue;
        uint32_t g = kNoParent;
        if ((memb >> j) & 1u) {
            const uint32_t rt = lds_find(sp, (uint32_t)c);
            const int rx = (int)(rt & (TX - 1)), ry = (int)((rt / TX) % TY), rz = (int)(rt / (TX * TY));
            g = (uint32_t)(((int64_t)(z0 + rz) * ny + (y0 + ry)) * nx + (x0 + rx));
        }
        P[((int64_t)z * ny + y) * nx + x] = g;
    }
}

// unions across the tile faces.  Each shell voxel of a tile once: the low z plane, then (lz > 0)
// the low / high y rows, then (lz > 0, 0 < ly < TY - 1) the low / high x columns.  A member unions
// with its backward neighbours outside the tile by the row rule of k_tc_tile applied to the whole
// row (the row (dz, dy) = (-1, +1) leaves through the high y face); in the planes and rows, where
// lanes walk x, a member that continues the run of its x predecessor (also on the shell, same
// rows) adds only q + 1 when q is no member.
__global__ void __launch_bounds__(256) k_tc_merge(TcParams p, uint32_t* __restrict__ P) {
    constexpr int TZ = kTcTZ, TY = kTcTY, TX = kTcTX;
    static_assert(TY > 2 && TZ > 1, "");
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const int ntx = (nx + TX - 1) / TX, nty = (ny + TY - 1) / TY, ntz = (nz + TZ - 1) / TZ;
    constexpr int fsz[5] = {TY * TX, (TZ - 1) * TX, (TZ - 1) * TX, (TZ - 1) * (TY - 2), (TZ - 1) * (TY - 2)};
    for (int t = blockIdx.x; t < ntx * nty * ntz; t += gridDim.x) {
        const int txi = t % ntx, tyi = (t / ntx) % nty, tzi = t / (ntx * nty);
        const int z0 = tzi * TZ, y0 = tyi * TY, x0 = txi * TX;
        for (int f = 0; f < 5; ++f) {
            for (int e = threadIdx.x; e < fsz[f]; e += 256) {
                int lz, ly, lx;
                if (f == 0) { lz = 0; ly = e / TX; lx = e % TX; }
                else if (f <= 2) { lz = 1 + e / TX; ly = f == 1 ? 0 : TY - 1; lx = e % TX; }
                else { lz = 1 + e / (TY - 2); ly = 1 + e % (TY - 2); lx = f == 3 ? 0 : TX - 1; }
                const int z = z0 + lz, y = y0 + ly, x = x0 + lx;
                if (z >= nz || y >= ny || x >= nx) continue;
                const int64_t i = ((int64_t)z * ny + y) * nx + x;
                if (P[i] == kNoParent) continue;
                if (lx == 0 && x > 0 && P[i - 1] != kNoParent) uf_union(P, (uint32_t)i, (uint32_t)(i - 1));
                const bool cont = f <= 2 && lx > 0 && P[i - 1] != kNoParent;
                const bool below = z > 0 && P[i - (int64_t)ny * nx] != kNoParent;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int dz = r < 3 ? -1 : 0, dy = r < 3 ? r - 1 : -1;
                    const int qz = z + dz, qy = y + dy;
                    if (qz < 0 || qy < 0 || qy >= ny) continue;
                    if ((r == 0 || r == 2) && below) continue;
                    const bool row_out = lz + dz < 0 || ly + dy < 0 || ly + dy >= TY;
                    if (!row_out && lx != 0 && lx != TX - 1) continue;  // the whole row is the tile's
                    const int64_t q = ((int64_t)qz * ny + qy) * nx + x;
                    const bool m0 = P[q] != kNoParent;
                    const bool mr = x + 1 < nx && P[q + 1] != kNoParent;
                    if (m0) {
                        if (row_out && !cont) uf_union(P, (uint32_t)i, (uint32_t)q);
                    } else {
                        const bool ml = !cont && x > 0 && P[q - 1] != kNoParent;
                        if (ml && (row_out || lx == 0)) uf_union(P, (uint32_t)i, (uint32_t)(q - 1));
                        if (mr && (row_out || lx == TX - 1)) uf_union(P, (uint32_t)i, (uint32_t)(q + 1));
                    }
                }
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_tc_roots(const uint32_t* __restrict__ P, int64_t n, uint64_t* __restrict__ bits) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool root = i < n && P[i] == (uint32_t)i;
    const uint64_t b = __ballot(root);
    if ((threadIdx.x & 63) == 0 && i < n) bits[i >> 6] = b;
}

// per-word exclusive offsets: chunk offset (256 words a chunk) + scan of the chunk's popcounts
__global__ void __launch_bounds__(256) k_tc_wordoff(const uint64_t* __restrict__ bits, int64_t nw,
                                                    const uint64_t* __restrict__ offs, uint32_t* __restrict__ woff) {
    __shared__ uint32_t tmp[256];
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t c = w < nw ? (uint32_t)__popcll(bits[w]) : 0u;
    tmp[threadIdx.x] = c;
    __syncthreads();
    for (int s = 1; s < 256; s <<= 1) {
        const uint32_t a = threadIdx.x >= (unsigned)s ? tmp[threadIdx.x - s] : 0u;
        __syncthreads();
        tmp[threadIdx.x] += a;
        __syncthreads();
    }
    if (w < nw) woff[w] = (uint32_t)offs[blockIdx.x] + tmp[threadIdx.x] - c;
}

__global__ void __launch_bounds__(256) k_tc_label(const uint32_t* __restrict__ P, int64_t n,
                                                  const uint64_t* __restrict__ bits, const uint32_t* __restrict__ woff,
                                                  uint64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t pi = P[i];
    uint64_t l = 0;
    if (pi != kNoParent) {
        const uint32_t r = tc_find(P, pi);
        const uint64_t below = (r & 63u) ? (bits[r >> 6] & ((1ull << (r & 63u)) - 1ull)) : 0ull;
        l = (uint64_t)woff[r >> 6] + (uint64_t)__popcll(below) + 1ull;
    }
    out[i] = l;
}

}  // namespace ctws
