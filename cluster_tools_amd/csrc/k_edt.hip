// k_edt.hip — _read_data/normalize, threshold and the exact Euclidean distance transform.
//
// Reference: cluster_tools/watershed/watershed.py:267-282 (_read_data), :139-160 (_apply_dt),
// utils/volume_utils.py:113-120 (normalize); vigra.filters.distanceTransform
// (separableMultiDistSquared).  For integer pixel pitch and dmax < 2^24 the squared
// distances are exact integers, so any exact separable EDT reproduces vigra bit for bit:
//   pass x : 1-D distance to the nearest foreground voxel on the row   (wave-level scans)
//   pass y : min_y' g(y') + p_y^2 (y - y')^2, LDS-staged columns, bounded search
//   pass z : same along z, then min(d2, ceil(dmax)) and sqrtf (correctly rounded)
// HBM traffic per outer voxel: x-pass reads the input (4 B f32 / 1 B u8) and writes the
// normalized input (4 B) and g^2 (4 B); y and z passes read 4 B and write 4 B each.
#include "ctws_kernels.h"

namespace ctws {

__device__ __forceinline__ float load_raw(const void* p, int dtype, int64_t i) {
    switch (dtype) {
        case 1: return (float)((const uint8_t*)p)[i];
        case 2: return (float)((const uint16_t*)p)[i];
        case 3: return ((const float*)p)[i];
        default: return (float)((const double*)p)[i];
    }
}

// ---- per-block min / max of the raw input over the channel range (normalize) -----------
__global__ void __launch_bounds__(256) k_input_minmax(const BlockDesc* __restrict__ D, BlockStat* S) {
    const BlockDesc& B = D[blockIdx.y];
    const int64_t n = (int64_t)B.C * B.N;
    const int64_t off = (int64_t)B.c0 * B.N;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t o = ordf(load_raw(B.input, B.dtype, off + i));
        mn = min(mn, o);
        mx = max(mx, o);
    }
    for (int s = 32; s > 0; s >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, s));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, s));
    }
    __shared__ uint32_t rmn[4], rmx[4];
    if ((threadIdx.x & 63) == 0) {
        rmn[threadIdx.x >> 6] = mn;
        rmx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomic_min_if(&S[blockIdx.y].in_min, min(min(rmn[0], rmn[1]), min(rmn[2], rmn[3])));
        atomic_max_if(&S[blockIdx.y].in_max, max(max(rmx[0], rmx[1]), max(rmx[2], rmx[3])));
    }
}

// ---- normalized input + threshold + EDT pass along x --------------------------------
// One wave per row (z, y).  fin = normalize(input) [channel agg, invert, mask -> 1];
// g2 = p_x^2 * (distance to the nearest voxel with fin > threshold on the row)^2.

__global__ void __launch_bounds__(256) k_prep_edt_x(const BlockDesc* __restrict__ D, BlockStat* S, PrepParams pp,
                                                    float* __restrict__ fin, uint32_t* __restrict__ g2) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    const BlockDesc& B = D[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    if (row >= (int64_t)B.Z * B.Y) return;
    const int X = B.X;
    int* sdist = smem_i + wave * X;  // per-wave row buffer: fg flag, then right distance
    const float mn = unordf(S[blockIdx.y].in_min);
    const float den = unordf(S[blockIdx.y].in_max) - mn;  // max(x - min) == max - min (monotone rounding)
    const int64_t rbase = row * X;
    uint32_t fgcount = 0;
    auto ld = [&](int x) -> float {
        const int64_t i = rbase + x;
        float v;
        if (B.n_channels == 0) {
            v = load_raw(B.input, B.dtype, i) - mn;
            if (den > 0.0f) v = v / den;
        } else {
            const int64_t cs = B.N;
            const int64_t o0 = (int64_t)B.c0 * cs + i;
            v = load_raw(B.input, B.dtype, o0) - mn;
            if (den > 0.0f) v = v / den;
            for (int c = 1; c < B.C; ++c) {
                float w = load_raw(B.input, B.dtype, o0 + c * cs) - mn;
                if (den > 0.0f) w = w / den;
                if (pp.agg == 0) v = v + w;
                else if (pp.agg == 1) v = fmaxf(v, w);
                else v = fminf(v, w);
            }
            if (pp.agg == 0) v = v / (float)B.C;
        }
        if (pp.invert) v = 1.0f - v;
        if (B.mask && !B.mask[i]) v = 1.0f;
        return v;
    };
    staged_loop<8>(lane, X, 64, ld, [&](int x, float v) {
        fin[B.base + rbase + x] = v;
        const int f = v > pp.threshold;
        sdist[x] = f;
        fgcount += f;
    });
    // any foreground in the block? (_apply_dt: np.sum(threshd) == 0 -> None)
    if (__ballot(fgcount != 0) != 0ull && lane == 0 && !*(volatile uint32_t*)&S[blockIdx.y].fg)
        atomicOr(&S[blockIdx.y].fg, 1u);
    __builtin_amdgcn_wave_barrier();
    // chunk per lane: [lane*K, lane*K + K)
    const int K = (X + 63) >> 6;
    const int x0 = lane * K, x1 = min(X, x0 + K);
    int last = -1, first = 0x3FFFFFFF;
    for (int x = x0; x < x1; ++x)
        if (sdist[x]) {
            last = x;
            if (first == 0x3FFFFFFF) first = x;
        }
    // exclusive max-scan of `last` from the left, exclusive min-scan of `first` from the right
    int lp = last, rn = first;
    for (int s = 1; s < 64; s <<= 1) {
        int a = __shfl_up(lp, s);
        if (lane >= s) lp = max(lp, a);
        int b = __shfl_down(rn, s);
        if (lane + s < 64) rn = min(rn, b);
    }
    int left = __shfl_up(lp, 1);
    if (lane == 0) left = -1;
    int right = __shfl_down(rn, 1);
    if (lane == 63) right = 0x3FFFFFFF;
    // backward over the lane's chunk: the distance to the nearest fg at or after x (0 exactly at
    // the fg voxels), in place; then forward: the nearer of that and the last fg before x
    {
        int r = right;
        for (int x = x1 - 1; x >= x0; --x) {
            if (sdist[x]) r = x;
            sdist[x] = (r >= 0x3FFFFFFF) ? 0x3FFFFFFF : r - x;
        }
        int l = left;
        for (int x = x0; x < x1; ++x) {
            int d = sdist[x];
            if (d == 0) l = x;
            d = min(d, (l < 0) ? 0x3FFFFFFF : x - l);
            sdist[x] = (d >= 0x3FFFFFFF) ? (int)kInfD2 : pp.px2 * d * d;
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int x = lane; x < X; x += 64) g2[B.base + rbase + x] = (uint32_t)sdist[x];
}

// Register variant (X <= 64 * KMAX): lane l owns the K = ceil(X / 64) consecutive voxels
// [l K, l K + K) of the row, so the nearest-foreground scans need no LDS: per-lane first/last
// foreground, then wave-level exclusive max/min scans, then the lane's own K distances.  f32
// rows of exactly 64 K voxels move as float4 / uint4 (16 B per lane per access).  Same results
// as k_prep_edt_x.
template <int KMAX>
__global__ void __launch_bounds__(256) k_prep_edt_x_reg(const BlockDesc* __restrict__ D, BlockStat* S, PrepParams pp,
                                                        float* __restrict__ fin, uint32_t* __restrict__ g2) {
    const BlockDesc& B = D[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    if (row >= (int64_t)B.Z * B.Y) return;
    const int X = B.X;
    const int K = (X + 63) >> 6;
    const float mn = unordf(S[blockIdx.y].in_min);
    const float den = unordf(S[blockIdx.y].in_max) - mn;  // max(x - min) == max - min (monotone rounding)
    const int64_t rbase = row * X;
    const int x0 = lane * K;
    float v[KMAX];
    const bool vec = (KMAX % 4 == 0) && K == KMAX && X == 64 * KMAX && B.n_channels == 0 && B.dtype == 3 &&
                     ((((uintptr_t)B.input) | (uintptr_t)(B.base * 4)) & 15u) == 0u;
    if (vec) {
        const float4* src = (const float4*)((const float*)B.input + rbase + x0);
#pragma unroll
        for (int q = 0; q < KMAX / 4; ++q) {
            const float4 t = src[q];
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            float a = v[k] - mn;
            if (den > 0.0f) a = a / den;
            if (pp.invert) a = 1.0f - a;
            if (B.mask && !B.mask[rbase + x0 + k]) a = 1.0f;
            v[k] = a;
        }
    } else {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            v[k] = 0.0f;
            const int x = x0 + k;
            if (k < K && x < X) {
                const int64_t i = rbase + x;
                float a;
                if (B.n_channels == 0) {
                    a = load_raw(B.input, B.dtype, i) - mn;
                    if (den > 0.0f) a = a / den;
                } else {
                    const int64_t cs = B.N;
                    const int64_t o0 = (int64_t)B.c0 * cs + i;
                    a = load_raw(B.input, B.dtype, o0) - mn;
                    if (den > 0.0f) a = a / den;
                    for (int c = 1; c < B.C; ++c) {
                        float w = load_raw(B.input, B.dtype, o0 + c * cs) - mn;
                        if (den > 0.0f) w = w / den;
                        if (pp.agg == 0) a = a + w;
                        else if (pp.agg == 1) a = fmaxf(a, w);
                        else a = fminf(a, w);
                    }
                    if (pp.agg == 0) a = a / (float)B.C;
                }
                if (pp.invert) a = 1.0f - a;
                if (B.mask && !B.mask[i]) a = 1.0f;
                v[k] = a;
            }
        }
    }
    // foreground bits of the lane's voxels, first / last foreground
    uint32_t fg = 0u;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
        if (k < K && x0 + k < X && v[k] > pp.threshold) fg |= 1u << k;
    // any foreground in the block? (_apply_dt: np.sum(threshd) == 0 -> None)
    if (__ballot(fg != 0u) != 0ull && lane == 0 && !*(volatile uint32_t*)&S[blockIdx.y].fg)
        atomicOr(&S[blockIdx.y].fg, 1u);
    int lp = fg ? x0 + 31 - __builtin_clz(fg) : -1;
    int rn = fg ? x0 + __builtin_ctz(fg) : 0x3FFFFFFF;
    // exclusive max-scan of `last` from the left, exclusive min-scan of `first` from the right
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
        const int a = __shfl_up(lp, s2);
        if (lane >= s2) lp = max(lp, a);
        const int b = __shfl_down(rn, s2);
        if (lane + s2 < 64) rn = min(rn, b);
    }
    int left = __shfl_up(lp, 1);
    if (lane == 0) left = -1;
    int right = __shfl_down(rn, 1);
    if (lane == 63) right = 0x3FFFFFFF;
    uint32_t out[KMAX];
    {
        int r = right;
#pragma unroll
        for (int k = KMAX - 1; k >= 0; --k) {
            const int x = x0 + k;
            if ((fg >> k) & 1u) r = x;
            out[k] = (uint32_t)((r >= 0x3FFFFFFF) ? 0x3FFFFFFF : r - x);
        }
        int l = left;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int x = x0 + k;
            if ((fg >> k) & 1u) l = x;
            const int dl = (l < 0) ? 0x3FFFFFFF : x - l;
            const int d = min((int)out[k], dl);
            out[k] = (d >= 0x3FFFFFFF) ? kInfD2 : (uint32_t)(pp.px2 * d * d);
        }
    }
    if (vec) {
        float4* fo = (float4*)(fin + B.base + rbase + x0);
        uint4* go = (uint4*)(g2 + B.base + rbase + x0);
#pragma unroll
        for (int q = 0; q < KMAX / 4; ++q) {
            fo[q] = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            go[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            const int x = x0 + k;
            if (k < K && x < X) {
                fin[B.base + rbase + x] = v[k];
                g2[B.base + rbase + x] = out[k];
            }
        }
    }
}
template __global__ void k_prep_edt_x_reg<4>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
template __global__ void k_prep_edt_x_reg<8>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
template __global__ void k_prep_edt_x_reg<16>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);

// Coalesced variant (X <= 64 * KMAX): lane l owns the voxels x = 64 k + l of the row, so every
// load and store of a wave covers 64 consecutive voxels (a row of 576 voxels is 9 fully
// coalesced 256-B accesses instead of 9 accesses strided by 36 B per lane).  The raw input
// type is a template parameter and the loads are unconditional (clamped x) global loads, so
// all KMAX loads of a lane are in flight together.  The foreground bits of each 64-voxel
// segment k are one ballot, mk[k] (wave-uniform); the nearest foreground to the left / right
// of x comes from mk[k] masked at the lane plus the last / first foreground of the segments
// before / after.  3-D datasets only (4-D inputs use k_prep_edt_x).  Same results as
// k_prep_edt_x.
template <int KMAX, class T>
__global__ void __launch_bounds__(256) k_prep_edt_x_co(const BlockDesc* __restrict__ D, BlockStat* S, PrepParams pp,
                                                       float* __restrict__ fin, uint32_t* __restrict__ g2) {
    const BlockDesc& B = D[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    if (row >= (int64_t)B.Z * B.Y) return;
    const int X = B.X;
    const int K = (X + 63) >> 6;
    const float mn = unordf(S[blockIdx.y].in_min);
    const float den = unordf(S[blockIdx.y].in_max) - mn;  // max(x - min) == max - min (monotone rounding)
    const int64_t rbase = row * X;
    const gptr_t<T> src = gbl((const T*)B.input) + rbase;
    const gptr_t<uint8_t> msk = B.mask ? gbl(B.mask) + rbase : nullptr;
    T raw[KMAX];
    uint8_t mv[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) raw[k] = src[min(64 * k + lane, X - 1)];
    if (msk) {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) mv[k] = msk[min(64 * k + lane, X - 1)];
    }
    uint64_t mk[KMAX];
    bool any = false;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int x = 64 * k + lane;
        const bool in = k < K && x < X;
        float a = (float)raw[k] - mn;
        if (den > 0.0f) a = a / den;
        if (pp.invert) a = 1.0f - a;
        if (msk && !mv[k]) a = 1.0f;
        if (in) fin[B.base + rbase + x] = a;
        mk[k] = __ballot(in && a > pp.threshold);
        any |= mk[k] != 0ull;
    }
    // any foreground in the block? (_apply_dt: np.sum(threshd) == 0 -> None)
    if (any && lane == 0 && !*(volatile uint32_t*)&S[blockIdx.y].fg) atomicOr(&S[blockIdx.y].fg, 1u);
    // last foreground at or before each segment, first at or after
    int lastk[KMAX], firstk[KMAX];
    {
        int l = -1;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (mk[k]) l = 64 * k + 63 - __builtin_clzll(mk[k]);
            lastk[k] = l;
        }
        int f = 0x3FFFFFFF;
#pragma unroll
        for (int k = KMAX - 1; k >= 0; --k) {
            if (mk[k]) f = 64 * k + __builtin_ctzll(mk[k]);
            firstk[k] = f;
        }
    }
    const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);  // bits <= lane
    const uint64_t ge = ~0ull << lane;                                    // bits >= lane
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int x = 64 * k + lane;
        const uint64_t ml = mk[k] & le, mr = mk[k] & ge;
        const int left = ml ? 64 * k + 63 - __builtin_clzll(ml) : (k > 0 ? lastk[k - 1] : -1);
        const int right = mr ? 64 * k + __builtin_ctzll(mr) : (k + 1 < KMAX ? firstk[k + 1] : 0x3FFFFFFF);
        const int dl = left < 0 ? 0x3FFFFFFF : x - left;
        const int dr = right >= 0x3FFFFFFF ? 0x3FFFFFFF : right - x;
        const int d = min(dl, dr);
        if (k < K && x < X) g2[B.base + rbase + x] = (d >= 0x3FFFFFFF) ? kInfD2 : (uint32_t)(pp.px2 * d * d);
    }
}
#define CTWS_PREP_CO(K)                                                                                \
    template __global__ void k_prep_edt_x_co<K, uint8_t>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);  \
    template __global__ void k_prep_edt_x_co<K, uint16_t>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*); \
    template __global__ void k_prep_edt_x_co<K, float>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);    \
    template __global__ void k_prep_edt_x_co<K, double>(const BlockDesc*, BlockStat*, PrepParams, float*, uint32_t*);
CTWS_PREP_CO(4)
CTWS_PREP_CO(8)
CTWS_PREP_CO(16)
#undef CTWS_PREP_CO

// per-block min / max of a 3-D input of type T: 8 global loads in flight per thread
template <class T>
__global__ void __launch_bounds__(256) k_input_minmax_t(const BlockDesc* __restrict__ D, BlockStat* S) {
    const BlockDesc& B = D[blockIdx.y];
    const gptr_t<T> src = gbl((const T*)B.input);
    const int64_t n = B.N;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    constexpr int U = 8;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride * U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[min(i0 + u * stride, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t o = ordf((float)v[u]);
            mn = min(mn, o);
            mx = max(mx, o);
        }
    }
    mn = wg_reduce_u32(mn, OpMin());
    mx = wg_reduce_u32(mx, OpMax());
    if (threadIdx.x == 0) {
        atomic_min_if(&S[blockIdx.y].in_min, mn);
        atomic_max_if(&S[blockIdx.y].in_max, mx);
    }
}
template __global__ void k_input_minmax_t<uint8_t>(const BlockDesc*, BlockStat*);
template __global__ void k_input_minmax_t<uint16_t>(const BlockDesc*, BlockStat*);
template __global__ void k_input_minmax_t<float>(const BlockDesc*, BlockStat*);
template __global__ void k_input_minmax_t<double>(const BlockDesc*, BlockStat*);

// Correctly rounded sqrtf of an integer n < 2^24 (vigra: sqrt on the float32 dest).  The
// hardware v_sqrt_f32 is not correctly rounded, so round a double sqrt to float and fix it
// with exact arithmetic: the float r is correct iff mid(r-,r)^2 < n < mid(r,r+)^2 (midpoints
// have <= 25 significant bits, so their squares are exact in double; no ties for n < 2^24).
// correctly rounded sqrt of a float >= 0 (v_sqrt_f32, what __fsqrt_rn lowers to, is not):
// the double sqrt rounded to float, corrected by the exact midpoint tests (the midpoint of two
// floats has 25 significant bits, its square 50: exact in double)
__device__ __forceinline__ float sqrt_rn_f(float x) {
    float r = (float)__dsqrt_rn((double)x);
    const double dx = (double)x;
    const float up = __uint_as_float(__float_as_uint(r) + 1u);
    const double mhi = 0.5 * ((double)r + (double)up);
    if (mhi * mhi < dx) return up;
    if (r > 0.0f) {
        const float lo = __uint_as_float(__float_as_uint(r) - 1u);
        const double mlo = 0.5 * ((double)r + (double)lo);
        if (mlo * mlo > dx) return lo;
    }
    return r;
}

// correctly rounded sqrtf of an integer n < 2^24 without double arithmetic: v_sqrt_f32 (1 ulp)
// gives r, the correctly rounded value is r - 1 ulp, r or r + 1 ulp, chosen by exact integer tests
// of the midpoints.  r = R 2^-k (R the 24-bit significand): the upper midpoint is (2R + 1)
// 2^-(k+1), below sqrt(n) iff (2R + 1)^2 < n 2^(2k+2); both sides are about 4 R^2 < 2^50.
__device__ __forceinline__ float sqrt_rn_int(uint32_t n) {
    if (n == 0u) return 0.0f;
    const float r = __builtin_amdgcn_sqrtf((float)n);  // n < 2^24: exact conversion
    const uint32_t bits = __float_as_uint(r);
    const uint64_t R = (uint64_t)((bits & 0x7FFFFFu) | 0x800000u);
    const int k = 150 - (int)(bits >> 23);  // r = R 2^-k, 12 <= k <= 23 for 1 <= n < 2^24
    const uint64_t n4 = (uint64_t)n << (2 * k + 2);
    if ((2 * R + 1) * (2 * R + 1) < n4) return __uint_as_float(bits + 1u);
    // lower midpoint: (2R - 1) 2^-(k+1), or (2^25 - 1) 2^-(k+2) when r is a power of two
    const bool pow2 = R == 0x800000ull;
    const uint64_t ml = pow2 ? (1ull << 25) - 1ull : 2 * R - 1;
    if (ml * ml > (pow2 ? n4 << 2 : n4)) return __uint_as_float(bits - 1u);
    return r;
}

// device self-check of sqrt_rn_int over [n0, n0 + count) (tests: every n < 2^24 against the
// correctly rounded float sqrt)
__global__ void __launch_bounds__(256) k_sqrt_int_check(uint32_t n0, uint32_t count, float* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < count) out[i] = sqrt_rn_int(n0 + i);
}

// ---- EDT pass along y (stride X) or z (stride Y*X), LDS-staged columns -----------------
// Tile: the full line (length L) x W consecutive x positions.  Bounded search:
//   best = g[p]; for r = 1.. while p2 r^2 < best: best = min(best, g[p +- r] + p2 r^2)
// exact (no candidate farther than sqrt(best / p2) can win) and O(distance) per voxel, which on
// boundary maps is a handful of LDS reads.  A voxel still searching after kEdtSearchCap steps
// (a line with no or far-away foreground) stops; its column is queued and k_edt_col_fh redoes
// the column with the Felzenszwalb-Huttenlocher lower envelope of parabolas, O(L) per column
// whatever the distances.  Capped voxels stay out of the dt statistics (k_edt_col_fh adds
// its column's).
// FINAL: clamp to maxDist = ceil(dmax) and write sqrtf(d2) as float, with dt statistics.

template <int W>
__global__ void __launch_bounds__(256) k_edt_col(const BlockDesc* __restrict__ D, BlockStat* S, EdtColParams ep,
                                                 const uint32_t* __restrict__ gin, uint32_t* __restrict__ gout,
                                                 float* __restrict__ dt, uint32_t* __restrict__ slice_min,
                                                 uint32_t* __restrict__ slice_max, unsigned long long* fh_list,
                                                 uint32_t* fh_cnt) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    uint32_t* col = (uint32_t*)smem_i;
    __shared__ unsigned long long capped_cols;  // bit c: a voxel of column c hit kEdtSearchCap
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int nxc = (B.X + W - 1) / W;
    const int L = (ep.axis == 1) ? B.Y : B.Z;
    const int other = (ep.axis == 1) ? B.Z : B.Y;  // the line index that is not x
    const int t = blockIdx.x;
    if (t >= other * nxc) return;
    const int o = t / nxc, xc = t % nxc;
    const int xb = xc * W;
    const int64_t lstride = (ep.axis == 1) ? B.X : (int64_t)B.Y * B.X;
    const int64_t obase = (ep.axis == 1) ? (int64_t)o * B.Y * B.X : (int64_t)o * B.X;
    const int c = threadIdx.x % W;
    const int r0 = threadIdx.x / W;
    constexpr int RS = 256 / W;
    const bool colok = xb + c < B.X;
    {
        const uint32_t* gsrc = gin + B.base + obase + xb + (colok ? c : 0);
        staged_loop<8>(
            r0, L, RS, [&](int p) { return colok ? gsrc[p * lstride] : kInfD2; },
            [&](int p, uint32_t v) { col[p * W + c] = v; });
    }
    if (threadIdx.x == 0) capped_cols = 0ull;
    __syncthreads();
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    const uint32_t maxd = ep.per_slice ? (uint32_t)(B.Y * B.Y + B.X * B.X) : B.maxd;
    bool capped_any = false;
    const uint32_t p2 = (uint32_t)ep.p2;
    for (int p = r0; p < L; p += RS) {
        uint32_t best = col[p * W + c];
        // radii r and r + 1 per step: four LDS reads in flight (clamped index, INF outside the
        // line; INF + p2 r^2 < 2^31 never wins)
        const int rlim = max(p, L - 1 - p);  // no candidates beyond
        const int rcap = min(rlim, kEdtSearchCap);
        int r = 1;
        for (; r <= rcap; r += 2) {
            const uint32_t rr0 = p2 * (uint32_t)(r * r);
            if (rr0 >= best) break;
            const uint32_t rr1 = p2 * (uint32_t)((r + 1) * (r + 1));
            const uint32_t a = col[max(p - r, 0) * W + c], b = col[min(p + r, L - 1) * W + c];
            const uint32_t a1 = col[max(p - r - 1, 0) * W + c], b1 = col[min(p + r + 1, L - 1) * W + c];
            const uint32_t m0 = min(p - r >= 0 ? a : kInfD2, p + r < L ? b : kInfD2);
            const uint32_t m1 = min(p - r - 1 >= 0 ? a1 : kInfD2, p + r + 1 < L ? b1 : kInfD2);
            best = min(best, min(m0 + rr0, m1 + rr1));
        }
        const bool capped = r <= rlim && p2 * (uint32_t)(r * r) < best;
        if (!colok) continue;
        capped_any |= capped;
        const int64_t gi = B.base + obase + p * lstride + xb + c;
        if (ep.final_pass && capped) {
            // k_edt_col_fh rewrites the column
        } else if (ep.final_pass) {
            const uint32_t d2 = min(best, maxd);
            const float v = sqrt_rn_int(d2);
            dt[gi] = v;
            const uint32_t ov = ordf(v);
            mn = min(mn, ov);
            mx = max(mx, ov);
        } else {
            gout[gi] = best;
        }
    }
    if (capped_any) atomicOr(&capped_cols, 1ull << c);
    __syncthreads();
    if (threadIdx.x < W && ((capped_cols >> threadIdx.x) & 1ull)) {
        const uint32_t e = atomicAdd(fh_cnt, 1u);
        fh_list[e] = ((unsigned long long)blockIdx.y << 48) | ((unsigned long long)o << 24) |
                     (unsigned long long)(xb + threadIdx.x);
    }
    if (ep.final_pass) {
        // workgroup reduce, then per block (3-D ws) and per slice (2-D dt: o is z)
        __shared__ uint32_t rmn[4], rmx[4];
        for (int s = 32; s > 0; s >>= 1) {
            mn = min(mn, (uint32_t)__shfl_xor((int)mn, s));
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, s));
        }
        const int wv = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            rmn[wv] = mn;
            rmx[wv] = mx;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            mn = min(min(rmn[0], rmn[1]), min(rmn[2], rmn[3]));
            mx = max(max(rmx[0], rmx[1]), max(rmx[2], rmx[3]));
            atomic_min_if(&S[blockIdx.y].dt_min, mn);
            atomic_max_if(&S[blockIdx.y].dt_max, mx);
            if (ep.axis == 1) {
                atomic_min_if(&slice_min[B.sbase + o], mn);
                atomic_max_if(&slice_max[B.sbase + o], mx);
            }
        }
    }
}

#define CTWS_EDT_COL(W)                                                                                          \
    template __global__ void k_edt_col<W>(const BlockDesc*, BlockStat*, EdtColParams, const uint32_t*, uint32_t*,   \
                                          float*, uint32_t*, uint32_t*, unsigned long long*, uint32_t*);
CTWS_EDT_COL(64)
CTWS_EDT_COL(32)
CTWS_EDT_COL(16)
CTWS_EDT_COL(8)
#undef CTWS_EDT_COL

// floor(a / b) for b > 0
__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// Columns queued by k_edt_col: the exact 1-D squared distance transform of the line by the lower
// envelope of the parabolas p2 (u - s)^2 + g[s] over the finite g[s] (Felzenszwalb-Huttenlocher,
// in Meijster's integer form: parabola u takes over from the stack top s at
// w = 1 + floor((p2 (u^2 - s^2) + g[u] - g[s]) / (2 p2 (u - s)))).  One thread per column.  The
// stack (s | t << 16 per entry, t = first position of the entry's interval) lives in the
// column's own output cells: entry k sits at position k <= t[k] <= u, so the backward pass
// reads an entry before the output of its position is written.  Same values as the bounded
// search (min over all finite g of g[s] + p2 (u - s)^2, kInfD2 on an all-INF line).
__global__ void __launch_bounds__(256) k_edt_col_fh(const BlockDesc* __restrict__ D, BlockStat* S, EdtColParams ep,
                                                    const uint32_t* __restrict__ gin, uint32_t* gout, float* dt,
                                                    uint32_t* __restrict__ slice_min, uint32_t* __restrict__ slice_max,
                                                    const unsigned long long* __restrict__ fh_list,
                                                    const uint32_t* __restrict__ fh_cnt) {
    const uint32_t n = *fh_cnt;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const unsigned long long ent = fh_list[e];
        const int bi = (int)(ent >> 48), o = (int)((ent >> 24) & 0xFFFFFFull), x = (int)(ent & 0xFFFFFFull);
        const BlockDesc& B = D[bi];
        const int L = (ep.axis == 1) ? B.Y : B.Z;
        const int64_t lstride = (ep.axis == 1) ? B.X : (int64_t)B.Y * B.X;
        const int64_t obase = (ep.axis == 1) ? (int64_t)o * B.Y * B.X : (int64_t)o * B.X;
        const int64_t cb = B.base + obase + x;
        const uint32_t* g = gin + cb;
        uint32_t* stk = (ep.final_pass ? (uint32_t*)dt : gout) + cb;
        const int64_t p2 = ep.p2;
        int q = -1, s_top = 0, t_top = 0;
        int64_t g_top = 0;
        for (int u = 0; u < L; ++u) {
            const uint32_t gu32 = g[u * lstride];
            if (gu32 >= kInfD2) continue;
            const int64_t gu = gu32;
            while (q >= 0) {
                const int64_t fs = p2 * (int64_t)(t_top - s_top) * (t_top - s_top) + g_top;
                const int64_t fu = p2 * (int64_t)(t_top - u) * (t_top - u) + gu;
                if (fs <= fu) break;
                if (--q >= 0) {
                    const uint32_t wd = stk[q * lstride];
                    s_top = (int)(wd & 0xFFFFu);
                    t_top = (int)(wd >> 16);
                    g_top = g[s_top * lstride];
                }
            }
            if (q < 0) {
                q = 0;
                s_top = u;
                t_top = 0;
                g_top = gu;
                stk[0] = (uint32_t)u;
            } else {
                const int64_t num = p2 * ((int64_t)u * u - (int64_t)s_top * s_top) + gu - g_top;
                const int64_t w = 1 + floor_div(num, 2 * p2 * (u - s_top));
                if (w < L) {
                    ++q;
                    s_top = u;
                    t_top = (int)w;
                    g_top = gu;
                    stk[q * lstride] = (uint32_t)u | ((uint32_t)w << 16);
                }
            }
        }
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;
        const uint32_t maxd = ep.per_slice ? (uint32_t)(B.Y * B.Y + B.X * B.X) : B.maxd;
        for (int u = L - 1; u >= 0; --u) {
            uint32_t best = kInfD2;
            if (q >= 0) {
                best = (uint32_t)min(p2 * (int64_t)(u - s_top) * (u - s_top) + g_top, (int64_t)kInfD2);
                if (u == t_top && --q >= 0) {
                    const uint32_t wd = stk[q * lstride];
                    s_top = (int)(wd & 0xFFFFu);
                    t_top = (int)(wd >> 16);
                    g_top = g[s_top * lstride];
                }
            }
            if (ep.final_pass) {
                const float v = sqrt_rn_int(min(best, maxd));
                dt[cb + u * lstride] = v;
                const uint32_t ov = ordf(v);
                mn = min(mn, ov);
                mx = max(mx, ov);
            } else {
                gout[cb + u * lstride] = best;
            }
        }
        if (ep.final_pass) {
            atomic_min_if(&S[bi].dt_min, mn);
            atomic_max_if(&S[bi].dt_max, mx);
            if (ep.axis == 1) {
                atomic_min_if(&slice_min[B.sbase + o], mn);
                atomic_max_if(&slice_max[B.sbase + o], mx);
            }
        }
    }
}

// per-slice min / max of dt (2-D ws on a 3-D dt): one workgroup per slice chunk
__global__ void __launch_bounds__(256) k_dt_slice_stats(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                        const float* __restrict__ dt, uint32_t* slice_min,
                                                        uint32_t* slice_max) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int z = blockIdx.x;
    if (z >= B.Z) return;
    const int64_t n = (int64_t)B.Y * B.X;
    const float* p = dt + B.base + (int64_t)z * n;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t o = ordf(p[i]);
        mn = min(mn, o);
        mx = max(mx, o);
    }
    for (int s = 32; s > 0; s >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, s));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, s));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&slice_min[B.sbase + z], mn);
        atomicMax(&slice_max[B.sbase + z], mx);
    }
}

}  // namespace ctws

namespace ctws {
// =========================================================================================
// vigra's real-valued distance path, for the configurations the exact integer kernels above do
// not cover: a non-integer pixel_pitch (watershed.py:157-158; vigra then works on a temporary
// array, T = double) and dmax >= 2^24 (squared distances are no longer exact integers in the
// float32 destination vigra works on directly, T = float).  separableMultiDistSquared: init
// f = (fg ? 0 : maxDist), then per axis 0, 1, 2 (2-D dt: y, x) detail::distParabola on every
// line with sigma = pitch[axis] -- the same double expressions in the same order as the
// restatement in oracle/ctws_oracle.cpp (dist_parabola), so the result is bit-identical -- then
// sqrt in float.  One thread per line, its parabola stack in a global scratch (element k of
// thread t at k * nthr + t); the few blocks that need this are not a throughput path.
// =========================================================================================
template <class T>
__global__ void __launch_bounds__(256) k_edt_real_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                       EdtRealParams ep, const uint32_t* __restrict__ xd2,
                                                       T* __restrict__ tmp) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    double dmax;
    if (ep.per_slice) dmax = (double)B.Y * B.Y + (double)B.X * B.X;
    else {
        const double a = ep.pitch[0] * B.Z, b = ep.pitch[1] * B.Y, c = ep.pitch[2] * B.X;
        dmax = a * a + b * b + c * c;
    }
    // real pitch: (Real)dmax; integer pitch (float destination): DestType(ceil(dmax))
    const T maxd = ep.real ? (T)dmax : (T)ceil(dmax);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.N; i += (int64_t)gridDim.x * blockDim.x)
        tmp[B.base + i] = xd2[B.base + i] == 0u ? (T)0 : maxd;  // x pass: 0 exactly at the foreground
}

template <class T>
__global__ void __launch_bounds__(256) k_edt_real_line(const BlockDesc* __restrict__ D, const BlockStat* S, int nb,
                                                       EdtRealParams ep, int axis, T* __restrict__ arr,
                                                       char* __restrict__ scratch, int max_len) {
    const int nthr = gridDim.x * blockDim.x;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    // scratch: line (T), left (double), right (double), apex values (T), centers (int)
    T* sline = (T*)scratch;
    double* sleft = (double*)(scratch + (size_t)nthr * max_len * sizeof(T));
    double* sright = sleft + (size_t)nthr * max_len;
    T* sval = (T*)(sright + (size_t)nthr * max_len);
    int* scen = (int*)(sval + (size_t)nthr * max_len);
    const double sigma = ep.per_slice ? 1.0 : ep.pitch[axis];
    const double sigma2 = sigma * sigma, sigma22 = 2.0 * sigma2;
    for (int bi = 0; bi < nb; ++bi) {
        const BlockDesc& B = D[bi];
        if (!S[bi].active) continue;
        const int L = axis == 0 ? B.Z : (axis == 1 ? B.Y : B.X);
        const int64_t lstride = axis == 0 ? (int64_t)B.Y * B.X : (axis == 1 ? B.X : 1);
        const int64_t nlines = B.N / L;
        for (int64_t ln = t; ln < nlines; ln += nthr) {
            int64_t base;
            if (axis == 0) base = ln;  // (y, x)
            else if (axis == 1) base = (ln / B.X) * (int64_t)B.Y * B.X + ln % B.X;  // (z, x)
            else base = ln * B.X;  // (z, y)
            T* a = arr + B.base + base;
            auto LN = [&](int i) -> T& { return sline[(size_t)i * nthr + t]; };
            auto LF = [&](int k) -> double& { return sleft[(size_t)k * nthr + t]; };
            auto RT = [&](int k) -> double& { return sright[(size_t)k * nthr + t]; };
            auto PV = [&](int k) -> T& { return sval[(size_t)k * nthr + t]; };
            auto CN = [&](int k) -> int& { return scen[(size_t)k * nthr + t]; };
            for (int i = 0; i < L; ++i) LN(i) = a[i * lstride];
            const double w = (double)L;
            int top = 0;
            LF(0) = 0.0;
            CN(0) = 0;
            RT(0) = w;
            PV(0) = LN(0);
            double current = 1.0;
            for (int is = 1; is < L; ++is, current += 1.0) {
                double intersection;
                while (true) {
                    const double diff = current - (double)CN(top);
                    intersection = current + ((double)(LN(is) - PV(top)) - sigma2 * (diff * diff)) / (sigma22 * diff);
                    if (intersection < LF(top)) {
                        if (--top < 0) {  // the stack ran empty
                            intersection = 0.0;
                            break;
                        }
                        continue;
                    } else if (intersection < RT(top)) {
                        RT(top) = intersection;
                    }
                    break;
                }
                ++top;
                LF(top) = intersection;
                CN(top) = is;
                RT(top) = w;
                PV(top) = LN(is);
            }
            int it = 0;
            double cur = 0.0;
            for (int o = 0; o < L; ++o, cur += 1.0) {
                while (cur >= RT(it)) ++it;
                const double diff = cur - (double)CN(it);
                a[o * lstride] = (T)(sigma2 * (diff * diff) + (double)PV(it));
            }
        }
    }
}

template <class T>
__global__ void __launch_bounds__(256) k_edt_real_final(const BlockDesc* __restrict__ D, BlockStat* S, EdtRealParams ep,
                                                        const T* __restrict__ tmp, float* __restrict__ dt,
                                                        uint32_t* __restrict__ slice_min, uint32_t* __restrict__ slice_max) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    uint32_t mn = 0xFFFFFFFFu, mx = 0u;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.N; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = sqrt_rn_f((float)tmp[B.base + i]);
        dt[B.base + i] = v;
        const uint32_t o = ordf(v);
        mn = min(mn, o);
        mx = max(mx, o);
        if (ep.per_slice) {
            const int z = (int)(i / YX);
            atomic_min_if(&slice_min[B.sbase + z], o);
            atomic_max_if(&slice_max[B.sbase + z], o);
        }
    }
    mn = wg_reduce_u32(mn, OpMin());
    mx = wg_reduce_u32(mx, OpMax());
    if (threadIdx.x == 0) {
        atomic_min_if(&S[blockIdx.y].dt_min, mn);
        atomic_max_if(&S[blockIdx.y].dt_max, mx);
    }
}

#define CTWS_EDT_REAL(T)                                                                                          \
    template __global__ void k_edt_real_init<T>(const BlockDesc*, const BlockStat*, EdtRealParams, const uint32_t*, \
                                                T*);                                                               \
    template __global__ void k_edt_real_line<T>(const BlockDesc*, const BlockStat*, int, EdtRealParams, int, T*, char*, \
                                                int);                                                              \
    template __global__ void k_edt_real_final<T>(const BlockDesc*, BlockStat*, EdtRealParams, const T*, float*,      \
                                                 uint32_t*, uint32_t*);
CTWS_EDT_REAL(float)
CTWS_EDT_REAL(double)
#undef CTWS_EDT_REAL
}  // namespace ctws

namespace ctws {
// a block takes part in the pipeline iff something is above the threshold (_apply_dt)
__global__ void k_set_active(const BlockDesc* __restrict__ D, BlockStat* S, int n) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n) S[b].active = S[b].fg != 0u;
}
}  // namespace ctws
