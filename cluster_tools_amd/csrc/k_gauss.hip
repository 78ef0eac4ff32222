// k_gauss.hip — vigra gaussianSmoothing, bit-exact, and the height map.
//
// Reference: utils/volume_utils.py:95-109 (apply_filter -> vigra.filters.gaussianSmoothing),
// watershed.py:163-169 (_make_hmap), :187-192 (seed map smoothing).
// vigra semantics restated (Kernel1D::initGaussian + convolveLine, BORDER_TREATMENT_REFLECT):
//   out[x] = float( sum_{p = x-r}^{x+r} k[x-p] * (double) in[reflect(p)] )
// accumulated in double, ascending p, separate multiply and add (this file is compiled with
// -ffp-contract=off: no FMA contraction), float32 between axes, axes in order z, y, x.
// The taps are computed on the host with the same libm exp() call vigra makes.
// One pass reads 4 B and writes 4 B per voxel; the first pass of the hmap smoothing reads
// fin and dt instead (8 B) and computes hmap = a*fin + b*(1 - normalize(dt)) on the fly.
#include "ctws_kernels.h"

namespace ctws {


// hmap value of voxel i (local index), slice z
__device__ __forceinline__ float hmap_value(const BlockDesc& B, const BlockStat& S, const HmapParams& hp,
                                            const float* fin, const float* dt, const uint32_t* smin,
                                            const uint32_t* smax, int64_t i, int z) {
    float mn, mx;
    if (hp.per_slice) {
        mn = unordf(smin[B.sbase + z]);
        mx = unordf(smax[B.sbase + z]);
    } else {
        mn = unordf(S.dt_min);
        mx = unordf(S.dt_max);
    }
    const float den = mx - mn;
    float d = dt[B.base + i] - mn;
    if (den > 0.0f) d = d / den;
    d = 1.0f - d;
    const float t1 = hp.a * fin[B.base + i];
    const float t2 = hp.b * d;
    return t1 + t2;
}

// plain hmap (no smoothing of the weights)
__global__ void __launch_bounds__(256) k_hmap(const BlockDesc* __restrict__ D, const BlockStat* S, HmapParams hp,
                                              const float* __restrict__ fin, const float* __restrict__ dt,
                                              const uint32_t* smin, const uint32_t* smax, float* __restrict__ out) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t yx = (int64_t)B.Y * B.X;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.N; i += (int64_t)gridDim.x * blockDim.x)
        out[B.base + i] = hmap_value(B, S[blockIdx.y], hp, fin, dt, smin, smax, i, (int)(i / yx));
}


__device__ __forceinline__ int reflect_idx(int p, int L) {
    return p < 0 ? -p : (p >= L ? 2 * (L - 1) - p : p);
}

// Column pass (axis z or y): tile = full line (L) x W consecutive x positions in LDS.
template <int W>
__global__ void __launch_bounds__(256) k_gauss_col(const BlockDesc* __restrict__ D, const BlockStat* S, GaussParams gp,
                                                   HmapParams hp, const double* __restrict__ taps,
                                                   const float* __restrict__ in, const float* __restrict__ dt,
                                                   const uint32_t* smin, const uint32_t* smax,
                                                   float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    double* k = (double*)smem_i;                        // 2r+1 taps (<= 128)
    float* col = (float*)(smem_i + 2 * 128);
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int nxc = (B.X + W - 1) / W;
    const int L = (gp.axis == 1) ? B.Y : B.Z;
    const int other = (gp.axis == 1) ? B.Z : B.Y;
    const int t = blockIdx.x;
    if (t >= other * nxc) return;
    const int o = t / nxc, xc = t % nxc;
    const int xb = xc * W;
    const int64_t lstride = (gp.axis == 1) ? B.X : (int64_t)B.Y * B.X;
    const int64_t obase = (gp.axis == 1) ? (int64_t)o * B.Y * B.X : (int64_t)o * B.X;
    const int c = threadIdx.x % W;
    const int r0 = threadIdx.x / W;
    constexpr int RS = 256 / W;
    const int ntap = 2 * gp.r + 1;
    for (int j = threadIdx.x; j < ntap; j += 256) k[j] = taps[j];
    const bool colok = xb + c < B.X;
    if (gp.hmap_src) {
        const BlockStat& st = S[blockIdx.y];
        staged_loop<8>(
            r0, L, RS,
            [&](int p) {
                const int64_t li = obase + p * lstride + xb + (colok ? c : 0);
                return hmap_value(B, st, hp, in, dt, smin, smax, li, (gp.axis == 1) ? o : p);
            },
            [&](int p, float v) { col[p * W + c] = colok ? v : 0.0f; });
    } else {
        const float* gsrc = in + B.base + obase + xb + (colok ? c : 0);
        staged_loop<8>(
            r0, L, RS, [&](int p) { return gsrc[p * lstride]; },
            [&](int p, float v) { col[p * W + c] = colok ? v : 0.0f; });
    }
    __syncthreads();
    if (!colok) return;
    const int r = gp.r;
    for (int p = r0; p < L; p += RS) {
        double sum = 0.0;
        if (p >= r && p + r < L) {
            for (int q = p - r, j = 2 * r; j >= 0; ++q, --j) sum += k[j] * (double)col[q * W + c];
        } else {
            for (int q = p - r, j = 2 * r; j >= 0; ++q, --j) sum += k[j] * (double)col[reflect_idx(q, L) * W + c];
        }
        out[B.base + obase + p * lstride + xb + c] = (float)sum;
    }
}

template __global__ void k_gauss_col<32>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*,
                                         const float*, const float*, const uint32_t*, const uint32_t*, float*);
template __global__ void k_gauss_col<16>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*,
                                         const float*, const float*, const uint32_t*, const uint32_t*, float*);
template __global__ void k_gauss_col<8>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams, const double*,
                                        const float*, const float*, const uint32_t*, const uint32_t*, float*);

// Row pass (axis x, contiguous): 4 rows per workgroup, one wave per row, row in LDS.
__global__ void __launch_bounds__(256) k_gauss_row(const BlockDesc* __restrict__ D, const BlockStat* S, GaussParams gp,
                                                   HmapParams hp, const double* __restrict__ taps,
                                                   const float* __restrict__ in, const float* __restrict__ dt,
                                                   const uint32_t* smin, const uint32_t* smax,
                                                   float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    double* k = (double*)smem_i;
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int X = B.X;
    float* rowb = (float*)(smem_i + 2 * 128) + wave * X;
    const int ntap = 2 * gp.r + 1;
    for (int j = threadIdx.x; j < ntap; j += 256) k[j] = taps[j];
    const int64_t row = (int64_t)blockIdx.x * 4 + wave;
    const bool rowok = row < (int64_t)B.Z * B.Y;
    const int64_t rbase = row * X;
    if (rowok) {
        const int z = (int)(row / B.Y);
        if (gp.hmap_src) {
            const BlockStat& st = S[blockIdx.y];
            staged_loop<8>(
                lane, X, 64, [&](int x) { return hmap_value(B, st, hp, in, dt, smin, smax, rbase + x, z); },
                [&](int x, float v) { rowb[x] = v; });
        } else {
            const float* gsrc = in + B.base + rbase;
            staged_loop<8>(lane, X, 64, [&](int x) { return gsrc[x]; }, [&](int x, float v) { rowb[x] = v; });
        }
    }
    __syncthreads();
    if (!rowok) return;
    const int r = gp.r;
    for (int x = lane; x < X; x += 64) {
        double sum = 0.0;
        if (x >= r && x + r < X) {
            for (int q = x - r, j = 2 * r; j >= 0; ++q, --j) sum += k[j] * (double)rowb[q];
        } else {
            for (int q = x - r, j = 2 * r; j >= 0; ++q, --j) sum += k[j] * (double)rowb[reflect_idx(q, X)];
        }
        out[B.base + rbase + x] = (float)sum;
    }
}

}  // namespace ctws
