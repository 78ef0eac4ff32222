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
    const double* k = taps;                             // 2r+1 taps (any radius: read through the cache)
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
    const double* k = taps;  // 2r+1 taps (any radius: read through the cache)
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int X = B.X;
    float* rowb = (float*)(smem_i + 2 * 128) + wave * X;
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

// =========================================================================================
// Sliding-window variants for radius R <= kGaussMaxR (compile time).  A thread computes a run
// of consecutive outputs and keeps the 2R+1 inputs of the current output in registers, already
// converted to double: per output one LDS read + one conversion instead of 2R+1 of each, and
// the taps sit in registers.  The arithmetic (double products summed over ascending source
// positions, separate multiply and add) is exactly that of the generic kernels above.
// =========================================================================================
template <int R>
__device__ __forceinline__ void load_taps(const double* __restrict__ taps, double (&k)[2 * R + 1]) {
#pragma unroll
    for (int j = 0; j <= 2 * R; ++j) k[j] = taps[j];
}

// out[p] for p in [p0, p1) from src(i) (i in [0, L), reflect border), written via put(p, v)
template <int R, class Src, class Put>
__device__ __forceinline__ void gauss_run(const double (&k)[2 * R + 1], int L, int p0, int p1, Src src, Put put) {
    double win[2 * R + 1];
#pragma unroll
    for (int m = 0; m <= 2 * R; ++m) win[m] = (double)src(reflect_idx(p0 - R + m, L));
    for (int p = p0; p < p1; ++p) {
        double sum = 0.0;
#pragma unroll
        for (int m = 0; m <= 2 * R; ++m) sum += k[2 * R - m] * win[m];
        put(p, (float)sum);
#pragma unroll
        for (int m = 0; m < 2 * R; ++m) win[m] = win[m + 1];
        win[2 * R] = (double)src(reflect_idx(p + 1 + R, L));
    }
}

template <int W, int R>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_gauss_col_r(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     GaussParams gp, HmapParams hp, const double* __restrict__ taps,
                                                     const float* __restrict__ in, const float* __restrict__ dt,
                                                     const uint32_t* smin, const uint32_t* smax,
                                                     float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    float* col = (float*)smem_i;
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
    double k[2 * R + 1];
    load_taps<R>(taps, k);
    __syncthreads();
    if (!colok) return;
    const int seg = (L + RS - 1) / RS;
    const int p0 = r0 * seg, p1 = min(L, p0 + seg);
    if (p0 >= p1) return;
    float* gdst = out + B.base + obase + xb + c;
    gauss_run<R>(
        k, L, p0, p1, [&](int i) { return col[i * W + c]; }, [&](int p, float v) { gdst[p * lstride] = v; });
}

// Row pass: a lane computes a run of kRowSeg consecutive x; a wave holds 64 / ceil(X / kRowSeg)
// rows.  The rows sit in LDS with one pad word per run (stride kRowSeg + 1: no bank
// conflicts); outputs go back through LDS so the global stores are coalesced.
constexpr int kRowSeg = 16;
constexpr int kRowWaveFloats = 64 * (kRowSeg + 1) + 64;  // per wave and buffer

__host__ __device__ constexpr int gauss_rows_per_wave(int X) { return 64 / ((X + kRowSeg - 1) / kRowSeg); }

template <int R>
__global__ void __launch_bounds__(256) k_gauss_row_r(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                     GaussParams gp, HmapParams hp, const double* __restrict__ taps,
                                                     const float* __restrict__ in, const float* __restrict__ dt,
                                                     const uint32_t* smin, const uint32_t* smax,
                                                     float* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) int smem_i[];
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int X = B.X;
    const int lpr = (X + kRowSeg - 1) / kRowSeg;  // lanes per row
    const int rpw = 64 / lpr;                      // rows per wave
    const int pitch = X + X / kRowSeg + 1;         // padded row length in LDS
    float* rowb = (float*)smem_i + wave * 2 * kRowWaveFloats;
    float* outb = rowb + kRowWaveFloats;
    auto pos = [&](int x) { return x + x / kRowSeg; };
    const int64_t nrows = (int64_t)B.Z * B.Y;
    const int64_t row0 = ((int64_t)blockIdx.x * 4 + wave) * rpw;
    if (row0 >= nrows) return;
    const int nr = (int)min((int64_t)rpw, nrows - row0);
    // stage nr rows (lane-strided, coalesced)
    const int nval = nr * X;
    if (gp.hmap_src) {
        const BlockStat& st = S[blockIdx.y];
        staged_loop<8>(
            lane, nval, 64,
            [&](int v) {
                const int rr = v / X, x = v - rr * X;
                const int64_t row = row0 + rr;
                return hmap_value(B, st, hp, in, dt, smin, smax, row * X + x, (int)(row / B.Y));
            },
            [&](int v, float val) {
                const int rr = v / X, x = v - rr * X;
                rowb[rr * pitch + pos(x)] = val;
            });
    } else {
        const float* gsrc = in + B.base + row0 * X;
        staged_loop<8>(
            lane, nval, 64, [&](int v) { return gsrc[v]; },
            [&](int v, float val) {
                const int rr = v / X, x = v - rr * X;
                rowb[rr * pitch + pos(x)] = val;
            });
    }
    double k[2 * R + 1];
    load_taps<R>(taps, k);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int rr = lane / lpr, sidx = lane - rr * lpr;
    if (rr < nr) {
        const int p0 = sidx * kRowSeg, p1 = min(X, p0 + kRowSeg);
        const float* rb = rowb + rr * pitch;
        float* ob = outb + rr * pitch;
        if (p0 < p1)
            gauss_run<R>(
                k, X, p0, p1, [&](int i) { return rb[pos(i)]; }, [&](int p, float v) { ob[pos(p)] = v; });
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float* gdst = out + B.base + row0 * X;
    for (int v = lane; v < nval; v += 64) {
        const int r2 = v / X, x = v - r2 * X;
        gdst[v] = outb[r2 * pitch + pos(x)];
    }
}

// =========================================================================================
// Fused y + x passes on a 2-D tile of one slice (both axes with radius R).  The separate
// passes write the y-smoothed volume to HBM and read it back (16 B per voxel for the pair);
// here the y result stays in LDS (as float, exactly the rounding between axes vigra does), so
// a pair costs 4 B in + 4 B out per voxel plus halo re-reads (mostly L2 hits).
//   tile: kYxTY rows x (128 - 2R) columns of outputs; the LDS window is (kYxTY + 2R) x 128,
//   rows/columns outside the block reflected at staging, so both passes read plain LDS.
//   y pass: thread = (column, half of the rows), a 16-output sliding window per thread;
//   x pass: thread = (row, eighth of the row); outputs go back through LDS for coalesced
//   stores.  Arithmetic per output as gauss_run: double products over ascending positions.
// Tiles of one XCD are contiguous (blockIdx round-robins over the 8 XCDs), so vertically
// adjacent tiles that share halo rows share an L2.
// =========================================================================================
constexpr int kYxTY = kGaussYxTY;
constexpr int kYxP = 129;  // LDS pitch: 128 + 1

__host__ __device__ constexpr int gauss_yx_tx(int R) { return 128 - 2 * R; }

template <int R>
__global__ void __launch_bounds__(256) k_gauss_yx(const BlockDesc* __restrict__ D, const BlockStat* S, int hmap_src,
                                                  HmapParams hp, const double* __restrict__ taps_y,
                                                  const double* __restrict__ taps_x, const float* __restrict__ in,
                                                  const float* __restrict__ dt, const uint32_t* smin,
                                                  const uint32_t* smax, float* __restrict__ out) {
    constexpr int TX = gauss_yx_tx(R);
    static_assert(kYxTY == 32, "the x pass maps 8 threads to each of the 32 tile rows");
    constexpr int NROW = kYxTY + 2 * R;
    constexpr int NL = NROW / 2;  // staged rows per thread
    __shared__ float win_s[NROW * kYxP];
    const BlockDesc& B = D[blockIdx.y];
    const BlockStat& st = S[blockIdx.y];
    if (!st.active) return;
    const int Y = B.Y, X = B.X;
    const int ntx = (X + TX - 1) / TX, nty = (Y + kYxTY - 1) / kYxTY;
    // XCD-contiguous tile order
    const int n = gridDim.x, per = n >> 3;
    const int bid = blockIdx.x;
    const int t = bid < (per << 3) ? (bid & 7) * per + (bid >> 3) : bid;
    if (t >= B.Z * nty * ntx) return;
    const int z = t / (nty * ntx), rem = t - z * (nty * ntx);
    const int y0 = (rem / ntx) * kYxTY, x0 = (rem % ntx) * TX;
    const int tid = threadIdx.x;
    const int c = tid & 127, half = tid >> 7;
    auto refl = [](int p, int L) { return min(max(reflect_idx(p, L), 0), L - 1); };
    const int64_t sbase = B.base + (int64_t)z * Y * X;
    const int gx = refl(x0 - R + c, X);
    // window rows and columns all inside the slice (the common case): no reflection, the row
    // addresses step by 2 X from one base (the kernel is VALU-bound: 806 FP64 mul / add per wave
    // and tile, and the reflected index arithmetic of the staging adds ~10 instructions per load).
    // A tile-uniform branch, so each path is one straight unrolled loop.
    const bool interior = y0 - R >= 0 && y0 + kYxTY + R <= Y && x0 - R >= 0 && x0 - R + 128 <= X;
    const int64_t ibase = sbase + (int64_t)(y0 - R + half) * X + (x0 - R + c);
    const int64_t X2 = 2 * (int64_t)X;
    auto gidx_in = [&](int i) -> int64_t { return ibase + i * X2; };
    auto gidx_refl = [&](int i) -> int64_t { return sbase + (int64_t)refl(y0 - R + 2 * i + half, Y) * X + gx; };
    // ---- stage: NL rows per thread, all loads in flight
    if (hmap_src) {
        float mn, mx;
        if (hp.per_slice) {
            mn = unordf(smin[B.sbase + z]);
            mx = unordf(smax[B.sbase + z]);
        } else {
            mn = unordf(st.dt_min);
            mx = unordf(st.dt_max);
        }
        const float den = mx - mn;
        float vf[NL], vd[NL];
        auto load2 = [&](auto gidx) {
#pragma unroll
            for (int i = 0; i < NL; ++i) {
                const int64_t gi = gidx(i);
                vf[i] = gbl(in)[gi];
                vd[i] = gbl(dt)[gi];
            }
        };
        if (interior) load2(gidx_in);
        else load2(gidx_refl);
#pragma unroll
        for (int i = 0; i < NL; ++i) {
            float d = vd[i] - mn;
            if (den > 0.0f) d = d / den;
            d = 1.0f - d;
            const float t1 = hp.a * vf[i];
            const float t2 = hp.b * d;
            win_s[(2 * i + half) * kYxP + c] = t1 + t2;
        }
    } else {
        float v[NL];
        auto load1 = [&](auto gidx) {
#pragma unroll
            for (int i = 0; i < NL; ++i) v[i] = gbl(in)[gidx(i)];
        };
        if (interior) load1(gidx_in);
        else load1(gidx_refl);
#pragma unroll
        for (int i = 0; i < NL; ++i) win_s[(2 * i + half) * kYxP + c] = v[i];
    }
    __syncthreads();
    // ---- y pass: column c, output rows [16 half, 16 half + 16)
    {
        double k[2 * R + 1];
        load_taps<R>(taps_y, k);
        const int p0 = half * (kYxTY / 2);
        double w[2 * R + 1];
#pragma unroll
        for (int m = 0; m < 2 * R; ++m) w[m] = (double)win_s[(p0 + m) * kYxP + c];
        float res[kYxTY / 2];
#pragma unroll
        for (int i = 0; i < kYxTY / 2; ++i) {
            w[(i + 2 * R) % (2 * R + 1)] = (double)win_s[(p0 + i + 2 * R) * kYxP + c];
            double sum = 0.0;
#pragma unroll
            for (int m = 0; m <= 2 * R; ++m) sum += k[2 * R - m] * w[(i + m) % (2 * R + 1)];
            res[i] = (float)sum;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kYxTY / 2; ++i) win_s[(p0 + i) * kYxP + c] = res[i];
    }
    __syncthreads();
    // ---- x pass: row p, columns [xs, xe) of the TX outputs
    constexpr int RUNX = (TX + 7) / 8;
    const int p = tid >> 3, j = tid & 7;
    const int xs = (j * TX) >> 3, xe = ((j + 1) * TX) >> 3;
    {
        double k[2 * R + 1];
        load_taps<R>(taps_x, k);
        const float* rb = win_s + p * kYxP + xs;
        double w[2 * R + 1];
#pragma unroll
        for (int m = 0; m < 2 * R; ++m) w[m] = (double)rb[m];
        float res[RUNX];
#pragma unroll
        for (int i = 0; i < RUNX; ++i) {
            // the phantom output of a short run reads at most column 128 (the pad word)
            w[(i + 2 * R) % (2 * R + 1)] = (double)rb[i + 2 * R];
            double sum = 0.0;
#pragma unroll
            for (int m = 0; m <= 2 * R; ++m) sum += k[2 * R - m] * w[(i + m) % (2 * R + 1)];
            res[i] = (float)sum;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < RUNX; ++i)
            if (xs + i < xe) win_s[p * kYxP + xs + i] = res[i];
    }
    __syncthreads();
    // ---- coalesced stores of the valid part of the tile (through LDS: storing each thread's
    // run from its registers measured 3.7 -> 6.1 ms per call on config 3 -- 64 lanes 14.5
    // voxels apart write partial lines)
    const int ny = min(kYxTY, Y - y0), nx = min(TX, X - x0);
    gwptr_t<float> o = gblw(out) + sbase + (int64_t)y0 * X + x0;
    for (int v = tid; v < kYxTY * TX; v += 256) {
        const int pp = v / TX, xx = v - pp * TX;
        if (pp < ny && xx < nx) o[(int64_t)pp * X + xx] = win_s[pp * kYxP + xx];
    }
}

#define CTWS_GAUSS_R(R)                                                                                          \
    template __global__ void k_gauss_yx<R>(const BlockDesc*, const BlockStat*, int, HmapParams, const double*,     \
                                           const double*, const float*, const float*, const uint32_t*,             \
                                           const uint32_t*, float*);                                               \
    template __global__ void k_gauss_col_r<32, R>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams,      \
                                                  const double*, const float*, const float*, const uint32_t*,       \
                                                  const uint32_t*, float*);                                        \
    template __global__ void k_gauss_col_r<16, R>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams,      \
                                                  const double*, const float*, const float*, const uint32_t*,       \
                                                  const uint32_t*, float*);                                        \
    template __global__ void k_gauss_col_r<8, R>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams,       \
                                                 const double*, const float*, const float*, const uint32_t*,        \
                                                 const uint32_t*, float*);                                         \
    template __global__ void k_gauss_row_r<R>(const BlockDesc*, const BlockStat*, GaussParams, HmapParams,          \
                                              const double*, const float*, const float*, const uint32_t*,           \
                                              const uint32_t*, float*);
CTWS_GAUSS_R(1)
CTWS_GAUSS_R(2)
CTWS_GAUSS_R(3)
CTWS_GAUSS_R(4)
CTWS_GAUSS_R(5)
CTWS_GAUSS_R(6)
CTWS_GAUSS_R(7)
CTWS_GAUSS_R(8)
CTWS_GAUSS_R(9)
CTWS_GAUSS_R(10)
CTWS_GAUSS_R(11)
CTWS_GAUSS_R(12)
#undef CTWS_GAUSS_R

}  // namespace ctws
