// k_cc.hip — local maxima seeds, connected components and vigra-scan-order numbering.
//
// Reference: watershed.py:179-207 (_make_seeds: localMaxima[3D](allowPlateaus,
// allowAtBorder) -> labelMultiArrayWithBackground), watershed.py:326-341 (halo crop,
// labelVolumeWithBackground, uint64 id offset), :310-321 (empty block).
//
// Numbering.  vigra numbers components 1..k by their first voxel in vigra scan order,
// which for a plain numpy array is the F-order index (axis 0 fastest).  The union-find
// parent arrays here are therefore keyed by the F-order key
//     3-D: f = z + Z*(y + Y*x)        2-D (per slice): f = z*Y*X + (y + Y*x)
// and union links the larger root under the smaller, so every root is its component's
// first voxel.  The label of a root is 1 + (number of roots with a smaller key), read from
// a per-block bitmap of roots (1 bit per key) and its per-word exclusive prefix.
#include "ctws_kernels.h"

namespace ctws {

#define BLOCK_LOOP(i, B)                                                                      \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).N;              \
         i += (int64_t)gridDim.x * blockDim.x)

// ---- local maxima classification ---------------------------------------------------------
// cls bit0: a neighbour is strictly greater; bit1: a neighbour is equal (plateau voxel).
// Neighbourhood: 6 (3-D ws) or 8 in-plane (2-D ws), as localMaxima3D / localMaxima.
__global__ void __launch_bounds__(256) k_localmax(const BlockDesc* __restrict__ D, BlockStat* S,
                                                  const float* __restrict__ v, uint8_t* __restrict__ cls) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int Y = B.Y, X = B.X;
    const int64_t YX = (int64_t)Y * X;
    const float* p = v + B.base;
    uint32_t nplat = 0;
    BLOCK_LOOP(i, B) {
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / X, x = rem - (rem / X) * X;
        const float c = p[i];
        bool gt = false, eq = false;
        auto chk = [&](int64_t j) {
            const float w = p[j];
            gt |= w > c;
            eq |= w == c;
        };
        if (B.nd_ws == 3) {
            if (z > 0) chk(i - YX);
            if (z + 1 < B.Z) chk(i + YX);
            if (y > 0) chk(i - X);
            if (y + 1 < Y) chk(i + X);
            if (x > 0) chk(i - 1);
            if (x + 1 < X) chk(i + 1);
        } else {
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (!dy && !dx) continue;
                    const int yy = y + dy, xx = x + dx;
                    if (yy < 0 || yy >= Y || xx < 0 || xx >= X) continue;
                    chk(i + dy * X + dx);
                }
        }
        cls[B.base + i] = (uint8_t)((gt ? 1 : 0) | (eq ? 2 : 0));
        nplat += eq;
    }
    if (nplat) atomicAdd(&S[blockIdx.y].plateau, nplat);
}

// ---- plateau resolution: CC of equal values over plateau voxels (C-order keys) -----------
__global__ void __launch_bounds__(256) k_plateau_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      const uint8_t* __restrict__ cls, uint32_t* __restrict__ P) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !S[blockIdx.y].plateau) return;
    BLOCK_LOOP(i, B) {
        if (cls[B.base + i] & 2) P[B.base + i] = (uint32_t)i;
    }
}

__global__ void __launch_bounds__(256) k_plateau_union(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                       const float* __restrict__ v, const uint8_t* __restrict__ cls,
                                                       uint32_t* __restrict__ Pg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !S[blockIdx.y].plateau) return;
    const int Y = B.Y, X = B.X;
    const int64_t YX = (int64_t)Y * X;
    const float* p = v + B.base;
    const uint8_t* cl = cls + B.base;
    uint32_t* P = Pg + B.base;
    BLOCK_LOOP(i, B) {
        if (!(cl[i] & 2)) continue;
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / X, x = rem - (rem / X) * X;
        const float c = p[i];
        auto un = [&](int64_t j) {
            if (p[j] == c) uf_union(P, (uint32_t)i, (uint32_t)j);
        };
        if (B.nd_ws == 3) {
            if (z > 0) un(i - YX);
            if (y > 0) un(i - X);
            if (x > 0) un(i - 1);
        } else {
            if (y > 0) {
                if (x > 0) un(i - X - 1);
                un(i - X);
                if (x + 1 < X) un(i - X + 1);
            }
            if (x > 0) un(i - 1);
        }
    }
}

// mark roots of plateaus that touch a strictly greater value (cls bit2 on the root)
__global__ void __launch_bounds__(256) k_plateau_flag(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      uint8_t* __restrict__ cls, uint32_t* __restrict__ Pg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !S[blockIdx.y].plateau) return;
    uint8_t* cl = cls + B.base;
    uint32_t* P = Pg + B.base;
    BLOCK_LOOP(i, B) {
        const uint8_t c = cl[i];
        if ((c & 3) == 3) {
            const uint32_t r = uf_find_compress(P, (uint32_t)i);
            cl[r] |= 4;  // benign race: every writer sets the same bit
        }
    }
}

// is voxel i a local maximum?
__device__ __forceinline__ bool is_max(const uint8_t* cl, const uint32_t* P, int64_t i) {
    const uint8_t c = cl[i];
    if (c & 1) return false;
    if (!(c & 2)) return true;
    return !(cl[uf_find(P, (uint32_t)i)] & 4);
}

// F-order key helpers
__device__ __forceinline__ uint32_t fkey3(int z, int y, int x, int Z, int Y) {
    return (uint32_t)(z + Z * (y + Y * x));
}

// ---- seed CC: init / union over maxima voxels (direct nbhd; in-plane in 2-D) -------------
// PF is keyed by F-order key.  Background keys get kNoParent so the bitmap sees no root.
__global__ void __launch_bounds__(256) k_seed_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   const uint8_t* __restrict__ cls, const uint32_t* __restrict__ Pp,
                                                   uint32_t* __restrict__ PF) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int Y = B.Y, X = B.X, Z = B.Z;
    const int64_t YX = (int64_t)Y * X;
    const uint8_t* cl = cls + B.base;
    const uint32_t* P = Pp + B.base;
    BLOCK_LOOP(i, B) {
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / X, x = rem - (rem / X) * X;
        const uint32_t f = (B.nd_ws == 3) ? fkey3(z, y, x, Z, Y) : (uint32_t)(z * YX + y + Y * x);
        PF[B.base + f] = is_max(cl, P, i) ? f : kNoParent;
    }
}

__global__ void __launch_bounds__(256) k_seed_union(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    uint32_t* __restrict__ PFg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int Y = B.Y, X = B.X, Z = B.Z;
    const int64_t YX = (int64_t)Y * X;
    uint32_t* PF = PFg + B.base;
    BLOCK_LOOP(i, B) {
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / X, x = rem - (rem / X) * X;
        if (B.nd_ws == 3) {
            const uint32_t f = fkey3(z, y, x, Z, Y);
            if (PF[f] == kNoParent) continue;
            if (z > 0 && PF[f - 1] != kNoParent) uf_union(PF, f, f - 1);
            if (y > 0 && PF[f - Z] != kNoParent) uf_union(PF, f, f - Z);
            if (x > 0 && PF[f - Z * Y] != kNoParent) uf_union(PF, f, f - (uint32_t)(Z * Y));
        } else {
            const uint32_t f = (uint32_t)(z * YX + y + Y * x);
            if (PF[f] == kNoParent) continue;
            if (y > 0 && PF[f - 1] != kNoParent) uf_union(PF, f, f - 1);
            if (x > 0 && PF[f - Y] != kNoParent) uf_union(PF, f, f - Y);
        }
    }
}

// ---- root bitmap + exclusive prefix -----------------------------------------------------
// keys per block: n = N (seeds, outer) or NI (crop, inner); words = n/64 + 1, chunks of 256
// words.  inner != 0 selects NI and the inner-sized parent array offset (ibase).
__global__ void __launch_bounds__(256) k_bitmap(const BlockDesc* __restrict__ D, const BlockStat* S, int inner,
                                                const uint32_t* __restrict__ PFg, uint64_t* __restrict__ Wg,
                                                uint32_t* __restrict__ csum) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || (inner && !B.crop)) return;
    const int64_t n = inner ? B.NI : B.N;
    const int64_t nw = n / 64 + 1;
    if ((int64_t)blockIdx.x * 256 >= nw) return;
    const uint32_t* PF = PFg + (inner ? B.ibase : B.base);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // each wave builds 64 words; one word = ballot over 64 consecutive keys (coalesced)
    uint32_t c = 0;
    for (int j = 0; j < 64; ++j) {
        const int64_t w = (int64_t)blockIdx.x * 256 + wv * 64 + j;
        if (w >= nw) break;
        const int64_t f = w * 64 + lane;
        const bool root = f < n && PF[f] == (uint32_t)f;
        const uint64_t bits = __ballot(root);
        if (lane == 0) Wg[B.wbase + w] = bits;
        c += (uint32_t)__popcll(bits);
    }
    __shared__ uint32_t red[4];
    if (lane == 0) red[wv] = c;
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
        else S[blockIdx.x].n_cc = carry;
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

// ---- seed labels + flood initialisation --------------------------------------------------
// labels = vigra label (| kFixedBit: seed), keys = (ordf(h) << 32) for seeds, INF otherwise.
__global__ void __launch_bounds__(256) k_seed_label(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const uint32_t* __restrict__ PFg, const uint64_t* __restrict__ Wg,
                                                    const uint32_t* __restrict__ Wpg, const float* __restrict__ h,
                                                    uint32_t* __restrict__ lab, uint64_t* __restrict__ key,
                                                    uint8_t* __restrict__ fixedv, int packed) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int Y = B.Y, X = B.X, Z = B.Z;
    const int64_t YX = (int64_t)Y * X;
    const uint32_t* PF = PFg + B.base;
    const uint64_t* W = Wg + B.wbase;
    const uint32_t* Wp = Wpg + B.wbase;
    BLOCK_LOOP(i, B) {
        const int z = (int)(i / YX);
        const int rem = (int)(i - z * YX);
        const int y = rem / X, x = rem - (rem / X) * X;
        const uint32_t f = (B.nd_ws == 3) ? fkey3(z, y, x, Z, Y) : (uint32_t)(z * YX + y + Y * x);
        uint32_t l = 0;
        uint64_t k = kInfKey;
        if (PF[f] != kNoParent) {
            const uint32_t r = uf_find(PF, f);
            const uint32_t lr = bitmap_rank(W, Wp, r) + 1u;
            l = lr | kFixedBit;
            k = ((uint64_t)ordf(h[B.base + i]) << 32) | (packed ? (uint64_t)lr : 0ull);
        }
        lab[B.base + i] = l;
        key[B.base + i] = k;
        fixedv[B.base + i] = l ? 1 : 0;
    }
}

// ---- halo crop CC (labelVolumeWithBackground, 6-nbhd, equal values, bg 0) -----------------
__device__ __forceinline__ void inner_coords(const BlockDesc& B, int64_t i, int& z, int& y, int& x) {
    const int64_t yx = (int64_t)B.IY * B.IX;
    z = (int)(i / yx);
    const int rem = (int)(i - z * yx);
    y = rem / B.IX;
    x = rem - y * B.IX;
}
__device__ __forceinline__ int64_t outer_of_inner(const BlockDesc& B, int z, int y, int x) {
    return ((int64_t)(z + B.iz0) * B.Y + (y + B.iy0)) * B.X + (x + B.ix0);
}

#define INNER_LOOP(i, B)                                                                      \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).NI;             \
         i += (int64_t)gridDim.x * blockDim.x)

__global__ void __launch_bounds__(256) k_crop_init(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                   const uint32_t* __restrict__ ws, uint32_t* __restrict__ PFg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !B.crop) return;
    uint32_t* PF = PFg + B.ibase;
    INNER_LOOP(i, B) {
        int z, y, x;
        inner_coords(B, i, z, y, x);
        const uint32_t f = fkey3(z, y, x, B.IZ, B.IY);
        PF[f] = ws[B.base + outer_of_inner(B, z, y, x)] ? f : kNoParent;
    }
}

__global__ void __launch_bounds__(256) k_crop_union(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    const uint32_t* __restrict__ ws, uint32_t* __restrict__ PFg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || !B.crop) return;
    uint32_t* PF = PFg + B.ibase;
    const uint32_t* w = ws + B.base;
    INNER_LOOP(i, B) {
        int z, y, x;
        inner_coords(B, i, z, y, x);
        const int64_t o = outer_of_inner(B, z, y, x);
        const uint32_t v = w[o];
        if (!v) continue;
        const uint32_t f = fkey3(z, y, x, B.IZ, B.IY);
        if (z > 0 && w[o - (int64_t)B.Y * B.X] == v) uf_union(PF, f, f - 1);
        if (y > 0 && w[o - B.X] == v) uf_union(PF, f, f - B.IZ);
        if (x > 0 && w[o - 1] == v) uf_union(PF, f, f - (uint32_t)(B.IZ * B.IY));
    }
}

// ---- uint64 output: (crop CC label | ws) + id offset on in-mask voxels ---------------------
__global__ void __launch_bounds__(256) k_output(const BlockDesc* __restrict__ D, BlockStat* S,
                                                const uint32_t* __restrict__ ws, const uint32_t* __restrict__ PFg,
                                                const uint64_t* __restrict__ Wg, const uint32_t* __restrict__ Wpg) {
    const BlockDesc& B = D[blockIdx.y];
    const bool active = S[blockIdx.y].active;
    uint32_t mx = 0;
    INNER_LOOP(i, B) {
        int z, y, x;
        inner_coords(B, i, z, y, x);
        const int64_t o = outer_of_inner(B, z, y, x);
        const bool inm = !B.mask || B.mask[o];
        uint64_t v;
        if (!active) {
            v = 0;  // empty block: constant offset (watershed.py:310-321)
        } else {
            uint32_t l = ws[B.base + o];
            if (B.crop && l) {
                const uint32_t r = uf_find(PFg + B.ibase, fkey3(z, y, x, B.IZ, B.IY));
                l = bitmap_rank(Wg + B.wbase, Wpg + B.wbase, r) + 1u;
            }
            mx = max(mx, l);
            v = l;
        }
        B.out[i] = inm ? v + B.id_offset : v;
    }
    for (int s = 32; s > 0; s >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, s));
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(&S[blockIdx.y].max_label, mx);
}

}  // namespace ctws

namespace ctws {
// point every element of a union-find forest directly at its root
__global__ void __launch_bounds__(256) k_flatten(const BlockDesc* __restrict__ D, const BlockStat* S, int inner,
                                                 uint32_t* __restrict__ PFg) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || (inner && !B.crop)) return;
    const int64_t n = inner ? B.NI : B.N;
    uint32_t* PF = PFg + (inner ? B.ibase : B.base);
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n; f += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = PF[f];
        if (p != kNoParent && p != (uint32_t)f) PF[f] = uf_find(PF, p);
    }
}
}  // namespace ctws
