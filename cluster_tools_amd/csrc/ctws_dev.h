// ctws_dev.h — device-side data layout and helpers shared by the gfx950 kernels.
//
// A *batch* is a set of blocks processed by one pipeline of launches.  Every per-voxel
// workspace array is the concatenation of the blocks' outer volumes (BlockDesc::base), so
// one launch covers all blocks of the batch (grid.y = block).  Per-block scalars live in
// BlockStat, per-slice scalars in arrays indexed by BlockDesc::sbase + z.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ctws {

constexpr uint32_t kInfD2 = 0x3FFFFFFFu;             // "no foreground" squared distance
constexpr uint64_t kInfKey = 0xFFFFFFFFFFFFFFFFull;  // flood key of an unreached voxel
constexpr uint32_t kNoParent = 0xFFFFFFFFu;          // union-find: background
constexpr uint32_t kFixedBit = 0x80000000u;          // flood label: voxel is a seed
constexpr uint32_t kRootBit = 0x80000000u;           // CC parent slot of a labelled root
constexpr int kRows = 4;                             // rows per workgroup iteration (row tiles)
constexpr uint32_t kDescRes = 0x80000000u;           // descent exit entry resolved: | seed label (0: open)

struct BlockDesc {
    int Z, Y, X, nd_ws;     // outer shape; nd_ws = 2 (per-slice ws) or 3
    int64_t N;              // Z*Y*X
    int64_t base;           // offset into outer-sized arrays
    int iz0, iy0, ix0, crop;
    int IZ, IY, IX, _p0;
    int64_t NI;             // inner voxels
    int64_t ibase;          // offset into inner-sized arrays
    int64_t wbase;          // offset into bitmap-word arrays (words = N/64 + 1)
    int64_t cbase;          // offset into bitmap-chunk arrays
    int64_t sbase;          // offset into per-slice arrays (Z entries)
    const void* input;      // raw outer input (device)
    const uint8_t* mask;    // outer mask or nullptr
    const uint64_t* init;   // pass-2 initial seeds or nullptr
    uint64_t* out;          // inner uint64 output
    uint32_t* out32;        // host path: inner uint32 codes instead (the host widens them, see k_output)
    int n_channels, c0, C, dtype;
    uint64_t id_offset;     // block_id * prod(block_shape)
    int tz, ty, tx, tbase;  // flood tile grid, offset into per-tile arrays
    uint32_t maxd;          // 3-D EDT: ceil(dmax) = sum_k (pitch_k n_k)^2
    uint32_t pass2;         // 1: _ws_pass2 (two_pass_watershed.py:210-255)
    int64_t hbase;          // pass 2: offset into the relabel hash arrays
    int64_t hcap;           // pass 2: hash capacity of this block (power of two)
    int64_t fbase;          // offset into the frontier bitmaps (Z*Y rows of ceil(X/64) words)
    int64_t p2hint;         // pass 2 (2-D): offset of the block's per-slice offset hint (-1: none)
    int64_t xcbase;         // crop CC: offset of the block's tiles in CcArgs::xface
    int64_t ptbase;         // plateau CC: offset of the block's tile flags (CcArgs::ptile)
};

struct BlockStat {
    uint32_t in_min, in_max;  // ordered-float bits of the raw (float-cast) input
    uint32_t fg;              // number of voxels above threshold (saturating flag use)
    uint32_t dt_min, dt_max;  // ordered-float bits of dt over the outer block
    uint32_t plateau;         // voxels with an equal-valued maxima-neighbour
    uint32_t n_seeds;         // seed components
    uint32_t max_label;       // local max label (before the id offset)
    uint32_t active;          // block takes part in the remaining pipeline
    uint32_t n_cc;            // crop CC components
    uint32_t err;             // kErr* bits: the block cannot be finished (per-block failure)
    uint32_t n_auto;          // auto-seeded regrow: strict hmap minima of the seedless slices
    uint32_t _p[4];
    uint32_t dsat;            // packed flood: a key's hop distance d reached kDMax (note_dsat)
    uint32_t _u;              // 2-D seeds: plateau maxima listed by k_seed_members<2>
    uint32_t sf_sparse;       // size filter: the removed segments are walked, not scanned (k_sf_plan)
    uint32_t _q;
};

// BlockStat::err bits (a failed block does not fail its batch; the caller sees the status)
constexpr uint32_t kErrHashFull = 1u;    // pass 2: relabel hash table full
constexpr uint32_t kErrCollision = 2u;   // pass 2 (2-D): wrapped new id == initial id (unresolved)
constexpr uint32_t kErrLabelBits = 4u;   // auto-seeded regrow: labels beyond the 20-bit key field
constexpr uint32_t kErrTakeDict = 8u;    // pass 2: auto-seed label without a new_to_old entry
constexpr uint32_t kErrUnsupported = 16u; // (unused since round 6: the wide keys auto-seed their regrow too)
constexpr uint32_t kErrVerify = 64u;     // the regrow's fixpoint check failed (CTWS_VERIFY=1): labels not written
constexpr uint32_t kErrOverflow = 32u;    // WatershedFromSeeds: seed id >= 2^32 - 1 (the reference's assert)

// Pointers read from the block descriptor are generic to the compiler: accesses through them
// become flat loads, and the waits the compiler puts around flat accesses serialise a wave's
// loads.  gbl() asserts the global address space, so they are global loads that stay in flight.
template <class T>
using gptr_t = const T __attribute__((address_space(1)))*;
template <class T>
__device__ __forceinline__ gptr_t<T> gbl(const T* p) {
    return (gptr_t<T>)p;
}
template <class T>
using gwptr_t = T __attribute__((address_space(1)))*;
template <class T>
__device__ __forceinline__ gwptr_t<T> gblw(T* p) {
    return (gwptr_t<T>)p;
}

// order-preserving float <-> uint32 mapping (total order for non-NaN floats)
__device__ __forceinline__ uint32_t ordf(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordf(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// union-find on an F-order keyed parent array.  Roots keep the smallest key, so the root
// of a component is its first voxel in vigra scan order (dim 0 fastest).
__device__ __forceinline__ uint32_t uf_find(const uint32_t* P, uint32_t a) {
    // follows parent pointers to the root (roots point to themselves)
    uint32_t p = P[a];
    while (p != a) {
        a = p;
        p = P[a];
    }
    return a;
}
__device__ __forceinline__ uint32_t uf_find_compress(uint32_t* P, uint32_t a) {
    uint32_t r = a;
    uint32_t p = P[r];
    while (p != r) {
        r = p;
        p = P[r];
    }
    // path compression (benign races: every write stores an ancestor)
    while (true) {
        uint32_t n = P[a];
        if (n == r || n == a) break;
        P[a] = r;
        a = n;
    }
    return r;
}
// find with path halving for the unions: a non-root's parent becomes its grandparent on the
// way up (benign races: a non-root never becomes a root again and every store is an ancestor),
// so the chains the merges build over many tiles stay short for the later finds
__device__ __forceinline__ uint32_t uf_find_halve(uint32_t* P, uint32_t a) {
    while (true) {
        const uint32_t p = P[a];
        if (p == a) return a;
        const uint32_t gp = P[p];
        if (gp == p) return p;
        P[a] = gp;
        a = gp;
    }
}
__device__ __forceinline__ void uf_union(uint32_t* P, uint32_t a, uint32_t b) {
    while (true) {
        a = uf_find_halve(P, a);
        b = uf_find_halve(P, b);
        if (a == b) return;
        if (a > b) {
            uint32_t t = a;
            a = b;
            b = t;
        }
        uint32_t old = atomicCAS(&P[b], b, a);
        if (old == b) return;
        b = old;
    }
}

// LDS union-find of the tile CC kernels (k_tilecc.hip, k_threshcc.hip)
// find with path halving: a non-root's parent is replaced by its grandparent (always an
// ancestor with a smaller key, so concurrent finds and CAS links stay consistent)
__device__ __forceinline__ uint32_t lds_find(uint32_t* sp, uint32_t a) {
    uint32_t p = __atomic_load_n(&sp[a], __ATOMIC_RELAXED);
    while (p != a) {
        const uint32_t gp = __atomic_load_n(&sp[p], __ATOMIC_RELAXED);
        if (gp != p) __atomic_store_n(&sp[a], gp, __ATOMIC_RELAXED);
        a = gp;
        p = __atomic_load_n(&sp[a], __ATOMIC_RELAXED);
    }
    return a;
}
// link the root with the larger order key under the one with the smaller; parents are indexed
// by tile C-order position (consecutive lanes: consecutive LDS words, no bank conflicts), the
// order key of a position is key(position)
template <typename Key>
__device__ __forceinline__ void lds_union(uint32_t* sp, uint32_t a, uint32_t b, Key key) {
    while (true) {
        a = lds_find(sp, a);
        b = lds_find(sp, b);
        if (a == b) return;
        if (key(a) > key(b)) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        const uint32_t old = atomicCAS(&sp[b], b, a);
        if (old == b) return;
        b = old;
    }
}

// vigra scan key (F order, axis 0 fastest; per slice and slice-major in 2-D ws mode)
__device__ __forceinline__ uint32_t scan_key_of(const BlockDesc& B, int z, int y, int x) {
    return (B.nd_ws == 3) ? (uint32_t)(z + B.Z * (y + B.Y * x))
                          : (uint32_t)((int64_t)z * B.Y * B.X + y + (int64_t)B.Y * x);
}
// scan key of a C-order index (outer block, or the inner block when inner != 0: 3-D F order)
__device__ __forceinline__ uint32_t scan_key_idx(const BlockDesc& B, int inner, uint32_t c) {
    const int Y = inner ? B.IY : B.Y, X = inner ? B.IX : B.X;
    const uint32_t yx = (uint32_t)Y * (uint32_t)X;
    const int z = (int)(c / yx);
    const uint32_t rem = c - (uint32_t)z * yx;
    const int y = (int)(rem / (uint32_t)X);
    const int x = (int)(rem - (uint32_t)y * (uint32_t)X);
    if (inner) return (uint32_t)(z + B.IZ * (y + B.IY * x));
    return scan_key_of(B, z, y, x);
}

// union by scan key: the root with the smaller key becomes the parent, so every root is its
// component's first voxel in vigra scan order
__device__ __forceinline__ void uf_union_scan(uint32_t* P, uint32_t a, uint32_t b, const BlockDesc& B, int inner) {
    while (true) {
        a = uf_find_halve(P, a);
        b = uf_find_halve(P, b);
        if (a == b) return;
        if (scan_key_idx(B, inner, a) > scan_key_idx(B, inner, b)) {
            const uint32_t t = a;
            a = b;
            b = t;
        }
        const uint32_t old = atomicCAS(&P[b], b, a);
        if (old == b) return;
        b = old;
    }
}

// voxel i of block B (outer C index) in a per-row-word bitmap (the frontier layout at fbase).
// 32-bit division: a block holds fewer than 2^31 voxels (block_refusal), and the emulated 64-bit
// one is a long instruction sequence per call (the pass-2 relabel calls this per voxel)
__device__ __forceinline__ bool bit_of(const uint64_t* bits, const BlockDesc& B, int64_t i) {
    const uint32_t ii = (uint32_t)i;
    const uint32_t row = ii / (uint32_t)B.X;
    const int x = (int)(ii - row * (uint32_t)B.X);
    return (bits[B.fbase + (int64_t)row * ((B.X + 63) >> 6) + (x >> 6)] >> (x & 63)) & 1ull;
}

// label of a CC member from its parent slot p = P[i] after k_root_label (0: background)
__device__ __forceinline__ uint32_t cc_label(const uint32_t* P, uint32_t p) {
    if (p == kNoParent) return 0u;
    if (p & kRootBit) return p & ~kRootBit;
    return P[p] & ~kRootBit;
}

// ---- contention-free updates of per-block / per-slice scalars ------------------------------
// Same-address atomics serialise (~3 ns each): one per wave on a batch-wide scalar costs more
// than the streaming pass itself.  Reduce over the workgroup first (every thread must call),
// then one lane updates, and only when the (possibly stale, monotone) value does not cover it.
template <class Op>
__device__ __forceinline__ uint32_t wg_reduce_u32(uint32_t v, Op op) {
    for (int s = 32; s > 0; s >>= 1) v = op(v, (uint32_t)__shfl_xor((int)v, s));
    __shared__ uint32_t red[16];
    const int nw = (int)((blockDim.x + 63) >> 6);
    __syncthreads();  // red[] may still be read by a previous reduction
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    v = red[0];
    for (int k = 1; k < nw; ++k) v = op(v, red[k]);
    return v;
}
struct OpMax {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
struct OpMin {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; }
};
struct OpAdd {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
__device__ __forceinline__ void atomic_max_if(uint32_t* p, uint32_t v) {
    if (v > *(volatile uint32_t*)p) atomicMax(p, v);
}
__device__ __forceinline__ void atomic_min_if(uint32_t* p, uint32_t v) {
    if (v < *(volatile uint32_t*)p) atomicMin(p, v);
}

// Strided staging loop with U independent loads in flight: for p in [begin, end) step
// `step`, st(p, ld(p)).  A plain loop issues one load, waits for it and stores it (one
// memory latency per element); here the U loads of a batch are issued back to back.  The
// tail batch is predicated rather than a scalar loop, so a short range (a 256-voxel row read
// by one wave: 4 elements per lane) costs one memory latency, not one per element.
template <int U, class LoadF, class StoreF>
__device__ __forceinline__ void staged_loop(int begin, int end, int step, LoadF ld, StoreF st) {
    using T = decltype(ld(0));
    int p = begin;
    for (; p + (U - 1) * step < end; p += U * step) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld(p + u * step);
#pragma unroll
        for (int u = 0; u < U; ++u) st(p + u * step, v[u]);
    }
    if (p < end) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p + u * step < end) v[u] = ld(p + u * step);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (p + u * step < end) st(p + u * step, v[u]);
    }
}

// label of voxel i after the flood: from the packed key (packed flood), else from lab
__device__ __forceinline__ uint32_t flood_label(const uint32_t* lab, const uint64_t* key, int packed, int64_t i) {
    if (packed) {
        const uint64_t k = key[i];
        return k == kInfKey ? 0u : (uint32_t)(k & ((1ull << 20) - 1ull));
    }
    return lab[i] & ~kFixedBit;
}

// ---- XCD-aware workgroup order -----------------------------------------------------------
// Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch),
// each with its own L2: consecutive workgroup ids land on different L2s, so a stencil's
// neighbour rows are fetched from HBM once per XCD.  The bijective remap gives the workgroups
// that share an XCD (equal id % 8) one contiguous range of logical ids.  Speed only: any
// placement computes the same result.  Launches using it keep gridDim.x a multiple of 8 when
// grid.y > 1, so that id % 8 labels the XCD for every grid row.
__device__ __forceinline__ int xcd_swizzle(int b, int n) {
    const int xcd = b & 7, q = n >> 3, r = n & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// ---- word tiles --------------------------------------------------------------------------
// A wave handles one 64-voxel word of a row (lane = x - 64 * word), kWordWaves_ waves per
// workgroup; each wave takes a contiguous run of the block's Z * Y * ceil(X / 64) words (the
// rows above / below of a word were just read by the same wave: L1 / L2 hits) and the runs of
// the workgroups on one XCD are contiguous (xcd_swizzle).  Rows whose length is
// not a multiple of 256 keep every lane busy (a row-tile loop x += 256 runs its last pass
// over a 576-voxel row with a quarter of the threads), x-neighbours are lane shuffles, and
// a word is exactly one word of the frontier bitmaps.  BODY sees z, y, x, i (block C-order
// index), row, xw (word in the row), wpr and `valid` (x < nx); every lane runs BODY (ballots
// are legal), invalid lanes must not touch memory.
#define WORD_TILES(nz, ny, nx, ...)                                                                          \
    {                                                                                                        \
        const int wpr = ((nx) + 63) >> 6;                                                                    \
        const int64_t nwords_ = (int64_t)(nz) * (ny) * wpr;                                                  \
        const int lane = threadIdx.x & 63;                                                                   \
        const int64_t nwaves_ = (int64_t)gridDim.x * (blockDim.x >> 6);                                      \
        const int64_t per_ = (nwords_ + nwaves_ - 1) / nwaves_;                                              \
        const int64_t wid_ = (int64_t)xcd_swizzle((int)blockIdx.x, (int)gridDim.x) * (blockDim.x >> 6) +     \
                             (threadIdx.x >> 6);                                                             \
        const int64_t wend_ = wid_ * per_ + per_ < nwords_ ? wid_ * per_ + per_ : nwords_;                   \
        /* (row, word, z, y) advanced word by word: one 64-bit division per wave, not per word */            \
        int64_t row_ = (wid_ * per_) / wpr;                                                                  \
        int xw_ = (int)(wid_ * per_ - row_ * wpr);                                                           \
        int z_ = (int)(row_ / (ny)), y_ = (int)(row_ - (int64_t)z_ * (ny));                                  \
        for (int64_t w_ = wid_ * per_; w_ < wend_; ++w_) {                                                   \
            const int64_t row = row_;                                                                        \
            const int xw = xw_;                                                                              \
            const int z = z_;                                                                                \
            const int y = y_;                                                                                \
            if (++xw_ == wpr) {                                                                              \
                xw_ = 0;                                                                                     \
                ++row_;                                                                                      \
                if (++y_ == (ny)) {                                                                          \
                    y_ = 0;                                                                                  \
                    ++z_;                                                                                    \
                }                                                                                            \
            }                                                                                                \
            const int x = xw * 64 + lane;                                                                    \
            const bool valid = x < (nx);                                                                     \
            const int64_t i = row * (nx) + x;                                                                \
            (void)z;                                                                                         \
            (void)y;                                                                                         \
            __VA_ARGS__                                                                                      \
        }                                                                                                    \
    }

// n / d for 0 <= n < 2^31, 0 < d and a quotient below 2^22, by the float reciprocal `inv` =
// 1.0f / d and one correction (the estimate's error is about q * 2^-23, so it is off by at most
// one): a few instructions instead of the emulated integer division's long dependent chain
__device__ __forceinline__ int div_small(int n, int d, float inv) {
    int q = (int)((float)n * inv);
    const int r = n - q * d;
    q += r < 0 ? -1 : (r >= d ? 1 : 0);
    return q;
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
    return (uint64_t)__shfl_up((long long)v, d);
}
__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    return (uint64_t)__shfl((long long)v, src);
}
__device__ __forceinline__ uint64_t shfl_down_u64(uint64_t v, int d) {
    return (uint64_t)__shfl_down((long long)v, d);
}

// ---- packed flood keys: C (ordered float bits, 32) | d (12, saturating) | label (20) ----------
constexpr uint64_t kPackInf = ~0ull;
constexpr uint32_t kLabelBits = 20;
constexpr uint64_t kLabelMask = (1ull << kLabelBits) - 1ull;
constexpr uint64_t kDOne = 1ull << kLabelBits;
constexpr uint64_t kDMask = 0xFFFull << kLabelBits;
// The tie order inside an equal-C plateau: d = hops since the plateau level was entered (the
// 12-bit field saturates at kDMax; INF has d = 0xFFF and stays INF).  d must grow along every
// parent edge: then (C, d) strictly increases from a voxel's argmin neighbour to the voxel, the
// fixpoint is unique, and any relaxation schedule reaches the sequential model's result.  A
// saturated d breaks that, so a final key with d = kDMax is reported (note_dsat below) and the
// block is flooded again on the wide keys, whose 32-bit d never saturates (round 6).
// Orders with d capped at 1 or without d measured closer to vigra's heap order on tie-dominated
// inputs (scripts/tie_order_experiment.py) but lose that: equal keys along a plateau path let a
// cycle of voxels keep a stale label, and the GPU converged to such a fixpoint (round 4,
// config-1 2-D test config: VI 0.029 against the model's 0) -- not adopted.
constexpr uint32_t kDMax = 4095;

// A packed key whose d field is at kDMax: the hop distance may have saturated, so the packed
// fixpoint may differ from the unbounded (C, d, label) one (a cycle of equal saturated keys can
// keep a stale label).  k_flood_verify (after every frontier flood) and the tile flood's writes
// report such a key in BlockStat::dsat; run_batch then floods those blocks again with the wide
// keys (k_flood: d is 32 bits there and never saturates).  If every final d is below kDMax, each
// final key is the exact f of its neighbours' minimum: a fixpoint of the unbounded order, which
// is unique, so a batch without a report is exact.
__device__ __forceinline__ bool key_dsat(uint64_t k) { return (k & kDMask) == kDMask && k != kPackInf; }
__device__ __forceinline__ void note_dsat(const BlockStat* S, int b) {
    uint32_t* p = const_cast<uint32_t*>(&S[b].dsat);
    if (!*(volatile uint32_t*)p) atomicOr(p, 1u);
}

// K(q) = f_q(min over the neighbours): a neighbour key `best` pushed into voxel q of height hb
__device__ __forceinline__ uint64_t f_packed(uint32_t hb, uint64_t best) {
    const uint32_t c = (uint32_t)(best >> 32);
    if (hb > c) return ((uint64_t)hb << 32) | (best & kLabelMask);
    return ((best & kDMask) >= ((uint64_t)kDMax << kLabelBits)) ? best : best + kDOne;
}

// seed test: from the seed CC parents (pass 1: `cc` = PF after k_root_label) or, when cc is
// null, from lab (kFixedBit; pass 2 and the fallbacks)
__device__ __forceinline__ bool is_seed(const uint32_t* lab, const uint32_t* cc, int64_t gi) {
    return cc ? cc[gi] != kNoParent : (lab[gi] & kFixedBit) != 0;
}

// rank of key f among set bits of a per-block bitmap with per-word exclusive prefix
__device__ __forceinline__ uint32_t bitmap_rank(const uint64_t* W, const uint32_t* Wp, uint32_t f) {
    uint32_t w = f >> 6;
    uint64_t m = W[w] & ((1ull << (f & 63)) - 1ull);
    return Wp[w] + (uint32_t)__popcll(m);
}

}  // namespace ctws
