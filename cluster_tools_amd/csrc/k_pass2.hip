// k_pass2.hip — the second pass of the two-pass (checkerboard) watershed on gfx950.
//
// Reference: watershed/two_pass_watershed.py:210-255 (_ws_pass2) and :122-207
// (_apply_watershed_with_seeds).  A pass-2 block is seeded by its own local maxima AND by the
// pass-1 labels of its neighbours found in its halo (`initial_seeds = ds_out[input_bb]`):
//
//   2-D ws only:  dt[z][initial_seeds[z] != 0] = 0                         (:139)
//   seeds = _make_seeds(dt);  seeds[outside mask] = 0                      (:141-144, :181-183)
//   seeds[seeds != 0] += offset         (uint32 array: wraps mod 2^32)     (:147, :184)
//   seeds[initial != 0] = initial       (uint64 -> uint32 setitem)         (:149, :187-188)
//   seeds = relabelConsecutive(seeds)   (first appearance in vigra order)  (:153, :192)
//   ws = watershed(hmap, seeds, size_filter, exclude=<initial ids>)        (:160, :199-202)
//   ws = takeDict(new_to_old, ws);  ws[outside mask] = 0;  write ws[inner] (no CC relabel)
//
// In 2-D mode `offset` grows slice by slice by the max_id of the previous slices (:166-168),
// which is only known after their floods.  relabelConsecutive numbers by first appearance,
// so the offset changes the numbering only where a shifted new seed value equals an initial
// value of the same slice (then both are one id: the new seed merges into the initial seed's
// segment).  The first run keys new seeds by (slice, tag 0, local seed id) and initial seeds
// by (slice, tag 1, value); once the slice offsets are known, k_p2_check flags a block where
// such an equality exists.  The host then runs the block again with the offsets as a hint:
// every seed is keyed by (slice, tag 1, its uint32 value), so equal values merge exactly as in
// relabelConsecutive, and it repeats until the offsets the run produces equal its hint (slice
// z's offset depends only on slices < z, so each run fixes at least one more slice).
// In 3-D mode the offset is the constant block_id * prod(block_shape), so keys are the exact
// uint32 values, as in the reference.
//
// relabelConsecutive is computed with a per-block open-addressing hash (key -> smallest
// vigra scan-order key f holding it): the first positions become roots of a bitmap, and the
// new id of a value is 1 + the rank of its first position (the machinery of k_cc.hip).
#include "ctws_kernels.h"

namespace ctws {

#define BLOCK_LOOP(i, B)                                                                      \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (B).N;              \
         i += (int64_t)gridDim.x * blockDim.x)

constexpr uint64_t kEmptyKey = ~0ull;
constexpr uint64_t kInitTag = 1ull << 32;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// slot of `k` in the block's table, or -1 (absent / table full: the error bit is set)
__device__ __forceinline__ int64_t hash_find(const uint64_t* hk, int64_t cap, uint64_t k) {
    int64_t s = (int64_t)(mix64(k) & (uint64_t)(cap - 1));
    for (int64_t p = 0; p < cap; ++p) {
        const uint64_t v = hk[s];
        if (v == k) return s;
        if (v == kEmptyKey) return -1;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

// (32-bit divisions: a block holds fewer than 2^31 voxels, ctws_api.cpp refuses larger ones)
__device__ __forceinline__ void inner_to_zyx(int64_t i, int64_t YX, int X, int& z, int& y, int& x) {
    const uint32_t ii = (uint32_t)i, yx = (uint32_t)YX;
    z = (int)(ii / yx);
    const int rem = (int)(ii - (uint32_t)z * yx);
    y = rem / X;
    x = rem - y * X;
}

// vigra scan-order key (F order; per slice in 2-D ws mode, slice-major across slices)
__device__ __forceinline__ uint32_t scan_key(const BlockDesc& B, int z, int y, int x) {
    return (B.nd_ws == 3) ? (uint32_t)(z + B.Z * (y + B.Y * x))
                          : (uint32_t)((int64_t)z * B.Y * B.X + y + (int64_t)B.Y * x);
}

// 2-D ws: no maxima on initial seeds (two_pass_watershed.py:139)
__global__ void __launch_bounds__(256) k_p2_zero_dt(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                    float* __restrict__ dt) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    BLOCK_LOOP(i, B) {
        if (gbl(B.init)[i] != 0) dt[B.base + i] = 0.0f;
    }
}

// the relabel key of voxel i (kEmptyKey: unlabelled) computed where it is used (k_p2_insert,
// k_p2_label) instead of a per-voxel key array in HBM (its write and two reads): 3-D keys are the
// seed values; 2-D keys carry the slice and tag the initial seeds.  sb0 (2-D): the slices' seed
// bases of the seed CC (k_slice_seed_base before the relabel rewrites w.sb); hint (2-D, blocks
// with B.p2hint >= 0): the slice offsets of the previous run, new seeds keyed by their uint32 value
__device__ __forceinline__ uint64_t p2_value(const BlockDesc& B, int64_t i, const uint32_t* PF, const uint64_t* sbits,
                                             const uint32_t* sb0, const uint32_t* hint, uint64_t* init_out = nullptr) {
    const uint64_t u = gbl(B.init)[i];
    if (init_out) *init_out = u;
    // the slice (2-D ws only: 3-D keys carry no position; a block holds fewer than 2^31 voxels)
    const int z = B.nd_ws == 3 ? 0 : (int)((uint32_t)i / (uint32_t)((int64_t)B.Y * B.X));
    if (u != 0) {
        // (uint32)u == 0: the setitem truncation makes the voxel background
        if ((uint32_t)u == 0) return kEmptyKey;
        return (B.nd_ws == 3) ? (uint64_t)(uint32_t)u : (((uint64_t)z << 33) | kInitTag | (uint32_t)u);
    }
    if (B.mask && !gbl(B.mask)[i]) return kEmptyKey;
    const uint32_t gl = bit_of(sbits, B, i) ? cc_label(PF, PF[i]) : 0u;  // seed label (0: background)
    if (!gl) return kEmptyKey;
    if (B.nd_ws == 3) {
        const uint32_t v = gl + (uint32_t)B.id_offset;  // wraps to 0: background
        return v ? (uint64_t)v : kEmptyKey;
    }
    if (B.p2hint >= 0) {
        // seeds[seeds != 0] += offset in uint32: a value that wraps to 0 is background
        const uint32_t v = (gl - sb0[B.sbase + z]) + (uint32_t)B.id_offset + hint[B.p2hint + z];
        return v ? (((uint64_t)z << 33) | kInitTag | v) : kEmptyKey;
    }
    return ((uint64_t)z << 33) | (uint64_t)(gl - sb0[B.sbase + z]);
}

// insert the keys of the voxels none of whose backward neighbours along the scan axes (3-D:
// z - 1, y - 1, x - 1; 2-D: y - 1, x - 1 in the slice) holds the same key: a voxel with such a
// neighbour has a smaller scan key with its value, so it cannot be the first appearance, and
// the first appearance itself passes (every voxel of smaller scan key that is a neighbour has
// a smaller key along some axis).  Only a few corner voxels per segment reach the atomics; the
// table keeps the smallest scan key per value.
__global__ void __launch_bounds__(256) k_p2_insert(const BlockDesc* __restrict__ D, BlockStat* S,
                                                   uint64_t* __restrict__ hkey, uint32_t* __restrict__ hpos,
                                                   const uint32_t* __restrict__ PFg, const uint64_t* __restrict__ sbits,
                                                   const uint32_t* __restrict__ sb0, const uint32_t* __restrict__ hint) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    uint64_t* hk = hkey + B.hbase;
    uint32_t* hp = hpos + B.hbase;
    const int64_t cap = B.hcap;
    const uint32_t* PF = PFg + B.base;
    auto value = [&](int64_t j) { return p2_value(B, j, PF, sbits, sb0, hint); };
    BLOCK_LOOP(i, B) {
        const uint64_t k = value(i);
        if (k == kEmptyKey) continue;
        int z, y, x;
        inner_to_zyx(i, YX, B.X, z, y, x);
        if (B.nd_ws == 3 && z > 0 && value(i - YX) == k) continue;
        if (y > 0 && value(i - B.X) == k) continue;
        if (x > 0 && value(i - 1) == k) continue;
        const uint32_t f = scan_key(B, z, y, x);
        int64_t s = (int64_t)(mix64(k) & (uint64_t)(cap - 1));
        bool done = false;
        for (int64_t p = 0; p < cap; ++p) {
            uint64_t v = hk[s];
            if (v == kEmptyKey) v = atomicCAS((unsigned long long*)&hk[s], (unsigned long long)kEmptyKey, k);
            if (v == kEmptyKey || v == k) {
                atomicMin(&hp[s], f);
                done = true;
                break;
            }
            s = (s + 1) & (cap - 1);
        }
        if (!done) atomicOr(&S[blockIdx.y].err, kErrHashFull);  // table full: this block fails
    }
}

// first positions -> bits of the root bitmap (zeroed beforehand)
__global__ void __launch_bounds__(256) k_p2_roots(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                  const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ hpos,
                                                  uint64_t* __restrict__ W) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < B.hcap; s += (int64_t)gridDim.x * blockDim.x) {
        if (hkey[B.hbase + s] == kEmptyKey) continue;
        const uint32_t f = hpos[B.hbase + s];
        atomicOr((unsigned long long*)&W[B.wbase + (f >> 6)], 1ull << (f & 63));
    }
}

// flood labels = new consecutive ids (block-global, slice-major in 2-D); old values per id
__global__ void __launch_bounds__(256) k_p2_label(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                  const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ hpos,
                                                  const uint64_t* __restrict__ Wg, const uint32_t* __restrict__ Wpg,
                                                  const float* __restrict__ h, uint32_t* __restrict__ lab,
                                                  uint64_t* __restrict__ key,
                                                  uint8_t* __restrict__ fixedv, uint32_t* __restrict__ oldv,
                                                  uint32_t* __restrict__ oldt, int packed, int write_keys,
                                                  const uint32_t* __restrict__ PFg, const uint64_t* __restrict__ sbits,
                                                  const uint32_t* __restrict__ sb0, const uint32_t* __restrict__ hint,
                                                  uint8_t* __restrict__ excl) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    const int lane = threadIdx.x & 63;
    const uint32_t* PF = PFg + B.base;
    const uint32_t nl = S[blockIdx.y].n_seeds;
    BLOCK_LOOP(i, B) {
        // a wave holds 64 consecutive voxels (only trailing lanes can be past the block's end):
        // keys come in runs, and the first lane of each run looks its key up for the run
        uint64_t u = 0;
        const uint64_t k = p2_value(B, i, PF, sbits, sb0, hint, &u);
        // excl (3-D): k_p2_excl's marks from the initial value read here (zeroed beforehand by
        // k_p2_excl_zero)
        if (excl && u != 0 && u <= nl && !excl[B.base + u]) excl[B.base + u] = 1;
        const uint64_t kp = shfl_u64(k, (lane + 63) & 63);
        const bool start = lane == 0 || kp != k;
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const int s0 = 63 - __builtin_clzll(__ballot(start) & upto);
        uint32_t pos = 0u, l = 0u;
        if (start && k != kEmptyKey) {
            const int64_t s = hash_find(hkey + B.hbase, B.hcap, k);
            pos = s >= 0 ? hpos[B.hbase + s] : 0u;  // s < 0 cannot happen after insert
            l = bitmap_rank(Wg + B.wbase, Wpg + B.wbase, pos) + 1u;
        }
        pos = (uint32_t)__shfl((int)pos, s0);
        l = (uint32_t)__shfl((int)l, s0);
        // write_keys = 0 (the descent flood): k_descent_init writes every key and fixed flag from
        // lab, so only lab is written here (and no height is read)
        if (k == kEmptyKey) {
            lab[B.base + i] = 0;
            if (write_keys) {
                // (the wide keys and the descent-less flood start from here: no stale key of an
                // earlier batch may stay in an unlabelled voxel)
                key[B.base + i] = kInfKey;
                fixedv[B.base + i] = 0;
            }
            continue;
        }
        lab[B.base + i] = l | kFixedBit;
        if (write_keys) {
            key[B.base + i] = ((uint64_t)ordf(h[B.base + i]) << 32) | (packed ? (uint64_t)l : 0ull);
            fixedv[B.base + i] = 1;
        }
        // the value's first voxel in scan order has the smallest x of its x run: a run start, or
        // a row's first voxel (its memory predecessor ends the previous row; N < 2^31)
        if (start || (uint32_t)i % (uint32_t)B.X == 0u) {
            int z, y, x;
            inner_to_zyx(i, YX, B.X, z, y, x);
            if (scan_key(B, z, y, x) == pos) {
                oldv[B.base + l] = (uint32_t)k;
                oldt[B.base + l] = (uint32_t)((k >> 32) & 1u);
            }
        }
    }
}

// size-filter exclusion (np.in1d(filter_ids, exclude)): a NEW id is kept when its numeric
// value equals an initial value (3-D: unique initial ids, :199-202; 2-D: the initial seeds of
// the slice, :160) — the mismatched id spaces of the reference
__global__ void __launch_bounds__(256) k_p2_excl(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                 const uint32_t* __restrict__ sb, uint8_t* __restrict__ excl) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    const uint32_t nl = S[blockIdx.y].n_seeds;
    BLOCK_LOOP(i, B) {
        const uint64_t u = gbl(B.init)[i];
        if (u == 0) continue;
        if (B.nd_ws == 3) {
            if (u <= nl) excl[B.base + u] = 1;
        } else {
            const int z = (int)((uint32_t)i / (uint32_t)YX);
            const uint32_t b0 = sb[B.sbase + z];
            const uint32_t b1 = (z + 1 < B.Z) ? sb[B.sbase + z + 1] : nl;
            if (u <= (uint64_t)(b1 - b0)) excl[B.base + b0 + u] = 1;
        }
    }
}

__global__ void __launch_bounds__(256) k_p2_excl_zero(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      uint8_t* __restrict__ excl) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t n = (int64_t)S[blockIdx.y].n_seeds + 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        excl[B.base + i] = 0;
}

// 2-D: with the slice offsets known, flag a shifted new seed equal to an initial value of its
// slice (relabelConsecutive merges them: the host re-runs the block with value keys)
__global__ void __launch_bounds__(256) k_p2_check(const BlockDesc* __restrict__ D, BlockStat* S,
                                                  const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ soff) {
    uint32_t* err = &S[blockIdx.y].err;
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active || B.nd_ws != 2 || B.p2hint >= 0) return;  // hint runs merge equal values
    const int64_t YX = (int64_t)B.Y * B.X;
    BLOCK_LOOP(i, B) {
        const uint64_t u = gbl(B.init)[i];
        const int z = (int)((uint32_t)i / (uint32_t)YX);
        if (i == (int64_t)z * YX) {
            // a shifted new seed that wraps to 0 would have become background
            const uint32_t t0 = 0u - (uint32_t)B.id_offset - soff[B.sbase + z];
            if (t0 && hash_find(hkey + B.hbase, B.hcap, ((uint64_t)z << 33) | t0) >= 0) atomicOr(err, kErrCollision);
        }
        if (u == 0 || (uint32_t)u == 0) continue;
        const uint32_t t = (uint32_t)u - (uint32_t)B.id_offset - soff[B.sbase + z];
        if (t == 0) continue;
        if (hash_find(hkey + B.hbase, B.hcap, ((uint64_t)z << 33) | t) >= 0) atomicOr(err, kErrCollision);
    }
}

// uint64 output of the inner block: takeDict(new_to_old), outside mask -> 0, no CC relabel,
// no offset (two_pass_watershed.py:171-173, 203-206, 252)
__global__ void __launch_bounds__(256) k_p2_output(const BlockDesc* __restrict__ D, BlockStat* S,
                                                   const uint32_t* __restrict__ lab, const uint64_t* __restrict__ key,
                                                   int keys_final, const uint32_t* __restrict__ oldv,
                                                   const uint32_t* __restrict__ oldt, const uint32_t* __restrict__ soff) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;  // dt is None: nothing is written (:240-242)
    const int64_t yx = (int64_t)B.IY * B.IX;
    uint32_t mx = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B.NI; i += (int64_t)gridDim.x * blockDim.x) {
        // (32-bit divisions: a block holds fewer than 2^31 voxels)
        const uint32_t ii = (uint32_t)i, yx32 = (uint32_t)yx;
        const int z = (int)(ii / yx32);
        const int rem = (int)(ii - (uint32_t)z * yx32);
        const int y = rem / B.IX, x = rem - y * B.IX;
        const int64_t o = ((int64_t)(z + B.iz0) * B.Y + (y + B.iy0)) * B.X + (x + B.ix0);
        // the final label: from the packed keys (keys_final: no unpack pass over the outer
        // block for the inner voxels read here) or from lab; the mask loaded with it
        const uint32_t l = flood_label(lab, key, keys_final, B.base + o);
        const bool inm = !B.mask || gbl(B.mask)[o];
        uint32_t v = 0;
        if (l && inm) {
            v = oldv[B.base + l];
            if (B.nd_ws == 2 && !oldt[B.base + l]) v = v + (uint32_t)B.id_offset + soff[B.sbase + z + B.iz0];
        }
        mx = max(mx, v);
        if (B.out32) gblw(B.out32)[i] = v;  // pass-2 values are uint32 (Appendix B.2)
        else gblw(B.out)[i] = v;
    }
    mx = wg_reduce_u32(mx, OpMax());
    if (threadIdx.x == 0 && mx) atomic_max_if(&S[blockIdx.y].max_label, mx);
}

}  // namespace ctws

namespace ctws {
// per slice (2-D ws) / block (3-D ws): 1 if any voxel lies inside the mask (all, without one)
__global__ void __launch_bounds__(256) k_slice_inmask(const BlockDesc* __restrict__ D, const BlockStat* S,
                                                      uint32_t* __restrict__ flag) {
    const BlockDesc& B = D[blockIdx.y];
    if (!S[blockIdx.y].active) return;
    const int64_t YX = (int64_t)B.Y * B.X;
    BLOCK_LOOP(i, B) {
        if (B.mask && !gbl(B.mask)[i]) continue;
        uint32_t* f = flag + B.sbase + (B.nd_ws == 2 ? (int)((uint32_t)i / (uint32_t)YX) : 0);
        if (!*f) *f = 1;
    }
}
}  // namespace ctws
