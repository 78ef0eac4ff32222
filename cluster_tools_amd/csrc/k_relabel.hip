// k_relabel.hip — RelabelWorkflow on gfx950: sorted uniques and table lookup of uint64 labels.
//
// Reference: relabel/find_uniques.py:93-159 (np.unique per block, per job), find_labeling.py:
// 84-126 (np.unique of all jobs' uniques -> consecutive new ids), write/write.py:153-226
// (nifty.tools.takeDict of every block through the assignment table).
//
// Sorted unique = bitmap over the value range: watershed ids of a block are
// block_id * prod(block_shape) + [1, n] (plus 0 for background), so the nonzero values of a
// block — and of a whole volume of up to 2^35 voxels — span a range that fits one bitmap in
// HBM.  One pass sets the bits (a wave of equal labels, the common case, costs one atomic),
// a popcount + exclusive scan over 256-word chunks gives every word its output position, and
// a compaction pass writes the set bits in ascending order: the uniques come out sorted with
// no sort at all.  0 is tracked with a flag and emitted first.
//
// When the values span too wide a range for a bitmap (sparse or arbitrary ids: more than 2^35
// values, or a bitmap larger than the labels themselves), or when the counts are wanted
// (np.unique(return_counts=True), find_uniques.py:104-106), the uniques come from a radix sort
// of the labels and a run-length encoding of the sorted run (hipcub, both device-wide).
//
// Lookup: every label is replaced by values[j] for keys[j] == label (keys ascending) by a
// binary search in the table; labels absent from the table are counted and left unchanged
// (takeDict would raise; the caller decides).
#include <hipcub/hipcub.hpp>

#include "ctws_kernels.h"

namespace ctws {

// red[0] = min nonzero label (atomicMin), red[1] = max label (atomicMax), red[2] = 1 if 0 occurs
__global__ void __launch_bounds__(256) k_u64_range(const uint64_t* __restrict__ v, int64_t n,
                                                   unsigned long long* __restrict__ red) {
    unsigned long long mn = ~0ull, mx = 0ull;
    bool zero = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = v[i];
        if (x == 0) zero = true;
        else mn = min(mn, (unsigned long long)x);
        mx = max(mx, (unsigned long long)x);
    }
    for (int s = 32; s > 0; s >>= 1) {
        mn = min(mn, (unsigned long long)__shfl_xor((long long)mn, s));
        mx = max(mx, (unsigned long long)__shfl_xor((long long)mx, s));
    }
    const bool anyz = __ballot(zero) != 0ull;
    if ((threadIdx.x & 63) == 0) {
        if (mn != ~0ull) atomicMin(&red[0], mn);
        if (mx) atomicMax(&red[1], mx);
        if (anyz && !red[2]) atomicOr(&red[2], 1ull);
    }
}

// bit (x - lo) for every nonzero label x
__global__ void __launch_bounds__(256) k_u64_bits(const uint64_t* __restrict__ v, int64_t n, uint64_t lo,
                                                  unsigned long long* __restrict__ bits) {
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + threadIdx.x;
        const uint64_t x = i < n ? v[i] : 0ull;
        const uint64_t x0 = (uint64_t)__shfl((long long)x, 0);
        const uint64_t nz = __ballot(x != 0ull);
        if (__ballot(x == x0 && x != 0ull) == nz) {
            // every labelled lane holds the same value: one atomic for the wave
            if ((threadIdx.x & 63) == 0 && nz) {
                const uint64_t b = x0 - lo;
                atomicOr(&bits[b >> 6], 1ull << (b & 63));
            }
        } else if (x != 0ull) {
            const uint64_t b = x - lo;
            atomicOr(&bits[b >> 6], 1ull << (b & 63));
        }
    }
}

// popcount of each 256-word chunk
__global__ void __launch_bounds__(256) k_bits_chunk_count(const uint64_t* __restrict__ bits, int64_t nw,
                                                          uint32_t* __restrict__ cnt) {
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t c = w < nw ? (uint32_t)__popcll(bits[w]) : 0u;
    c = wg_reduce_u32(c, OpAdd());
    if (threadIdx.x == 0) cnt[blockIdx.x] = c;
}

// one workgroup: exclusive scan of the chunk counts into uint64 offsets; total -> offs[nc]
__global__ void __launch_bounds__(256) k_scan_chunks(const uint32_t* __restrict__ cnt, int64_t nc,
                                                     uint64_t* __restrict__ offs) {
    __shared__ uint64_t tmp[256];
    uint64_t carry = 0;
    for (int64_t c0 = 0; c0 < nc; c0 += 256) {
        const int64_t c = c0 + threadIdx.x;
        const uint64_t v = c < nc ? cnt[c] : 0ull;
        tmp[threadIdx.x] = v;
        __syncthreads();
        for (int s = 1; s < 256; s <<= 1) {
            const uint64_t a = threadIdx.x >= (unsigned)s ? tmp[threadIdx.x - s] : 0ull;
            __syncthreads();
            tmp[threadIdx.x] += a;
            __syncthreads();
        }
        if (c < nc) offs[c] = carry + tmp[threadIdx.x] - v;
        carry += tmp[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) offs[nc] = carry;
}

// ascending values of the set bits: out[first + rank] = lo + bit position
__global__ void __launch_bounds__(256) k_bits_compact(const uint64_t* __restrict__ bits, int64_t nw,
                                                      const uint64_t* __restrict__ offs, uint64_t lo, uint64_t first,
                                                      uint64_t* __restrict__ out) {
    const int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint64_t b = w < nw ? bits[w] : 0ull;
    const uint32_t c = (uint32_t)__popcll(b);
    // workgroup exclusive scan of the word counts
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = c;
    for (int s = 1; s < 64; s <<= 1) {
        const uint32_t a = (uint32_t)__shfl_up((int)x, s);
        if (lane >= s) x += a;
    }
    __shared__ uint32_t wt[4];
    if (lane == 63) wt[wv] = x;
    __syncthreads();
    uint32_t woff = 0;
    for (int k = 0; k < wv; ++k) woff += wt[k];
    uint64_t pos = first + offs[blockIdx.x] + woff + x - c;
    while (b) {
        const int p = __builtin_ctzll(b);
        b &= b - 1;
        out[pos++] = lo + (uint64_t)w * 64 + (uint64_t)p;
    }
}

// labels[i] <- values[j] with keys[j] == labels[i] (keys ascending); misses are counted
__global__ void __launch_bounds__(256) k_u64_lookup(uint64_t* __restrict__ v, int64_t n,
                                                    const uint64_t* __restrict__ keys,
                                                    const uint64_t* __restrict__ vals, int64_t nt,
                                                    unsigned long long* __restrict__ missing) {
    unsigned long long miss = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = v[i];
        int64_t lo = 0, hi = nt;  // first key >= x
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        if (lo < nt && keys[lo] == x) v[i] = vals[lo];
        else ++miss;
    }
    for (int s = 32; s > 0; s >>= 1) miss += (unsigned long long)__shfl_xor((long long)miss, s);
    if ((threadIdx.x & 63) == 0 && miss) atomicAdd(missing, miss);
}

// Device -> pinned host copy by a few workgroups (16-B stores, grid-stride).  The runtime moves
// large device-to-host copies with a blit kernel over every CU, which starves the compute
// kernels running concurrently; this copy leaves all but gridDim.x CUs to them.
__global__ void __launch_bounds__(256) k_copy_to_host(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                      size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// sort-based unique: radix sort of the uint64 keys, then (value, count) runs.  With tmp ==
// nullptr the temporary storage is only sized.
hipError_t u64_sort(void* tmp, size_t& bytes, const uint64_t* in, uint64_t* out, int64_t n, hipStream_t stream) {
    return hipcub::DeviceRadixSort::SortKeys(tmp, bytes, in, out, n, 0, 64, stream);
}
hipError_t u64_runs(void* tmp, size_t& bytes, const uint64_t* sorted, uint64_t* uniq, uint64_t* counts,
                    uint64_t* n_runs, int64_t n, hipStream_t stream) {
    return hipcub::DeviceRunLengthEncode::Encode(tmp, bytes, sorted, uniq, counts, n_runs, n, stream);
}

}  // namespace ctws
