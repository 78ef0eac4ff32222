// k_eval.hip — segmentation evaluation (VI split / merge, adapted Rand) on gfx950.
//
// Reference: evaluation/measures.py:80-164 (contingency table from the seg x gt overlaps,
// then utils/validation_utils.py:60-76 compute_vi_scores(use_log2=True) and :178-198
// compute_rand_scores), with the overlaps of evaluation_workflow.py:53-67 (NodeLabelWorkflow,
// gt label 0 ignored when ignore_label).  The reference gathers the overlaps with nifty over
// blocks and reduces them in one Python job; here the contingency table is built in HBM:
//
//   A: gt id  -> voxel count     (open-addressing hash, the slot index is the id's dense index)
//   B: seg id -> voxel count
//   P: (slot_A << 32 | slot_B) -> voxel count
//
// A wave first merges runs of equal (gt, seg) pairs among its 64 consecutive voxels (labels
// are spatially coherent: one atomic per run instead of one per voxel on the hot ids), then
// the run leaders insert / count.  Tables persist across ctws_eval_add calls (blockwise
// accumulation); k_eval_reduce sums the entropy and Rand terms in double.
#include "ctws_kernels.h"

namespace ctws {

constexpr uint64_t kEvEmpty = ~0ull;

__device__ __forceinline__ uint64_t ev_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// slot of k (inserted if absent); -1 when the table is full.  The label 2^64 - 1 (= the empty
// marker) has the extra slot `cap` of its own (arrays hold cap + 1 entries): present iff counted.
__device__ __forceinline__ int64_t ev_insert(uint64_t* keys, int64_t cap, uint64_t k) {
    if (k == kEvEmpty) return cap;
    int64_t s = (int64_t)(ev_mix(k) & (uint64_t)(cap - 1));
    for (int64_t p = 0; p < cap; ++p) {
        uint64_t v = keys[s];
        if (v == kEvEmpty) v = atomicCAS((unsigned long long*)&keys[s], (unsigned long long)kEvEmpty, (unsigned long long)k);
        if (v == kEvEmpty || v == k) return s;
        s = (s + 1) & (cap - 1);
    }
    return -1;
}

// gt / seg label arrays (uint64) of n voxels; ignore: drop voxels with gt == 0.
// state[0] = counted voxels, state[1] = table-full flag.
__global__ void __launch_bounds__(256) k_eval_add(const uint64_t* __restrict__ seg, const uint64_t* __restrict__ gt,
                                                  int64_t n, int ignore, uint64_t* __restrict__ ka,
                                                  unsigned long long* __restrict__ ca, int64_t cap_a,
                                                  uint64_t* __restrict__ kb, unsigned long long* __restrict__ cb,
                                                  int64_t cap_b, uint64_t* __restrict__ kp,
                                                  unsigned long long* __restrict__ cp, int64_t cap_p,
                                                  unsigned long long* __restrict__ state) {
    const int lane = threadIdx.x & 63;
    unsigned long long counted = 0;
    bool full = false;
    for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63)); i0 < n;
         i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + lane;
        const bool valid = i < n;
        const uint64_t g = valid ? gt[i] : 0ull;
        const uint64_t s = valid ? seg[i] : 0ull;
        const bool use = valid && !(ignore && g == 0ull);
        // runs of equal (g, s) among the used lanes: a lane leads when the previous lane differs
        const uint64_t gp = (uint64_t)__shfl_up((long long)g, 1), sp = (uint64_t)__shfl_up((long long)s, 1);
        const bool usep = __shfl_up((int)use, 1) != 0;
        const bool lead = use && (lane == 0 || !usep || gp != g || sp != s);
        const uint64_t lm = __ballot(lead), um = __ballot(use);
        if (!lead) continue;
        // run = used lanes from this leader up to the next leader (or the end of the used run)
        const uint64_t after = lane == 63 ? 0ull : (lm >> (lane + 1)) << (lane + 1);
        const int next = after ? __builtin_ctzll(after) : 64;
        const uint64_t span = (next >= 64 ? ~0ull : ((1ull << next) - 1ull)) & ~((1ull << lane) - 1ull);
        const unsigned long long len = (unsigned long long)__popcll(um & span);
        counted += len;
        const int64_t sa = ev_insert(ka, cap_a, g), sb = ev_insert(kb, cap_b, s);
        if (sa < 0 || sb < 0) {
            full = true;
            continue;
        }
        atomicAdd(&ca[sa], len);
        atomicAdd(&cb[sb], len);
        const int64_t sp2 = ev_insert(kp, cap_p, ((uint64_t)sa << 32) | (uint64_t)sb);
        if (sp2 < 0) {
            full = true;
            continue;
        }
        atomicAdd(&cp[sp2], len);
    }
    for (int o = 32; o > 0; o >>= 1) counted += (unsigned long long)__shfl_xor((long long)counted, o);
    if (lane == 0 && counted) atomicAdd(&state[0], counted);
    if (__ballot(full) && lane == 0) atomicOr(&state[1], 1ull);
}

// sums: out[0] = sum_a  (-c/n log2(c/n) over gt ids), out[1] = sum_b (seg ids),
// out[2] = sum_ab (c/n log2(n c / (a b)) over pairs), out[3] = sum a^2, out[4] = sum b^2, out[5] = sum pairs^2
__global__ void __launch_bounds__(256) k_eval_reduce(const uint64_t* __restrict__ ka, const unsigned long long* __restrict__ ca,
                                                     int64_t cap_a, const uint64_t* __restrict__ kb,
                                                     const unsigned long long* __restrict__ cb, int64_t cap_b,
                                                     const uint64_t* __restrict__ kp,
                                                     const unsigned long long* __restrict__ cp, int64_t cap_p,
                                                     const unsigned long long* __restrict__ state, double* __restrict__ out) {
    const double n = (double)state[0];
    double v[6] = {0, 0, 0, 0, 0, 0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= cap_a; s += stride)
        if (s < cap_a ? ka[s] != kEvEmpty : ca[s] != 0ull) {
            const double c = (double)ca[s];
            v[0] += -c / n * log2(c / n);
            v[3] += c * c;
        }
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= cap_b; s += stride)
        if (s < cap_b ? kb[s] != kEvEmpty : cb[s] != 0ull) {
            const double c = (double)cb[s];
            v[1] += -c / n * log2(c / n);
            v[4] += c * c;
        }
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < cap_p; s += stride) {
        const uint64_t k = kp[s];
        if (k == kEvEmpty) continue;
        const double c = (double)cp[s];
        const double a = (double)ca[k >> 32], b = (double)cb[k & 0xFFFFFFFFull];
        v[2] += c / n * log2(n * c / (a * b));
        v[5] += c * c;
    }
    __shared__ double red[6][4];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double x = v[k];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        double x = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) x += red[threadIdx.x][w];
        if (x != 0.0) atomicAdd(&out[threadIdx.x], x);
    }
}

}  // namespace ctws
