// Calibration of rocprofv3 FETCH_SIZE on gfx950 for the access shapes of the flood (VERDICT r03
// #4: the x2 correction is documented for wide coalesced reads only).  Each kernel moves a known
// number of bytes from a buffer far larger than the caches (2 GiB, cold: every line is first
// touched once by a kernel); scripts/pmc_gather_calibration.py divides FETCH_SIZE by that count.
//   stream16  16 B per lane, coalesced, every byte of 1 GiB once
//   stream8    8 B per lane, coalesced, every byte of 1 GiB once
//   seg512     each wave one 512-B segment (8 B per lane) at a random place; every segment of
//              1 GiB once (the frontier's row words: a wave's 64 lanes on one row)
//   line8      each lane 8 B in its own 128-B line, lines in random order, every line of 2 GiB
//              once (the frontier's neighbour gathers: a lane per voxel, rows apart)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <random>

__global__ void stream16(const uint4* __restrict__ a, size_t n, unsigned long long* out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) atomicAdd(out, 1ull);
}
__global__ void stream8(const uint64_t* __restrict__ a, size_t n, unsigned long long* out) {
    uint64_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s ^= a[i];
    if (s == 0x12345678ull) atomicAdd(out, 1ull);
}
// perm: a permutation of the segment / line ids
__global__ void seg512(const uint64_t* __restrict__ a, const uint32_t* __restrict__ perm, size_t nseg,
                       unsigned long long* out) {
    uint64_t s = 0;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t w = wave; w < nseg; w += nw) s ^= a[(size_t)perm[w] * 64 + lane];
    if (s == 0x12345678ull) atomicAdd(out, 1ull);
}
__global__ void line8(const uint64_t* __restrict__ a, const uint32_t* __restrict__ perm, size_t nlines,
                      unsigned long long* out) {
    uint64_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nlines; i += (size_t)gridDim.x * blockDim.x)
        s ^= a[(size_t)perm[i] * 16 + (i & 15)];
    if (s == 0x12345678ull) atomicAdd(out, 1ull);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t big = (size_t)2 << 30;  // 2 GiB
    uint8_t* buf;
    unsigned long long* out;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&out, 8));
    CK(hipMemset(buf, 1, big));
    // a 1 GiB region for the streams, the whole buffer for the line gathers
    const size_t gib = (size_t)1 << 30;
    const size_t nseg = gib / 512, nlines = big / 128;
    std::vector<uint32_t> ps(nseg), pl(nlines);
    for (size_t i = 0; i < nseg; ++i) ps[i] = (uint32_t)i;
    for (size_t i = 0; i < nlines; ++i) pl[i] = (uint32_t)i;
    std::mt19937_64 rng(7);
    std::shuffle(ps.begin(), ps.end(), rng);
    std::shuffle(pl.begin(), pl.end(), rng);
    uint32_t *dps, *dpl;
    CK(hipMalloc(&dps, nseg * 4));
    CK(hipMalloc(&dpl, nlines * 4));
    CK(hipMemcpy(dps, ps.data(), nseg * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpl, pl.data(), nlines * 4, hipMemcpyHostToDevice));
    // evict the region from L2 / MALL between kernels: stream the other GiB in between
    auto flush = [&]() { stream16<<<4096, 256>>>((const uint4*)(buf + gib), gib / 16, out); };
    flush();
    stream16<<<4096, 256>>>((const uint4*)buf, gib / 16, out);
    flush();
    stream8<<<4096, 256>>>((const uint64_t*)buf, gib / 8, out);
    flush();
    seg512<<<4096, 256>>>((const uint64_t*)buf, dps, nseg, out);
    line8<<<4096, 256>>>((const uint64_t*)buf, dpl, nlines, out);
    CK(hipDeviceSynchronize());
    printf("{\"stream16_bytes\": %zu, \"stream8_bytes\": %zu, \"seg512_bytes\": %zu, \"line8_lines\": %zu, "
           "\"line8_bytes_8B\": %zu, \"flush_bytes\": %zu, \"permutation_bytes_seg512\": %zu, "
           "\"permutation_bytes_line8\": %zu}\n", gib, gib, gib, nlines, nlines * 8, gib, nseg * 4, nlines * 4);
    return 0;
}
