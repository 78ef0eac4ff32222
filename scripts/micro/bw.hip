// micro-benchmark: achievable HBM rates for the streaming patterns of the pipeline
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) k_copy48(const uint32_t* __restrict__ a, uint64_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i] + 7ull;
}
template <int U>
__global__ void __launch_bounds__(256) k_copy48_u(const uint32_t* __restrict__ a, uint64_t* __restrict__ b, int64_t n) {
    for (int64_t i0 = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += (int64_t)gridDim.x * 256 * U) {
        uint32_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = a[min(i0 + u * 256, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * 256 < n) b[i0 + u * 256] = v[u] + 7ull;
    }
}
__global__ void __launch_bounds__(256) k_copy44v(const uint4* __restrict__ a, uint4* __restrict__ b, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
        uint4 v = a[i];
        v.x += 1;
        b[i] = v;
    }
}
__global__ void __launch_bounds__(256) k_copy44(const uint32_t* __restrict__ a, uint32_t* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i] + 1;
}

int main() {
    const int64_t n = 134217728;  // 512^3
    uint32_t* a;
    uint64_t* b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 8));
    CK(hipMemset(a, 1, n * 4));
    CK(hipMemset(b, 0, n * 8));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, double bytes, auto launch) {
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
    };
    for (int g : {1024, 4096, 16384, 131072}) {
        char nm[64];
        snprintf(nm, 64, "copy 4->8 grid %d", g);
        run(nm, n * 12.0, [&] { k_copy48<<<g, 256>>>(a, b, n); });
    }
    run("copy 4->8 U4 grid 4096", n * 12.0, [&] { k_copy48_u<4><<<4096, 256>>>(a, b, n); });
    run("copy 4->8 U8 grid 2048", n * 12.0, [&] { k_copy48_u<8><<<2048, 256>>>(a, b, n); });
    run("copy 4->4 grid 16384", n * 8.0, [&] { k_copy44<<<16384, 256>>>(a, (uint32_t*)b, n); });
    run("copy 4->4 uint4 grid 8192", n * 8.0, [&] { k_copy44v<<<8192, 256>>>((const uint4*)a, (uint4*)b, n / 4); });
    run("memcpy d2d 512MB", n * 8.0, [&] { hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice); });
    return 0;
}
