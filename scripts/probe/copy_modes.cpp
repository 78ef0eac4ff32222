// H2D copy rate + interference with a streaming kernel for several pinned-memory / stream
// setups (which of them does the runtime move with SDMA rather than a blit kernel?).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void k_stream(const float* a, float* out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.f) out[0] = s;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t bytes = (size_t)1 << 31;  // 2 GiB
    const size_t nk = (size_t)1 << 30;     // 4 GiB streamed by the kernel
    float *dev, *big, *out;
    hipMalloc(&dev, bytes);
    hipMalloc(&big, nk * 4);
    hipMalloc(&out, 4);
    hipMemset(big, 0, nk * 4);
    hipStream_t sk, sc_nb, sc_b;
    hipStreamCreateWithFlags(&sk, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&sc_nb, hipStreamNonBlocking);
    hipStreamCreate(&sc_b);
    struct Mode { const char* name; void* p; bool reg; };
    void *p_def, *p_nc, *p_port, *p_reg;
    hipHostMalloc(&p_def, bytes, hipHostMallocDefault);
    hipHostMalloc(&p_nc, bytes, hipHostMallocNonCoherent);
    hipHostMalloc(&p_port, bytes, hipHostMallocPortable);
    p_reg = aligned_alloc(4096, bytes);
    memset(p_reg, 0, bytes);
    hipHostRegister(p_reg, bytes, hipHostRegisterDefault);
    Mode modes[] = {{"hipHostMalloc default", p_def, false}, {"hipHostMalloc NonCoherent", p_nc, false},
                    {"hipHostMalloc Portable", p_port, false}, {"malloc + hipHostRegister", p_reg, true}};
    // kernel alone
    k_stream<<<4096, 256, 0, sk>>>(big, out, nk);
    hipStreamSynchronize(sk);
    double t = now();
    for (int i = 0; i < 10; ++i) k_stream<<<4096, 256, 0, sk>>>(big, out, nk);
    hipStreamSynchronize(sk);
    const double tk = (now() - t) / 10;
    printf("kernel alone %.2f ms\n", tk * 1e3);
    for (auto& m : modes) {
        for (int sb = 0; sb < 1; ++sb) {
            hipStream_t sc = sb ? sc_b : sc_nb;
            hipMemcpyAsync(dev, m.p, bytes, hipMemcpyHostToDevice, sc);
            hipStreamSynchronize(sc);
            t = now();
            hipMemcpyAsync(dev, m.p, bytes, hipMemcpyHostToDevice, sc);
            hipStreamSynchronize(sc);
            const double th = now() - t;
            t = now();
            hipMemcpyAsync(dev, m.p, bytes, hipMemcpyHostToDevice, sc);
            for (int i = 0; i < 20; ++i) k_stream<<<4096, 256, 0, sk>>>(big, out, nk);
            hipStreamSynchronize(sc);
            hipStreamSynchronize(sk);
            const double tb = now() - t;
            t = now();
            hipMemcpyAsync(m.p, dev, bytes, hipMemcpyDeviceToHost, sc);
            hipStreamSynchronize(sc);
            const double td = now() - t;
            // D2H concurrent with the kernels: whole, and in 64 MiB pieces
            t = now();
            hipMemcpyAsync(m.p, dev, bytes, hipMemcpyDeviceToHost, sc);
            for (int i = 0; i < 20; ++i) k_stream<<<4096, 256, 0, sk>>>(big, out, nk);
            hipStreamSynchronize(sc);
            hipStreamSynchronize(sk);
            const double tdb = now() - t;
            t = now();
            for (size_t o = 0; o < bytes; o += (size_t)64 << 20)
                hipMemcpyAsync((char*)m.p + o, (char*)dev + o, (size_t)64 << 20, hipMemcpyDeviceToHost, sc);
            for (int i = 0; i < 20; ++i) k_stream<<<4096, 256, 0, sk>>>(big, out, nk);
            hipStreamSynchronize(sc);
            hipStreamSynchronize(sk);
            const double tdc = now() - t;
            printf("    D2H + 20 kernels: whole %.1f ms, 64 MiB pieces %.1f ms\n", tdb * 1e3, tdc * 1e3);
            printf("%-28s %-9s H2D %5.1f GB/s D2H %5.1f GB/s | copy + 20 kernels %.1f ms (copy %.1f, kernels %.1f)\n",
                   m.name, sb ? "blocking" : "nonblock", bytes / th / 1e9, bytes / td / 1e9, tb * 1e3, th * 1e3,
                   20 * tk * 1e3);
        }
    }
    return 0;
}
