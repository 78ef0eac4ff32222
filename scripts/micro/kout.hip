// micro-benchmark: the library's k_output / k_finalize_ws on the bench layout (32 blocks of
// 64x256x256) vs a plain stream kernel, to find what limits the streaming stages.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../cluster_tools_amd/csrc/ctws_kernels.h"
using namespace ctws;

__global__ void __launch_bounds__(256) k_plain(const BlockDesc* __restrict__ D, const uint32_t* __restrict__ ws) {
    const BlockDesc& B = D[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B.NI; i += (int64_t)gridDim.x * 256)
        B.out[i] = ws[B.base + i] + B.id_offset;
}

int main() {
    const int nb = 32, Z = 64, Y = 256, X = 256;
    const int64_t N = (int64_t)Z * Y * X;
    uint32_t* lab;
    hipMalloc(&lab, N * nb * 4);
    hipMemset(lab, 1, N * nb * 4);
    std::vector<uint64_t*> outs(nb);
    for (auto& o : outs) hipMalloc(&o, N * 8);
    std::vector<BlockDesc> d(nb);
    std::vector<BlockStat> s(nb);
    for (int b = 0; b < nb; ++b) {
        memset(&d[b], 0, sizeof(BlockDesc));
        memset(&s[b], 0, sizeof(BlockStat));
        d[b].Z = Z; d[b].Y = Y; d[b].X = X; d[b].nd_ws = 3; d[b].N = N; d[b].base = N * b;
        d[b].IZ = Z; d[b].IY = Y; d[b].IX = X; d[b].NI = N; d[b].ibase = N * b;
        d[b].out = outs[b];
        d[b].id_offset = 1000;
        s[b].active = 1;
    }
    BlockDesc* dd;
    BlockStat* ds;
    hipMalloc(&dd, sizeof(BlockDesc) * nb);
    hipMalloc(&ds, sizeof(BlockStat) * nb);
    hipMemcpy(dd, d.data(), sizeof(BlockDesc) * nb, hipMemcpyHostToDevice);
    hipMemcpy(ds, s.data(), sizeof(BlockStat) * nb, hipMemcpyHostToDevice);
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
        printf("%-36s %8.3f ms  %7.1f GB/s  err=%s\n", name, ms, bytes / ms / 1e6, hipGetErrorString(hipGetLastError()));
    };
    const double bytes = (double)N * nb * 12;
    run("plain via BlockDesc (4096 x nb)", bytes, [&] { k_plain<<<dim3(4096, nb), 256>>>(dd, lab); });
    run("k_output rows (4096 x nb)", bytes, [&] { k_output<<<dim3(4096, nb), 256>>>(dd, ds, lab, lab); });
    run("k_output rows (1024 x nb)", bytes, [&] { k_output<<<dim3(1024, nb), 256>>>(dd, ds, lab, lab); });
    run("k_finalize_ws (4096 x nb)", (double)N * nb * 8, [&] { k_finalize_ws<<<dim3(4096, nb), 256>>>(dd, ds, lab, lab, lab); });
    run("k_unpack_labels (4096 x nb)", (double)N * nb * 16, [&] { k_unpack_labels<<<dim3(4096, nb), 256>>>(dd, ds, (uint64_t*)outs[0], lab); });
    return 0;
}
