// h2d_lab.hip -- development harness (not product code): host -> device rates on
// the GPU box for the end-to-end decode path (1.08 GB of table bytes):
//   sdma1        one hipMemcpyAsync of the whole buffer (pinned host memory)
//   sdmaK        the buffer split over K streams (K SDMA queues), K = 2, 4
//   zcopy        a copy kernel that reads the pinned host buffer directly
//                (host-mapped, coalesced 16-B loads over PCIe) into HBM
//   zread        the same kernel reading only (no HBM store)
//   dec_mapped   bhg_decode_batch straight on the host-mapped table bytes
//                (handles and descriptors in HBM): the decode kernel's own
//                loads cross PCIe, no staging copy at all
// build: make -C scripts/lab h2d_lab      run: scripts/lab/h2d_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/bithashgpu.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool STORE>
__global__ __launch_bounds__(256) void k_zcopy(const u32x4 *__restrict__ h, u32x4 *__restrict__ d, uint64_t n16,
                                               uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(h + i);
        if (STORE) d[i] = v;
        else acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (!STORE && acc == 0x12345678u) sink[threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const uint32_t n = 1000000, L = 1076;
    const uint32_t R = (uint32_t)((128ull << 20) / L + 1);
    const uint64_t tbytes = (uint64_t)R * L + 12;
    std::vector<bhg_handle> hh(n);
    for (uint32_t i = 0; i < n; i++) hh[i] = bhg_handle{(uint64_t)(i / R) * tbytes + (uint64_t)(i % R) * L, L, 0};
    const uint64_t len = hh[n - 1].offset + L + 12;
    uint8_t *host;
    CK(hipHostMalloc(&host, len + 4096, hipHostMallocMapped));
    for (uint32_t i = 0; i < n; i++) {  // valid records: header {40, 1024, fn}, key/value bytes
        uint8_t *r = host + hh[i].offset;
        const uint32_t hdr[3] = {40, 1024, 1 + i / R};
        memcpy(r, hdr, 12);
        for (uint32_t b = 12; b < L; b++) r[b] = (uint8_t)(48 + ((i * 131u + b * 7u) % 75));
    }
    uint8_t *hdev;
    CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&hdev), host, 0));
    uint8_t *dev;
    uint32_t *sink;
    bhg_handle *dh;
    bhg_desc *dd, *dd2;
    CK(hipMalloc(&dev, len + 4096));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&dh, n * sizeof(bhg_handle)));
    CK(hipMalloc(&dd, n * sizeof(bhg_desc)));
    CK(hipMalloc(&dd2, n * sizeof(bhg_desc)));
    CK(hipMemcpy(dh, hh.data(), n * sizeof(bhg_handle), hipMemcpyHostToDevice));
    hipStream_t st[4];
    for (int k = 0; k < 4; k++) CK(hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    auto timeit = [&](const char *name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        std::vector<double> ts;
        for (int r = 0; r < reps; r++) {
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a, st[0]));
            fn();
            for (int k = 1; k < 4; k++) {  // join the side streams into st[0]
                hipEvent_t e;
                CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                CK(hipEventRecord(e, st[k]));
                CK(hipStreamWaitEvent(st[0], e, 0));
            }
            CK(hipEventRecord(b, st[0]));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-12s median %.3f ms  %.2f GB/s  (%.2f GiB/s of table bytes)\n", name, ts[ts.size() / 2],
               len / ts[ts.size() / 2] / 1e6, len / ts[ts.size() / 2] * 1e3 / (1ull << 30));
        fflush(stdout);
    };
    auto fence_side = [&]() {  // side streams start after st[0]'s start event
        hipEvent_t e;
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        CK(hipEventRecord(e, st[0]));
        for (int k = 1; k < 4; k++) CK(hipStreamWaitEvent(st[k], e, 0));
    };
    timeit("sdma1", [&] { CK(hipMemcpyAsync(dev, host, len, hipMemcpyHostToDevice, st[0])); });
    for (int K : {2, 4}) {
        char nm[16];
        snprintf(nm, sizeof nm, "sdma%d", K);
        timeit(nm, [&] {
            fence_side();
            const uint64_t part = (len / K + 4095) & ~4095ull;
            for (int k = 0; k < K; k++) {
                const uint64_t o = (uint64_t)k * part, l = o >= len ? 0 : std::min(part, len - o);
                if (l) CK(hipMemcpyAsync(dev + o, host + o, l, hipMemcpyHostToDevice, st[k]));
            }
        });
    }
    const uint64_t n16 = len / 16;
    timeit("zcopy", [&] {
        hipLaunchKernelGGL(k_zcopy<true>, dim3(cus * 8), dim3(256), 0, st[0], (const u32x4 *)hdev, (u32x4 *)dev, n16, sink);
    });
    timeit("zread", [&] {
        hipLaunchKernelGGL(k_zcopy<false>, dim3(cus * 8), dim3(256), 0, st[0], (const u32x4 *)hdev, (u32x4 *)dev, n16, sink);
    });
    bhg_ctx *ctx = bhg_create(0, 0);
    if (!ctx) { fprintf(stderr, "bhg_create failed\n"); return 1; }
    if (bhg_decode_batch(ctx, dev, len, dh, n, 0, nullptr, dd2, nullptr, 0, nullptr, st[0]) != 0) return 1;
    timeit("dec_hbm", [&] {
        if (bhg_decode_batch(ctx, dev, len, dh, n, 0, nullptr, dd, nullptr, 0, nullptr, st[0]) != 0) exit(1);
    });
    timeit("dec_mapped", [&] {
        if (bhg_decode_batch(ctx, hdev, len, dh, n, 0, nullptr, dd, nullptr, 0, nullptr, st[0]) != 0) exit(1);
    });
    CK(hipDeviceSynchronize());
    std::vector<bhg_desc> a(n), b(n);
    CK(hipMemcpy(a.data(), dd, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), dd2, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
    printf("dec_mapped descriptors %s the HBM decode's\n", memcmp(a.data(), b.data(), n * sizeof(bhg_desc)) ? "DIFFER from" : "equal");
    bhg_destroy(ctx);
    return 0;
}
