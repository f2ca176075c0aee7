// pmc_calib.hip -- lab (not product code): calibrates rocprofv3 FETCH_SIZE on gfx950
// for the access shapes of the C2 decode kernel, on the 1M x 1076 B batch layout:
//   k_lin      every byte once, 16 B per lane, coalesced (1.076 GB)
//   k_heads    lane = record: 4 x 16 B at each record start (the phase-1 head, 64 MB)
//   k_hdl      the 16-B handles, coalesced (16 MB)
//   k_tail4    lane = record: one 4-B load 128 B past a window start (the 132-B window's tail word)
// run: rocprofv3 --pmc FETCH_SIZE -- scripts/lab/pmc_calib ; compare with the byte counts printed
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
constexpr uint64_t N = 1000000, L = 1076;

__global__ void k_lin(const uint8_t *src, uint64_t len, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t o = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 16; o + 16 <= len; o += (uint64_t)gridDim.x * blockDim.x * 16) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(src + o);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_heads(const uint8_t *src, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = (i * L) & ~3ull;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const u32x4 v = *reinterpret_cast<const u32x4_a4 *>(src + a + 16 * t);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_hdl(const uint8_t *hdl, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(hdl + 16 * i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ void k_tail4(const uint8_t *src, uint32_t *sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= *reinterpret_cast<const uint32_t *>(src + ((i * L + 52) & ~3ull) + 128);
    if (acc == 0x12345678u) sink[0] = acc;
}
int main() {
    const uint64_t len = N * L + 4096;
    uint8_t *src, *hdl;
    uint32_t *sink;
    CK(hipMalloc(&src, len));
    CK(hipMalloc(&hdl, N * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 0x5a, len));
    CK(hipMemset(hdl, 0x11, N * 16));
    const int grid = 256 * 8, block = 256;
    for (int r = 0; r < 5; r++) {
        // a 300 MB sweep between launches evicts the 256 MiB infinity cache
        hipLaunchKernelGGL(k_lin, dim3(grid), dim3(block), 0, 0, src, len, sink);
        hipLaunchKernelGGL(k_heads, dim3(grid), dim3(block), 0, 0, src + 0, sink);
        hipLaunchKernelGGL(k_lin, dim3(grid), dim3(block), 0, 0, src, len, sink);
        hipLaunchKernelGGL(k_hdl, dim3(grid), dim3(block), 0, 0, hdl, sink);
        hipLaunchKernelGGL(k_lin, dim3(grid), dim3(block), 0, 0, src, len, sink);
        hipLaunchKernelGGL(k_tail4, dim3(grid), dim3(block), 0, 0, src, sink);
    }
    CK(hipDeviceSynchronize());
    printf("bytes: k_lin %llu, k_heads %llu (4 x 16 B per record), k_hdl %llu, k_tail4 %llu (4 B per record)\n",
           (unsigned long long)(len / 16 * 16), (unsigned long long)(N * 64), (unsigned long long)(N * 16),
           (unsigned long long)(N * 4));
    return 0;
}
