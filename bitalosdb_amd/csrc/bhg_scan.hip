// bhg_scan.hip -- exclusive prefix sum over u64 (decoded-size -> output
// offsets for snappy values, record lengths -> record positions for encode).
// Reduce-then-scan: per-workgroup chunk sums, then a chunk-local scan plus base, the base
// summed by each workgroup from the chunk sums before it (up to 4,096 chunks = 8M elements;
// larger inputs scan the sums recursively).  Each workgroup covers 2048 elements (256
// threads x 8), so 1M sizes need 489 workgroups.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

#define SCAN_T 256
#define SCAN_PER 8
#define SCAN_CHUNK (SCAN_T * SCAN_PER)

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += t;
    }
    return v;
}

// block-wide exclusive scan of one value per thread; returns exclusive prefix, *total = sum
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[SCAN_T / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_T / 64; k++) {
        if (k < w) before += wsum[k];
        tot += wsum[k];
    }
    __syncthreads();
    *total = tot;
    return before + inc - v;
}

__global__ __launch_bounds__(SCAN_T) void k_chunk_sums(const uint64_t *__restrict__ in, uint64_t n,
                                                       uint64_t *__restrict__ sums) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_CHUNK;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        uint64_t idx = b0 + (uint64_t)threadIdx.x * SCAN_PER + k;
        if (idx < n) s += in[idx];
    }
    uint64_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// chunk-local exclusive scan + base (base = bases[blockIdx.x] or 0); in may alias out
__global__ __launch_bounds__(SCAN_T) void k_chunk_scan(const uint64_t *in, uint64_t *out, uint64_t n,
                                                       const uint64_t *__restrict__ bases, int write_total) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_CHUNK;
    uint64_t v[SCAN_PER];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        uint64_t idx = b0 + (uint64_t)threadIdx.x * SCAN_PER + k;
        v[k] = idx < n ? in[idx] : 0;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan(s, &tot) + (bases ? bases[blockIdx.x] : 0);
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        uint64_t idx = b0 + (uint64_t)threadIdx.x * SCAN_PER + k;
        if (idx < n) out[idx] = run;
        run += v[k];
    }
    if (write_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_T - 1) out[n] = run;
}

// chunk-local exclusive scan whose base is summed here from the chunk sums before it (nb <=
// kDirectChunks: at most 16 per thread, read from L2), the last chunk writing the total: two
// launches per scan instead of four (sums, recursive scan of the sums, chunk scan, total copy)
constexpr uint64_t kDirectChunks = SCAN_T * 16;
__global__ __launch_bounds__(SCAN_T) void k_chunk_scan_direct(const uint64_t *in, uint64_t *out, uint64_t n,
                                                              const uint64_t *__restrict__ sums) {
    uint64_t pre = 0;
    for (uint32_t k = threadIdx.x; k < blockIdx.x; k += SCAN_T) pre += sums[k];
    uint64_t base;
    block_excl_scan(pre, &base);
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_CHUNK;
    uint64_t v[SCAN_PER];
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        uint64_t idx = b0 + (uint64_t)threadIdx.x * SCAN_PER + k;
        v[k] = idx < n ? in[idx] : 0;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = block_excl_scan(s, &tot) + base;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        uint64_t idx = b0 + (uint64_t)threadIdx.x * SCAN_PER + k;
        if (idx < n) out[idx] = run;
        run += v[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == SCAN_T - 1) out[n] = run;
}

size_t scan_scratch_bytes(uint64_t n) {
    size_t bytes = 0;
    while (n > SCAN_CHUNK) {
        n = (n + SCAN_CHUNK - 1) / SCAN_CHUNK;
        bytes += (n + 1) * sizeof(uint64_t);
    }
    return bytes + 64;
}

// p[i * stride] += add (mod 2^64) over n entries: the pipelined snappy host path rebases a chunk's
// scanned value offsets onto the batch (stride 1) and its handles onto the chunk's staged bytes
// (stride 2: bhg_handle.offset, add = -lo)
__global__ __launch_bounds__(256) void k_add_u64(uint64_t *p, uint64_t n, uint64_t add, uint32_t stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i * stride] += add;
}

hipError_t launch_add_u64(const Launch &L, uint64_t *p, uint64_t n, uint64_t add, uint32_t stride) {
    if (n == 0 || add == 0) return hipSuccess;
    uint64_t grid = (n + 255) / 256;
    const uint64_t cap = (uint64_t)L.num_cus * 4;
    if (grid > cap) grid = cap;
    hipLaunchKernelGGL(k_add_u64, dim3((uint32_t)grid), dim3(256), 0, L.stream, p, n, add, stride);
    return hipGetLastError();
}

// dst <- src, n bytes, dst in page-locked host memory mapped into the device (the pipelined
// snappy host path's values: a copy kernel writes them over PCIe at the link rate, where a
// D2H copy may take a DMA engine that runs at half of it, scripts/lab/e2e_snappy/).  The
// caller places src so that src and dst agree mod 16: the bulk moves in aligned 16-B units,
// only a head and a tail of under 16 bytes go bytewise.
__global__ __launch_bounds__(256) void k_copy_out(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                  uint64_t n) {
    const uint64_t mis = (16u - ((uint64_t)dst & 15u)) & 15u;
    const uint64_t head = mis < n ? mis : n;
    const uint64_t nv = (n - head) / 16, t0 = head + nv * 16;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
    const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src + head);
    u32x4 *d4 = reinterpret_cast<u32x4 *>(dst + head);
    for (uint64_t i = tid; i < nv; i += stride) d4[i] = s4[i];
    if (tid < head) dst[tid] = src[tid];
    if (tid < n - t0) dst[t0 + tid] = src[t0 + tid];
}

hipError_t launch_copy_out(const Launch &L, const uint8_t *src, uint8_t *dst, uint64_t n) {
    if (n == 0) return hipSuccess;
    uint64_t grid = (n / 16 + 255) / 256;
    // one workgroup per 4 CUs: the link, not the grid, sets the rate (64 .. 1,024 workgroups
    // measured within 1 % on the snappy host path, profiles/r4/e2e_snappy/copy_out_grid.txt)
    const uint64_t cap = (uint64_t)L.num_cus / 4;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_copy_out, dim3((uint32_t)grid), dim3(256), 0, L.stream, src, dst, n);
    return hipGetLastError();
}

// exclusive scan of in[0..n) into out[0..n], out[n] = total.  in may equal out.
hipError_t launch_exclusive_scan_u64(const Launch &L, const uint64_t *in, uint64_t *out, uint64_t n, void *scratch) {
    if (n == 0) {
        return hipMemsetAsync(out, 0, sizeof(uint64_t), L.stream);
    }
    const uint64_t nb = (n + SCAN_CHUNK - 1) / SCAN_CHUNK;
    if (nb == 1) {
        hipLaunchKernelGGL(k_chunk_scan, dim3(1), dim3(SCAN_T), 0, L.stream, in, out, n, (const uint64_t *)nullptr, 1);
        return hipGetLastError();
    }
    uint64_t *sums = reinterpret_cast<uint64_t *>(scratch);
    uint8_t *rest = reinterpret_cast<uint8_t *>(scratch) + (nb + 1) * sizeof(uint64_t);
    hipLaunchKernelGGL(k_chunk_sums, dim3((uint32_t)nb), dim3(SCAN_T), 0, L.stream, in, n, sums);
    if (nb <= kDirectChunks) {
        hipLaunchKernelGGL(k_chunk_scan_direct, dim3((uint32_t)nb), dim3(SCAN_T), 0, L.stream, in, out, n,
                           (const uint64_t *)sums);
        return hipGetLastError();
    }
    hipError_t e = launch_exclusive_scan_u64(L, sums, sums, nb, rest);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_chunk_scan, dim3((uint32_t)nb), dim3(SCAN_T), 0, L.stream, in, out, n, (const uint64_t *)sums, 0);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // total = sums[nb]
    return hipMemcpyAsync(out + n, sums + nb, sizeof(uint64_t), hipMemcpyDeviceToDevice, L.stream);
}

}  // namespace bhg
