// bhg_sort.hip -- stable LSD radix sort of (u64 key, u32 value) pairs for the
// table tail (bhg_tail.hip sorts the adds of a batch by (table, khash) with
// the add order kept inside equal keys, as Writer.updateHash sees them).
//
// 8-bit digits over key bits [0, end_bit), one pass per digit:
//   k_rs_hist     wave per 1,024-item block: digit counts in LDS ->
//                 counts[digit * nblocks + block]
//   scan          exclusive scan of counts (bhg_scan.hip): the output base of
//                 every (digit, block), digit-major, so blocks keep their order
//   k_rs_scatter  wave per block, items in order 64 at a time: an item's rank
//                 among the lanes with its digit comes from 8 ballots (one per
//                 digit bit) and a popcount below the lane; the last lane of a
//                 digit advances that digit's base in LDS.  A single wave walks
//                 its block in order, so the pass is stable.
// Off the hot path (one sort per table-tail call); no library code.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

constexpr uint32_t kRsItems = 1024;  // items per block (16 per lane)

__global__ __launch_bounds__(64) void k_rs_hist(const uint64_t *__restrict__ keys, uint32_t n, uint32_t shift,
                                                uint32_t nblocks, uint64_t *__restrict__ counts) {
    __shared__ uint32_t h[256];
    const uint32_t lane = threadIdx.x, b = blockIdx.x;
    for (uint32_t d = lane; d < 256; d += 64) h[d] = 0;
    __syncthreads();
    const uint32_t i0 = b * kRsItems;
    for (uint32_t it = 0; it < kRsItems / 64; it++) {
        const uint32_t i = i0 + it * 64 + lane;
        if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    for (uint32_t d = lane; d < 256; d += 64) counts[(size_t)d * nblocks + b] = h[d];
}

__global__ __launch_bounds__(64) void k_rs_scatter(const uint64_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                   uint64_t *__restrict__ kout, uint32_t *__restrict__ vout, uint32_t n,
                                                   uint32_t shift, uint32_t nblocks,
                                                   const uint64_t *__restrict__ offs) {
    __shared__ uint64_t base[256];
    const uint32_t lane = threadIdx.x, b = blockIdx.x;
    for (uint32_t d = lane; d < 256; d += 64) base[d] = offs[(size_t)d * nblocks + b];
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t i0 = b * kRsItems;
    for (uint32_t it = 0; it < kRsItems / 64; it++) {
        const uint32_t i = i0 + it * 64 + lane;
        const bool v = i < n;
        const uint64_t k = v ? kin[i] : 0ull;
        const uint32_t x = v ? vin[i] : 0u;
        const uint32_t d = (uint32_t)(k >> shift) & 255u;
        // lanes holding an item with this lane's digit
        uint64_t eq = __ballot(v);
#pragma unroll
        for (uint32_t bit = 0; bit < 8; bit++) {
            const uint64_t m = __ballot((d >> bit) & 1u);
            eq &= ((d >> bit) & 1u) ? m : ~m;
        }
        if (v) {
            const uint64_t pos = base[d] + (uint64_t)__builtin_popcountll(eq & below);
            kout[pos] = k;
            vout[pos] = x;
            if ((eq >> lane) == 1ull) base[d] += (uint64_t)__builtin_popcountll(eq);  // the digit's last lane
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

size_t radix_sort_scratch_bytes(uint32_t n) {
    const uint64_t nb = ((uint64_t)n + kRsItems - 1) / kRsItems, nc = 256 * (nb ? nb : 1);
    return ((nc * 8 + 255) & ~(uint64_t)255) + scan_scratch_bytes(nc);
}

hipError_t launch_radix_sort_pairs(const Launch &L, uint64_t *keys, uint64_t *keys_out, uint32_t *vals,
                                   uint32_t *vals_out, uint32_t n, uint32_t end_bit, void *scratch) {
    if (n == 0) return hipSuccess;
    const uint32_t nb = (uint32_t)(((uint64_t)n + kRsItems - 1) / kRsItems);
    const uint64_t nc = 256ull * nb;
    uint64_t *counts = reinterpret_cast<uint64_t *>(scratch);
    void *scan_s = reinterpret_cast<uint8_t *>(scratch) + ((nc * 8 + 255) & ~(uint64_t)255);
    const uint32_t passes = end_bit == 0 ? 1u : (end_bit + 7) / 8;
    // pass p reads src and writes dst; the last pass writes keys_out / vals_out
    uint64_t *ka = keys, *kb = keys_out;
    uint32_t *va = vals, *vb = vals_out;
    if ((passes & 1u) == 0) {  // an even number of passes ends where it started: start in the output
        if (hipError_t e = hipMemcpyAsync(keys_out, keys, (size_t)n * 8, hipMemcpyDeviceToDevice, L.stream)) return e;
        if (hipError_t e = hipMemcpyAsync(vals_out, vals, (size_t)n * 4, hipMemcpyDeviceToDevice, L.stream)) return e;
        ka = keys_out; kb = keys;
        va = vals_out; vb = vals;
    }
    for (uint32_t p = 0; p < passes; p++) {
        const uint32_t shift = 8 * p;
        hipLaunchKernelGGL(k_rs_hist, dim3(nb), dim3(64), 0, L.stream, (const uint64_t *)ka, n, shift, nb, counts);
        if (hipError_t e = hipGetLastError()) return e;
        if (hipError_t e = launch_exclusive_scan_u64(L, counts, counts, nc, scan_s)) return e;
        hipLaunchKernelGGL(k_rs_scatter, dim3(nb), dim3(64), 0, L.stream, (const uint64_t *)ka, (const uint32_t *)va,
                           kb, vb, n, shift, nb, (const uint64_t *)counts);
        if (hipError_t e = hipGetLastError()) return e;
        uint64_t *tk = ka; ka = kb; kb = tk;
        uint32_t *tv = va; va = vb; vb = tv;
    }
    return hipSuccess;
}

}  // namespace bhg
