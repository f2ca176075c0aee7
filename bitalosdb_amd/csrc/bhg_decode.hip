// bhg_decode.hip -- batched CRC / FNV-1 primitives and the decode dispatch.
//
//   k_crc_ranges / k_fnv_ranges   lane per range: crc.New(b).Value() and
//                                 hash.Fnv32 (internal/crc/crc.go:23-33,
//                                 internal/hash/fnv.go:19-23)
//   k_crc_long                    workgroup per LONG range (the per-table
//                                 indexhash_checksum, writer.go:476-478)
//   launch_decode                 NoCompressor: k_decode_tile
//                                 (bhg_decode_tile.hip); snappy: the header /
//                                 CRC pass of k_decode_stream
//                                 (bhg_decode_stream.hip), then k_snappy_rt
//                                 (bhg_snappy_dec.hip) after the size scan
#include "bhg_decode_stream.h"
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

// ---------------------------------------------------------------------------
// batched primitives
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_crc_ranges(const uint8_t *__restrict__ src, uint64_t src_len,
                                                    const bhg_handle *__restrict__ handles, uint32_t n,
                                                    uint32_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<8>::kWords];
    Crc4Lds<8>::fill(T);
    __syncthreads();
    const Crc4Lds<8> crc(T);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const bhg_handle h = handles[i];
        uint32_t r = 0;
        if (h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset)
            r = crc_mask(~crc_range(crc, 0xffffffffu, base + h.offset, h.length, end));
        out[i] = r;
    }
}

__global__ __launch_bounds__(256) void k_fnv_ranges(const uint8_t *__restrict__ src, uint64_t src_len,
                                                    const bhg_handle *__restrict__ handles, uint32_t n,
                                                    uint32_t *__restrict__ out) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const bhg_handle h = handles[i];
        uint32_t r = 0;
        if (h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset) r = fnv1_range(base + h.offset, h.length, end);
        out[i] = r;
    }
}

// k_crc_long: masked CRC-32C of a few LONG ranges -- the per-table
// indexhash_checksum verify of SURVEY 8(a) A6(ii): writer.go:476-478 stores
// crc.New(indexhash_data).Value() (internal/crc/crc.go:23-33) and a table open
// re-computes it over ~1.5 MB.  k_crc_ranges gives a range one lane, which
// walks 1.5 MB serially (~20 ms); here one workgroup takes a range:
//   * the range is cut into kLongChunk-byte chunks aligned to its END; chunk 0
//     holds the remainder (1..kLongChunk bytes) and runs from Go's initial
//     state ^0, every other chunk from state 0; one lane per chunk;
//   * lane 0 folds the chunk states in order, state = Z_4096(state) ^ crc0(chunk)
//     (CRC linearity: crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B));
//   * Z_4096 is built in LDS from the context's Z_1024 table (four applications
//     per entry); chunks are taken kLongPass at a time, the state carried over.
constexpr uint32_t kLongChunk = 4096, kLongPass = 2048, kLongThreads = 512;

__device__ __forceinline__ uint32_t zapply_tab(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

__global__ __launch_bounds__(kLongThreads) void k_crc_long(const uint8_t *__restrict__ src, uint64_t src_len,
                                                           const bhg_handle *__restrict__ handles, uint32_t n,
                                                           uint32_t *__restrict__ out, const uint32_t *__restrict__ gz1024) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<8>::kWords];
    __shared__ uint32_t Z1[1024], Z[1024], C[kLongPass];
    Crc4Lds<8>::fill(T);
    for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) Z1[t] = gz1024[t];
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) {
        uint32_t x = (t & 255u) << (8 * (t >> 8));  // S[k][i] = Z_4096(i << 8k)
#pragma unroll
        for (int r = 0; r < 4; r++) x = zapply_tab(Z1, x);
        Z[t] = x;
    }
    __syncthreads();
    const Crc4Lds<8> crc(T);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const bhg_handle h = handles[i];
        if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {  // as k_crc_ranges: 0
            if (threadIdx.x == 0) out[i] = 0;
            continue;
        }
        const uint64_t len = h.length, p = base + h.offset;
        const uint64_t nch = len ? (len + kLongChunk - 1) / kLongChunk : 0;
        const uint64_t t0 = len - (uint64_t)kLongChunk * (nch ? nch - 1 : 0);  // chunk 0 length
        uint32_t state = 0xffffffffu;  // crc.New: Go starts from ^0
        for (uint64_t k0 = 0; k0 < nch; k0 += kLongPass) {
            const uint64_t kend = nch - k0 < kLongPass ? nch : k0 + kLongPass;
            for (uint64_t k = k0 + threadIdx.x; k < kend; k += blockDim.x) {
                const uint64_t a = k == 0 ? p : p + t0 + (uint64_t)kLongChunk * (k - 1);
                C[k - k0] = crc_range(crc, k == 0 ? 0xffffffffu : 0u, a, k == 0 ? t0 : kLongChunk, end);
            }
            __syncthreads();
            if (threadIdx.x == 0)
                for (uint64_t k = k0; k < kend; k++) state = k == 0 ? C[0] : zapply_tab(Z, state) ^ C[k - k0];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[i] = crc_mask(~state);  // crc.go:31-33
    }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_decode(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         int codec, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    if (codec == BHG_CODEC_NONE) return launch_decode_tile(L, src, src_len, h, n, expected_crc, out);
    return launch_decode_stream(L, src, src_len, h, n, 1, expected_crc, out, sizes);
}

hipError_t launch_crc_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out) {
    hipLaunchKernelGGL(k_crc_ranges, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, out);
    return hipGetLastError();
}

hipError_t launch_crc_long(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           uint32_t *out) {
    const uint32_t grid = n < 65535u ? n : 65535u;
    hipLaunchKernelGGL(k_crc_long, dim3(grid), dim3(kLongThreads), 0, L.stream, src, src_len, h, n, out, L.ztab);
    return hipGetLastError();
}

hipError_t launch_fnv_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out) {
    hipLaunchKernelGGL(k_fnv_ranges, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, out);
    return hipGetLastError();
}

}  // namespace bhg
