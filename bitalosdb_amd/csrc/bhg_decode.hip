// bhg_decode.hip -- batched CRC / FNV-1 primitives and the decode dispatch.
//
//   k_crc_ranges / k_fnv_ranges   lane per range: crc.New(b).Value() and
//                                 hash.Fnv32 (internal/crc/crc.go:23-33,
//                                 internal/hash/fnv.go:19-23)
//   k_crc_long_part / _join       LONG ranges, up to 64 workgroups each (the
//                                 per-table indexhash_checksum, writer.go:476-478)
//   launch_decode                 NoCompressor: k_decode_tile
//                                 (bhg_decode_tile.hip); snappy: the header /
//                                 CRC pass of k_decode_stream
//                                 (bhg_decode_stream.hip), then k_snappy_rt
//                                 (bhg_snappy_dec.hip) after the size scan
#include "bhg_crc_tables.h"
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

// k_crc_long_part + k_crc_long_join: masked CRC-32C of LONG ranges -- the per-table
// indexhash_checksum of SURVEY 8(a) A6(ii): writer.go:476-478 stores
// crc.New(indexhash_data).Value() (internal/crc/crc.go:23-33); a table open re-computes it,
// and the table tail (bhg_tail.hip) writes it.  A range is cut into 64 x 256 spans of
// 2^(8+s) bytes aligned to its END (s the smallest with 64 x 256 x 2^(8+s) >= its length),
// so every span is full except the first non-empty one, which starts at byte 0 and runs from
// Go's initial state ^0; every other span runs from state 0.  A lane CRCs one span as four
// interleaved chains over its quarters (chain 0 from the span's initial state, the others
// from 0), folded with Z_{quarter}; a partial first span runs as one chain.  Then, by CRC
// linearity over GF(2),
//     crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B),
// a workgroup (one of 64 parts) folds its 256 span states as a tree whose right subtrees are
// always full (level l shifts by Z_{2^l spans}), and one wave per range folds the 64 part
// states the same way (Z_{2^(8+l) spans}).  Empty spans left of the first hold 0, and Z(0) = 0.
// The shift tables Z_{2^(6+j)} come from the context (bhg_crc_tables.h kXLong).
// History: round 3's one-workgroup-per-range kernel took ~0.6 ms for a 10-MB index (one CU);
// round 4 spread a range over up to 64 workgroups with one serial 1-KiB chain per lane (23 x
// 1.51 MB: 0.057 ms, the chain's dependent LDS lookups); round 5: 256-B spans, four chains
// (0.0295 ms; k_crc_long_part 21.8-23.5 us + k_crc_long_join 4.1-4.5 us).
// 256 lanes per part: 512 (8 waves, two workgroups per CU) measured 28.5 against 23.5 us, and
// the conflict-free CrcR8 (two VALU per lookup address) 27.8 against Crc4Lds<8>'s 23.5 us
// (23 x 1.51 MB, profiles/r5/crc_long/)
constexpr uint32_t kLongTLog = 8;  // log2 of the spans (lanes) per part
constexpr uint32_t kLongParts = 64, kLongThreads = 1u << kLongTLog, kLongSpan0 = 8;
// every shift the kernels take exists: the quarter fold Z_{2^(6+s)} up to the join's last level
// Z_{2^31} (64 x 256 spans of 2^18 B at s = 10 cover any u32 length)
static_assert(kLongSpan0 - 2 >= kXLongLo && 31 - kXLongLo < kXLongN, "long shift set");

__device__ __forceinline__ uint32_t zapply_tab(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

// the range's span exponent s and span count (spans of 2^(8+s) bytes covering len)
__device__ __forceinline__ void long_geo(uint64_t len, uint32_t &s, uint64_t &nspan) {
    s = 0;
    while (((uint64_t)kLongParts * kLongThreads << (kLongSpan0 + s)) < len) s++;
    nspan = (len + (1ull << (kLongSpan0 + s)) - 1) >> (kLongSpan0 + s);
}

// Z_{2^x} in the context's long set
__device__ __forceinline__ const uint32_t *zlong(const uint32_t *zl, uint32_t x) {
    return zl + (uint64_t)(x - kXLongLo) * 1024;
}

// raw CRC of the full span [A, A + 2^(8+s)) (any alignment, inside the source): four chains over
// its quarters of 2^(6+s) bytes, 64 B of each per step, chain 0 from c0; folded with Zq = Z_quarter
template <class Tab>
__device__ __forceinline__ uint32_t span_crc4(const Tab &crc, const uint32_t *Zq, uint32_t c0, uint64_t A, uint32_t s,
                                              uint64_t end) {
    const uint64_t aa = A & ~3ull, Q = 64ull << s;
    const uint32_t z = (uint32_t)(A & 3);
    uint32_t cc[4] = {c0, 0u, 0u, 0u};
    for (uint32_t it = 0; it < (1u << s); it++) {
        uint32_t w[4][17];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t a = aa + (uint64_t)j * Q + 64ull * it;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = gld<u32x4_a4>(a + 16 * q);  // inside the span: below end
                w[j][4 * q] = x.x; w[j][4 * q + 1] = x.y; w[j][4 * q + 2] = x.z; w[j][4 * q + 3] = x.w;
            }
            w[j][16] = z ? ld32_safe(a + 64, end) : 0u;  // the last quarter's may pass the source end
        }
#pragma unroll
        for (int t = 0; t < 16; t++)
#pragma unroll
            for (int j = 0; j < 4; j++) cc[j] = crc.word(cc[j], __builtin_amdgcn_alignbyte(w[j][t + 1], w[j][t], z));
    }
    return zapply_tab(Zq, zapply_tab(Zq, zapply_tab(Zq, cc[0]) ^ cc[1]) ^ cc[2]) ^ cc[3];
}

__global__ __launch_bounds__(kLongThreads) void k_crc_long_part(const uint8_t *__restrict__ src, uint64_t src_len,
                                                                const bhg_handle *__restrict__ handles,
                                                                uint32_t *__restrict__ part,
                                                                const uint32_t *__restrict__ zl) {
    const uint32_t i = blockIdx.y, p = blockIdx.x, t = threadIdx.x;
    const bhg_handle h = handles[i];
    const bool ok = h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
    const uint64_t len = ok ? h.length : 0;
    uint32_t s;
    uint64_t nspan;
    long_geo(len, s, nspan);
    const uint64_t first = (uint64_t)kLongParts * kLongThreads - nspan;  // global index of the first non-empty span
    if ((uint64_t)(p + 1) * kLongThreads <= first) {                    // an empty part (whole workgroup)
        if (t == 0) part[(uint64_t)i * kLongParts + p] = 0;
        return;
    }
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Lds<8>::kWords];
    Crc4Lds<8>::fill(T);
    const Crc4Lds<8> crc(T);
    __shared__ uint32_t Z[kLongTLog * 1024], Zq[1024], st[kLongThreads];
    const uint32_t *zs = zlong(zl, kLongSpan0 + s);  // Z_{span 2^l}, l < kLongTLog: contiguous in the set
    for (uint32_t w = t; w < kLongTLog * 1024; w += kLongThreads) Z[w] = zs[w];
    const uint32_t *zq = zlong(zl, kLongSpan0 - 2 + s);  // Z_{span / 4}
    for (uint32_t w = t; w < 1024; w += kLongThreads) Zq[w] = zq[w];
    __syncthreads();
    const uint64_t g = (uint64_t)p * kLongThreads + t;
    uint32_t c = 0;
    if (g >= first) {
        const uint64_t span = 1ull << (kLongSpan0 + s), k = g - first;  // k: span index from the range start
        const uint64_t e = len - (nspan - 1 - k) * span;               // end of the span (exclusive)
        const uint64_t b = k == 0 ? 0 : e - span;
        const uint64_t A = (uint64_t)src + h.offset + b, end = (uint64_t)src + src_len;
        if (e - b == span) c = span_crc4(crc, Zq, k == 0 ? 0xffffffffu : 0u, A, s, end);
        else c = crc_range(crc, 0xffffffffu, A, e - b, end);  // a partial first span
    }
    st[t] = c;
    __syncthreads();
#pragma unroll
    for (uint32_t l = 0; l < kLongTLog; l++) {
        const uint32_t w = 1u << l;
        if ((t & (2 * w - 1)) == 2 * w - 1) st[t] = zapply_tab(Z + l * 1024, st[t - w]) ^ st[t];
        __syncthreads();
    }
    if (t == kLongThreads - 1) part[(uint64_t)i * kLongParts + p] = st[t];
}

// one wave per range: lane = part
__global__ __launch_bounds__(64) void k_crc_long_join(uint64_t src_len, const bhg_handle *__restrict__ handles,
                                                      const uint32_t *__restrict__ part, const uint32_t *__restrict__ zl,
                                                      uint32_t *__restrict__ out) {
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    const bhg_handle h = handles[i];
    const bool ok = h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
    const uint64_t len = ok ? h.length : 0;
    uint32_t s;
    uint64_t nspan;
    long_geo(len, s, nspan);
    uint32_t v = part[(uint64_t)i * kLongParts + lane];
#pragma unroll
    for (uint32_t l = 0; l < 6; l++) {
        const uint32_t w = 1u << l;
        const uint32_t left = __shfl(v, (int)(lane >= w ? lane - w : 0), 64);
        if ((lane & (2 * w - 1)) == 2 * w - 1) v = zapply_tab(zlong(zl, kLongSpan0 + s + kLongTLog + l), left) ^ v;  // 2^l parts
    }
    if (lane == 63) {
        const uint32_t state = len ? v : 0xffffffffu;  // crc.New of nothing: ^0
        out[i] = ok ? crc_mask(~state) : 0u;           // crc.go:31-33; out of bounds: 0, as k_crc_ranges
    }
}

size_t crc_long_scratch_bytes(uint32_t n) { return (size_t)n * kLongParts * 4; }

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_decode(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         int codec, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes, uint32_t *lists,
                         void *long_scratch) {
    if (codec == BHG_CODEC_NONE) return launch_decode_tile(L, src, src_len, h, n, expected_crc, out);
    if (lists)  // the list sizes (the header pass appends, launch_snappy reads)
        if (hipError_t e = hipMemsetAsync(lists, 0, 4 * kSnapListHdr, L.stream)) return e;
    return launch_decode_stream(L, src, src_len, h, n, 1, expected_crc, out, sizes, lists, long_scratch);
}

hipError_t launch_crc_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out) {
    hipLaunchKernelGGL(k_crc_ranges, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, out);
    return hipGetLastError();
}

hipError_t launch_crc_long(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           uint32_t *out, void *scratch) {
    uint32_t *part = reinterpret_cast<uint32_t *>(scratch);
    const uint32_t *zl = L.xtab + kXLong;
    for (uint32_t i0 = 0; i0 < n; i0 += 65535u) {  // gridDim.y <= 65535
        const uint32_t m = n - i0 < 65535u ? n - i0 : 65535u;
        hipLaunchKernelGGL(k_crc_long_part, dim3(kLongParts, m), dim3(kLongThreads), 0, L.stream, src, src_len, h + i0,
                           part, zl);
        hipLaunchKernelGGL(k_crc_long_join, dim3(m), dim3(64), 0, L.stream, src_len, h + i0, part, zl, out + i0);
        if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
}

hipError_t launch_fnv_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out) {
    hipLaunchKernelGGL(k_fnv_ranges, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, out);
    return hipGetLastError();
}

}  // namespace bhg
