// bhg_longcrc.hip -- the masked CRC-32C of LONG records (crc.New(record).Value(),
// internal/crc/crc.go:19-33, over Reader.readData's buffer, bithash/reader.go:233-272) with the
// whole chip, for NoCompressor batches of long records (bithash holds KKV
// values up to 256 MiB, bithash/writer.go:43).
//
// Why: the tile kernel (bhg_decode_tile.hip) gives a record 8 lanes of one wave, and a record of
// 1-4 MiB then takes thousands of synchronous window loads while the rest of the GPU idles:
// 21.8 ms for a batch of 7,000 values of 4 KiB - 4 MiB (bench.py --config bigval, rocprofv3,
// profiles/r6/bigval/).  Here every record longer than kLongRec is cut into 64-KiB chunks
// aligned to its END (chunk 0, the first, may be partial and holds Go's initial state ^0), and
// every chunk of every record is one work item of a persistent grid:
//   k_lc_count  lane per handle: chunks of a long in-bounds record (else 0)
//   (scan)      chunk base per record, total
//   k_lc_emit   lane per record: the (record, chunk) list; per-record accumulators zeroed
//   k_lc_chunk  workgroup per chunk: 512 lanes x 128-B spans (two chains each), the spans'
//               states folded as a tree whose right subtrees are full (level l: Z_{128 * 2^l}),
//               then shifted to the record end (Z_{64 KiB * j} by the bits of j) and XOR-ed into
//               the record's accumulator -- by CRC linearity over GF(2),
//                   crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B),
//               the record state is the XOR of its chunks' shifted states, in any order.  The
//               workgroup that adds the last chunk (a device-scope counter per record) writes
//               the descriptor's crc and, against expected_crc, its status.
// The tile kernel's LONG instantiation left those descriptors with crc 0 and an unchecked status.
#include "bhg_crc_tables.h"
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

constexpr uint32_t kLcChunk = 65536;  // bytes per work item
constexpr uint32_t kLcThreads = 512;  // lanes per workgroup: one 128-B span each
constexpr uint32_t kLcTree = 9;       // fold levels: Z_128 .. Z_32K
constexpr uint32_t kLcDist = 6;       // end shifts Z_64K .. Z_2M in LDS (longer records: the context's set)
static_assert(kLcThreads * 128 == kLcChunk && (1u << kLcTree) == kLcThreads, "chunk geometry");

// LDS layout (bytes): CrcR8 tables, tree shifts, Z_64 (chain fold), end shifts, span states
constexpr uint32_t kLcT = 0, kLcZt = CrcR8::kBytes, kLcZq = kLcZt + kLcTree * 4096, kLcZd = kLcZq + 4096,
                   kLcSt = kLcZd + kLcDist * 4096, kLcBytes = kLcSt + kLcThreads * 4;

__device__ __forceinline__ uint32_t zap(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

__device__ __forceinline__ bool long_rec(const bhg_handle &h, uint64_t src_len) {
    return h.length > kLongRec && h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
}

// Z_{2^x} in the context's long shift set (bhg_crc_tables.h kXLong: x = 6 .. 31)
__device__ __forceinline__ const uint32_t *zlong(const uint32_t *zl, uint32_t x) { return zl + 1024u * (x - kXLongLo); }

// crc from the record's final state: the descriptor's crc, and its status against expected_crc
// (the tile kernel checked every other field; RECORD_NIL records get their CRC too)
__device__ __forceinline__ void lc_finish(bhg_desc *out, uint32_t i, uint32_t state, const uint32_t *expected_crc) {
    uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
    const uint32_t crc = crc_mask(~state);  // crc.go:31-33
    dw[8] = crc;
    if (dw[9] == BHG_ST_OK && expected_crc != nullptr && expected_crc[i] != crc) dw[9] = BHG_ST_CRC_MISMATCH;
}

// raw CRC of the full 128-B span [A, A + 128) from state c0: two chains over its halves, folded with Z_64
__device__ __forceinline__ uint32_t span128(const CrcR8 &crc, const uint32_t *Z64, uint32_t c0, uint64_t A, uint64_t end) {
    const uint64_t aa = A & ~3ull;
    const uint32_t z = (uint32_t)(A & 3);
    uint32_t w[2][17];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const uint64_t a = aa + 64ull * j;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 x = gld<u32x4_a4>(a + 16 * q);
            w[j][4 * q] = x.x; w[j][4 * q + 1] = x.y; w[j][4 * q + 2] = x.z; w[j][4 * q + 3] = x.w;
        }
        w[j][16] = z ? ld32_safe(a + 64, end) : 0u;
    }
    uint32_t c[2] = {c0, 0u};
#pragma unroll
    for (int t = 0; t < 16; t++)
#pragma unroll
        for (int j = 0; j < 2; j++) c[j] = crc.word(c[j], __builtin_amdgcn_alignbyte(w[j][t + 1], w[j][t], z));
    return zap(Z64, c[0]) ^ c[1];
}

}  // namespace

__global__ __launch_bounds__(256) void k_lc_count(const bhg_handle *__restrict__ h, uint32_t n, uint64_t src_len,
                                                  uint64_t *__restrict__ cnt) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const bhg_handle x = h[i];
        cnt[i] = long_rec(x, src_len) ? ((uint64_t)x.length + kLcChunk - 1) / kLcChunk : 0ull;
    }
}

// acc[2 i] the record's XOR of shifted chunk states, acc[2 i + 1] its chunks done.  A record whose
// chunks would pass the list's capacity (only when handles overlap: the capacity holds every chunk
// of records that do not) goes to the overflow list, walked chunk by chunk by one workgroup.
__global__ __launch_bounds__(256) void k_lc_emit(const uint64_t *__restrict__ base, uint32_t n, uint64_t cap,
                                                 uint2 *__restrict__ ent, uint32_t *__restrict__ acc,
                                                 uint32_t *__restrict__ ovf) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b0 = base[i], b1 = base[i + 1];
        if (b1 == b0) continue;
        acc[2 * i] = 0;
        acc[2 * i + 1] = 0;
        if (b1 <= cap) {
            for (uint64_t k = 0; k < b1 - b0; k++) ent[b0 + k] = make_uint2(i, (uint32_t)k);
        } else {
            ovf[1 + atomicAdd(ovf, 1u)] = i;
            // the list ends inside this record (base is non-decreasing: every later record
            // overflows too): its list slots up to cap are marked empty
            for (uint64_t k = b0; k < cap; k++) ent[k] = make_uint2(0xffffffffu, 0u);
        }
    }
}

__global__ __launch_bounds__(kLcThreads) void k_lc_chunk(const uint8_t *__restrict__ src, uint64_t src_len,
                                                        const bhg_handle *__restrict__ h, uint32_t n,
                                                        const uint32_t *__restrict__ expected_crc,
                                                        bhg_desc *__restrict__ out, const uint64_t *__restrict__ base,
                                                        uint64_t cap, const uint2 *__restrict__ ent,
                                                        uint32_t *__restrict__ acc, const uint32_t *__restrict__ ovf,
                                                        const uint32_t *__restrict__ zl) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLcBytes / 4];
    const uint32_t t = threadIdx.x;
    const uint64_t total = base[n], nlist = total < cap ? total : cap;
    const uint32_t novf = *ovf;
    if (blockIdx.x >= nlist && blockIdx.x >= novf) return;
    const uint32_t tb = lds_addr(lds);
    CrcR8::fill(tb + kLcT);
    uint32_t *Zt = lds + kLcZt / 4, *Zq = lds + kLcZq / 4, *Zd = lds + kLcZd / 4, *st = lds + kLcSt / 4;
    for (uint32_t w = t; w < kLcTree * 1024; w += kLcThreads) Zt[w] = zlong(zl, 7)[w];  // Z_128 .. Z_32K: contiguous
    for (uint32_t w = t; w < 1024; w += kLcThreads) Zq[w] = zlong(zl, 6)[w];
    for (uint32_t w = t; w < kLcDist * 1024; w += kLcThreads) Zd[w] = zlong(zl, 16)[w];  // Z_64K .. Z_2M
    __syncthreads();
    const CrcR8 crc(tb + kLcT);
    const uint64_t sb = (uint64_t)src, end = sb + src_len;
    // the state of chunk k of record i, as a raw CRC contribution ending at the chunk's end
    // (every thread returns it; the tree leaves it in st[kLcThreads - 1])
    auto chunk_state = [&](uint32_t i, uint32_t k) -> uint32_t {
        const bhg_handle x = h[i];
        const uint32_t L = x.length, nch = (uint32_t)(((uint64_t)L + kLcChunk - 1) / kLcChunk);
        const uint64_t P = sb + x.offset;
        const uint32_t ce = L - kLcChunk * (nch - 1 - k), cb = k == 0 ? 0u : ce - kLcChunk;
        const int64_t se = (int64_t)ce - 128 * (int64_t)(kLcThreads - 1 - t), ss = se - 128;
        uint32_t c = 0;
        if (se > (int64_t)cb) {
            if (ss >= (int64_t)cb) c = span128(crc, Zq, (k == 0 && ss == 0) ? 0xffffffffu : 0u, P + (uint64_t)ss, end);
            else c = crc_range(crc, 0xffffffffu, P, (uint64_t)se, end);  // the partial first span (chunk 0)
        }
        st[t] = c;
        __syncthreads();
#pragma unroll
        for (uint32_t l = 0; l < kLcTree; l++) {
            const uint32_t w = 1u << l;
            if ((t & (2 * w - 1)) == 2 * w - 1) st[t] = zap(Zt + 1024 * l, st[t - w]) ^ st[t];
            __syncthreads();
        }
        const uint32_t v = st[kLcThreads - 1];
        __syncthreads();  // st is rewritten by the next chunk
        return v;
    };
    // the list: chunk g, its state shifted to the record end and XOR-ed in; the last chunk of a
    // record completes its descriptor
    for (uint64_t g = blockIdx.x; g < nlist; g += gridDim.x) {
        const uint2 e = ent[g];
        if (e.x == 0xffffffffu) continue;  // past the last record that fits (workgroup-uniform)
        const uint32_t v = chunk_state(e.x, e.y);
        if (t == 0) {
            const uint32_t L = h[e.x].length, nch = (uint32_t)(((uint64_t)L + kLcChunk - 1) / kLcChunk);
            uint32_t c = v;
            for (uint32_t j = nch - 1 - e.y, b = 0; j; j >>= 1, b++)
                if (j & 1) c = zap(b < kLcDist ? Zd + 1024 * b : zlong(zl, 16 + b), c);  // Z_{64 KiB * 2^b}
            atomicXor(acc + 2 * e.x, c);
            __threadfence();
            if (atomicAdd(acc + 2 * e.x + 1, 1u) == nch - 1) {
                __threadfence();
                lc_finish(out, e.x, atomicXor(acc + 2 * e.x, 0u), expected_crc);
            }
        }
    }
    // overflow records: one workgroup walks all chunks of one record, Horner over Z_64K
    for (uint32_t q = blockIdx.x; q < novf; q += gridDim.x) {
        const uint32_t i = ovf[1 + q];
        const uint32_t L = h[i].length, nch = (uint32_t)(((uint64_t)L + kLcChunk - 1) / kLcChunk);
        uint32_t s = 0;
        for (uint32_t k = 0; k < nch; k++) {
            const uint32_t v = chunk_state(i, k);
            s = k == 0 ? v : zap(Zd, s) ^ v;
        }
        if (t == 0) lc_finish(out, i, s, expected_crc);
    }
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static uint64_t lc_cap(uint32_t n, uint64_t src_len) { return src_len / kLcChunk + n + 1; }

size_t long_crc_scratch_bytes(uint32_t n, uint64_t src_len) {
    return al256(((size_t)n + 1) * 8) + al256(scan_scratch_bytes(n)) + al256((size_t)n * 8) +
           al256((size_t)lc_cap(n, src_len) * 8) + al256(((size_t)n + 1) * 4);
}

hipError_t launch_long_crc(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           const uint32_t *expected_crc, bhg_desc *out, void *scratch) {
    uint8_t *sp = static_cast<uint8_t *>(scratch);
    uint64_t *base = reinterpret_cast<uint64_t *>(sp);
    sp += al256(((size_t)n + 1) * 8);
    void *scan = sp;
    sp += al256(scan_scratch_bytes(n));
    uint32_t *acc = reinterpret_cast<uint32_t *>(sp);
    sp += al256((size_t)n * 8);
    uint2 *ent = reinterpret_cast<uint2 *>(sp);
    const uint64_t cap = lc_cap(n, src_len);
    sp += al256((size_t)cap * 8);
    uint32_t *ovf = reinterpret_cast<uint32_t *>(sp);
    hipLaunchKernelGGL(k_lc_count, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, h, n, src_len, base);
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = launch_exclusive_scan_u64(L, base, base, n, scan)) return e;
    if (hipError_t e = hipMemsetAsync(ovf, 0, 4, L.stream)) return e;
    hipLaunchKernelGGL(k_lc_emit, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, base, n, cap, ent, acc, ovf);
    // persistent: one workgroup per CU (the LDS tables), chunks grid-strided
    hipLaunchKernelGGL(k_lc_chunk, dim3(L.num_cus), dim3(kLcThreads), 0, L.stream, src, src_len, h, n, expected_crc, out,
                       base, cap, ent, acc, ovf, L.xtab + kXLong);
    return hipGetLastError();
}

}  // namespace bhg
