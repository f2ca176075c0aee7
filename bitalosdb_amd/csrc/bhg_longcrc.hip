// bhg_longcrc.hip -- the masked CRC-32C of LONG records (crc.New(record).Value(),
// internal/crc/crc.go:19-33, over Reader.readData's buffer, bithash/reader.go:233-272) with the
// whole chip, for batches of long records (bithash holds KKV values up to 256
// MiB, bithash/writer.go:43): the NoCompressor decode and the snappy header pass leave them here.
//
// Why: the tile kernel (bhg_decode_tile.hip) gives a record 8 lanes of one wave, and a record of
// 1-4 MiB then takes thousands of synchronous window loads while the rest of the GPU idles:
// 21.8 ms for a batch of 7,000 values of 4 KiB - 4 MiB (bench.py --config bigval, rocprofv3,
// profiles/r6/bigval/).  Here every record longer than kLongRec is cut into 8-KiB pieces aligned
// to its END (piece 0, the first, may be partial and holds Go's initial state ^0), and every piece
// of every record is one WAVE's work item of a persistent grid:
//   k_lc_count  lane per handle: pieces of a long in-bounds record (else 0)
//   (scan)      piece base per record, total
//   k_lc_emit   lane per record: its list entries {piece end address, bytes, first?, shift}
//   k_lc_piece  wave per piece: 64 lanes x 128-B spans (two chains each), the spans' states folded
//               by a 6-level tree across the lanes (level l: Z_{128 * 2^l}, ds_bpermute), then
//               shifted to the record end (Z_{8 KiB * j} by the bits of j) and stored -- by CRC
//               linearity over GF(2),
//                   crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B),
//               the record state is the XOR of its pieces' shifted states, in any order.  The
//               next piece's spans are loaded while this one is computed; no barriers, no atomics.
//   k_lc_fin    lane per record: the XOR of its pieces' states -> the descriptor's crc and, against
//               expected_crc, its status.
// (Round 6's first cut took 64-KiB chunks per 512-thread workgroup with a 9-level tree across
// waves (a barrier per level) and an atomic hand-off per chunk: bigval NoCompressor 2.16 ms.)
// The tile kernel's LONG instantiation left those descriptors with crc 0 and an unchecked status.
#include "bhg_crc_tables.h"
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

constexpr uint32_t kLcPiece = 8192;   // bytes per work item (one wave: 64 lanes x 128 B)
// 16 waves per workgroup (one workgroup per CU: the LDS tables; 128 VGPRs): 8 waves (169 VGPRs)
// measured 2,316 against 2,550-2,573 GiB/s for the bigval NoCompressor decode
constexpr uint32_t kLcThreads = 1024;
constexpr uint32_t kLcTree = 9;       // shift tables Z_128 .. Z_32K (tree levels 0-5, end shifts 6-8)
constexpr uint32_t kLcDist = 6;       // end shifts Z_64K .. Z_2M in LDS (longer records: the context's set)

// LDS layout (bytes): CrcR8 tables, Z_128 .. Z_32K, Z_64 (chain fold), Z_64K .. Z_2M
constexpr uint32_t kLcT = 0, kLcZt = CrcR8::kBytes, kLcZq = kLcZt + kLcTree * 4096, kLcZd = kLcZq + 4096,
                   kLcBytes = kLcZd + kLcDist * 4096;

__device__ __forceinline__ uint32_t zap(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

__device__ __forceinline__ bool long_rec(const bhg_handle &h, uint64_t src_len) {
    return h.length > kLongRec && h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
}

// Z_{2^x} in the context's long shift set (bhg_crc_tables.h kXLong: x = 6 .. 31)
__device__ __forceinline__ const uint32_t *zlong(const uint32_t *zl, uint32_t x) { return zl + 1024u * (x - kXLongLo); }

// crc from the record's final state: the descriptor's crc, and its status against expected_crc
// (the tile kernel checked every other field; RECORD_NIL records get their CRC too) -- or, for the
// encoder (crc_out non-null), crc_out[i] alone
__device__ __forceinline__ void lc_finish(bhg_desc *out, uint32_t *crc_out, uint32_t i, uint32_t state,
                                          const uint32_t *expected_crc) {
    const uint32_t crc = crc_mask(~state);  // crc.go:31-33
    if (crc_out != nullptr) {
        crc_out[i] = crc;
        return;
    }
    uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
    dw[8] = crc;
    if (dw[9] == BHG_ST_OK && expected_crc != nullptr && expected_crc[i] != crc) dw[9] = BHG_ST_CRC_MISMATCH;
}

// a 128-B span [A, A + 128): span_load issues its loads, span_crc its raw CRC from state c0 (two
// chains over its halves, folded with Z_64)
struct Span {
    uint32_t w[2][17];
};
__device__ __forceinline__ void span_load(Span &S, uint64_t A, uint64_t end) {
    const uint64_t aa = A & ~3ull;
    const uint32_t z = (uint32_t)(A & 3);
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const uint64_t a = aa + 64ull * j;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 x = gld<u32x4_a4>(a + 16 * q);
            S.w[j][4 * q] = x.x; S.w[j][4 * q + 1] = x.y; S.w[j][4 * q + 2] = x.z; S.w[j][4 * q + 3] = x.w;
        }
        S.w[j][16] = z ? ld32_safe(a + 64, end) : 0u;
    }
}
__device__ __forceinline__ uint32_t span_crc(const CrcR8 &crc, const uint32_t *Z64, uint32_t c0, uint64_t A, const Span &S) {
    const uint32_t z = (uint32_t)(A & 3);
    uint32_t c[2] = {c0, 0u};
#pragma unroll
    for (int t = 0; t < 16; t++)
#pragma unroll
        for (int j = 0; j < 2; j++) c[j] = crc.word(c[j], __builtin_amdgcn_alignbyte(S.w[j][t + 1], S.w[j][t], z));
    return zap(Z64, c[0]) ^ c[1];
}

// a list entry: the piece's end (absolute), its bytes (bit 31: the record's first piece), and j,
// the pieces after it in the record (its state is shifted by Z_{8 KiB * j})
struct LcEnt {
    uint64_t end;
    uint32_t len, j;
};

}  // namespace

__global__ __launch_bounds__(256) void k_lc_count(const bhg_handle *__restrict__ h, uint32_t n, uint64_t src_len,
                                                  uint64_t *__restrict__ cnt) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const bhg_handle x = h[i];
        cnt[i] = long_rec(x, src_len) ? ((uint64_t)x.length + kLcPiece - 1) / kLcPiece : 0ull;
    }
}

// A record whose pieces would pass the list's capacity (only when handles overlap: the capacity
// holds every piece of records that do not) goes to the overflow list, walked piece by piece by
// one wave.
__global__ __launch_bounds__(256) void k_lc_emit(const uint8_t *__restrict__ src, const bhg_handle *__restrict__ h,
                                                 const uint64_t *__restrict__ base, uint32_t n, uint64_t cap,
                                                 LcEnt *__restrict__ ent, uint32_t *__restrict__ ovf) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b0 = base[i], b1 = base[i + 1];
        if (b1 == b0) continue;
        if (b1 <= cap) {
            const bhg_handle x = h[i];
            const uint32_t nch = (uint32_t)(b1 - b0);
            for (uint32_t k = 0; k < nch; k++) {
                const uint32_t ce = x.length - kLcPiece * (nch - 1 - k), cb = k == 0 ? 0u : ce - kLcPiece;
                ent[b0 + k] = LcEnt{(uint64_t)src + x.offset + ce, (ce - cb) | (k == 0 ? 0x80000000u : 0u), nch - 1 - k};
            }
        } else {
            ovf[1 + atomicAdd(ovf, 1u)] = i;
            // the list ends inside this record (base is non-decreasing: every later record
            // overflows too): its list slots up to cap are marked empty
            for (uint64_t k = b0; k < cap; k++) ent[k] = LcEnt{0, 0, 0};
        }
    }
}

__global__ __launch_bounds__(kLcThreads) void k_lc_piece(const uint8_t *__restrict__ src, uint64_t src_len,
                                                        const bhg_handle *__restrict__ h, uint32_t n,
                                                        const uint32_t *__restrict__ expected_crc,
                                                        bhg_desc *__restrict__ out, uint32_t *__restrict__ crc_out,
                                                        const uint64_t *__restrict__ base,
                                                        uint64_t cap, const LcEnt *__restrict__ ent,
                                                        uint32_t *__restrict__ pst, const uint32_t *__restrict__ ovf,
                                                        const uint32_t *__restrict__ zl) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLcBytes / 4];
    const uint32_t t = threadIdx.x, lane = t & 63;
    const uint64_t total = base[n], nlist = total < cap ? total : cap;
    const uint32_t novf = *ovf;
    const uint32_t tb = lds_addr(lds);
    CrcR8::fill(tb + kLcT);
    uint32_t *Zt = lds + kLcZt / 4, *Zq = lds + kLcZq / 4, *Zd = lds + kLcZd / 4;
    for (uint32_t w = t; w < kLcTree * 1024; w += kLcThreads) Zt[w] = zlong(zl, 7)[w];  // Z_128 .. Z_32K: contiguous
    for (uint32_t w = t; w < 1024; w += kLcThreads) Zq[w] = zlong(zl, 6)[w];
    for (uint32_t w = t; w < kLcDist * 1024; w += kLcThreads) Zd[w] = zlong(zl, 16)[w];  // Z_64K .. Z_2M
    __syncthreads();
    const CrcR8 crc(tb + kLcT);
    const uint64_t end = (uint64_t)src + src_len;
    // Z_{8 KiB * 2^b}: Z_8K .. Z_32K, Z_64K .. Z_2M in LDS, longer shifts from the context's set
    auto shift_table = [&](uint32_t b) -> const uint32_t * {
        return b < 3 ? Zt + 1024 * (6 + b) : b < 3 + kLcDist ? Zd + 1024 * (b - 3) : zlong(zl, 13 + b);
    };
    // this lane's span of a piece: [se - 128, se), se = len - 128 (63 - lane) inside the piece; the
    // record's first piece may start with a partial span (and holds Go's initial state ^0)
    struct Lane {
        uint64_t A, P;
        int32_t ss, se;
        bool first, full, part;
    };
    auto lane_of = [&](const LcEnt &e) {
        Lane L;
        const uint32_t len = e.len & 0x7fffffffu;
        L.first = (e.len >> 31) != 0;
        L.P = e.end - len;  // the piece's start
        L.se = (int32_t)len - 128 * (int32_t)(63 - lane);
        L.ss = L.se - 128;
        L.full = L.se > 0 && L.ss >= 0;
        L.part = L.se > 0 && L.ss < 0;
        L.A = L.P + (uint64_t)(L.full ? L.ss : 0);
        return L;
    };
    // the piece's state at its end: the spans' states folded across the lanes (lane 63 holds it)
    auto piece_state = [&](const Lane &L, const Span &S) -> uint32_t {
        uint32_t c = 0;
        if (L.full) c = span_crc(crc, Zq, (L.first && L.ss == 0) ? 0xffffffffu : 0u, L.A, S);
        else if (L.part) c = crc_range(crc, 0xffffffffu, L.P, (uint64_t)L.se, end);
#pragma unroll
        for (uint32_t l = 0; l < 6; l++) {
            const uint32_t w = 1u << l;
            const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane - w) & 63u) * 4u), (int)c);
            if ((lane & (2 * w - 1)) == 2 * w - 1) c = zap(Zt + 1024 * l, v) ^ c;
        }
        return c;
    };
    // the list: piece g by wave g mod (waves of the grid), the next piece's spans in flight
    const uint64_t nw = (uint64_t)gridDim.x * (kLcThreads / 64), w0 = (uint64_t)blockIdx.x * (kLcThreads / 64) + (t >> 6);
    if (w0 < nlist) {
        LcEnt e = ent[w0];
        Lane L = lane_of(e);
        Span S;
        if (e.len) span_load(S, L.full ? L.A : L.P, end);  // (an empty entry: no address to load from)
        for (uint64_t g = w0; g < nlist; g += nw) {
            const LcEnt ec = e;
            const Lane Lc = L;
            const Span Sc = S;
            if (g + nw < nlist) {
                e = ent[g + nw];
                L = lane_of(e);
                if (e.len) span_load(S, L.full ? L.A : L.P, end);
            }
            if (ec.len == 0) continue;  // past the last record that fits (the overflow list holds it)
            uint32_t c = piece_state(Lc, Sc);
            if (lane == 63) {
                for (uint32_t j = ec.j, b = 0; j; j >>= 1, b++)
                    if (j & 1) c = zap(shift_table(b), c);
                pst[g] = c;
            }
        }
    }
    // overflow records: one wave walks all pieces of one record, Horner over Z_8K
    for (uint64_t q = w0; q < novf; q += nw) {
        const uint32_t i = ovf[1 + q];
        const bhg_handle x = h[i];
        const uint32_t nch = (uint32_t)(((uint64_t)x.length + kLcPiece - 1) / kLcPiece);
        uint32_t s = 0;
        for (uint32_t k = 0; k < nch; k++) {
            const uint32_t ce = x.length - kLcPiece * (nch - 1 - k), cb = k == 0 ? 0u : ce - kLcPiece;
            const LcEnt e = {(uint64_t)src + x.offset + ce, (ce - cb) | (k == 0 ? 0x80000000u : 0u), 0};
            const Lane L = lane_of(e);
            Span S;
            span_load(S, L.full ? L.A : L.P, end);
            const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)piece_state(L, S), 63);
            s = k == 0 ? v : zap(Zt + 1024 * 6, s) ^ v;
        }
        if (lane == 0) lc_finish(out, crc_out, i, s, expected_crc);
    }
}

// lane per long record of the list: the XOR of its pieces' shifted states
__global__ __launch_bounds__(256) void k_lc_fin(const uint64_t *__restrict__ base, uint32_t n, uint64_t cap,
                                                const uint32_t *__restrict__ pst, const uint32_t *__restrict__ expected_crc,
                                                bhg_desc *__restrict__ out, uint32_t *__restrict__ crc_out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b0 = base[i], b1 = base[i + 1];
        if (b1 == b0 || b1 > cap) continue;  // not long, or walked by the overflow pass
        uint32_t s = 0;
        for (uint64_t k = b0; k < b1; k++) s ^= pst[k];
        lc_finish(out, crc_out, i, s, expected_crc);
    }
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static uint64_t lc_cap(uint32_t n, uint64_t src_len) { return src_len / kLcPiece + n + 1; }

size_t long_crc_scratch_bytes_cap(uint32_t n, uint64_t cap) {
    return al256(((size_t)n + 1) * 8) + al256(scan_scratch_bytes(n)) + al256((size_t)cap * sizeof(LcEnt)) +
           al256((size_t)cap * 4) + al256(((size_t)n + 1) * 4);
}
size_t long_crc_scratch_bytes(uint32_t n, uint64_t src_len) { return long_crc_scratch_bytes_cap(n, lc_cap(n, src_len)); }

hipError_t launch_long_crc(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           const uint32_t *expected_crc, bhg_desc *out, void *scratch, uint32_t *crc_out,
                           uint64_t list_cap) {
    uint8_t *sp = static_cast<uint8_t *>(scratch);
    uint64_t *base = reinterpret_cast<uint64_t *>(sp);
    sp += al256(((size_t)n + 1) * 8);
    void *scan = sp;
    sp += al256(scan_scratch_bytes(n));
    const uint64_t cap = list_cap ? list_cap : lc_cap(n, src_len);
    LcEnt *ent = reinterpret_cast<LcEnt *>(sp);
    sp += al256((size_t)cap * sizeof(LcEnt));
    uint32_t *pst = reinterpret_cast<uint32_t *>(sp);
    sp += al256((size_t)cap * 4);
    uint32_t *ovf = reinterpret_cast<uint32_t *>(sp);
    hipLaunchKernelGGL(k_lc_count, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, h, n, src_len, base);
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = launch_exclusive_scan_u64(L, base, base, n, scan)) return e;
    if (hipError_t e = hipMemsetAsync(ovf, 0, 4, L.stream)) return e;
    hipLaunchKernelGGL(k_lc_emit, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, h, base, n, cap, ent, ovf);
    // persistent: one workgroup per CU (the LDS tables), pieces wave-strided
    hipLaunchKernelGGL(k_lc_piece, dim3(L.num_cus), dim3(kLcThreads), 0, L.stream, src, src_len, h, n, expected_crc, out,
                       crc_out, base, cap, ent, pst, ovf, L.xtab + kXLong);
    hipLaunchKernelGGL(k_lc_fin, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, base, n, cap, pst, expected_crc, out,
                       crc_out);
    return hipGetLastError();
}

}  // namespace bhg
