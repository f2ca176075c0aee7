// bhg_decode.hip -- batched bithash block decode for gfx950.
//
// Kernel map:
//   k_decode_lane<MODE>  one LANE per block.  Each lane walks its own record:
//                        CRC-32C chain over [0, L) out of the replicated LDS
//                        table, header parse + readRecord validation
//                        (bithash/block2.go:57-66), trailer/UserKey split
//                        (readKV :38-55), FNV-1 of the UserKey
//                        (internal/hash/fnv.go:19-23), descriptor store.
//                        MODE_NONE is the whole NoCompressor decode
//                        (compress.go:57-59 returns src -> zero-copy view).
//                        MODE_SNAPPY additionally parses the snappy varint
//                        header (decodedLen) and emits the decoded size.
//   k_snappy_wave        one WAVE per snappy block: golang/snappy v0.0.4
//                        decode (decode_other.go) with the output window in
//                        LDS and a wave-uniform tag walk.
//   k_crc_ranges / k_fnv_ranges   batched primitives.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

enum { MODE_NONE = 0, MODE_SNAPPY = 1 };

struct DescOut {
    uint32_t key_off, key_len, val_off, val_len;
    uint64_t trailer;
    uint32_t file_num, fnv1, crc, status;
};

__device__ __forceinline__ void store_desc(bhg_desc *out, const DescOut &d) {
    // 40 B = 5 x 8 B stores (descriptor array is 8-byte aligned)
    uint2 *o = reinterpret_cast<uint2 *>(out);
    o[0] = make_uint2(d.key_off, d.key_len);
    o[1] = make_uint2(d.val_off, d.val_len);
    o[2] = make_uint2((uint32_t)d.trailer, (uint32_t)(d.trailer >> 32));
    o[3] = make_uint2(d.file_num, d.fnv1);
    o[4] = make_uint2(d.crc, d.status);
}

// Go encoding/binary.Uvarint + snappy decodedLen: returns false on corrupt.
__device__ __forceinline__ bool snappy_varint(uint64_t p, uint32_t n, uint64_t end, uint64_t &v, uint32_t &hdr) {
    uint64_t x = 0;
    uint32_t s = 0;
    for (uint32_t i = 0; i < 10; i++) {
        if (i >= n) return false;
        uint32_t b = gld<uint8_t>(p + i);
        if (b < 0x80) {
            if (i == 9 && b > 1) return false;
            x |= (uint64_t)b << s;
            if (x > 0xffffffffull) return false;
            v = x;
            hdr = i + 1;
            return true;
        }
        x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    return false;
}

// Table flavours for the lane kernels: slice-by-1 (byte table replicated 32x,
// 32 KiB) or slice-by-4 (4 tables replicated R x, 4 KiB * R).
template <int SLICE, int R>
struct TabSel;
template <int R>
struct TabSel<1, R> {
    typedef CrcLds type;
    static constexpr uint32_t words = BHG_CRC_LDS_WORDS;
    static __device__ __forceinline__ void fill(uint32_t *T) { crc_lds_fill(T); }
};
template <int R>
struct TabSel<0, R> {   // diagnostic: loads only
    typedef XorTab type;
    static constexpr uint32_t words = 4;
    static __device__ __forceinline__ void fill(uint32_t *) {}
};
template <int R>
struct TabSel<4, R> {
    typedef Crc4Lds<R> type;
    static constexpr uint32_t words = Crc4Lds<R>::kWords;
    static __device__ __forceinline__ void fill(uint32_t *T) { Crc4Lds<R>::fill(T); }
};

// Record prefix: the first 64 B of a record as 15 record-aligned words
// (RW[j] = bytes [4j, 4j+4) of the record), fetched by 4 dwordx4 loads issued
// together with the CRC walk's first window.  Header, user key (FNV-1) and
// trailer come from these registers whenever 20 + keyLen <= 60.
struct Prefix {
    uint32_t rw[15];
    __device__ __forceinline__ void load(uint64_t p, uint64_t end) {
        const uint64_t a = p & ~3ull;
        const uint32_t sh = (uint32_t)(p & 3);
        uint32_t w[16];
        if (a + 64 <= end) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 v = gld<u32x4_a4>(a + 16 * q);
                w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) w[j] = ld32_safe(a + 4 * j, end);
        }
#pragma unroll
        for (int j = 0; j < 15; j++) rw[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    }
    // bytes [4t + s, 4t + s + 4) of the record for dynamic t in 3..12, s in 0..3
    __device__ __forceinline__ uint32_t word_at(uint32_t byte) const {
        const uint32_t t = byte >> 2, s = byte & 3;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (uint32_t j = 3; j < 14; j++) {
            lo = t == j ? rw[j] : lo;
            hi = t == j ? rw[j + 1] : hi;
        }
        return __builtin_amdgcn_alignbyte(hi, lo, s);
    }
    // FNV-1 over record bytes [12, 12 + klen), klen <= 48
    __device__ __forceinline__ uint32_t fnv_key(uint32_t klen) const {
        uint32_t h = BHG_FNV_OFFSET;
        const uint32_t stop = 12 + klen;
#pragma unroll
        for (uint32_t j = 3; j < 15; j++) {
            if (4 * j >= stop) break;
#pragma unroll
            for (uint32_t b = 0; b < 4; b++) {
                const uint32_t hn = (h * BHG_FNV_PRIME) ^ ((rw[j] >> (8 * b)) & 0xffu);
                h = 4 * j + b < stop ? hn : h;
            }
        }
        return h;
    }
};

template <int MODE, int SLICE, int R, int WG, int WIN, int PF>
__global__ __launch_bounds__(WG) void k_decode_lane(const uint8_t *__restrict__ src, uint64_t src_len,
                                                    const bhg_handle *__restrict__ handles, uint32_t n,
                                                    const uint32_t *__restrict__ expected_crc,
                                                    bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes) {
    typedef TabSel<SLICE, R> TS;
    __shared__ __attribute__((aligned(16))) uint32_t T[TS::words];
    TS::fill(T);
    __syncthreads();
    const typename TS::type crc(T);
    const uint64_t base = (uint64_t)src;
    const uint64_t end = base + src_len;
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bhg_handle hn = {0, 0, 0};
    if (i < n) hn = handles[i];
    for (; i < n; i += stride) {
        const bhg_handle h = hn;
        if (i + stride < n) hn = handles[i + stride];     // next block's handle in flight
        DescOut d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        uint64_t dsize = 0;
        if (h.length == 0) {
            d.status = BHG_ST_ILLEGAL_LENGTH;              // reader.go:234-236
        } else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {
            d.status = BHG_ST_INCOMPLETE;                  // ReadAt short
        } else {
            const uint64_t p = base + h.offset;
            const uint32_t L = h.length;
            Prefix P;
            P.load(p, end);                                 // header / key / trailer registers
            const uint32_t k = L >= 12 ? P.rw[0] : 0, v = L >= 12 ? P.rw[1] : 0, fn = P.rw[2];
            const bool valid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            // everything that needs only the prefix is done before the CRC walk
            uint32_t key_len = 0, fnv = BHG_FNV_OFFSET;
            uint64_t trailer = 255;
            if (valid) {
                if (k >= 8) {
                    key_len = k - 8;
                    if (key_len <= 36) {
                        fnv = P.fnv_key(key_len);
                        trailer = (uint64_t)P.word_at(12 + key_len) | ((uint64_t)P.word_at(16 + key_len) << 32);
                    } else {
                        fnv = fnv1_range(p + 12, key_len, end);
                        trailer = ldu64(p + 12 + k - 8, end);
                    }
                }
            }
            if (PF == 1)
                d.crc = crc_mask(~crc_range_w<WIN, true>(crc, 0xffffffffu, p, L, end));
            else if (PF == 2)
                d.crc = crc_mask(~crc_range_a<WIN, typename TS::type, true>(crc, 0xffffffffu, p, L, end));
            else if (PF == 3)
                d.crc = crc_mask(~crc_range_pp<WIN>(crc, 0xffffffffu, p, L, end));

            else
                d.crc = crc_mask(~crc_range_a<WIN>(crc, 0xffffffffu, p, L, end));
            if (!valid) {
                d.status = BHG_ST_RECORD_NIL;              // block2.go:59-62 (L < 12: Go would panic)
            } else {
                d.file_num = fn;
                d.key_off = 12;
                d.key_len = key_len;
                d.trailer = trailer;
                d.fnv1 = fnv;
                if (MODE == MODE_NONE) {
                    d.val_off = 12 + k;
                    d.val_len = v;
                } else {
                    uint64_t dl;
                    uint32_t hdr;
                    if (!snappy_varint(p + 12 + k, v, end, dl, hdr) || dl * 3 > (uint64_t)(v - hdr) * 64) {
                        d.status = BHG_ST_SNAPPY_CORRUPT;
                    } else {
                        dsize = dl;
                        d.val_len = (uint32_t)dl;           // provisional; k_snappy_wave finalises
                        d.val_off = 12 + k;                 // provisional: compressed payload offset
                    }
                }
            }
            if (expected_crc != nullptr && d.status == BHG_ST_OK && expected_crc[i] != d.crc)
                d.status = BHG_ST_CRC_MISMATCH;
        }
        if (d.status == BHG_ST_RECORD_NIL) {
            const uint32_t c = d.crc;
            d = DescOut{0, 0, 0, 0, 0, 0, 0, c, BHG_ST_RECORD_NIL};
        }
        store_desc(out + i, d);
        if (MODE == MODE_SNAPPY) sizes[i] = dsize;
    }
}

// ---------------------------------------------------------------------------
// golang/snappy v0.0.4 decode, one wave per block (decode_other.go `decode`).
// The tag walk is wave-uniform (scalar); literal / copy bytes are moved by the
// 64 lanes in parallel through an LDS output window.  LDS in-order execution
// within a wave orders each copy's reads after the writes it depends on.
// Blocks whose compressed payload or output exceeds the LDS window use the
// same walk directly on global memory executed by lane 0.
// ---------------------------------------------------------------------------
#define SNAPPY_WAVES_PER_WG 4
#define SNAPPY_IN_CAP 2048
#define SNAPPY_OUT_CAP 4096

__device__ __forceinline__ uint32_t lds_u8(const uint8_t *b, uint32_t i) { return b[i]; }

// Serial decode on global memory (lane 0 only); returns true when ok.
__device__ bool snappy_decode_global(const uint8_t *s, uint64_t slen, uint8_t *dst, uint64_t dlen) {
    uint64_t d = 0, si = 0;
    while (si < slen) {
        uint32_t tag = s[si];
        uint64_t length, offset;
        if ((tag & 3) == 0) {
            uint32_t x = tag >> 2;
            if (x < 60) { si += 1; }
            else {
                uint32_t nb = x - 59;
                si += 1 + nb;
                if (si > slen) return false;
                x = 0;
                for (uint32_t j = 0; j < nb; j++) x |= (uint32_t)s[si - nb + j] << (8 * j);
            }
            length = (uint64_t)x + 1;
            if (length > dlen - d || length > slen - si) return false;
            for (uint64_t j = 0; j < length; j++) dst[d + j] = s[si + j];
            d += length;
            si += length;
            continue;
        } else if ((tag & 3) == 1) {
            si += 2;
            if (si > slen) return false;
            length = 4 + ((tag >> 2) & 7);
            offset = ((uint64_t)(tag & 0xe0) << 3) | s[si - 1];
        } else if ((tag & 3) == 2) {
            si += 3;
            if (si > slen) return false;
            length = 1 + (tag >> 2);
            offset = (uint64_t)s[si - 2] | ((uint64_t)s[si - 1] << 8);
        } else {
            si += 5;
            if (si > slen) return false;
            length = 1 + (tag >> 2);
            offset = (uint64_t)s[si - 4] | ((uint64_t)s[si - 3] << 8) | ((uint64_t)s[si - 2] << 16) |
                     ((uint64_t)s[si - 1] << 24);
        }
        if (offset == 0 || d < offset || length > dlen - d) return false;
        for (uint64_t j = 0; j < length; j++) dst[d + j] = dst[d - offset + j];
        d += length;
    }
    return d == dlen;
}

__global__ __launch_bounds__(64 * SNAPPY_WAVES_PER_WG) void k_snappy_wave(
    const uint8_t *__restrict__ src, uint64_t src_len, const bhg_handle *__restrict__ handles, uint32_t n,
    bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals, uint64_t out_cap,
    const uint64_t *__restrict__ val_off) {
    __shared__ __attribute__((aligned(16))) uint8_t lin[SNAPPY_WAVES_PER_WG][SNAPPY_IN_CAP + 16];
    __shared__ __attribute__((aligned(16))) uint8_t lout[SNAPPY_WAVES_PER_WG][SNAPPY_OUT_CAP + 16];
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *in = lin[wave];
    const uint64_t base = (uint64_t)src;
    const uint32_t nwaves = gridDim.x * SNAPPY_WAVES_PER_WG;
    for (uint32_t i = blockIdx.x * SNAPPY_WAVES_PER_WG + wave; i < n; i += nwaves) {
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = __builtin_amdgcn_readfirstlane(dw[9]);
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t cpos = __builtin_amdgcn_readfirstlane(dw[2]);   // provisional val_off
        const uint32_t dlen32 = __builtin_amdgcn_readfirstlane(dw[3]);  // provisional val_len
        const uint64_t dlen = dlen32;
        const uint64_t rec = base + handles[i].offset;
        const uint32_t L = handles[i].length;
        const uint32_t clen = L - cpos;
        const uint64_t o0 = val_off[i];
        const uint64_t o1 = val_off[i + 1];
        uint32_t fin = status;
        if (o1 > out_cap || o1 - o0 < dlen) {
            fin = BHG_ST_SNAPPY_TOO_LARGE;
        } else {
            const uint64_t cp = rec + cpos;
            // varint header (already validated by the lane pass)
            uint32_t hdr = 0;
            for (;;) {
                uint32_t b = gld<uint8_t>(cp + hdr);
                hdr++;
                if (b < 0x80) break;
            }
            const uint32_t slen = clen - hdr;
            uint8_t *dstg = out_vals + o0;
            bool ok;
            if (slen <= SNAPPY_IN_CAP && dlen <= SNAPPY_OUT_CAP) {
                // stage the compressed stream in LDS (bytes; slen <= 2 KiB)
                const uint64_t sp = cp + hdr;
                for (uint32_t j = lane; j < slen; j += 64) in[j] = gld<uint8_t>(sp + j);
                // output window placed so that LDS byte (o) and global byte (o) share alignment
                const uint32_t ash = (uint32_t)((uint64_t)dstg & 3);
                uint8_t *ob = lout[wave] + ash;
                uint64_t d = 0, s = 0;
                ok = true;
                while (s < slen) {
                    const uint32_t tag = in[s];
                    uint32_t length, offset = 0;
                    bool literal = false;
                    if ((tag & 3) == 0) {
                        uint32_t x = tag >> 2;
                        if (x < 60) { s += 1; }
                        else {
                            const uint32_t nb = x - 59;
                            s += 1 + nb;
                            if (s > slen) { ok = false; break; }
                            x = 0;
                            for (uint32_t j = 0; j < nb; j++) x |= (uint32_t)in[s - nb + j] << (8 * j);
                        }
                        const uint64_t l64 = (uint64_t)x + 1;
                        if (l64 > dlen - d || l64 > slen - s) { ok = false; break; }
                        length = (uint32_t)l64;
                        literal = true;
                    } else if ((tag & 3) == 1) {
                        s += 2;
                        if (s > slen) { ok = false; break; }
                        length = 4 + ((tag >> 2) & 7);
                        offset = ((tag & 0xe0) << 3) | in[s - 1];
                    } else if ((tag & 3) == 2) {
                        s += 3;
                        if (s > slen) { ok = false; break; }
                        length = 1 + (tag >> 2);
                        offset = (uint32_t)in[s - 2] | ((uint32_t)in[s - 1] << 8);
                    } else {
                        s += 5;
                        if (s > slen) { ok = false; break; }
                        length = 1 + (tag >> 2);
                        const uint64_t o64 = (uint64_t)in[s - 4] | ((uint64_t)in[s - 3] << 8) |
                                             ((uint64_t)in[s - 2] << 16) | ((uint64_t)in[s - 1] << 24);
                        if (o64 > d) { ok = false; break; }
                        offset = (uint32_t)o64;
                    }
                    if (literal) {
                        for (uint32_t j = lane; j < length; j += 64) ob[d + j] = in[s + j];
                        d += length;
                        s += length;
                    } else {
                        if (offset == 0 || d < offset || length > dlen - d) { ok = false; break; }
                        // forward copy; for offset < length the source repeats with period `offset`
                        for (uint32_t j = lane; j < length; j += 64) {
                            const uint32_t jj = offset >= length ? j : j % offset;
                            ob[d + j] = ob[d - offset + jj];
                        }
                        d += length;
                    }
                }
                ok = ok && d == dlen;
                if (ok) {
                    // coalesced write-out: bytes up to 4-alignment, dwords, tail bytes
                    const uint64_t g0 = (uint64_t)dstg;
                    const uint32_t head = (uint32_t)((4 - (g0 & 3)) & 3) < dlen32 ? (uint32_t)((4 - (g0 & 3)) & 3) : dlen32;
                    if (lane < head) dstg[lane] = ob[lane];
                    const uint32_t nwd = (dlen32 - head) >> 2;
                    const uint32_t *obw = reinterpret_cast<const uint32_t *>(ob + head);
                    uint32_t *gw = reinterpret_cast<uint32_t *>(dstg + head);
                    for (uint32_t j = lane; j < nwd; j += 64) gw[j] = obw[j];
                    const uint32_t tb = head + 4 * nwd;
                    if (lane < dlen32 - tb) dstg[tb + lane] = ob[tb + lane];
                }
            } else {
                uint32_t r = 0;
                if (lane == 0) r = snappy_decode_global(reinterpret_cast<const uint8_t *>(cp + hdr), slen, dstg, dlen) ? 1u : 0u;
                ok = __builtin_amdgcn_readfirstlane(r) != 0;
            }
            if (!ok) fin = BHG_ST_SNAPPY_CORRUPT;
        }
        if (lane == 0) {
            if (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) {
                dw[2] = 0;
                dw[3] = dlen32;
            } else {
                dw[2] = 0;
                dw[3] = 0;
            }
            dw[9] = fin;
        }
    }
}

// ---------------------------------------------------------------------------
// golang/snappy v0.0.4 decode, one LANE per block (decode_other.go `decode`).
// gfx950 runs unaligned global dword/dwordx4 accesses natively, so a lane
// moves literals and non-overlapping copies 16 B at a time straight from the
// record (input) / its own output (copy source) into its output slot; the
// last chunk may overshoot into bytes that later elements overwrite (never
// past the block's dlen).  Overlapping copies go 4 B (offset >= 4) or 1 B
// at a time.  ~64 x 32 x 256 blocks are in flight chip-wide, which hides
// the per-element load latency that a wave-per-block walk exposes.
// A lane's loads of its own earlier stores are ordered by the memory
// pipeline (same wave, same address).
// ---------------------------------------------------------------------------
typedef uint32_t u32a1 __attribute__((aligned(1)));
typedef uint64_t u64a1 __attribute__((aligned(1)));
typedef u32x4 u32x4a1 __attribute__((aligned(1)));

__device__ __forceinline__ uint64_t ldu64_g(uint64_t a, uint64_t end) {
    if (a + 8 <= end) return gld<u64a1>(a);
    uint64_t x = 0;
    for (uint32_t b = 0; b < 8; b++)
        if (a + b < end) x |= (uint64_t)gld<uint8_t>(a + b) << (8 * b);
    return x;
}

// returns true on success; cp/dst absolute addresses
__device__ __forceinline__ bool snappy_lane_decode(uint64_t cp, uint32_t slen, uint64_t dst, uint32_t dlen,
                                                   uint64_t end) {
    uint32_t s = 0, d = 0;
    while (s < slen) {
        const uint64_t t8 = ldu64_g(cp + s, end);
        const uint32_t tag = (uint32_t)t8 & 0xffu;
        uint32_t length, offset;
        if ((tag & 3) == 0) {
            uint32_t x = tag >> 2;
            uint64_t l64;
            if (x < 60) {
                s += 1;
                l64 = (uint64_t)x + 1;
            } else {
                const uint32_t nb = x - 59;
                if ((uint64_t)s + 1 + nb > slen) return false;
                s += 1 + nb;
                x = (uint32_t)(t8 >> 8) & (nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u));
                l64 = (uint64_t)x + 1;
            }
            if (l64 > (uint64_t)(dlen - d) || l64 > (uint64_t)(slen - s)) return false;
            length = (uint32_t)l64;
            uint32_t k = 0;
            for (; k + 16 <= length || (k < length && d + k + 16 <= dlen && cp + s + k + 16 <= end); k += 16)
                gst<u32x4a1>(dst + d + k, gld<u32x4a1>(cp + s + k));
            for (; k < length; k++) gst<uint8_t>(dst + d + k, gld<uint8_t>(cp + s + k));
            d += length;
            s += length;
            continue;
        } else if ((tag & 3) == 1) {
            if ((uint64_t)s + 2 > slen) return false;
            s += 2;
            length = 4 + ((tag >> 2) & 7);
            offset = ((tag & 0xe0) << 3) | ((uint32_t)(t8 >> 8) & 0xffu);
        } else if ((tag & 3) == 2) {
            if ((uint64_t)s + 3 > slen) return false;
            s += 3;
            length = 1 + (tag >> 2);
            offset = (uint32_t)(t8 >> 8) & 0xffffu;
        } else {
            if ((uint64_t)s + 5 > slen) return false;
            s += 5;
            length = 1 + (tag >> 2);
            offset = (uint32_t)(t8 >> 8);
        }
        if (offset == 0 || d < offset || length > dlen - d) return false;
        const uint64_t o = dst + d, from = o - offset;
        if (offset >= 16) {
            uint32_t k = 0;
            for (; k + 16 <= length || (k < length && d + k + 16 <= dlen); k += 16)
                gst<u32x4a1>(o + k, gld<u32x4a1>(from + k));
            for (; k < length; k++) gst<uint8_t>(o + k, gld<uint8_t>(from + k));
        } else if (offset >= 4) {
            uint32_t k = 0;
            for (; k + 4 <= length || (k < length && d + k + 4 <= dlen); k += 4)
                gst<u32a1>(o + k, gld<u32a1>(from + k));
            for (; k < length; k++) gst<uint8_t>(o + k, gld<uint8_t>(from + k));
        } else {
            for (uint32_t k = 0; k < length; k++) gst<uint8_t>(o + k, gld<uint8_t>(from + k));
        }
        d += length;
    }
    return d == dlen;
}

__global__ __launch_bounds__(256) void k_snappy_lane(const uint8_t *__restrict__ src, uint64_t src_len,
                                                     const bhg_handle *__restrict__ handles, uint32_t n,
                                                     bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                     uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = dw[9];
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t cpos = dw[2], dlen = dw[3];
        const bhg_handle h = handles[i];
        const uint64_t rec = base + h.offset;
        const uint32_t clen = h.length - cpos;
        const uint64_t o0 = val_off[i], o1 = val_off[i + 1];
        uint32_t fin = status;
        if (o1 > out_cap || o1 - o0 < dlen) {
            fin = BHG_ST_SNAPPY_TOO_LARGE;
        } else {
            const uint64_t cp = rec + cpos;
            uint32_t hdr = 0;
            for (;;) {  // varint already validated by the lane pass
                const uint32_t b = gld<uint8_t>(cp + hdr);
                hdr++;
                if (b < 0x80) break;
            }
            if (!snappy_lane_decode(cp + hdr, clen - hdr, (uint64_t)out_vals + o0, dlen, end)) fin = BHG_ST_SNAPPY_CORRUPT;
        }
        dw[2] = 0;
        dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? dlen : 0u;
        dw[9] = fin;
    }
}

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
__device__ __forceinline__ u32x4 ld16_bounded(uint64_t a, uint64_t lo, uint64_t hi) {
    if (a >= lo && a + 16 <= hi) return gld<u32x4_a4>(a);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint64_t q = a + 4 * k + b;
            if (q >= lo && q < hi) x |= (uint32_t)gld<uint8_t>(q) << (8 * b);
        }
        w[k] = x;
    }
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// ---------------------------------------------------------------------------
// k_decode_lanebuf: the production lane kernel.  Work is walked in wave tiles
// of 64 consecutive handles (every lane of a wave takes part in the
// wave-wide min/max that build the buffer descriptor).  Per block: handle ->
// prefix registers (header, key, trailer, FNV-1) -> CRC over 128 B
// line-aligned windows fetched by range-checked buffer loads, ping-ponged
// two windows deep -> 40 B descriptor.  A wave whose blocks span >= 4 GiB
// (a 32-bit buffer offset cannot reach) takes the global-load walk instead.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = shfl_xor64(v, o);
        v = t < v ? t : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t t = shfl_xor64(v, o);
        v = t > v ? t : v;
    }
    return v;
}

template <int MODE, int R, int WG, int WIN>
__global__ __launch_bounds__(WG) void k_decode_lanebuf(const uint8_t *__restrict__ src, uint64_t src_len,
                                                       const bhg_handle *__restrict__ handles, uint32_t n,
                                                       const uint32_t *__restrict__ expected_crc,
                                                       bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes) {
    typedef Crc4Lds<R> Tab;
    __shared__ __attribute__((aligned(16))) uint32_t T[Tab::kWords];
    Tab::fill(T);
    __syncthreads();
    const Tab crc(T);
    const uint64_t base = (uint64_t)src;
    const uint64_t end = base + src_len;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves = gridDim.x * (WG / 64);
    const uint32_t ntiles = (n + 63) / 64;
    constexpr uint32_t WB = 16 * WIN;
    uint32_t tile = blockIdx.x * (WG / 64) + (threadIdx.x >> 6);
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    for (; tile < ntiles; tile += waves) {
        const uint32_t i = tile * 64 + lane;
        const bool active = i < n;
        const bhg_handle h = hn;
        {
            const uint32_t nt = tile + waves;
            hn = bhg_handle{0, 0, 0};
            if (nt < ntiles && nt * 64 + lane < n) hn = handles[nt * 64 + lane];   // next tile's handle in flight
        }
        DescOut d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        bool inb = false;
        if (active) {
            if (h.length == 0) d.status = BHG_ST_ILLEGAL_LENGTH;                 // reader.go:234-236
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) d.status = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = inb ? base + h.offset : base;
        const uint32_t L = inb ? h.length : 0u;
        // prefix registers (header / key / trailer / FNV-1)
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool valid = false;
        if (inb) {
            Prefix P;
            P.load(p, end);
            k = L >= 12 ? P.rw[0] : 0;
            v = L >= 12 ? P.rw[1] : 0;
            fn = P.rw[2];
            valid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (valid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    fnv = P.fnv_key(key_len);
                    trailer = (uint64_t)P.word_at(12 + key_len) | ((uint64_t)P.word_at(16 + key_len) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // wave-uniform descriptor over [lo, hi)
        const uint64_t lo = wave_min_u64(inb ? ((p & ~3ull) & ~127ull) : ~0ull);
        const uint64_t hi = wave_max_u64(inb ? p + L : 0ull);
        const uint32_t myw = inb ? crc_buf_windows(p, L, WB) : 0u;
        uint32_t nwin = myw;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nwin = max(nwin, (uint32_t)__shfl_xor(nwin, o, 64));
        uint32_t c = 0xffffffffu;
        if (lo != ~0ull) {
            const uint64_t rbase = __builtin_amdgcn_readfirstlane((uint32_t)lo) |
                                   ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(lo >> 32)) << 32);
            const uint64_t span = end - rbase;
            if (hi - rbase < 0xFFFF0000ull) {
                const uint32_t nrec = span > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)span;
                const __amdgpu_buffer_rsrc_t rsrc =
                    __builtin_amdgcn_make_buffer_rsrc((void *)rbase, (short)0, (int)nrec, 0x00020000);
                uint32_t cc = crc_range_buf<WIN>(crc, 0xffffffffu, inb ? p : rbase, inb ? L : 0, rsrc, rbase, nwin,
                                                  rbase + nrec);
                c = cc;
            } else if (inb) {
                c = crc_range_pp<WIN>(crc, 0xffffffffu, p, L, end);
            }
        }
        if (active) {
            uint64_t dsize = 0;
            if (inb) {
                d.crc = crc_mask(~c);
                if (!valid) {
                    d.status = BHG_ST_RECORD_NIL;              // block2.go:59-62 (L < 12: Go would panic)
                } else {
                    d.file_num = fn;
                    d.key_off = 12;
                    d.key_len = key_len;
                    d.trailer = trailer;
                    d.fnv1 = fnv;
                    if (MODE == MODE_NONE) {
                        d.val_off = 12 + k;
                        d.val_len = v;
                    } else {
                        uint64_t dl;
                        uint32_t hdr;
                        if (!snappy_varint(p + 12 + k, v, end, dl, hdr) || dl * 3 > (uint64_t)(v - hdr) * 64) {
                            d.status = BHG_ST_SNAPPY_CORRUPT;
                        } else {
                            dsize = dl;
                            d.val_len = (uint32_t)dl;
                            d.val_off = 12 + k;
                        }
                    }
                }
                if (expected_crc != nullptr && d.status == BHG_ST_OK && expected_crc[i] != d.crc)
                    d.status = BHG_ST_CRC_MISMATCH;
                if (d.status == BHG_ST_RECORD_NIL) {
                    const uint32_t cc = d.crc;
                    d = DescOut{0, 0, 0, 0, 0, 0, 0, cc, BHG_ST_RECORD_NIL};
                }
            }
            store_desc(out + i, d);
            if (MODE == MODE_SNAPPY) sizes[i] = dsize;
        }
    }
}

// ---------------------------------------------------------------------------
// k_decode_coop: one lane per block for the CRC chain, but the record bytes
// arrive through WAVE-COOPERATIVE loads.  A wave owns a tile of 64 blocks.
// Step s fetches, for every block r of the tile, the 64 B-aligned chunk
// s of its record: 4 lanes x 16 B per record, so one dwordx4 instruction
// covers 16 whole 64 B chunks (the per-lane pattern issues one request per
// 16 B and measured 0.29 ms for loads alone).  The chunks are transposed
// through a per-wave LDS tile (row = one block, 80 B stride: conflict-free
// ds_write_b128 / ds_read_b128) and lane r absorbs row r.  Two steps of
// loads stay in flight in registers (G0/G1).
// ---------------------------------------------------------------------------
#define COOP_ROW 80

template <int MODE, int SLICE, int R, int WAVES>
__global__ __launch_bounds__(64 * WAVES, 4) void k_decode_coop(const uint8_t *__restrict__ src, uint64_t src_len,
                                                            const bhg_handle *__restrict__ handles, uint32_t n,
                                                            const uint32_t *__restrict__ expected_crc,
                                                            bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes) {
    typedef TabSel<SLICE, R> TS;
    __shared__ __attribute__((aligned(16))) uint32_t T[TS::words];
    __shared__ __attribute__((aligned(16))) uint8_t stage[WAVES][64 * COOP_ROW];
    TS::fill(T);
    __syncthreads();
    const typename TS::type crc(T);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint8_t *tile_lds = stage[wave];
    const uint8_t *my_row = tile_lds + lane * COOP_ROW;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    for (uint32_t tile = blockIdx.x * WAVES + wave; tile < ntiles; tile += gridDim.x * WAVES) {
        const uint32_t i = tile * 64 + lane;
        bhg_handle h = {0, 0, 0};
        if (i < n) h = handles[i];
        DescOut d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        bool inb = false;
        if (i < n) {
            if (h.length == 0) d.status = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) d.status = BHG_ST_INCOMPLETE;
            else inb = true;
        }
        const uint64_t p = base + h.offset;
        const uint64_t e = p + h.length;
        const uint64_t a0 = p & ~63ull;
        const uint32_t steps = inb ? (uint32_t)((e - a0 + 63) >> 6) : 0u;
        uint32_t maxs = steps;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) maxs = max(maxs, (uint32_t)__shfl_xor(maxs, o, 64));
        // my 4 load slots: block r_j = 16 j + lane/4, piece lane%4
        uint64_t sa[4];
        uint32_t sst[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int r = 16 * j + (lane >> 2);
            sa[j] = shfl64(a0, r) + 16 * (lane & 3);
            sst[j] = (uint32_t)__shfl(steps, r, 64);
        }
        u32x4 G0[4], G1[4];
        auto issue = [&](u32x4 *G, uint32_t s) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                G[j] = s < sst[j] ? ld16_bounded(sa[j] + 64ull * s, base, end) : u32x4{0, 0, 0, 0};
        };
        issue(G0, 0);
        issue(G1, 1);
        // prefix registers: header / key / trailer
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;
        bool valid = false;
        if (inb) {
            Prefix P;
            P.load(p, end);
            const uint32_t L = h.length;
            k = L >= 12 ? P.rw[0] : 0;
            v = L >= 12 ? P.rw[1] : 0;
            fn = P.rw[2];
            valid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (valid && k >= 8) {
                key_len = k - 8;
                if (key_len <= 36) {
                    fnv = P.fnv_key(key_len);
                    trailer = (uint64_t)P.word_at(12 + key_len) | ((uint64_t)P.word_at(16 + key_len) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        const uint64_t pa = (p + 3) & ~3ull, pe = e & ~3ull;
        const uint32_t z = (uint32_t)(p & 3);
        uint32_t c = 0xffffffffu;
        auto absorb = [&](const u32x4 *G, uint32_t s) {
#pragma unroll
            for (int j = 0; j < 4; j++)
                *reinterpret_cast<u32x4 *>(tile_lds + (16 * j + (lane >> 2)) * COOP_ROW + 16 * (lane & 3)) = G[j];
            u32x4 W[4];
#pragma unroll
            for (int q = 0; q < 4; q++) W[q] = *reinterpret_cast<const u32x4 *>(my_row + 16 * q);
            const uint64_t cb = a0 + 64ull * s;
            if (s < steps) {
                if (cb >= pa && cb + 64 <= pe) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        c = crc.word(c, W[q].x); c = crc.word(c, W[q].y);
                        c = crc.word(c, W[q].z); c = crc.word(c, W[q].w);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 16; q++) {
                        const uint32_t w = q % 4 == 0 ? W[q / 4].x : q % 4 == 1 ? W[q / 4].y : q % 4 == 2 ? W[q / 4].z : W[q / 4].w;
                        const uint64_t ws = cb + 4 * q;
                        if (ws >= pa && ws < pe) c = crc.word(c, w);
                        else if (ws < pa && ws + 4 > p) c = crc.partial(c, w >> (8 * z), (uint32_t)((pa < e ? pa : e) - p));
                        else if (ws == pe && pe < e && pe >= pa) c = crc.partial(c, w, (uint32_t)(e - pe));
                    }
                }
            }
        };
        for (uint32_t s = 0; s < maxs; s += 2) {
            absorb(G0, s);
            if (s + 2 < maxs) issue(G0, s + 2);
            if (s + 1 < maxs) {
                absorb(G1, s + 1);
                if (s + 3 < maxs) issue(G1, s + 3);
            }
        }
        if (i < n) {
            uint64_t dsize = 0;
            if (inb) {
                d.crc = crc_mask(~c);
                if (!valid) {
                    d.status = BHG_ST_RECORD_NIL;
                } else {
                    d.file_num = fn;
                    d.key_off = 12;
                    d.key_len = key_len;
                    d.trailer = trailer;
                    d.fnv1 = fnv;
                    if (MODE == MODE_NONE) {
                        d.val_off = 12 + k;
                        d.val_len = v;
                    } else {
                        uint64_t dl;
                        uint32_t hdr;
                        if (!snappy_varint(p + 12 + k, v, end, dl, hdr) || dl * 3 > (uint64_t)(v - hdr) * 64) {
                            d.status = BHG_ST_SNAPPY_CORRUPT;
                        } else {
                            dsize = dl;
                            d.val_len = (uint32_t)dl;
                            d.val_off = 12 + k;
                        }
                    }
                }
                if (expected_crc != nullptr && d.status == BHG_ST_OK && expected_crc[i] != d.crc)
                    d.status = BHG_ST_CRC_MISMATCH;
                if (d.status == BHG_ST_RECORD_NIL) {
                    const uint32_t cc = d.crc;
                    d = DescOut{0, 0, 0, 0, 0, 0, 0, cc, BHG_ST_RECORD_NIL};
                }
            }
            store_desc(out + i, d);
            if (MODE == MODE_SNAPPY) sizes[i] = dsize;
        }
    }
}

// ---------------------------------------------------------------------------
// DIAGNOSTIC kernel (variant 26/27): memory ceiling of the wave-per-record
// pattern -- each wave streams NR records at a time with 1 KiB contiguous
// dwordx4 instructions and folds them with xor (no CRC).  Writes only the
// status/crc words of the descriptor.  Never a default.
// ---------------------------------------------------------------------------
template <int NR>
__global__ __launch_bounds__(256) void k_diag_wave(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t r0 = gw * NR; r0 < n; r0 += nw * NR) {
        uint32_t acc[NR];
        uint64_t p[NR], e[NR];
#pragma unroll
        for (int k = 0; k < NR; k++) {
            acc[k] = 0;
            const uint32_t r = r0 + k;
            const bhg_handle h = r < n ? handles[r] : bhg_handle{0, 0, 0};
            p[k] = (base + h.offset) & ~15ull;
            e[k] = base + h.offset + h.length;
        }
        for (uint32_t off = 0;; off += 1024) {
            bool any = false;
            u32x4 v[NR];
#pragma unroll
            for (int k = 0; k < NR; k++) {
                const uint64_t a = p[k] + off + 16 * lane;
                v[k] = a + 16 <= e[k] && a + 16 <= end ? gld<u32x4>(a) : u32x4{0, 0, 0, 0};
                any |= p[k] + off < e[k];
            }
#pragma unroll
            for (int k = 0; k < NR; k++) acc[k] ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
            if (!__any(any)) break;
        }
#pragma unroll
        for (int k = 0; k < NR; k++) {
            uint32_t x = acc[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
            if (lane == 0 && r0 + k < n) {
                uint32_t *dw = reinterpret_cast<uint32_t *>(out + r0 + k);
                dw[8] = x;
                dw[9] = 0;
            }
        }
    }
}

// DIAGNOSTIC (variants 31/32): pure linear read of src (grid-stride, 16 B per
// lane, UNR loads in flight), xor-folded; the chip's streaming-read ceiling
// for the same bytes.  Writes one word per workgroup.
template <int UNR>
__global__ __launch_bounds__(256) void k_diag_stream(const uint8_t *__restrict__ src, uint64_t src_len,
                                                     bhg_desc *__restrict__ out) {
    const uint64_t base = (uint64_t)src;
    const uint64_t nvec = src_len / 16;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride * UNR) {
        u32x4 x[UNR];
#pragma unroll
        for (int u = 0; u < UNR; u++) x[u] = v + u * stride < nvec ? gld<u32x4>(base + 16 * (v + u * stride)) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < UNR; u++) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
    }
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) reinterpret_cast<uint32_t *>(out)[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc;
}

// Decode variants (BHG_DECODE_VARIANT / ctx setting): slice, replication,
// workgroup size, resident workgroups per CU.
struct LaneVariant { int slice, repl, wg, wgs_per_cu, win, pf; };
static const LaneVariant kLaneVariants[] = {
    {1, 32, 256, 4, 4, 1},    // 0: byte table x32, 32 KiB/WG, 64 B windows
    {4, 32, 1024, 1, 4, 1},   // 1: slice-4 x32, 128 KiB/WG (conflict free)
    {4, 16, 512, 2, 4, 1},    // 2: slice-4 x16, 64 KiB/WG
    {4, 8, 256, 4, 4, 1},     // 3: slice-4 x8, 32 KiB/WG
    {4, 4, 256, 8, 4, 1},     // 4: slice-4 x4, 16 KiB/WG
    {4, 16, 1024, 2, 4, 1},   // 5: slice-4 x16, 64 KiB/WG, 32 waves/CU
    {4, 8, 512, 4, 4, 1},     // 6: slice-4 x8, 32 KiB/WG, 32 waves/CU
    {4, 16, 512, 2, 8, 1},    // 7: 128 B windows, prefetched
    {4, 8, 256, 4, 8, 1},     // 8
    {4, 8, 256, 4, 16, 0},    // 9: 256 B windows, no prefetch
    {4, 16, 512, 2, 16, 0},   // 10
    {4, 32, 1024, 1, 8, 1},   // 11
    {4, 8, 256, 4, 8, 0},     // 12: 128 B windows, no prefetch
    {4, 16, 512, 2, 8, 0},    // 13: 128 B line-aligned windows
    {4, 8, 512, 4, 8, 0},     // 14
    {4, 16, 1024, 2, 8, 0},   // 15
    {4, 32, 1024, 1, 16, 0},  // 16
    {0, 1, 512, 4, 8, 1},     // 17: DIAG loads only (xor fold), 128 B windows prefetched
    {0, 1, 512, 4, 4, 1},     // 18: DIAG loads only, 64 B windows prefetched
    {0, 1, 512, 4, 8, 0},     // 19: DIAG loads only, line-aligned 128 B windows
    {-1, 8, 512, 2, 0, 0},    // 20: cooperative loads, slice-4 x8, 8 waves/WG (72 KiB/WG)
    {-1, 8, 256, 4, 0, 0},    // 21: cooperative, x8, 4 waves/WG (52 KiB/WG)
    {-1, 16, 512, 1, 0, 0},   // 22: cooperative, x16, 8 waves/WG (104 KiB/WG)
    {-1, 4, 512, 3, 0, 0},    // 23: cooperative, x4, 8 waves/WG (56 KiB/WG)
    {-1, 16, 256, 2, 0, 0},   // 24: cooperative, x16, 4 waves/WG (84 KiB/WG)
    {-1, 0, 512, 2, 0, 0},    // 25: DIAG cooperative loads only (xor fold)
    {-2, 4, 256, 8, 0, 0},    // 26: DIAG wave-per-record loads only, 4 records in flight
    {-2, 2, 256, 8, 0, 0},    // 27: DIAG wave-per-record loads only, 2 records in flight
    {4, 16, 512, 2, 8, 2},    // 28: per-lane, line-aligned 128 B windows, prefetched
    {0, 1, 512, 4, 8, 2},     // 29: DIAG per-lane loads only, line-aligned prefetched
    {4, 8, 512, 2, 8, 2},     // 30: per-lane aligned prefetched, x8
    {-3, 4, 256, 8, 0, 0},    // 31: DIAG linear stream, 4 loads in flight per lane
    {-3, 8, 256, 8, 0, 0},    // 32: DIAG linear stream, 8 loads in flight per lane
    {4, 16, 512, 2, 8, 3},    // 33: per-lane, line-aligned, ping-pong 128 B windows, x16
    {4, 32, 1024, 1, 8, 3},   // 34: ping-pong, x32 (conflict free), 16 waves/CU
    {4, 8, 512, 2, 8, 3},     // 35: ping-pong, x8
    {0, 1, 512, 4, 8, 3},     // 36: DIAG ping-pong loads only
    {4, 16, 512, 2, 4, 3},    // 37: ping-pong 64 B windows, x16
    {4, 8, 256, 4, 8, 3},     // 38: ping-pong, x8, 4 waves/WG
    {-4, 16, 512, 2, 8, 0},   // 39: lanebuf (buffer-load ping-pong), x16, 128 B windows
    {-4, 32, 1024, 1, 8, 0},  // 40: lanebuf, x32 conflict-free, 16 waves/CU
    {-4, 8, 512, 2, 8, 0},    // 41: lanebuf, x8
    {-4, 16, 512, 2, 4, 0},   // 42: lanebuf, 64 B windows
    {-4, 8, 256, 4, 8, 0},    // 43: lanebuf, x8, 4-wave WGs
};
static const int kNumLaneVariants = sizeof(kLaneVariants) / sizeof(kLaneVariants[0]);

template <int MODE, int S, int R, int WG, int WIN = 4, int PF = 1>
static void launch_lane_t(const Launch &L, int wpc, const uint8_t *src, uint64_t src_len, const bhg_handle *h,
                          uint32_t n, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    uint64_t need = (n + WG - 1) / WG;
    uint64_t cap = (uint64_t)L.num_cus * (uint64_t)wpc;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_decode_lane<MODE, S, R, WG, WIN, PF>), dim3(grid), dim3(WG), 0, L.stream, src, src_len, h, n,
                       expected_crc, out, sizes);
}

template <int MODE, int R, int WAVES, int SLICE = 4>
static void launch_coop_t(const Launch &L, int wpc, const uint8_t *src, uint64_t src_len, const bhg_handle *h,
                          uint32_t n, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    const uint64_t tiles = (n + 63) / 64;
    uint64_t need = (tiles + WAVES - 1) / WAVES;
    uint64_t cap = (uint64_t)L.num_cus * (uint64_t)wpc;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_decode_coop<MODE, SLICE, R, WAVES>), dim3(grid), dim3(64 * WAVES), 0, L.stream, src, src_len, h,
                       n, expected_crc, out, sizes);
}

template <int MODE, int R, int WG, int WIN>
static void launch_lanebuf_t(const Launch &L, int wpc, const uint8_t *src, uint64_t src_len, const bhg_handle *h,
                             uint32_t n, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    const uint64_t tiles = (n + 63) / 64;
    uint64_t need = (tiles + WG / 64 - 1) / (WG / 64);
    uint64_t cap = (uint64_t)L.num_cus * (uint64_t)wpc;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_decode_lanebuf<MODE, R, WG, WIN>), dim3(grid), dim3(WG), 0, L.stream, src, src_len, h, n,
                       expected_crc, out, sizes);
}

template <int MODE>
static void launch_lane_mode(const Launch &L, int variant, const uint8_t *src, uint64_t src_len, const bhg_handle *h,
                             uint32_t n, const uint32_t *e, bhg_desc *out, uint64_t *sizes) {
    const LaneVariant &v = kLaneVariants[variant];
    const int w = L.lane_wgs_per_cu > 0 ? L.lane_wgs_per_cu : v.wgs_per_cu;
    switch (variant) {
    case 0: launch_lane_t<MODE, 1, 32, 256>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 1: launch_lane_t<MODE, 4, 32, 1024>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 2: launch_lane_t<MODE, 4, 16, 512>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 3: launch_lane_t<MODE, 4, 8, 256>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 4: launch_lane_t<MODE, 4, 4, 256>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 5: launch_lane_t<MODE, 4, 16, 1024>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 6: launch_lane_t<MODE, 4, 8, 512>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 7: launch_lane_t<MODE, 4, 16, 512, 8, 1>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 8: launch_lane_t<MODE, 4, 8, 256, 8, 1>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 9: launch_lane_t<MODE, 4, 8, 256, 16, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 10: launch_lane_t<MODE, 4, 16, 512, 16, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 11: launch_lane_t<MODE, 4, 32, 1024, 8, 1>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 12: launch_lane_t<MODE, 4, 8, 256, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 13: launch_lane_t<MODE, 4, 16, 512, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 14: launch_lane_t<MODE, 4, 8, 512, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 15: launch_lane_t<MODE, 4, 16, 1024, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 16: launch_lane_t<MODE, 4, 32, 1024, 16, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 17: launch_lane_t<MODE, 0, 1, 512, 8, 1>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 18: launch_lane_t<MODE, 0, 1, 512, 4, 1>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 19: launch_lane_t<MODE, 0, 1, 512, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 20: launch_coop_t<MODE, 8, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 21: launch_coop_t<MODE, 8, 4>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 22: launch_coop_t<MODE, 16, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 23: launch_coop_t<MODE, 4, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 24: launch_coop_t<MODE, 16, 4>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 25: launch_coop_t<MODE, 1, 8, 0>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 26: {
        uint32_t grid = (uint32_t)L.num_cus * 8;
        hipLaunchKernelGGL((k_diag_wave<4>), dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out);
        break;
    }
    case 27: {
        uint32_t grid = (uint32_t)L.num_cus * 8;
        hipLaunchKernelGGL((k_diag_wave<2>), dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out);
        break;
    }
    case 28: launch_lane_t<MODE, 4, 16, 512, 8, 2>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 29: launch_lane_t<MODE, 0, 1, 512, 8, 2>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 30: launch_lane_t<MODE, 4, 8, 512, 8, 2>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 31: hipLaunchKernelGGL((k_diag_stream<4>), dim3(L.num_cus * 8), dim3(256), 0, L.stream, src, src_len, out); break;
    case 32: hipLaunchKernelGGL((k_diag_stream<8>), dim3(L.num_cus * 8), dim3(256), 0, L.stream, src, src_len, out); break;
    case 33: launch_lane_t<MODE, 4, 16, 512, 8, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 34: launch_lane_t<MODE, 4, 32, 1024, 8, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 35: launch_lane_t<MODE, 4, 8, 512, 8, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 36: launch_lane_t<MODE, 0, 1, 512, 8, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 37: launch_lane_t<MODE, 4, 16, 512, 4, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 38: launch_lane_t<MODE, 4, 8, 256, 8, 3>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 39: launch_lanebuf_t<MODE, 16, 512, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 40: launch_lanebuf_t<MODE, 32, 1024, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 41: launch_lanebuf_t<MODE, 8, 512, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    case 42: launch_lanebuf_t<MODE, 16, 512, 4>(L, w, src, src_len, h, n, e, out, sizes); break;
    default: launch_lanebuf_t<MODE, 8, 256, 8>(L, w, src, src_len, h, n, e, out, sizes); break;
    }
}

hipError_t launch_decode_lane(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              int codec, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    int variant = L.variant;
    if (codec == BHG_CODEC_NONE && variant == kTileVariant)
        return launch_decode_tile(L, src, src_len, h, n, expected_crc, out);
    if (codec == BHG_CODEC_NONE && variant == kTile2Variant)
        return launch_decode_tile2(L, src, src_len, h, n, expected_crc, out);
    if (variant < 0 || variant >= kNumLaneVariants) variant = 28;
    if (codec == BHG_CODEC_NONE)
        launch_lane_mode<MODE_NONE>(L, variant, src, src_len, h, n, expected_crc, out, sizes);
    else
        launch_lane_mode<MODE_SNAPPY>(L, variant, src, src_len, h, n, expected_crc, out, sizes);
    return hipGetLastError();
}

hipError_t launch_snappy_wave(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
    if (L.snappy_variant == 2) return launch_snappy_rt(L, src, src_len, h, n, out, out_vals, out_cap, val_off);
    if (L.snappy_variant == 3) return launch_snappy_grp(L, src, src_len, h, n, out, out_vals, out_cap, val_off);
    if (L.snappy_variant == 4) return launch_snappy_rt(L, src, src_len, h, n, out, out_vals, out_cap, val_off, true);
    if (L.snappy_variant == 0) {
        uint32_t grid = (n + 255) / 256;
        const uint32_t cap = (uint32_t)L.num_cus * 8;
        if (grid > cap) grid = cap;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL(k_snappy_lane, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals,
                           out_cap, val_off);
        return hipGetLastError();
    }
    uint32_t grid = (n + SNAPPY_WAVES_PER_WG - 1) / SNAPPY_WAVES_PER_WG;
    const uint32_t cap = (uint32_t)L.num_cus * 16;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_snappy_wave, dim3(grid), dim3(64 * SNAPPY_WAVES_PER_WG), 0, L.stream, src, src_len, h, n,
                       out, out_vals, out_cap, val_off);
    return hipGetLastError();
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
