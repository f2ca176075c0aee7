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

template <int MODE>
__global__ __launch_bounds__(256) void k_decode_lane(const uint8_t *__restrict__ src, uint64_t src_len,
                                                     const bhg_handle *__restrict__ handles, uint32_t n,
                                                     const uint32_t *__restrict__ expected_crc,
                                                     bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes) {
    __shared__ __attribute__((aligned(16))) uint32_t T[BHG_CRC_LDS_WORDS];
    crc_lds_fill(T);
    __syncthreads();
    const CrcLds crc(T);
    const uint64_t base = (uint64_t)src;
    const uint64_t end = base + src_len;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const bhg_handle h = handles[i];
        DescOut d = {0, 0, 0, 0, 0, 0, 0, 0, BHG_ST_OK};
        uint64_t dsize = 0;
        if (h.length == 0) {
            d.status = BHG_ST_ILLEGAL_LENGTH;              // reader.go:234-236
        } else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) {
            d.status = BHG_ST_INCOMPLETE;                  // ReadAt short
        } else {
            const uint64_t p = base + h.offset;
            const uint32_t L = h.length;
            d.crc = crc_mask(~crc_range(crc, 0xffffffffu, p, L, end));
            if (L < 12) {
                d.status = BHG_ST_RECORD_NIL;
            } else {
                const uint32_t k = ldu32(p, end), v = ldu32(p + 4, end), fn = ldu32(p + 8, end);
                if (k == 0 || v == 0 || (uint64_t)12 + k + v != (uint64_t)L) {
                    d.status = BHG_ST_RECORD_NIL;          // block2.go:59-62
                    d.crc = d.crc;                          // crc stays (bytes were readable)
                } else {
                    d.file_num = fn;
                    d.key_off = 12;
                    if (k >= 8) {
                        d.key_len = k - 8;
                        d.trailer = ldu64(p + 12 + k - 8, end);
                    } else {
                        d.key_len = 0;
                        d.trailer = 255;                    // InternalKeyKindInvalid
                    }
                    d.fnv1 = fnv1_range(p + 12, d.key_len, end);
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
                            d.val_len = (uint32_t)dl;       // provisional; k_snappy_wave finalises
                            d.val_off = 12 + k;             // provisional: compressed payload offset
                        }
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
// batched primitives
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_crc_ranges(const uint8_t *__restrict__ src, uint64_t src_len,
                                                    const bhg_handle *__restrict__ handles, uint32_t n,
                                                    uint32_t *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint32_t T[BHG_CRC_LDS_WORDS];
    crc_lds_fill(T);
    __syncthreads();
    const CrcLds crc(T);
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

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
hipError_t launch_decode_lane(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              int codec, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    const uint32_t grid = lane_grid(L, n, 256);
    if (codec == BHG_CODEC_NONE)
        hipLaunchKernelGGL(k_decode_lane<MODE_NONE>, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n,
                           expected_crc, out, sizes);
    else
        hipLaunchKernelGGL(k_decode_lane<MODE_SNAPPY>, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n,
                           expected_crc, out, sizes);
    return hipGetLastError();
}

hipError_t launch_snappy_wave(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
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

hipError_t launch_fnv_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out) {
    hipLaunchKernelGGL(k_fnv_ranges, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, out);
    return hipGetLastError();
}

}  // namespace bhg
