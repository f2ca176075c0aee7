// snappy_ls_lab.hip -- lab record (not built into the product): k_snappy_ls, the
// C3 snappy decode with a lane per block and the block staged in LDS (stream
// staged with contiguous 16-B loads, elements walked in LDS, output written back
// with contiguous 16-B stores), round 2 session 2.
//
// Measured on MI355X against k_snappy_rt (bench c3 step, 1M blocks, header pass
// included): k_snappy_rt 2.74 ms; this kernel with the plain walk 3.9-5.8 ms
// (BPW 16/20/28/32 blocks per wave, 4/4/3/2 waves per CU) -- slower although it
// removes the over-fetch entirely (PMC FETCH_SIZE 0.65 GB vs 11.7 GB per launch):
// 62 % of wave time waiting, ~200 VALU+SALU instructions per element step,
// 11 % of LDS cycles in unaligned-access stalls, one wave per SIMD.
// The branch-light walk (snappy_decode_lds2) is bit-exact in a host emulation
// (scripts: 200k fuzzed streams + C3 values) but its BPW=20 build aborted twice
// on the GPU inside tests/test_gpu_decode.py::test_snappy_values and passed once
// in isolation.  Cause found in session 3 (the product k_snappy_lds hit it too):
// `(uint64_t)__builtin_amdgcn_readlane(lo32, b)` sign-extends (readlane returns int)
// an address whose bit 31 is set, and lanes that hand LDS bytes to each other need
// a wavefront fence + may_alias LDS types.  Kept here as the record.
#include "../../bitalosdb_amd/csrc/bhg_device.h"

namespace bhg {
typedef u32x4 u32x4_lds_u __attribute__((aligned(1)));
#ifndef BHG_LS_WALK
#define BHG_LS_WALK 2
#endif
typedef uint64_t u64_lds_u __attribute__((aligned(1)));

// The same element walk on a block staged in LDS: stream [sp, sp + slen), output [op, op + dlen),
// both byte offsets into one LDS slot.  Sources are read 4 x 16 B before any store of the element
// (LDS is ordered per wave, so a later read sees every earlier store); stores overshoot the
// element's end by up to 15 B, into bytes the next elements rewrite (the output area keeps 16 B
// of slack after dlen).
__device__ __forceinline__ bool snappy_decode_lds(uint8_t *lds, uint32_t sp, uint32_t slen, uint32_t op,
                                                  uint32_t dlen) {
    uint32_t s = 0, d = 0;
    while (s < slen) {
        const uint64_t t8 = *reinterpret_cast<const u64_lds_u *>(lds + sp + s);  // may read past the stream: masked below
        const uint32_t tag = (uint32_t)t8 & 0xffu;
        uint32_t n, R, a;
        if ((tag & 3) == 0) {  // literal
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
            n = (uint32_t)l64;
            a = sp + s;
            R = n;
            s += n;
        } else {
            uint32_t offset;
            if ((tag & 3) == 1) {
                if ((uint64_t)s + 2 > slen) return false;
                s += 2;
                n = 4 + ((tag >> 2) & 7);
                offset = ((tag & 0xe0) << 3) | ((uint32_t)(t8 >> 8) & 0xffu);
            } else if ((tag & 3) == 2) {
                if ((uint64_t)s + 3 > slen) return false;
                s += 3;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8) & 0xffffu;
            } else {
                if ((uint64_t)s + 5 > slen) return false;
                s += 5;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8);
            }
            if (offset == 0 || d < offset || n > dlen - d) return false;
            a = op + d - offset;
            R = offset < n ? offset : n;
        }
        const uint32_t o = op + d;
        const bool lit = (tag & 3) == 0;
        for (uint32_t k = 0; k < n;) {
            const uint32_t seg = lit ? (n - k < 64u ? n - k : 64u) : n;  // copies are <= 64 B
            const uint32_t src = lit ? a + k : a;
            const uint32_t rb = lit ? seg : R;
            const u32x4 c0 = *reinterpret_cast<const u32x4_lds_u *>(lds + src);
            const u32x4 c1 = *reinterpret_cast<const u32x4_lds_u *>(lds + src + 16);
            const u32x4 c2 = *reinterpret_cast<const u32x4_lds_u *>(lds + src + 32);
            const u32x4 c3 = *reinterpret_cast<const u32x4_lds_u *>(lds + src + 48);
            for (uint32_t t = 0; t < seg; t += rb) {
                uint8_t *q = lds + o + k + t;
                *reinterpret_cast<u32x4_lds_u *>(q) = c0;
                if (rb > 16 && t + 16 < seg) *reinterpret_cast<u32x4_lds_u *>(q + 16) = c1;
                if (rb > 32 && t + 32 < seg) *reinterpret_cast<u32x4_lds_u *>(q + 32) = c2;
                if (rb > 48 && t + 48 < seg) *reinterpret_cast<u32x4_lds_u *>(q + 48) = c3;
            }
            k += seg;
        }
        d += n;
    }
    return d == dlen;
}

// Branch-light form of the same walk for SIMT: every element is decoded with selects (no
// per-type branches), and moved as 16-B chunks at period R (R >= 16: chunk k reads src + 16k,
// which lies below the chunk's own destination; R < 16: the same 16 B -- the R-byte pattern --
// written at dst, dst + R, dst + 2R, ...).  Tag bytes come from three aligned dword reads.
__device__ __forceinline__ bool snappy_decode_lds2(uint8_t *lds, uint32_t sp, uint32_t slen, uint32_t op,
                                                   uint32_t dlen) {
    const uint32_t *l32 = reinterpret_cast<const uint32_t *>(lds);
    uint32_t s = 0, d = 0;
    bool ok = true;
    while (s < slen) {
        const uint32_t a = sp + s, wa = a >> 2, sh = a & 3;
        const uint32_t w0 = l32[wa], w1 = l32[wa + 1], w2 = l32[wa + 2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
        const uint32_t tag = lo & 0xffu, ty = tag & 3u, x = tag >> 2;
        const uint32_t b14 = (lo >> 8) | (hi << 24);  // bytes 1..4 after the tag
        const bool lit = ty == 0;
        const uint32_t nb = (lit && x >= 60) ? x - 59 : 0u;  // extra length bytes of a long literal
        const uint32_t lmask = nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
        const uint64_t l64 = lit ? (nb ? (uint64_t)(b14 & lmask) + 1 : (uint64_t)x + 1)
                                 : (uint64_t)(ty == 1 ? 4u + (x & 7u) : 1u + x);
        const uint32_t adv = lit ? 1u + nb : (ty == 1 ? 2u : ty == 2 ? 3u : 5u);
        const uint32_t off = ty == 1 ? (((tag & 0xe0u) << 3) | (b14 & 0xffu)) : ty == 2 ? (b14 & 0xffffu) : b14;
        const bool hdr_bad = (uint64_t)s + adv > slen;
        const bool bad = lit ? (hdr_bad || l64 > (uint64_t)(dlen - d) || l64 > (uint64_t)slen - s - adv)
                             : (hdr_bad || off == 0 || d < off || l64 > (uint64_t)(dlen - d));
        if (bad) {
            ok = false;
            break;
        }
        const uint32_t n = (uint32_t)l64;
        const uint32_t src = lit ? a + adv : op + d - off;
        const uint32_t R = lit ? n : (off < n ? off : n);
        const uint32_t step = R >= 16 ? 16u : R, rstep = R >= 16 ? 16u : 0u;
        const uint32_t o = op + d;
        for (uint32_t t = 0, r = 0; t < n; t += step, r += rstep)
            *reinterpret_cast<u32x4_lds_u *>(lds + o + t) = *reinterpret_cast<const u32x4_lds_u *>(lds + src + r);
        s += adv + (lit ? n : 0u);
        d += n;
    }
    return ok && d == dlen;
}


// ---------------------------------------------------------------------------
// k_snappy_ls: lane per block, the block staged in LDS.  A wave takes BPW
// consecutive blocks; the whole wave copies each block's stream into the
// block's LDS slot with contiguous 16-B loads (one 1-KB request per wave
// instruction), lane b walks block b's elements entirely in LDS (tag reads,
// literal and copy-source reads, stores: an LDS round trip per element instead
// of an HBM/L2 one, and no line of the stream or of the output is fetched
// twice), then the whole wave writes each decoded block out with contiguous
// 16-B stores.  Blocks whose stream or output exceed the slot decode in their
// lane with snappy_decode_rt (global memory), as before.
// Slot = SO stream bytes + OB output bytes + 16 B of store slack (+ 64 B of
// read slack for the 4 x 16 B source reads near the slot end).
// ---------------------------------------------------------------------------
template <int BPW, int SO, int OB>
__global__ __launch_bounds__(64) void k_snappy_ls(const uint8_t *__restrict__ src, uint64_t src_len,
                                                  const bhg_handle *__restrict__ handles, uint32_t n,
                                                  bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                  uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    constexpr uint32_t SLOT = SO + OB + 16 + 64;
    __shared__ __attribute__((aligned(16))) uint8_t lds[BPW * SLOT];
    const uint32_t lane = threadIdx.x;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    const uint32_t ngroups = (n + BPW - 1) / BPW;
    for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        const uint32_t i = g * BPW + lane;
        // ---- per block (lane < BPW): provisional descriptor from the header pass
        uint32_t status = BHG_ST_RECORD_NIL, cpos = 0, dlen = 0, clen = 0, fin = 0;
        uint64_t cp = 0, o0 = 0;
        bool act = false, staged = false;
        if (lane < BPW && i < n) {
            const uint32_t *dw = reinterpret_cast<const uint32_t *>(out + i);
            status = dw[9];
            if (status == BHG_ST_OK || status == BHG_ST_CRC_MISMATCH) {
                cpos = dw[2];
                dlen = dw[3];
                const bhg_handle h = handles[i];
                cp = base + h.offset + cpos;
                clen = h.length - cpos;
                o0 = val_off[i];
                const uint64_t o1 = val_off[i + 1];
                act = true;
                fin = status;
                if (o1 > out_cap || o1 - o0 < dlen) {
                    fin = BHG_ST_SNAPPY_TOO_LARGE;
                    act = false;
                } else {
                    staged = clen <= SO && dlen <= OB;
                }
            }
        }
        uint8_t *const slot = lds + (lane < BPW ? lane : 0) * SLOT;
        // ---- stage: block b's stream [cp, cp + clen) -> slot b, 16 B per lane per instruction
        const uint32_t scl = staged ? clen : 0u;
        for (uint32_t b = 0; b < BPW; b++) {
            const uint32_t cl = __builtin_amdgcn_readlane(scl, b);
            if (cl == 0) continue;  // wave-uniform
            const uint64_t c = (uint64_t)__builtin_amdgcn_readlane((uint32_t)cp, b) |
                               ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(cp >> 32), b) << 32);
            for (uint32_t off = 16 * lane; off < cl; off += 1024)
                *reinterpret_cast<u32x4 *>(lds + b * SLOT + off) = ld16_hi(c + off, c + cl);
        }
        // ---- decode: lane b walks block b in LDS
        if (staged) {
            uint32_t hdr = 0;
            while (slot[hdr] >= 0x80) hdr++;  // uvarint decodedLen, validated by the header pass
            hdr++;
            if (!(BHG_LS_WALK == 2 ? snappy_decode_lds2(slot, hdr, clen - hdr, SO, dlen)
                                   : snappy_decode_lds(slot, hdr, clen - hdr, SO, dlen)))
                fin = BHG_ST_SNAPPY_CORRUPT;
        } else if (act) {
            uint32_t hdr = 0;
            for (;;) {
                const uint32_t bb = gld<uint8_t>(cp + hdr);
                hdr++;
                if (bb < 0x80) break;
            }
            if (!snappy_decode_rt(cp + hdr, clen - hdr, (uint64_t)out_vals + o0, dlen, end, oend))
                fin = BHG_ST_SNAPPY_CORRUPT;
        }
        // ---- write out: block b's decoded bytes -> out_vals[o0, o0 + dlen), 16 B per lane per instruction
        const bool good = staged && (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH);
        const uint32_t gdl = good ? dlen : 0u;
        for (uint32_t b = 0; b < BPW; b++) {
            const uint32_t dl = __builtin_amdgcn_readlane(gdl, b);
            if (dl == 0) continue;  // wave-uniform
            const uint64_t o = (uint64_t)out_vals + ((uint64_t)__builtin_amdgcn_readlane((uint32_t)o0, b) |
                                                     ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(o0 >> 32), b) << 32));
            for (uint32_t off = 16 * lane; off < dl; off += 1024)
                st16_clip(o + off, *reinterpret_cast<const u32x4 *>(lds + b * SLOT + SO + off), o + dl);
        }
        if (lane < BPW && i < n && (status == BHG_ST_OK || status == BHG_ST_CRC_MISMATCH)) {
            uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
            dw[2] = 0;
            dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? dlen : 0u;
            dw[9] = fin;
        }
    }
}


/* launcher as it was in bhg_snappy_dec.hip:
#ifndef BHG_SNAPPY_LS
#define BHG_SNAPPY_LS 0
#endif
#ifndef BHG_LS_BPW
#define BHG_LS_BPW 20
#endif
hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
    if (BHG_SNAPPY_LS) {
        constexpr uint32_t BPW = BHG_LS_BPW;
        const uint32_t groups = (n + BPW - 1) / BPW;
        const uint32_t cap = (uint32_t)L.num_cus * 16;
        uint32_t grid = groups < cap ? groups : cap;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL((k_snappy_ls<BPW, 768, 1024>), dim3(grid), dim3(64), 0, L.stream, src, src_len, h, n, out,
                           out_vals, out_cap, val_off);
        return hipGetLastError();
    }
*/
}  // namespace bhg
