// Lab record (not built into the product): the LDS-staged group snappy
// decoder tried in round 2.  Bit-exact (tests/test_gpu_decode.py snappy cases,
// full-size C3) but slower than k_snappy_rt on MI355X:
//   G=16 byte lanes, SLOT 3072, 12 waves/CU       4.07 ms per 1M C3 blocks
//   G=4, 16-B unaligned LDS chunks, 4 waves/CU    3.26 ms (PMC: 456M SALU, 292M
//        VALU, 18M LDS instr; 52M LDS unaligned-stall and 35M bank-conflict cycles)
//   G=8, SLOT 1600, 12 waves/CU                   1.94 ms for the blocks that fit
// k_snappy_rt: 2.4 ms.  Per element the group pays an LDS tag read, a
// dependent decode and an LDS move with no other work to hide them; 96-100
// resident blocks per CU (1.6 KB of LDS each) are not enough.
#include "../../bitalosdb_amd/csrc/bhg_device.h"

namespace bhg {
// ---------------------------------------------------------------------------
// k_snappy_lds: the same decode with every block staged in LDS.  A group of
// G lanes owns a block and a SLOT-byte LDS slot: the block's stream
// (staged with 16-B loads) and, 16-B aligned after it, the decoded bytes.
// All lanes of a group parse the same tag (LDS broadcast reads; the parse is
// branch-free selects, so the groups of a wave stay converged), then one
// element is moved as up to G 16-B unaligned LDS chunks, one per lane:
//   literal              out[d + k] = stream[s + k]
//   copy, offset >= 16   split into sub-copies of at most `offset` bytes,
//                        each reading only bytes below its own start (final)
//   copy, offset < 16    one byte per lane step: out[d + k] = out[d - o + k mod o]
// A chunk's tail beyond the element's end writes bytes that the next
// elements overwrite (the slot keeps 16 B of slack after the output).  The
// decoded block leaves LDS as 16-B stores.  Blocks that do not fit a slot
// keep their provisional descriptor and are decoded by k_snappy_rt.
// ---------------------------------------------------------------------------
typedef u32x4 u32x4_lds_u __attribute__((aligned(1)));

template <int G, int SLOT, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_snappy_lds(const uint8_t *__restrict__ src, uint64_t src_len,
                                                         const bhg_handle *__restrict__ handles, uint32_t n,
                                                         bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                         uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    constexpr uint32_t BPW = 64 / G;
    constexpr uint32_t STRIDE = SLOT + 16;  // slot bases 4 banks apart: groups at equal offsets spread over banks
    __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * BPW * STRIDE];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane / G, t = lane % G;
    uint8_t *const slot = lds + (w * BPW + q) * STRIDE;
    const uint64_t base = (uint64_t)src;
    const uint32_t ngroups = (n + BPW - 1) / BPW;
    for (uint32_t g = blockIdx.x * WPB + w; g < ngroups; g += gridDim.x * WPB) {
        const uint32_t i = g * BPW + q;
        bool act = false;
        uint32_t status = 0, dlen = 0, clen = 0, so = 0;
        uint64_t o0 = 0, rec = 0, rend = 0;
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + (i < n ? i : 0));
        if (i < n) {
            status = dw[9];
            const uint32_t cpos = dw[2];  // provisional (header pass): value position in the record
            if ((status == BHG_ST_OK || status == BHG_ST_CRC_MISMATCH) && cpos != 0) {
                dlen = dw[3];
                const bhg_handle h = handles[i];
                clen = h.length - cpos;
                rec = base + h.offset + cpos;
                rend = base + h.offset + h.length;
                o0 = val_off[i];
                const uint64_t o1 = val_off[i + 1];
                so = (clen + 15) & ~15u;
                if (o1 > out_cap || o1 - o0 < dlen) {
                    if (t == 0) {
                        dw[2] = 0;
                        dw[3] = 0;
                        dw[9] = BHG_ST_SNAPPY_TOO_LARGE;
                    }
                } else {
                    act = (uint64_t)so + dlen + 16 <= SLOT;  // 16 B of slack for chunk tails
                }
            }
        }
        if (act)
            for (uint32_t off = 16 * t; off < clen; off += 16 * G)
                *reinterpret_cast<u32x4 *>(slot + off) = ld16_hi(rec + off, rend);
        uint32_t s = 0, d = 0;
        bool ok = true;
        if (act) {  // decodedLen uvarint (validated by the header pass): skip it
            while (slot[s] >= 0x80) s++;
            s++;
        }
        uint8_t *const ob = slot + so;
        // one element per group per iteration; the loop and the common move are wave-uniform
        // (predicated), only the rare long / overlapping elements take a divergent slow path
        for (;;) {
            if (act && s >= clen) {
                ok = d == dlen;
                act = false;
            }
            if (__ballot(act) == 0) break;
            uint32_t len = 0, adv = 0, off = 0;
            bool lit = false;
            if (act) {
                // ---- parse one tag (decode_other.go decode), branch-free
                const uint32_t a = s & ~3u, sh = s & 3u;
                const uint32_t w0 = *reinterpret_cast<const uint32_t *>(slot + a);
                const uint32_t w1 = *reinterpret_cast<const uint32_t *>(slot + a + 4);
                const uint32_t w2 = *reinterpret_cast<const uint32_t *>(slot + a + 8);
                const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
                const uint32_t tag = lo & 0xffu, ty = tag & 3u, x = tag >> 2;
                lit = ty == 0;
                const bool llong = lit && x >= 60;
                const uint32_t nb = llong ? x - 59 : 0u;  // extra length bytes of a long literal (1..4)
                const uint64_t t8 = (uint64_t)lo | ((uint64_t)hi << 32);
                const uint64_t lmask = nb >= 4 ? 0xffffffffull : ((1ull << (8 * nb)) - 1);
                const uint64_t l64 = lit ? (llong ? ((t8 >> 8) & lmask) + 1 : (uint64_t)x + 1)
                                         : (ty == 1 ? 4u + (x & 7u) : 1u + x);
                adv = lit ? 1 + nb : (ty == 1 ? 2u : ty == 2 ? 3u : 5u);
                off = ty == 1 ? (((tag & 0xe0u) << 3) | ((lo >> 8) & 0xffu))
                              : ty == 2 ? ((lo >> 8) & 0xffffu) : ((lo >> 8) | (hi << 24));
                const bool hdr_bad = (uint64_t)s + adv > clen;
                const bool bad = lit ? (hdr_bad || l64 > (uint64_t)(dlen - d) || l64 > (uint64_t)clen - s - adv)
                                     : (hdr_bad || off == 0 || d < off || l64 > (uint64_t)(dlen - d));
                len = (uint32_t)l64;
                if (bad) {
                    ok = false;
                    act = false;
                    len = 0;
                }
            }
            // ---- move: up to 64 B as one 16-B chunk per lane, when no byte depends on this element
            const bool fast = act && len <= 16 * G && (lit || off >= len);
            const uint32_t sbase = lit ? s + adv : so + d - off;
            if (fast && 16 * t < len) {
                const u32x4 v = *reinterpret_cast<const u32x4_lds_u *>(slot + sbase + 16 * t);
                *reinterpret_cast<u32x4_lds_u *>(ob + d + 16 * t) = v;
            }
            if (__ballot(act && !fast) != 0 && act && !fast) {
                if (lit || off >= 16) {
                    // non-overlapping pieces of at most `step` bytes; a piece reads only bytes below its start
                    const uint32_t step = lit ? 16 * G : (off < 16 * G ? off : 16 * G);
                    for (uint32_t p0 = 0; p0 < len; p0 += step) {
                        const uint32_t pl = len - p0 < step ? len - p0 : step;
                        for (uint32_t c = 16 * t; c < pl; c += 16 * G) {
                            const u32x4 v = *reinterpret_cast<const u32x4_lds_u *>(slot + sbase + p0 + c);
                            *reinterpret_cast<u32x4_lds_u *>(ob + d + p0 + c) = v;
                        }
                    }
                } else {  // offset 1..15: the LZ77 run, a byte per lane per step from the period below d
                    uint32_t km = t % off;
                    for (uint32_t k = t; k < len; k += G) {
                        ob[d + k] = slot[sbase + km];
                        km += G;
                        km = km >= off ? km - off : km;
                        km = km >= off ? km - off : km;
                        km = km >= off ? km - off : km;
                        km = km >= off ? km - off : km;
                    }
                }
            }
            if (act) {
                s += adv + (lit ? len : 0u);
                d += len;
            }
        }
        if (act && ok)
            for (uint32_t off = 16 * t; off < dlen; off += 16 * G)
                st16_clip((uint64_t)out_vals + o0 + off, *reinterpret_cast<const u32x4 *>(ob + off),
                          (uint64_t)out_vals + o0 + dlen);
        if (act && t == 0) {
            dw[2] = 0;
            dw[3] = ok ? dlen : 0u;
            dw[9] = ok ? status : BHG_ST_SNAPPY_CORRUPT;
        }
    }
}


}  // namespace bhg
