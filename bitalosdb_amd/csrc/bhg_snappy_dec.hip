// bhg_snappy_dec.hip -- golang/snappy v0.0.4 block decode (decode_other.go
// `decode`, called by internal/compress/compress.go:83-85), one LANE per
// block, with every element moved by ONE round trip to memory.
//
// Why: the first lane decoder (round 1's k_snappy_lane) copied an
// element 16, 4 or 1 byte(s) at a time with a load of its own earlier
// output inside the loop.  On CDNA4 vmcnt counts stores as well as loads, so
// each such load also waits for every store before it: an overlapping copy
// of offset 1..3 cost one L2 round trip per BYTE, and the wave-wide element
// step is set by the slowest of 64 lanes.
//
// Here an element is (source address A, period R, length n):
//   literal            A = input + s,      R = n (walked in 64-B segments)
//   copy, offset >= n  A = output + d - o, R = n
//   copy, offset <  n  A = output + d - o, R = o   (LZ77 overlap: the output
//                      is the o bytes before d repeated, out[d+k] =
//                      out[d - o + k mod o])
// Up to 4 x 16 B of A are loaded at once (all of it lies below d, i.e. was
// stored by earlier elements), then the 16-B chunks are stored at d, d+R,
// d+2R, ...: a later store overwrites the garbage tail of an earlier one,
// so nothing is read back.  The next element's tag is loaded before this
// element's data, so one wait covers both.  Chunks never store at or past
// the block's end (dlen); bytes between d+n and dlen they overshoot into are
// rewritten by the following elements in program order.
//
// The validation is the reference decoder's, check for check: literal
// length fields past the input, literal longer than the remaining input or
// output, copy offset 0 or beyond the bytes written, copy past dlen, and
// d == dlen at the end (snappy.ErrCorrupt otherwise).
//
// Measured at C3 (1M blocks, ~526 B streams -> 1 KiB): 2.39 ms per launch
// vs 2.96 ms for k_snappy_lane; rocprofv3 FETCH_SIZE says 12.1 GB of HBM
// reads per launch for ~1.3 GB of stream + copy-source bytes -- every lane
// walks its own lines 8-16 B at a time and the lines are evicted between
// its consecutive touches (profiles/r1_s4_pmc_snappy_rt.json).  Residency
// 4..32 waves per CU changes the time by < 15 %.  Knock-outs (timing only):
// no copy-source loads 2.20 ms / 6.6 GB, no stores 1.95 ms / 12.2 GB, neither
// 1.24 ms / 6.6 GB -- the tag and literal loads alone fetch 6.6 GB.  Reading
// the tag stream through a per-lane 128-B LDS window cut the fetch to 8.2 GB
// but not the time (2.83 ms): the walk is bound by the latency of its
// dependent element steps, not by HBM bandwidth.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

typedef u32x4 u32x4u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1)));

__device__ __forceinline__ uint64_t ld64_bounded(uint64_t a, uint64_t hi) {
    if (a + 8 <= hi) return gld<u64u>(a);
    uint64_t x = 0;
    for (uint32_t b = 0; b < 8; b++)
        if (a + b < hi) x |= (uint64_t)gld<uint8_t>(a + b) << (8 * b);
    return x;
}

__device__ __forceinline__ u32x4 ld16_hi(uint64_t a, uint64_t hi) {
    if (a + 16 <= hi) return gld<u32x4u>(a);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < 16; b++)
        if (a + b < hi) w[b >> 2] |= (uint32_t)gld<uint8_t>(a + b) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

// 16 bytes at a, clipped at oe (exclusive)
__device__ __forceinline__ void st16_clip(uint64_t a, u32x4 v, uint64_t oe) {
    if (a + 16 <= oe) {
        gst<u32x4u>(a, v);
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t b = 0; b < 16; b++)
        if (a + b < oe) gst<uint8_t>(a + b, (uint8_t)(w[b >> 2] >> (8 * (b & 3))));
}

// cp/dst absolute; the stream is [cp, cp + slen), the block's output [dst, dst + dlen);
// end bounds input reads, oend bounds output reads (the out_vals allocation)
__device__ __forceinline__ bool snappy_decode_rt(uint64_t cp, uint32_t slen, uint64_t dst, uint32_t dlen, uint64_t end,
                                                 uint64_t oend) {
    const uint64_t oe = dst + dlen;
    uint32_t s = 0, d = 0;
    auto tag8 = [&](uint64_t p) -> uint64_t { return ld64_bounded(p, end); };
    uint64_t t8 = slen ? tag8(cp) : 0;
    while (s < slen) {
        const uint32_t tag = (uint32_t)t8 & 0xffu;
        uint32_t n, R;
        uint64_t A, hi;
        bool lit;
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
            A = cp + s;
            R = n;
            hi = end;
            lit = true;
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
            A = dst + d - offset;
            R = offset < n ? offset : n;
            hi = oend;
            lit = false;
        }
        if (s < slen) t8 = tag8(cp + s);  // next tag: in flight with this element's data
        const uint64_t o = dst + d;
        for (uint32_t k = 0; k < n;) {
            const uint32_t seg = lit ? (n - k < 64u ? n - k : 64u) : n;  // copies are <= 64 B
            const uint64_t a = lit ? A + k : A;
            const uint32_t rb = lit ? seg : R;
            const u32x4 z = {0, 0, 0, 0};
            const u32x4 c0 = ld16_hi(a, hi);
            const u32x4 c1 = rb > 16 ? ld16_hi(a + 16, hi) : z;
            const u32x4 c2 = rb > 32 ? ld16_hi(a + 32, hi) : z;
            const u32x4 c3 = rb > 48 ? ld16_hi(a + 48, hi) : z;
            for (uint32_t t = 0; t < seg; t += rb) {
                const uint64_t q = o + k + t;
                st16_clip(q, c0, oe);
                if (rb > 16 && t + 16 < seg) st16_clip(q + 16, c1, oe);
                if (rb > 32 && t + 32 < seg) st16_clip(q + 32, c2, oe);
                if (rb > 48 && t + 48 < seg) st16_clip(q + 48, c3, oe);
            }
            k += seg;
        }
        d += n;
    }
    return d == dlen;
}

}  // namespace

__global__ __launch_bounds__(256) void k_snappy_rt(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                   uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = dw[9];
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t cpos = dw[2], dlen = dw[3];  // provisional: value position in the record, decoded length
        if (cpos == 0) continue;                    // finalized by k_snappy_lds
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
            for (;;) {  // uvarint decodedLen, validated by the header pass
                const uint32_t b = gld<uint8_t>(cp + hdr);
                hdr++;
                if (b < 0x80) break;
            }
            if (!snappy_decode_rt(cp + hdr, clen - hdr, (uint64_t)out_vals + o0, dlen, end, oend))
                fin = BHG_ST_SNAPPY_CORRUPT;
        }
        dw[2] = 0;
        dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? dlen : 0u;
        dw[9] = fin;
    }
}

// ---------------------------------------------------------------------------
// k_snappy_lds: the same decode with each block staged in LDS and its
// elements moved by a group of G = 16 lanes.  A wave decodes 4 blocks at a
// time; each group owns a SLOT-byte LDS slot holding the block's stream
// (loaded with 16-B coalesced reads) and, 16-B aligned after it, the decoded
// bytes.  Every lane of a group parses the same tag (LDS broadcast reads, no
// divergence inside a group), then the element's bytes move one per lane per
// step: out[d + k] = literal ? stream[s + k] : out[d - o + (k mod o)] -- the
// LZ77 overlap of a copy with o < length reads only bytes below d, which are
// final, so the lanes of a step are independent.  The decoded block leaves
// LDS as 16-B stores.  Blocks that do not fit a slot are left for
// k_snappy_rt (their provisional descriptor is untouched).
// ---------------------------------------------------------------------------
template <int SLOT, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_snappy_lds(const uint8_t *__restrict__ src, uint64_t src_len,
                                                         const bhg_handle *__restrict__ handles, uint32_t n,
                                                         bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                         uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    constexpr uint32_t G = 16, BPW = 64 / G;
    __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * BPW * SLOT];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, q = lane / G, t = lane % G;
    uint8_t *const slot = lds + (w * BPW + q) * SLOT;
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
                    act = (uint64_t)so + (dlen > 16 ? dlen : 16) <= SLOT;
                }
            }
        }
        // stage the stream: 16 B per lane per step, zero past the record
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
        while (act) {
            if (s >= clen) {
                ok = d == dlen;
                break;
            }
            const uint32_t a = s & ~3u, sh = s & 3u;
            const uint32_t w0 = *reinterpret_cast<const uint32_t *>(slot + a);
            const uint32_t w1 = *reinterpret_cast<const uint32_t *>(slot + a + 4);
            const uint32_t w2 = *reinterpret_cast<const uint32_t *>(slot + a + 8);
            const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh), hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
            const uint32_t tag = lo & 0xffu;
            uint32_t len, adv, off = 0;
            bool lit = false, bad;
            if ((tag & 3) == 0) {  // literal
                const uint32_t x = tag >> 2;
                uint64_t l64;
                if (x < 60) {
                    adv = 1;
                    l64 = (uint64_t)x + 1;
                    bad = false;
                } else {
                    const uint32_t nb = x - 59;
                    adv = 1 + nb;
                    const uint64_t t8 = (uint64_t)lo | ((uint64_t)hi << 32);
                    l64 = ((t8 >> 8) & (nb >= 4 ? 0xffffffffull : ((1ull << (8 * nb)) - 1))) + 1;
                    bad = (uint64_t)s + adv > clen;
                }
                bad = bad || l64 > (uint64_t)(dlen - d) || l64 > (uint64_t)clen - s - adv;
                len = (uint32_t)l64;
                lit = true;
            } else {
                if ((tag & 3) == 1) {
                    adv = 2;
                    len = 4 + ((tag >> 2) & 7);
                    off = ((tag & 0xe0u) << 3) | ((lo >> 8) & 0xffu);
                } else if ((tag & 3) == 2) {
                    adv = 3;
                    len = 1 + (tag >> 2);
                    off = (lo >> 8) & 0xffffu;
                } else {
                    adv = 5;
                    len = 1 + (tag >> 2);
                    off = (lo >> 8) | (hi << 24);
                }
                bad = (uint64_t)s + adv > clen || off == 0 || d < off || len > dlen - d;
            }
            if (bad) {
                ok = false;
                break;
            }
            const uint32_t sp = lit ? s + adv : so + d - off;  // source of element byte 0 in the slot
            const bool wrap = !lit && off < len;
            const float rcp = __builtin_amdgcn_rcpf((float)(off ? off : 1u));
            for (uint32_t k0 = 0; k0 < len; k0 += G) {
                const uint32_t k = k0 + t;
                if (k < len) {
                    uint32_t kk = k;
                    if (wrap) {  // k mod off, k < 64: float quotient, one correction each way
                        uint32_t qq = (uint32_t)((float)k * rcp);
                        int32_t r = (int32_t)(k - qq * off);
                        r = r < 0 ? r + (int32_t)off : r;
                        r = r >= (int32_t)off ? r - (int32_t)off : r;
                        kk = (uint32_t)r;
                    }
                    ob[d + k] = slot[sp + kk];
                }
            }
            if (lit) s += len;
            s += adv;
            d += len;
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

hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
    constexpr int SLOT = 3072, WPB = 4;  // 48 KiB of LDS per workgroup: three per CU
    const uint64_t groups = (n + 3) / 4;
    uint64_t gl = (groups + WPB - 1) / WPB;
    const uint64_t capl = (uint64_t)L.num_cus * 3;
    if (gl > capl) gl = capl;
    if (gl == 0) gl = 1;
    hipLaunchKernelGGL((k_snappy_lds<SLOT, WPB>), dim3((uint32_t)gl), dim3(64 * WPB), 0, L.stream, src, src_len, h, n,
                       out, out_vals, out_cap, val_off);
    // the blocks too large for a slot (their descriptors are still provisional)
    uint32_t grid = (n + 255) / 256;
    const uint32_t cap = (uint32_t)L.num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_snappy_rt, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals, out_cap,
                       val_off);
    return hipGetLastError();
}

}  // namespace bhg
