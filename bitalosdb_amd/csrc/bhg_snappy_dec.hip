// bhg_snappy_dec.hip -- golang/snappy v0.0.4 block decode (decode_other.go
// `decode`, called by internal/compress/compress.go:83-85), one LANE per
// block, with every element moved by ONE round trip to memory.
//
// Why: the first lane decoder (k_snappy_lane, bhg_decode.hip) copied an
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
// the tag stream through a per-lane 128-B LDS window (WIN, snappy_variant 4)
// cuts the fetch to 8.2 GB but not the time (2.83 ms): the walk is bound by
// the latency of its dependent element steps, not by HBM bandwidth.  This is
// the default (snappy_variant 2) and the next kernel to rework.
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
// WIN: the tag stream is read through a per-lane 128-B LDS window (win, 16-B
// aligned, 144 B) refilled with 8 whole 16-B loads; without it every tag is an
// 8-B global load, and at C3 those loads alone fetched 6.6 GB from HBM for
// 0.58 GB of stream (lines evicted between a lane's consecutive touches)
template <bool WIN>
__device__ __forceinline__ bool snappy_decode_rt(uint64_t cp, uint32_t slen, uint64_t dst, uint32_t dlen, uint64_t end,
                                                 uint64_t oend, uint8_t *win = nullptr) {
    const uint64_t oe = dst + dlen;
    uint32_t s = 0, d = 0;
    uint64_t wb = 0;  // absolute address of win[0]
    auto tag8 = [&](uint64_t p) -> uint64_t {
        if (!WIN) return ld64_bounded(p, end);
        if (wb == 0 || p < wb || p + 8 > wb + 128) {
            wb = p & ~15ull;
#pragma unroll
            for (uint32_t t = 0; t < 8; t++)
                *reinterpret_cast<u32x4 *>(win + 16 * t) = ld16_hi(wb + 16 * t, end);
        }
        const uint32_t q = (uint32_t)(p - wb), qa = q & ~3u, qs = q & 3u;
        const uint32_t w0 = *reinterpret_cast<const uint32_t *>(win + qa);
        const uint32_t w1 = *reinterpret_cast<const uint32_t *>(win + qa + 4);
        const uint32_t w2 = *reinterpret_cast<const uint32_t *>(win + qa + 8);
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, qs) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, qs) << 32);
    };
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

template <bool WIN>
__global__ __launch_bounds__(256) void k_snappy_rt(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                   uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    __shared__ __attribute__((aligned(16))) uint8_t wins[WIN ? 256 * 144 : 16];
    uint8_t *win = wins + (WIN ? threadIdx.x * 144 : 0);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = dw[9];
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t cpos = dw[2], dlen = dw[3];  // provisional: value position in the record, decoded length
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
            if (!snappy_decode_rt<WIN>(cp + hdr, clen - hdr, (uint64_t)out_vals + o0, dlen, end, oend, win))
                fin = BHG_ST_SNAPPY_CORRUPT;
        }
        dw[2] = 0;
        dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? dlen : 0u;
        dw[9] = fin;
    }
}

// ---------------------------------------------------------------------------
// k_snappy_grp: G lanes per block, the block's compressed stream and its
// decoded output both in LDS.
//
// Profiling k_snappy_rt at C3 showed 12.1 GB of HBM reads per launch for
// 1.6 GB of algorithmic traffic: half a million lanes each touching its own
// input line, output line and copy-source line 8-16 B at a time thrash the
// 4 MB L2 of every XCD.  Here a group of G lanes loads its block's stream
// with 16-B loads G wide (whole lines, once), decodes entirely inside LDS,
// and writes the decoded value back 16 B x G wide (whole lines, once).
//
// One code path serves every element: bytes out[d + k] = buf[i0 + k mod R]
// for k < n, with buf/i0/R = input/s/n for a literal, output/d-offset/n for
// a copy with offset >= n, and output/d-offset/offset for an overlapping
// copy (the LZ77 repeat); lane j of the group moves k = j, j+G, ...  All
// sources lie below d, written by earlier elements of the same wave (LDS
// operations of a wave complete in order).  Blocks whose stream or output
// exceeds the LDS slot are decoded by the group's first lane with
// snappy_decode_rt straight from/to global memory.
//
// Status: bit-exact, but at C3 3.23 ms per step vs 2.83 for k_snappy_rt:
// LDS caps residency at 72 blocks per CU (2.2 KB each) and an element costs
// ~1-2 k cycles of dependent LDS/VALU latency, so the kernel is latency
// bound where k_snappy_rt is bandwidth bound on over-fetch.  Kept as
// snappy_variant 3.
// ---------------------------------------------------------------------------
constexpr uint32_t kGrpInCap = 1152;   // compressed bytes + 3 alignment bytes
constexpr uint32_t kGrpOutCap = 1024;  // decoded bytes
constexpr uint32_t kGrpSlot = kGrpInCap + 16 + kGrpOutCap + 16;

template <int G>
__device__ __forceinline__ bool snappy_decode_lds(const uint8_t *inb, uint32_t s, uint32_t send, uint8_t *outb,
                                                  uint32_t dlen, uint32_t j) {
    uint32_t d = 0;
    while (s < send) {
        const uint32_t a = s & ~3u, sb = s & 3u;
        const uint32_t w0 = *reinterpret_cast<const uint32_t *>(inb + a);
        const uint32_t w1 = *reinterpret_cast<const uint32_t *>(inb + a + 4);
        const uint32_t w2 = *reinterpret_cast<const uint32_t *>(inb + a + 8);
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sb), hi = __builtin_amdgcn_alignbyte(w2, w1, sb);
        const uint64_t t8 = (uint64_t)lo | ((uint64_t)hi << 32);
        const uint32_t tag = lo & 0xffu;
        uint32_t n, R, i0;
        const uint8_t *buf;
        if ((tag & 3) == 0) {  // literal
            uint32_t x = tag >> 2;
            uint64_t l64;
            if (x < 60) {
                s += 1;
                l64 = (uint64_t)x + 1;
            } else {
                const uint32_t nb = x - 59;
                if ((uint64_t)s + 1 + nb > send) return false;
                s += 1 + nb;
                x = (uint32_t)(t8 >> 8) & (nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u));
                l64 = (uint64_t)x + 1;
            }
            if (l64 > (uint64_t)(dlen - d) || l64 > (uint64_t)(send - s)) return false;
            n = (uint32_t)l64;
            buf = inb;
            i0 = s;
            R = n;
            s += n;
        } else {
            uint32_t offset;
            if ((tag & 3) == 1) {
                if ((uint64_t)s + 2 > send) return false;
                s += 2;
                n = 4 + ((tag >> 2) & 7);
                offset = ((tag & 0xe0) << 3) | ((uint32_t)(t8 >> 8) & 0xffu);
            } else if ((tag & 3) == 2) {
                if ((uint64_t)s + 3 > send) return false;
                s += 3;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8) & 0xffffu;
            } else {
                if ((uint64_t)s + 5 > send) return false;
                s += 5;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8);
            }
            if (offset == 0 || d < offset || n > dlen - d) return false;
            buf = outb;
            i0 = d - offset;
            R = offset < n ? offset : n;
        }
        uint8_t *o = outb + d;
        if (R == n) {
            for (uint32_t k = j; k < n; k += 4 * G) {
                uint8_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
                b0 = buf[i0 + k];
                if (k + G < n) b1 = buf[i0 + k + G];
                if (k + 2 * G < n) b2 = buf[i0 + k + 2 * G];
                if (k + 3 * G < n) b3 = buf[i0 + k + 3 * G];
                o[k] = b0;
                if (k + G < n) o[k + G] = b1;
                if (k + 2 * G < n) o[k + 2 * G] = b2;
                if (k + 3 * G < n) o[k + 3 * G] = b3;
            }
        } else {  // overlapping copy: period R < n
            uint32_t km = j % R;
            const uint32_t step = (uint32_t)G % R;
            for (uint32_t k = j; k < n; k += G) {
                o[k] = buf[i0 + km];
                km += step;
                km = km >= R ? km - R : km;
            }
        }
        d += n;
        __atomic_signal_fence(__ATOMIC_SEQ_CST);  // keep this element's LDS writes before the next element's reads
    }
    return d == dlen;
}

template <int G, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_snappy_grp(const uint8_t *__restrict__ src, uint64_t src_len,
                                                         const bhg_handle *__restrict__ handles, uint32_t n,
                                                         bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                         uint64_t out_cap, const uint64_t *__restrict__ val_off) {
    constexpr uint32_t BPW = 64 / G;  // blocks per wave
    __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * BPW * kGrpSlot];
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane / G, j = lane % G;
    uint8_t *inb = lds + (wave * BPW + g) * kGrpSlot;
    uint8_t *outb = inb + kGrpInCap + 16;
    const uint32_t wstride = gridDim.x * WPB * BPW;
    for (uint32_t wb = (blockIdx.x * WPB + wave) * BPW; wb < n; wb += wstride) {
        const uint32_t i = wb + g;
        if (i >= n) continue;
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = dw[9];
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t cpos = dw[2], dlen = dw[3];  // provisional: value position in the record, decoded length
        const bhg_handle h = handles[i];
        const uint32_t clen = h.length - cpos;
        const uint64_t o0 = val_off[i], o1 = val_off[i + 1];
        uint32_t fin = status;
        if (o1 > out_cap || o1 - o0 < dlen) {
            fin = BHG_ST_SNAPPY_TOO_LARGE;
        } else {
            const uint64_t cp = base + h.offset + cpos;
            const uint32_t sh = (uint32_t)(cp & 3);
            const uint64_t ca = cp - sh;
            bool ok;
            if (clen + sh <= kGrpInCap && dlen <= kGrpOutCap) {
                const uint32_t nch = (clen + sh + 15) / 16;
                for (uint32_t t = j; t < nch; t += G) {
                    const uint64_t a = ca + 16ull * t;
                    u32x4 v;
                    if (a + 16 <= end) {
                        v = gld<u32x4_a4>(a);
                    } else {
                        v = u32x4{ld32_safe(a, end), ld32_safe(a + 4, end), ld32_safe(a + 8, end), ld32_safe(a + 12, end)};
                    }
                    *reinterpret_cast<u32x4 *>(inb + 16 * t) = v;
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                uint32_t s = sh;
                while (inb[s] >= 0x80) s++;  // uvarint decodedLen, validated by the header pass
                s++;
                ok = snappy_decode_lds<G>(inb, s, sh + clen, outb, dlen, j);
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
                if (ok) {
                    const uint64_t dst = (uint64_t)out_vals + o0;
                    for (uint32_t t = 16 * j; t < dlen; t += 16 * G)
                        st16_clip(dst + t, *reinterpret_cast<const u32x4 *>(outb + t), dst + dlen);
                }
                __atomic_signal_fence(__ATOMIC_SEQ_CST);
            } else {
                uint32_t r = 0;
                if (j == 0) {
                    uint32_t hdr = 0;
                    for (;;) {
                        const uint32_t b = gld<uint8_t>(cp + hdr);
                        hdr++;
                        if (b < 0x80) break;
                    }
                    r = snappy_decode_rt<false>(cp + hdr, clen - hdr, (uint64_t)out_vals + o0, dlen, end, oend) ? 1u : 0u;
                }
                ok = __shfl(r, g * G, 64) != 0;
            }
            if (!ok) fin = BHG_ST_SNAPPY_CORRUPT;
        }
        if (j == 0) {
            dw[2] = 0;
            dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? dlen : 0u;
            dw[9] = fin;
        }
    }
}

}  // namespace

hipError_t launch_snappy_rt(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                            bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off, bool win) {
    uint32_t grid = (n + 255) / 256;
    const uint32_t cap = (uint32_t)L.num_cus * (L.lane_wgs_per_cu > 0 ? L.lane_wgs_per_cu : 8);
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    if (win)
        hipLaunchKernelGGL(k_snappy_rt<true>, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals,
                           out_cap, val_off);
    else
        hipLaunchKernelGGL(k_snappy_rt<false>, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals,
                           out_cap, val_off);
    return hipGetLastError();
}

hipError_t launch_snappy_grp(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
    constexpr int G = 8, WPB = 1;  // 8 blocks per wave, 17.5 KB of LDS per workgroup: 9 workgroups per CU
    constexpr uint32_t bpw = 64 / G;
    uint64_t need = ((uint64_t)n + bpw * WPB - 1) / (bpw * WPB);
    const uint64_t cap = (uint64_t)L.num_cus * 9;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_snappy_grp<G, WPB>), dim3(grid), dim3(64 * WPB), 0, L.stream, src, src_len, h, n, out,
                       out_vals, out_cap, val_off);
    return hipGetLastError();
}

}  // namespace bhg
