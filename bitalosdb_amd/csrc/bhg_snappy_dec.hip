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

hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off) {
    uint32_t grid = (n + 255) / 256;
    const uint32_t cap = (uint32_t)L.num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_snappy_rt, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals, out_cap,
                       val_off);
    return hipGetLastError();
}

}  // namespace bhg
