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

// One CHUNK of a block (the big-block path below): the elements from stream position s0 to s_end
// (positions after the uvarint header), writing output [d0, d_end) of the block's dlen.  The same
// checks as snappy_decode_rt, plus: a copy reaching before d0 (into another chunk, which another lane
// may not have written yet), an element passing s_end or d_end, or not ending exactly at (s_end,
// d_end) -> false, and the block is decoded again serially (k_snappy_rt), which gives the exact
// status.  (golang/snappy encodes every 64-KiB input block on its own, so its copies never reach
// before their block, and a chunk starts at a block's first element or later.)
__device__ __forceinline__ bool snappy_decode_chunk(uint64_t cp, uint32_t s0, uint32_t s_end, uint64_t dst, uint32_t d0,
                                                    uint32_t d_end, uint64_t end, uint64_t oend) {
    const uint64_t oe = dst + d_end;
    uint32_t s = s0, d = d0;
    auto tag8 = [&](uint64_t p) -> uint64_t { return ld64_bounded(p, end); };
    uint64_t t8 = s < s_end ? tag8(cp + s) : 0;
    while (s < s_end) {
        const uint32_t tag = (uint32_t)t8 & 0xffu;
        uint32_t n, R;
        uint64_t A, hi;
        bool lit;
        if ((tag & 3) == 0) {
            uint32_t x = tag >> 2;
            uint64_t l64;
            if (x < 60) {
                s += 1;
                l64 = (uint64_t)x + 1;
            } else {
                const uint32_t nb = x - 59;
                if ((uint64_t)s + 1 + nb > s_end) return false;
                s += 1 + nb;
                x = (uint32_t)(t8 >> 8) & (nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u));
                l64 = (uint64_t)x + 1;
            }
            if (l64 > (uint64_t)(d_end - d) || l64 > (uint64_t)(s_end - s)) return false;
            n = (uint32_t)l64;
            A = cp + s;
            R = n;
            hi = end;
            lit = true;
            s += n;
        } else {
            uint32_t offset;
            if ((tag & 3) == 1) {
                if ((uint64_t)s + 2 > s_end) return false;
                s += 2;
                n = 4 + ((tag >> 2) & 7);
                offset = ((tag & 0xe0) << 3) | ((uint32_t)(t8 >> 8) & 0xffu);
            } else if ((tag & 3) == 2) {
                if ((uint64_t)s + 3 > s_end) return false;
                s += 3;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8) & 0xffffu;
            } else {
                if ((uint64_t)s + 5 > s_end) return false;
                s += 5;
                n = 1 + (tag >> 2);
                offset = (uint32_t)(t8 >> 8);
            }
            if (offset == 0 || d - d0 < offset || n > d_end - d) return false;
            A = dst + d - offset;
            R = offset < n ? offset : n;
            hi = oend;
            lit = false;
        }
        if (s < s_end) t8 = tag8(cp + s);
        const uint64_t o = dst + d;
        for (uint32_t k = 0; k < n;) {
            const uint32_t seg = lit ? (n - k < 64u ? n - k : 64u) : n;
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
    return s == s_end && d == d_end;
}

}  // namespace

// list_cnt/list_ent: null (every block) or the count and block indices k_snappy_lds left
__global__ __launch_bounds__(256) void k_snappy_rt(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                   uint64_t out_cap, const uint64_t *__restrict__ val_off,
                                                   const uint32_t *__restrict__ list_cnt,
                                                   const uint32_t *__restrict__ list_ent) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    const uint32_t cnt = list_cnt ? *list_cnt : n;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
        const uint32_t i = list_ent ? list_ent[j] : j;
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

// ---------------------------------------------------------------------------
// k_snappy_lds: lane per block, the block staged in LDS, a branch-free element
// step, and the next group's streams prefetched into registers while this
// group decodes.
//
// A workgroup is one wave and owns BPW LDS slots of SLOT bytes.  The block
// decodes IN PLACE: its output grows from the slot start, its stream is staged
// at the slot end (P = (SLOT - 8 - round16(clen)) & ~15), and the walk checks
// before every element that its writes (which overshoot by up to 15 B) stay
// below the next unread tag; a block that would break that (or does not fit)
// is listed for the lane-per-block k_snappy_rt pass from global memory.  At C3
// (1 KiB values, streams <= 721 B) a 1,088-B slot never falls back, so 144
// blocks are resident per CU (8 waves x 18) instead of 80 with separate
// stream and output areas (measured: 1,152-B slots x 17 blocks 1.080 ms per C3
// step, 1,088 x 18 1.044, 1,088 x 17 1.077, 1,072 x 19 1.178).  Per group of BPW consecutive blocks:
//   1. the group's streams (prefetched into VGPRs, one 16-B chunk per lane per
//      block) are written into the slots;
//   2. the NEXT group's streams are requested (loads in flight during 3-5),
//      and the descriptors of the group after it;
//   3. lane b walks block b entirely in LDS;
//   4. the wave stores each decoded block with contiguous 16-B stores;
//   5. the descriptors are finalised.
// The element step moves every element as "ops" of 16 B (84 % of C3 elements
// are <= 16 B), one 16-B read and one 16-B write, no masking:
//   literal, or copy of offset o >= 16:  op j reads src + 16 j, writes d + 16 j
//     (a copy's source of op j lies below d + 16 j: written by ops < j)
//   copy of offset o < 16:  op t reads the 16 B at d - o (its first o bytes
//     valid), writes them at d + t o
// A write past the element's end lands in bytes later elements (or the pad)
// own and is overwritten by them in program order; for a short-offset copy
// the last write to every byte comes from the op whose period holds it (LDS
// is in order per wave, so a read sees every earlier write of its lane).  So
// every byte of [0, dlen) ends up right, and a typical element is one op with
// the next tag's read in flight alongside it.  (64-B ops measured 18 % slower:
// 4x the LDS bytes, and unaligned LDS accesses stall -- PMC: 55 % of LDS-active
// cycles; dword-aligned stores with a read-back head merge measured 21 % slower.)
// Checks are the reference decoder's, as in snappy_decode_rt.
// ---------------------------------------------------------------------------
constexpr uint32_t kSlBpw = 18;     // blocks (lanes) per wave
constexpr uint32_t kSlSlot = 1088;  // in-place slot bytes per block

// Every LDS access of k_snappy_lds goes through these may_alias types: the slot
// is written as 16-B chunks and read as bytes, 8-B tags and 16-B chunks, and
// type-based alias analysis must not reorder those accesses.
typedef uint64_t u64_lds_u __attribute__((aligned(1), may_alias));
typedef u32x4 u32x4_lds_u __attribute__((aligned(1), may_alias));


namespace {

// Lanes of the wave hand LDS bytes to each other (staging -> walk -> store-out
// -> next staging): LDS runs a wave's accesses in program order, but the
// compiler sees one thread and could move a read above another lane's write,
// so each hand-over is a wavefront-scope fence.
__device__ __forceinline__ void sl_wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// mode of a block in k_snappy_lds
enum : uint32_t { SL_SKIP = 0, SL_LDS = 1, SL_GLOBAL = 2, SL_TOOLARGE = 3 };

struct SlInfo {
    uint64_t cp, o0;  // stream (absolute, varint header included), output offset in out_vals
    uint32_t clen, dlen, status, mode, i;
};

// in-place slot: where a stream of clen bytes is staged (16-B aligned, 8 B of
// tag over-read room after it)
template <int SLOT>
__device__ __forceinline__ uint32_t sl_pos(uint32_t clen) {
    return ((uint32_t)SLOT - 8u - ((clen + 15u) & ~15u)) & ~15u;
}

// A block's descriptor fields, loaded a group before they are used: sl_load issues the loads
// (unconditional, index clamped to n - 1) and nothing reads the values until sl_finish, a
// whole group later -- computing the mode right after the loads made the compiler wait for
// them on the spot (a memory round trip per group).
struct SlRaw {
    uint64_t hoff, o0, o1;
    uint32_t hlen, st, cpos, dlen, i;
};
__device__ __forceinline__ SlRaw sl_load(uint32_t i, uint32_t n, const bhg_desc *out, const bhg_handle *handles,
                                         const uint64_t *val_off) {
    const uint32_t ii = i < n ? i : n - 1;
    const uint32_t *dw = reinterpret_cast<const uint32_t *>(out + ii);
    SlRaw r;
    r.st = dw[9];
    r.cpos = dw[2];  // provisional (header pass): value position in the record
    r.dlen = dw[3];  // ... decoded length
    const bhg_handle h = handles[ii];
    r.hoff = h.offset;
    r.hlen = h.length;
    r.o0 = val_off[ii];
    r.o1 = val_off[ii + 1];
    r.i = i;
    return r;
}
template <int SLOT>
__device__ __forceinline__ SlInfo sl_finish(const SlRaw &w, uint32_t n, uint64_t base, uint64_t out_cap) {
    SlInfo r;
    r.cp = base + w.hoff + w.cpos;
    r.o0 = w.o0;
    r.clen = w.hlen - w.cpos;
    r.dlen = w.dlen;
    r.status = w.st;
    r.i = w.i;
    if (w.i >= n || (w.st != BHG_ST_OK && w.st != BHG_ST_CRC_MISMATCH))
        r.mode = SL_SKIP;
    else if (w.o1 > out_cap || w.o1 - w.o0 < w.dlen)
        r.mode = SL_TOOLARGE;
    else
        r.mode = (w.dlen <= (uint32_t)SLOT - 64u && r.clen + 24u <= (uint32_t)SLOT) ? SL_LDS : SL_GLOBAL;
    return r;
}

// block staged in LDS: tag stream [sp, se), output at op (LDS byte addresses,
// op < sp: in place).  Returns 0 (ok), 1 (snappy.ErrCorrupt) or 2 (an element
// would write into the unread stream: decode the block from global memory).
// The element decode is straight-line (selects, non-short-circuit checks) so
// the 64 lanes of a wave do not split into per-tag-type paths; the tag read is
// unconditional (a read at se lies inside the slot).
// G lanes per block (lane g of its group): all G decode the same elements; a literal or a copy that
// does not overlap its own output (offset >= length) moves its 16-B ops G at a time, one per lane
// (they read only bytes below the element's output, or the stream); an overlapping copy runs its
// ops one after another on every lane of the group (the same addresses and bytes).  The lanes of a
// group hand bytes to each other through LDS in the wave's program order: a round of the parallel
// loop is one read instruction, then one write instruction, for all G lanes -- a literal in an
// in-place slot reads its stream just above the output it writes, so its round k + 1 reads bytes
// at or above where round k wrote only because every read of a round precedes the round's writes
// (tests/test_snappy_walk_host.py runs the walk on the host in exactly this order).
template <int G>
__device__ __forceinline__ uint32_t snappy_walk_lds(uint8_t *lds, uint32_t sp, uint32_t se, uint32_t op,
                                                    uint32_t dlen, uint32_t g) {
    uint32_t s = sp, d = 0, res = 0;
    // the tag and the 4 bytes after it (one unaligned ds_read_b64; two aligned dword reads
    // measured no faster)
    auto tag_at = [&](uint32_t p) -> uint64_t { return *reinterpret_cast<const u64_lds_u *>(lds + p); };
    uint64_t t8 = tag_at(s);
    // lgkmcnt(0) here: the first tag is then complete on entry as on the back edge (where the
    // next tag's read completes before the op's write), and the loop head needs no wait -- it
    // used to wait there for the previous element's last write
    __builtin_amdgcn_s_waitcnt(0xC07F);
    while (s < se) {
        const uint32_t tag = (uint32_t)t8 & 0xffu, ty = tag & 3u, x = tag >> 2;
        const uint32_t b14 = (uint32_t)(t8 >> 8);  // the 4 bytes after the tag
        // per-type constants from shifts of packed nibble/byte tables (straight-line; the
        // ?: form compiled to per-type exec-mask branches):
        //   adv: literal 1, copy-1 2, copy-2 3, copy-4 5;  offset mask: ~0 >> {-, 24, 16, 0}
        const uint32_t mlit = 0u - (uint32_t)(ty == 0u), m1 = 0u - (uint32_t)(ty == 1u);
        uint32_t n = (m1 & (4u + (x & 7u))) | (~m1 & (x + 1u));
        uint32_t adv = (0x5321u >> (4u * ty)) & 0xfu;
        const uint32_t off = (b14 & (0xffffffffu >> ((0x00101800u >> (8u * ty)) & 0xffu))) | (m1 & ((tag >> 5) << 8));
        if (ty == 0u && x >= 60u) {  // long literal: 1-4 length bytes (rare; divergent)
            const uint32_t nb = x - 59u;
            const uint32_t lmask = nb >= 4u ? 0xffffffffu : ((1u << (8u * nb)) - 1u);
            n = (b14 & lmask) + 1u;
            adv = 1u + nb;
        }
        // checks of decode_other.go, three compares: n - 1 >= dlen - d is n == 0 (a 4-byte literal
        // length of 2^32 - 1) or an element past dlen; sn > se is a tag (or a literal's bytes)
        // past the stream -- sn cannot wrap once n <= dlen - d <= 1 KiB; off - 1 >= d is a copy
        // offset of 0 or past the bytes written
        const uint32_t sn = s + adv + (mlit & n);
        const bool bad = ((uint32_t)(n - 1u >= dlen - d) | (uint32_t)(sn > se) | (~mlit & (uint32_t)(off - 1u >= d))) != 0u;
        const bool spill = op + d + n + 16u > sn;  // 16-B ops write below op + d + n + 16; the next tag is at sn
        if (bad | spill) {
            res = bad ? 1u : 2u;
            break;
        }
        const uint64_t t8n = tag_at(sn);  // next tag, in flight
        const uint32_t a = (mlit & (s + adv)) | (~mlit & (op + d - off));
        const uint32_t o = op + d;
        // 16-B ops (84 % of C3 elements are <= 16 B): a literal or a copy of offset >= 16 moves
        // 16 B at a time (a copy's op j reads bytes below o + 16 j, written by ops < j); a copy of
        // offset < 16 writes the 16 B at a (its first `off` bytes valid) at o, o + off, ...
        const uint32_t big = mlit | (0u - (uint32_t)(off >= 16u));
        const uint32_t sstep = big & 16u;
        const uint32_t dstep = (big & 16u) | (~big & off);
        // n >= 1 here (n == 0 is `bad`): a do-while, so the compiler sees that the next tag's read
        // (issued before the first op's read, which the op waits for) is complete at the loop head
        // and does not wait there for the last op's write as well
        if (G > 1 && (mlit | (0u - (uint32_t)(off >= n))) != 0u) {
            for (uint32_t t = 16 * g; t < n; t += 16 * G)
                *reinterpret_cast<u32x4_lds_u *>(lds + o + t) = *reinterpret_cast<const u32x4_lds_u *>(lds + a + t);
        } else {
            uint32_t t = 0, r = 0;
            do {
                *reinterpret_cast<u32x4_lds_u *>(lds + o + t) = *reinterpret_cast<const u32x4_lds_u *>(lds + a + r);
                t += dstep;
                r += sstep;
            } while (t < n);
        }
        d += n;
        s = sn;
        t8 = t8n;
    }
    return res ? res : (d == dlen ? 0u : 1u);
}

}  // namespace

// The LDS walk runs in "roles": a slot shape (BPW blocks per wave in SLOT-byte in-place slots, CH
// 16-B stream chunks per lane per block prefetched into VGPRs, the rest of a longer stream loaded
// at the dump) over one list of blocks.  The header pass (k_decode_stream<1>) sorted the blocks to
// decode into 64 sub-lists per class (in_cnt: the sub-lists' sizes, in_ent: sub-list 0, sub_cap
// entries apart): <= 1 KiB decoded with the stream fitting 1,088 B (tier 1), and 4 buckets of
// decoded size above it (tier 2).  k_snappy_lds_nat walks the batch in its own order when >= 7/8
// of it is small (C3); k_snappy_lds_multi runs every list in one launch, largest slots first: the
// buckets in 4,160 / 3,392 / 2,624 / 1,856-B slots (4 / 5 / 7 / 10 blocks per wave), then tier 1's
// list (18 per wave) unless the batch went in its own order.  What neither holds (over 4 KiB, an
// in-place spill) goes to k_snappy_rt (out_cnt / out_ent).
// Measured on the C4-shaped decode (bench.py --config mixdec: 1M values U[64, 4096], 76 % of
// them > 1 KiB; profiles/r5/snappy_*): the > 1 KiB blocks took 5.83 ms per step in k_snappy_rt
// (6.90-ms step, 137.6 GiB/s); one 4,160-B tier 5.27 ms per step; tier 1 from the header pass's
// list instead of walking all blocks 4.89; tier 2 in size buckets 4.28; slots sized per bucket
// 3.98; all lists in one launch 3.75-3.77 (252 GiB/s).  Dropped: 4 x 4 / 3 x 4 / 2 x 4 blocks x
// chunks in the 4-KiB tier (5.44-5.77 vs 5.27), 64-B ops (4 reads in flight per element: 6.3 ms,
// C3 +12 %), a 2-KiB class before the buckets (5.30-5.47), one WAVE per block (wave-uniform SALU
// decode, byte-per-lane copies: 7.3 ms for the tier alone, ~75 SALU instructions per element for
// one block where a lane walk spends ~80 VALU per element step for 6), 8 / 12 buckets.
// ORDER: 0 the list; 1 the list unless the batch is mostly this class, 2 the batch's own order
// only when it is (tier 1 in two kernels, each role returning at once when not its case, so
// neither carries the other's code)
// the work of one slot shape over its list (a "role"): lds holds BPW * SLOT + 64 bytes (+ 64:
// literal reads past the last slot); the workgroup takes groups blockIdx.x, + gridDim.x, ...
template <int BPW, int SLOT, int CH, int ORDER, int NSUB, int GL = 1>
__device__ __forceinline__ void sl_role(uint8_t *__restrict__ lds, const uint8_t *__restrict__ src, uint64_t src_len,
                                        const bhg_handle *__restrict__ handles, uint32_t n,
                                        bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals, uint64_t out_cap,
                                        const uint64_t *__restrict__ val_off, const uint32_t *__restrict__ in_cnt,
                                        const uint32_t *__restrict__ in_ent, uint32_t sub_cap,
                                        uint32_t *__restrict__ out_cnt, uint32_t *__restrict__ out_ent) {
    static_assert(SLOT % 16 == 0, "16-B aligned slots");
    constexpr uint32_t DMAX = SLOT - 64;            // longest decoded block a slot takes
    constexpr uint32_t DCH = (DMAX + 1023) / 1024;  // 1-KiB rows of the store-out
    const uint32_t lane = threadIdx.x;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    // the sub-lists as one list: lane k holds the inclusive / exclusive prefix of their sizes at k
    // NSUB sub-lists as one list: lane k of register r holds the inclusive / exclusive prefix of
    // their sizes at sub-list 64 r + k
    static_assert(NSUB % 64 == 0 && NSUB <= 1024, "sub-lists");
    constexpr int NR = NSUB / 64;
    uint32_t incl[NR], excl[NR];
    uint32_t lcnt = 0;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const uint32_t sz = in_cnt[64 * r + lane];
        incl[r] = wave_incl_add(sz) + lcnt;
        excl[r] = incl[r] - sz;
        lcnt = (uint32_t)__builtin_amdgcn_readlane((int)incl[r], 63);
    }
    // tier 1: when at least 7/8 of the batch is in this class, walk the batch in its own order
    // instead (the blocks of the other class skipped): the list's lookups and its order cost the
    // all-1-KiB C3 step 4 % (0.958 -> 0.998 ms); mixed sizes gain from the list
    const bool mostly = (uint64_t)lcnt * 8 >= (uint64_t)n * 7;
    if ((ORDER == 1 && mostly) || (ORDER == 2 && !mostly)) return;
    constexpr bool natural = ORDER == 2;
    const uint32_t cnt = natural ? n : lcnt;
    const uint32_t ngroups = (cnt + BPW - 1) / BPW;
    const uint32_t G = gridDim.x;
    uint32_t g = blockIdx.x;
    if (g >= ngroups) return;
    // sub-list t's prefix (t wave-uniform)
    auto rl = [](const uint32_t *v, uint32_t t) {
        uint32_t x = 0;
#pragma unroll
        for (int r = 0; r < NR; r++)
            if ((t >> 6) == (uint32_t)r) x = (uint32_t)__builtin_amdgcn_readlane((int)v[r], (int)(t & 63u));
        return x;
    };
    // block index of this lane in group grp (n: none): list position j = grp * BPW + lane, found in
    // its sub-list by a wave-uniform search for the group's first position and a walk over the
    // (usually no) sub-list ends the group spans; one load, issued a group before the descriptor
    // loads that need it
    auto index = [&](uint32_t grp) -> uint32_t {
        const uint32_t j0 = grp * BPW, j = j0 + lane;
        if (grp >= ngroups) return n;
        const bool ok = lane < BPW && j < cnt;
        if (natural) return ok ? j : n;
        uint32_t sidx = 0;
        for (uint32_t step = NSUB / 2; step; step >>= 1)
            if (rl(incl, sidx + step - 1) <= j0) sidx += step;
        uint32_t sl = sidx, b0 = rl(excl, sidx);
        const uint32_t jl = j0 + BPW - 1 < cnt - 1 ? j0 + BPW - 1 : cnt - 1;
        for (uint32_t t = sidx; t < NSUB - 1; t++) {
            const uint32_t it = rl(incl, t);
            if (it > jl) break;
            if (j >= it) {
                sl = t + 1;
                b0 = it;
            }
        }
        const uint32_t x = in_ent[(size_t)sl * sub_cap + (ok ? j - b0 : 0u)];
        return ok ? x : n;
    };
    auto load = [&](uint32_t i) -> SlRaw { return sl_load(i < n ? i : n, n, out, handles, val_off); };
    u32x4 v[BPW * CH];
    // CH 16-B chunks per lane per staged block, loaded unconditionally (lanes
    // past the stream load src + 0; the dump drops them) and clamped to end
    // src (a chunk that would cross the end is loaded from end - 16 and
    // shifted into place at the dump), so no branch and no wait is tied to the
    // loads until the next dump.  (The launcher sends src_len < 64 elsewhere.)
    auto prefetch = [&](const SlInfo &I) {
#pragma unroll
        for (int b = 0; b < BPW; b++) {
            const uint32_t clb = __builtin_amdgcn_readlane(I.mode == SL_LDS ? I.clen : 0u, b);
            const uint64_t cpb = readlane_u64(I.cp, b);
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const uint32_t off = 1024u * c + 16u * lane;
                const uint64_t a = off < clb ? cpb + off : base;
                v[b * CH + c] = gld<u32x4u>(a + 16 <= end ? a : end - 16);
            }
        }
    };
    // in natural order, a block this tier cannot hold belongs to the other class's list: skipped
    auto finish = [&](const SlRaw &w) -> SlInfo {
        SlInfo r = sl_finish<SLOT>(w, n, base, out_cap);
        if (natural && r.mode == SL_GLOBAL) r.mode = SL_SKIP;
        return r;
    };
    SlInfo cur = finish(load(index(g)));
    prefetch(cur);
    SlInfo nxt = finish(load(index(g + G)));
    uint32_t ix2 = index(g + 2 * G);
    for (; g < ngroups; g += G) {
        // 1. this group's streams -> slots
#pragma unroll
        for (int b = 0; b < BPW; b++) {
            const uint32_t clb = __builtin_amdgcn_readlane(cur.mode == SL_LDS ? cur.clen : 0u, b);
            const uint64_t cpb = readlane_u64(cur.cp, b);
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const uint32_t off = 1024u * c + 16u * lane;
                const uint64_t a = cpb + off;
                u32x4 x4 = v[b * CH + c];
                if (off < clb && a + 16 > end) {  // the chunk was loaded from end - 16: its bytes start at a - (end - 16)
                    const uint32_t sh = (uint32_t)(a - (end - 16));
                    unsigned __int128 x = (unsigned __int128)x4.x | ((unsigned __int128)x4.y << 32) |
                                          ((unsigned __int128)x4.z << 64) | ((unsigned __int128)x4.w << 96);
                    x >>= 8 * sh;
                    x4 = u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
                }
                if (off < clb) *reinterpret_cast<u32x4_lds_u *>(lds + b * SLOT + sl_pos<SLOT>(clb) + off) = x4;
            }
        }
        // streams past CH KiB (tier 1: 1,025 .. SLOT - 24 B, values snappy could not shrink, ~1
        // in 3,000 dict values): the rest loaded here, synchronously -- rare, and it keeps them
        // out of the global-memory pass
        for (uint64_t lm = __ballot(cur.mode == SL_LDS && cur.clen > 1024u * CH); lm; lm &= lm - 1) {
            const int b = __builtin_ctzll(lm);
            const uint32_t clb = __builtin_amdgcn_readlane(cur.clen, b);
            for (uint32_t off = 1024u * CH + 16 * lane; off < clb; off += 1024u) {
                const u32x4 c = ld16_hi(readlane_u64(cur.cp, b) + off, end);
                *reinterpret_cast<u32x4_lds_u *>(lds + b * SLOT + sl_pos<SLOT>(clb) + off) = c;
            }
        }
        sl_wsync();
        // 2. descriptors of the group after next (and the list entries of the one after
        // that), then the next group's streams in flight
        const SlRaw nn = load(ix2);
        ix2 = index(g + 3 * G);
        prefetch(nxt);
        // 3. decode
        uint32_t fin = cur.status, mode = cur.mode;
        if (GL == 1) {
            if (mode == SL_LDS) {
                const uint32_t sb = lane * SLOT, sp = sb + sl_pos<SLOT>(cur.clen);
                uint32_t hdr = 0;
                while (hdr < 5 && lds[sp + hdr] >= 0x80) hdr++;  // uvarint decodedLen, validated by the header pass
                hdr++;
                const uint32_t r = snappy_walk_lds<1>(lds, sp + hdr, sp + cur.clen, sb, cur.dlen, 0);
                if (r == 1) fin = BHG_ST_SNAPPY_CORRUPT;
                if (r == 2) mode = SL_GLOBAL;
            }
        } else {
            // lane l walks block l / G (its fields from lane l / G), then lane b < BPW takes block b's
            // result from its group's first lane
            static_assert(BPW * GL <= 64, "groups fit the wave");
            const uint32_t bl = lane / GL;
            const uint32_t gm = (uint32_t)__shfl((int)mode, (int)bl, 64), gc = (uint32_t)__shfl((int)cur.clen, (int)bl, 64);
            const uint32_t gd = (uint32_t)__shfl((int)cur.dlen, (int)bl, 64);
            uint32_t r = 0;
            if (bl < (uint32_t)BPW && gm == SL_LDS) {
                const uint32_t sb = bl * SLOT, sp = sb + sl_pos<SLOT>(gc);
                uint32_t hdr = 0;
                while (hdr < 5 && lds[sp + hdr] >= 0x80) hdr++;
                hdr++;
                r = snappy_walk_lds<GL>(lds, sp + hdr, sp + gc, sb, gd, lane % GL);
            }
            r = (uint32_t)__shfl((int)r, (int)(lane * GL < 64 ? lane * GL : 0u), 64);
            if (mode == SL_LDS) {
                if (r == 1) fin = BHG_ST_SNAPPY_CORRUPT;
                if (r == 2) mode = SL_GLOBAL;
            }
        }
        if (mode == SL_TOOLARGE) {
            fin = BHG_ST_SNAPPY_TOO_LARGE;
        }
        // 4. decoded blocks -> out_vals
        sl_wsync();
        {
            const bool good = mode == SL_LDS && (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH);
            const uint32_t dl = good ? cur.dlen : 0u;
#pragma unroll
            for (int b = 0; b < BPW; b++) {
                const uint32_t dlb = __builtin_amdgcn_readlane(dl, b);
                const uint64_t ob = (uint64_t)out_vals + readlane_u64(cur.o0, b);
#pragma unroll
                for (uint32_t c = 0; c < DCH; c++) {
                    const uint32_t off = 1024u * c + 16u * lane;
                    if (off < dlb)
                        st16_clip(ob + off, *reinterpret_cast<const u32x4_lds_u *>(lds + b * SLOT + off), ob + dlb);
                }
            }
        }
        sl_wsync();
        // 5. descriptors (SL_GLOBAL blocks stay provisional, listed for the next tier)
        if (mode == SL_GLOBAL) {
            const uint32_t k = atomicAdd(out_cnt, 1u);
            out_ent[k] = cur.i;
        }
        if (mode == SL_LDS || mode == SL_TOOLARGE) {
            uint32_t *dw = reinterpret_cast<uint32_t *>(out + cur.i);
            dw[2] = 0;
            dw[3] = (fin == BHG_ST_OK || fin == BHG_ST_CRC_MISMATCH) ? cur.dlen : 0u;
            dw[9] = fin;
        }
        cur = nxt;
        nxt = finish(nn);
    }
}

// tier 1 in the batch's own order (when >= 7/8 of the blocks are small; else it returns at once)
template <int G1>
__global__ __launch_bounds__(64) void k_snappy_lds_nat(const uint8_t *__restrict__ src, uint64_t src_len,
                                                       const bhg_handle *__restrict__ handles, uint32_t n,
                                                       bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                       uint64_t out_cap, const uint64_t *__restrict__ val_off,
                                                       const uint32_t *__restrict__ c_small,
                                                       const uint32_t *__restrict__ e_small, uint32_t sub_cap,
                                                       uint32_t *__restrict__ c_rt, uint32_t *__restrict__ e_rt) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSlBpw * kSlSlot + 64];
    sl_role<kSlBpw, kSlSlot, 1, 2, 64, G1>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_small, e_small,
                                       sub_cap, c_rt, e_rt);
}

// every list in one launch, largest slots first: the 4 size buckets of the 4-KiB tier, each in
// slots sized to it, then tier 1's list (unless tier 1 ran in batch order).  One launch, so the
// empty roles of an all-1-KiB batch cost one start-up, and a role's tail overlaps the next one's
// groups.
// The role shapes are sized for 8 one-wave workgroups per CU (2 waves per SIMD): 19.2 KiB of LDS each.
// The round-5 shapes (6 / 7 / 9 / 13 / 23 blocks, 24.5 KiB) left 6 waves per CU, 2-2-1-1 over the
// SIMDs: mixdec 288.8-289.4 -> 305.6-306.7 GiB/s (3 alternating runs, profiles/r6/lab_r6b/ item 9).
constexpr uint32_t kMultiLds = 18 * 1088 + 64;  // the largest role (10 x 1,856 + 64 = 18,624 B is next)
template <int G1, int G2>
__global__ __launch_bounds__(64) void k_snappy_lds_multi(const uint8_t *__restrict__ src, uint64_t src_len,
                                                         const bhg_handle *__restrict__ handles, uint32_t n,
                                                         bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                         uint64_t out_cap, const uint64_t *__restrict__ val_off,
                                                         uint32_t *__restrict__ list, uint32_t sub_cap) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMultiLds];
    static_assert(kSnapBuckets == 4 && kSnapBucketBytes == 768, "the bucket slot sizes below");
    static_assert(4 * 4160 + 64 <= kMultiLds && 5 * 3392 + 64 <= kMultiLds && 7 * 2624 + 64 <= kMultiLds && 10 * 1856 + 64 <= kMultiLds &&
                      18 * 1088 + 64 <= kMultiLds, "roles fit the LDS");
    const uint32_t *c_small = list, *c_large = list + 64;
    uint32_t *c_rt = list + kSnapRtCount;
    const uint32_t *e_small = list + kSnapListHdr, *e_large = e_small + (size_t)64 * sub_cap;
    uint32_t *e_rt = list + kSnapListHdr + (size_t)kSnapSubs * sub_cap;
    const size_t bs = (size_t)64 * sub_cap;
    sl_role<4, 4160, 2, 0, 64, G2>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_large, e_large, sub_cap,
                               c_rt, e_rt);
    sl_role<5, 3392, 2, 0, 64, G2>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_large + 64,
                               e_large + bs, sub_cap, c_rt, e_rt);
    sl_role<7, 2624, 2, 0, 64, G2>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_large + 128,
                               e_large + 2 * bs, sub_cap, c_rt, e_rt);
    sl_role<10, 1856, 1, 0, 64, G2>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_large + 192,
                                e_large + 3 * bs, sub_cap, c_rt, e_rt);
    sl_role<18, 1088, 1, 1, 64, G1>(lds, src, src_len, handles, n, out, out_vals, out_cap, val_off, c_small, e_small,
                                sub_cap, c_rt, e_rt);
}

// ---------------------------------------------------------------------------
// Blocks past the LDS tiers (the global-memory list: decoded > 4 KiB, or an in-place spill):
// chunk-parallel.  One lane walking a whole 1-4 MiB value took 170 ms for a batch of 7,000 values
// of 4 KiB - 4 MiB (bench.py --config bigval, profiles/r6/bigval/): the step was the longest value's
// serial walk.  Here
//   k_sb_parse  one WAVE per listed block: a tag-only parse of its stream -- 64 positions at a time,
//               every lane the element length and output length of a tag at its byte, then the
//               element chain followed with v_readlane -- that cuts the block at the first element
//               starting at or past every 64 KiB of output: chunks (stream start, output start).
//               Blocks of <= 64 KiB are one chunk without a parse.  Anything irregular (a length
//               past the stream, output past dlen, not ending exactly at the stream end) sends the
//               block to the serial pass.
//   k_sb_walk   LANE per chunk: snappy_decode_chunk.  The last chunk of a block (a device-scope
//               counter per block) finalises its descriptor, or lists the block for the serial pass
//               when any of its chunks failed (a copy into an earlier chunk, a corrupt element).
//   k_snappy_rt the serial pass over that list (exact golang/snappy statuses).
// ---------------------------------------------------------------------------
constexpr uint32_t kSbChunk = 65536;  // decoded bytes per chunk (at least: a chunk starts at an element)
constexpr uint32_t kSbSeg = 16384;    // stream bytes per segment of a long stream's parse
constexpr uint32_t kSbSegMin = 2 * kSbSeg;  // streams longer than this: the segment parse
constexpr uint32_t kSbBad = 0x10000u; // a window exit: the chain met an irregular element
struct SbEnt {
    uint32_t i, s0, d0, last;  // block, stream start (after the uvarint header), output start; ~0 = unused slot
};
struct SbBig {
    uint32_t i, seg0, nseg, b0;  // block, its first segment, segments, first chunk slot
};
// layout of the big path's scratch: [0] chunk slots reserved, [1] serial list size, [2] segments
// reserved, [3] segment-parsed blocks; from 256 B the chunk entries (cap), the per-block words
// {chunks left, failed} (n), the serial list (n), the segment-parsed blocks (n), then per segment
// (segcap) its block's index in that list, its entry (stream position, output), and the 64 chain
// results of the speculative parse
static size_t al256_(size_t x) { return (x + 255) & ~(size_t)255; }
static uint64_t sb_cap(uint32_t n, uint64_t out_cap) { return out_cap / kSbChunk + n + 1; }
static uint64_t sb_segcap(uint32_t n, uint64_t out_cap) { return out_cap / kSbSeg + n + 1; }
constexpr uint32_t kSbMark = 1024;              // checkpoint spacing along a chain of a segment
constexpr uint32_t kSbMarks = kSbSeg / kSbMark; // checkpoints per chain (index 0 unused)
constexpr uint32_t kSbCk = 4;                    // chains with checkpoints: lanes 0, 16, 32, 48
size_t snappy_big_bytes(uint32_t n, uint64_t out_cap) {
    const uint64_t sc = sb_segcap(n, out_cap);
    return 256 + al256_(sb_cap(n, out_cap) * sizeof(SbEnt)) + al256_((size_t)n * 8) + al256_((size_t)n * 4) +
           al256_((size_t)n * sizeof(SbBig)) + al256_(sc * 4) + al256_(sc * 8) + al256_(sc * 64 * 8) +
           al256_(sc * kSbCk * kSbMarks * 8);
}
struct SbScratch {
    uint32_t *ctr;
    SbEnt *ent;
    uint32_t *blk, *ser;
    SbBig *bigs;
    uint32_t *segblk;
    uint2 *segent, *res, *ck;
    uint64_t cap, segcap;
};
static SbScratch sb_layout(void *p, uint32_t n, uint64_t out_cap) {
    SbScratch S;
    uint8_t *b = static_cast<uint8_t *>(p);
    S.ctr = reinterpret_cast<uint32_t *>(b);
    S.cap = sb_cap(n, out_cap);
    S.segcap = sb_segcap(n, out_cap);
    b += 256;
    S.ent = reinterpret_cast<SbEnt *>(b);
    b += al256_(S.cap * sizeof(SbEnt));
    S.blk = reinterpret_cast<uint32_t *>(b);
    b += al256_((size_t)n * 8);
    S.ser = reinterpret_cast<uint32_t *>(b);
    b += al256_((size_t)n * 4);
    S.bigs = reinterpret_cast<SbBig *>(b);
    b += al256_((size_t)n * sizeof(SbBig));
    S.segblk = reinterpret_cast<uint32_t *>(b);
    b += al256_(S.segcap * 4);
    S.segent = reinterpret_cast<uint2 *>(b);
    b += al256_(S.segcap * 8);
    S.res = reinterpret_cast<uint2 *>(b);
    b += al256_(S.segcap * 64 * 8);
    S.ck = reinterpret_cast<uint2 *>(b);
    return S;
}

constexpr uint32_t kSbBuf = 4096;  // staged stream bytes per wave (+ 128 of look-ahead)
constexpr uint32_t kSbLanes = 8;   // chunks per wave in k_sb_walk

// a listed block's stream: S (absolute, after the uvarint header), slen, dlen
struct SbStream {
    uint64_t S;
    uint32_t slen, dlen;
};
__device__ __forceinline__ SbStream sb_stream(uint64_t base, const bhg_handle *handles, const bhg_desc *out, uint32_t i) {
    const uint32_t *dw = reinterpret_cast<const uint32_t *>(out + i);
    const bhg_handle hh = handles[i];
    const uint64_t cp = base + hh.offset + dw[2];
    uint32_t hdr = 0;
    while (hdr < 10 && gld<uint8_t>(cp + hdr) >= 0x80) hdr++;  // uvarint decodedLen (validated by the header pass)
    hdr++;
    return SbStream{cp + hdr, hh.length - dw[2] - hdr, dw[3]};
}

// [bb, bb + kSbBuf + 128) of the stream into buf (bytes past the stream: 0)
__device__ __forceinline__ void sb_stage(uint8_t *buf, const SbStream &T, uint32_t bb, uint32_t lane) {
    sl_wsync();
    for (uint32_t t = 16 * lane; t < kSbBuf + 128; t += 1024) {
        u32x4 v = {0, 0, 0, 0};
        if ((uint64_t)bb + t + 16 <= T.slen) v = gld<u32x4u>(T.S + bb + t);
        else if (bb + t < T.slen) v = ld16_hi(T.S + bb + t, T.S + T.slen);
        *reinterpret_cast<u32x4_lds_u *>(buf + t) = v;
    }
    sl_wsync();
}

// One window of the tag-only parse: the positions e .. e + lim - 1 (lim <= 64; buf holds the
// stream from bb).  Lane q: the element a tag at e + q would be (elen: its stream length, 0 when
// its length bytes or data pass the stream, or a literal is longer than dlen or 2^26 -- never
// golang/snappy's, whose blocks are 64 KiB -- so that a window's output sum cannot wrap; olen: its
// output length), then by pointer doubling (ds_bpermute) nx = the position (relative to e) after
// the elements from e + q up to the first one at or past lim, kSbBad or more when one of them is
// irregular, and sm = their output.  6 levels cover the <= 32 elements of 64 bytes.
struct SbWin {
    uint32_t elen, olen, nx, sm;
};
__device__ __forceinline__ SbWin sb_window(const uint8_t *buf, uint32_t bb, uint32_t e, uint32_t lim, uint32_t slen,
                                           uint32_t dlen, uint32_t lane) {
    const uint32_t p = e + lane, x = p - bb;
    uint32_t elen = 0, olen = 0;
    if (p < slen) {
        const uint32_t tag = buf[x], ty = tag & 3u, v = tag >> 2;
        if (ty == 0) {
            uint32_t ln = v + 1, nb = 0;
            if (v >= 60) {
                nb = v - 59;
                uint32_t lv = 0;
                for (uint32_t q = 0; q < 4; q++) lv |= q < nb ? (uint32_t)buf[x + 1 + q] << (8 * q) : 0u;
                ln = lv + 1;  // 0 for a 4-byte 2^32 - 1: irregular
            }
            const uint64_t el = 1ull + nb + ln;
            if (p + 1 + nb <= slen && ln != 0 && ln <= dlen && ln <= (1u << 26) && p + el <= slen) {
                elen = (uint32_t)el;
                olen = ln;
            }
        } else {
            const uint32_t el = ty == 1 ? 2u : ty == 2 ? 3u : 5u;
            if (p + el <= slen) { elen = el; olen = ty == 1 ? 4 + (v & 7) : 1 + v; }
        }
    }
    uint32_t nx = elen ? lane + elen : kSbBad, sm = olen;
#pragma unroll
    for (int lv = 0; lv < 6; lv++) {
        const bool in = nx < lim;
        const int a = (int)((in ? nx : 0u) * 4u);
        const uint32_t nn = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)nx);
        const uint32_t ns = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)sm);
        if (in) { nx = nn; sm += ns; }
    }
    return SbWin{elen, olen, nx, sm};
}

// Blocks past the LDS tiers, one WAVE per listed block.  A block of <= 64 KiB decoded is one chunk
// without a parse.  A stream of <= kSbSegMin bytes is parsed here, window by window (the chain from
// the block start; at a window that holds a 64-KiB output boundary its elements one by one, with
// v_readlane), cutting the block at the first element at or past every 64 KiB of output.  Longer
// streams are handed to the segment parse (k_sb_seg -> k_sb_stitch -> k_sb_emit): the round-6
// bigval batch's 4-MiB values took 14.7 ms here, one window after another.  Anything irregular (a
// length past the stream, output past dlen, not ending exactly at the stream end) sends the block
// to the serial pass.
__global__ __launch_bounds__(256) void k_sb_parse(const uint8_t *__restrict__ src, uint64_t src_len,
                                                  const bhg_handle *__restrict__ handles, uint32_t n,
                                                  bhg_desc *__restrict__ out, uint64_t out_cap,
                                                  const uint64_t *__restrict__ val_off,
                                                  const uint32_t *__restrict__ rt_cnt, const uint32_t *__restrict__ rt_ent,
                                                  uint32_t *__restrict__ ctr, SbEnt *__restrict__ ent, uint64_t cap,
                                                  uint32_t *__restrict__ blk, uint32_t *__restrict__ ser,
                                                  SbBig *__restrict__ bigs, uint32_t *__restrict__ segblk, uint64_t segcap) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[4][kSbBuf + 128];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *buf = bufs[w];
    const uint64_t base = (uint64_t)src;
    const uint32_t cnt = *rt_cnt;
    for (uint32_t j = blockIdx.x * 4 + w; j < cnt; j += gridDim.x * 4) {
        const uint32_t i = rt_ent[j];
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t status = dw[9];
        if (status != BHG_ST_OK && status != BHG_ST_CRC_MISMATCH) continue;
        const uint32_t dlen = dw[3];
        const uint64_t o0 = val_off[i], o1 = val_off[i + 1];
        if (o1 > out_cap || o1 - o0 < dlen) {  // as k_snappy_rt
            if (lane == 0) { dw[2] = 0; dw[3] = 0; dw[9] = BHG_ST_SNAPPY_TOO_LARGE; }
            continue;
        }
        const SbStream T = sb_stream(base, handles, out, i);
        // chunk slots: at most one per 64 KiB of output, plus the first
        const uint32_t k = dlen / kSbChunk + 1;
        uint32_t b0 = 0;
        if (lane == 0) b0 = atomicAdd(ctr, k);
        b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0);
        if ((uint64_t)b0 + k > cap) {  // (cannot happen: the chunks of all blocks fit out_cap / 64 KiB + n)
            if (lane == 0) ser[atomicAdd(ctr + 1, 1u)] = i;
            for (uint32_t q = lane; (uint64_t)b0 + q < cap && q < k; q += 64) ent[b0 + q] = SbEnt{~0u, 0, 0, 0};
            continue;
        }
        if (dlen > kSbChunk && T.slen > kSbSegMin) {  // the segment parse, when its scratch holds the segments
            const uint32_t nseg = (T.slen + kSbSeg - 1) / kSbSeg;
            uint32_t s0 = 0;
            if (lane == 0) s0 = atomicAdd(ctr + 2, nseg);
            s0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)s0);
            if ((uint64_t)s0 + nseg <= segcap) {
                uint32_t t = 0;
                if (lane == 0) t = atomicAdd(ctr + 3, 1u);  // < n: one entry per listed block at most
                t = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
                if (lane == 0) bigs[t] = SbBig{i, s0, nseg, b0};
                for (uint32_t q = lane; q < nseg; q += 64) segblk[s0 + q] = t;
                continue;
            }
            // (the one reservation that crosses segcap: its segments below it are marked unused)
            for (uint64_t q = (uint64_t)s0 + lane; q < segcap; q += 64) segblk[q] = ~0u;
        }
        uint32_t ci = 1;
        bool bad = false;
        if (dlen > kSbChunk) {
            uint32_t e = 0, d = 0, nextb = kSbChunk, bb = ~0u;
            while (e < T.slen) {
                if (bb == ~0u || e + 64 + 8 > bb + kSbBuf) sb_stage(buf, T, bb = e, lane);
                const uint32_t lim = min(64u, T.slen - e);
                const SbWin W = sb_window(buf, bb, e, lim, T.slen, dlen, lane);
                const uint32_t wx = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.nx);
                const uint32_t ws = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.sm);
                if (wx >= kSbBad || ws > dlen - d) { bad = true; break; }
                if (d + ws < nextb) {  // no chunk boundary in this window (the common case)
                    d += ws;
                    e += wx;
                    continue;
                }
                // a chunk boundary: the window's elements one by one
                uint32_t q = 0;
                while (q < lim) {
                    const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)W.elen, (int)q);
                    const uint32_t ol = (uint32_t)__builtin_amdgcn_readlane((int)W.olen, (int)q);
                    if (el == 0 || ol > dlen - d) { bad = true; break; }
                    if (d >= nextb) {
                        if (lane == 0) ent[b0 + ci] = SbEnt{i, e + q, d, 0};
                        ci++;
                        nextb = (d / kSbChunk + 1) * kSbChunk;
                    }
                    d += ol;
                    q += el;
                }
                if (bad) break;
                e += q;
            }
            if (!bad && (e != T.slen || d != dlen)) bad = true;
        }
        if (bad) {
            for (uint32_t q = lane; q < k; q += 64) ent[b0 + q] = SbEnt{~0u, 0, 0, 0};
            if (lane == 0) ser[atomicAdd(ctr + 1, 1u)] = i;
            continue;
        }
        for (uint32_t q = ci + lane; q < k; q += 64) ent[b0 + q] = SbEnt{~0u, 0, 0, 0};
        if (lane == 0) {
            ent[b0] = SbEnt{i, 0, 0, ci == 1 ? 1u : 0u};
            if (ci > 1) ent[b0 + ci - 1].last = 1;
            blk[2 * i] = ci;
            blk[2 * i + 1] = 0;
        }
    }
}

// The segment parse of a long stream, in three launches.
//   k_sb_seg     one WAVE per segment (kSbSeg stream bytes at X0): 64 chains at once, from X0 + b for
//                every lane b, each to the first element at or past the segment's end -- where it
//                ends and its output (or that it met an irregular element).  Every window (at the
//                lowest chain still in the segment) is one sb_window, each chain in it then one
//                ds_bpermute.  The chains merge within a few elements.
//   k_sb_stitch  one WAVE per block, its segments in order: the block's chain enters segment k at
//                position P; the chain from X0 + (P - X0) is the block's, and ends where the next
//                one starts.  When P >= X0 + 64 (a literal longer than 64 bytes over X0) the wave
//                walks the segment from P itself.  Then the totals are checked as in k_sb_parse.
//   k_sb_emit    one WAVE per segment, the block's chain through it from its entry, writing chunk
//                slot m at the element after the one that reaches m * 64 KiB of output: the first
//                element at or past that output.
// (golang/snappy's stream is a sequence of 64-KiB blocks, so every chunk decodes on its own.)
__global__ __launch_bounds__(256) void k_sb_seg(const uint8_t *__restrict__ src, const bhg_handle *__restrict__ handles,
                                                const bhg_desc *__restrict__ out, const uint32_t *__restrict__ ctr,
                                                const SbBig *__restrict__ bigs, const uint32_t *__restrict__ segblk,
                                                uint64_t segcap, uint2 *__restrict__ res, uint2 *__restrict__ ck) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[4][kSbBuf + 128];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *buf = bufs[w];
    const uint64_t total = ctr[2] < segcap ? ctr[2] : segcap;
    for (uint64_t j = (uint64_t)blockIdx.x * 4 + w; j < total; j += (uint64_t)gridDim.x * 4) {
        const uint32_t sb = segblk[j];
        if (sb == ~0u) continue;  // reserved by a block that did not fit
        const SbBig B = bigs[sb];
        const SbStream T = sb_stream((uint64_t)src, handles, out, B.i);
        const uint32_t k = (uint32_t)(j - B.seg0), x0 = k * kSbSeg, x1 = min(x0 + kSbSeg, T.slen);
        uint32_t P = x0 + lane, O = 0, bb = ~0u, cn = 1;  // cn: the chain's next checkpoint (lanes 16 q)
        bool act = P < x1;
        const bool ckl = (lane & 15) == 0;
        uint2 *const ckj = ck + (j * kSbCk + (lane >> 4)) * kSbMarks;
        for (;;) {
            const uint32_t key = act ? P : ~0u;
            const uint32_t E = ~(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(~key), 63);  // the lowest chain
            if (E == ~0u) break;
            if (bb == ~0u || E + 64 + 8 > bb + kSbBuf) sb_stage(buf, T, bb = E, lane);
            // windows end at the checkpoint marks x0 + c kSbMark too (k_sb_stitch walks the same way)
            const uint32_t lim = min(min(64u, x1 - E), x0 + ((E - x0) / kSbMark + 1) * kSbMark - E);
            const SbWin W = sb_window(buf, bb, E, lim, T.slen, T.dlen, lane);
            const uint32_t q = P - E;
            const bool mv = act && q < lim;
            const int a = (int)((mv ? q : 0u) * 4u);
            const uint32_t nx = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)W.nx);
            const uint32_t sm = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)W.sm);
            if (mv) {
                if (nx >= kSbBad) {
                    P = ~0u;
                    act = false;
                } else {
                    P = E + nx;
                    O += sm;
                    act = P < x1;
                    // chains 0, 16, 32, 48 at every mark they reach: their first element at or past it
                    for (; ckl && cn < kSbMarks && P >= x0 + cn * kSbMark; cn++) ckj[cn] = uint2{P, O};
                }
            }
        }
        for (; ckl && cn < kSbMarks; cn++) ckj[cn] = uint2{~0u, 0};
        res[j * 64 + lane] = uint2{P, O};  // P = ~0: an irregular element on the chain from x0 + lane
    }
}

__global__ __launch_bounds__(256) void k_sb_stitch(const uint8_t *__restrict__ src, const bhg_handle *__restrict__ handles,
                                                   const bhg_desc *__restrict__ out, uint32_t *__restrict__ ctr,
                                                   SbEnt *__restrict__ ent, uint32_t *__restrict__ blk,
                                                   uint32_t *__restrict__ ser, const SbBig *__restrict__ bigs,
                                                   uint64_t segcap, uint2 *__restrict__ segent,
                                                   const uint2 *__restrict__ res, const uint2 *__restrict__ ck) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[4][kSbBuf + 128];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *buf = bufs[w];
    const uint32_t nb = ctr[3];
    for (uint32_t t = blockIdx.x * 4 + w; t < nb; t += gridDim.x * 4) {
        const SbBig B = bigs[t];
        const SbStream T = sb_stream((uint64_t)src, handles, out, B.i);
        uint32_t P = 0, bb = ~0u;
        uint64_t D = 0;
        bool bad = false;
        // the chain results of the next kSbPf segments in flight, lane b holding chain b's (a step
        // is then a v_readlane, not a memory round trip: 0.73 -> ms per bigval step)
        constexpr uint32_t kSbPf = 4;
#ifdef BHG_SB_PROF
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        uint32_t nmiss = 0, nwin = 0, nmerge = 0;
#endif
        uint2 rr[kSbPf];
#pragma unroll
        for (uint32_t q = 0; q < kSbPf; q++)
            rr[q] = res[(uint64_t)(B.seg0 + (q < B.nseg ? q : 0u)) * 64 + lane];
        for (uint32_t k = 0; k < B.nseg && !bad; k++) {
            const uint32_t x0 = k * kSbSeg, x1 = min(x0 + kSbSeg, T.slen);
            const uint2 rk = rr[0];
#pragma unroll
            for (uint32_t q = 0; q + 1 < kSbPf; q++) rr[q] = rr[q + 1];
            rr[kSbPf - 1] = res[(uint64_t)(B.seg0 + (k + kSbPf < B.nseg ? k + kSbPf : 0u)) * 64 + lane];
            if (lane == 0) segent[B.seg0 + k] = uint2{P, (uint32_t)D};
            if (P - x0 < 64u) {  // (P >= x0: the previous segment's chain ended at or past x0)
                const uint32_t b = P - x0;
                const uint2 r = {(uint32_t)__builtin_amdgcn_readlane((int)rk.x, (int)b),
                                 (uint32_t)__builtin_amdgcn_readlane((int)rk.y, (int)b)};
                if (r.x == ~0u) bad = true;
                P = r.x;
                D += r.y;
            } else {
                // the chain from P, in windows that end at the marks as k_sb_seg's do, until it meets
                // one of the segment's checkpointed chains at a mark (then that chain's exit is the
                // block's) or ends.  (Four chains: a chain from inside a long literal's bytes parses
                // them as tags and can die on a garbage length before it meets the block's.)
                const uint64_t sj = (uint64_t)(B.seg0 + k);
#ifdef BHG_SB_PROF
                nmiss++;
#endif
                while (P < x1) {
#ifdef BHG_SB_PROF
                    nwin++;
#endif
                    if (bb == ~0u || P + 64 + 8 > bb + kSbBuf) sb_stage(buf, T, bb = P, lane);
                    const uint32_t nm = x0 + ((P - x0) / kSbMark + 1) * kSbMark;
                    const uint32_t lim = min(min(64u, x1 - P), nm - P);
                    const SbWin W = sb_window(buf, bb, P, lim, T.slen, T.dlen, lane);
                    const uint32_t wx = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.nx);
                    if (wx >= kSbBad) { bad = true; break; }
                    D += (uint32_t)__builtin_amdgcn_readfirstlane((int)W.sm);
                    P += wx;
                    if (P >= nm && P < x1) {
                        // lane q: checkpoint set q's entry at this mark
                        const uint2 c = ck[((uint64_t)sj * kSbCk + (lane < kSbCk ? lane : 0u)) * kSbMarks + (P - x0) / kSbMark];
                        const uint64_t hit = __ballot(lane < kSbCk && c.x == P);
                        if (hit) {  // the same element: from here on the chains are one
#ifdef BHG_SB_PROF
                            nmerge++;
#endif
                            const uint32_t q = (uint32_t)__builtin_ctzll(hit);
                            const uint32_t cy = (uint32_t)__builtin_amdgcn_readlane((int)c.y, (int)q);
                            const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)rk.x, (int)(16 * q));
                            const uint32_t ey = (uint32_t)__builtin_amdgcn_readlane((int)rk.y, (int)(16 * q));
                            if (ex == ~0u) { bad = true; break; }
                            D += ey - cy;
                            P = ex;
                            break;
                        }
                    }
                }
            }
        }
        bad = bad || P != T.slen || D != T.dlen;
#ifdef BHG_SB_PROF
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0 && t1 - t0 > 20000)
            printf("stitch blk %u nseg %u miss %u win %u merge %u bad %d cycles %llu\n", B.i, B.nseg, nmiss, nwin, nmerge,
                   (int)bad, (unsigned long long)(t1 - t0));
#endif
        const uint32_t m_last = (T.dlen - 1) / kSbChunk, k_res = T.dlen / kSbChunk + 1;
        // every slot unused until k_sb_emit writes it (and for good, on a failed block)
        for (uint32_t q = lane; q < k_res; q += 64) ent[B.b0 + q] = SbEnt{~0u, 0, 0, 0};
        if (lane == 0) {
            if (bad) {
                blk[2 * B.i] = 0;
                blk[2 * B.i + 1] = 1;  // k_sb_emit skips the block
                ser[atomicAdd(ctr + 1, 1u)] = B.i;
            } else {
                blk[2 * B.i] = m_last + 1;
                blk[2 * B.i + 1] = 0;
            }
        }
        sl_wsync();
        if (!bad && lane == 0) ent[B.b0] = SbEnt{B.i, 0, 0, m_last == 0 ? 1u : 0u};
    }
}

__global__ __launch_bounds__(256) void k_sb_emit(const uint8_t *__restrict__ src, const bhg_handle *__restrict__ handles,
                                                 const bhg_desc *__restrict__ out, const uint32_t *__restrict__ ctr,
                                                 SbEnt *__restrict__ ent, const uint32_t *__restrict__ blk,
                                                 const SbBig *__restrict__ bigs, const uint32_t *__restrict__ segblk,
                                                 uint64_t segcap, const uint2 *__restrict__ segent) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[4][kSbBuf + 128];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *buf = bufs[w];
    const uint64_t total = ctr[2] < segcap ? ctr[2] : segcap;
    for (uint64_t j = (uint64_t)blockIdx.x * 4 + w; j < total; j += (uint64_t)gridDim.x * 4) {
        const uint32_t sb = segblk[j];
        if (sb == ~0u) continue;
        const SbBig B = bigs[sb];
        if (blk[2 * B.i + 1]) continue;  // the stitch failed: the block is on the serial list
        const SbStream T = sb_stream((uint64_t)src, handles, out, B.i);
        const uint32_t k = (uint32_t)(j - B.seg0), x1 = min(k * kSbSeg + kSbSeg, T.slen);
        const uint32_t m_last = (T.dlen - 1) / kSbChunk;
        const uint2 en = segent[j];
        uint32_t e = en.x, d = en.y, bb = ~0u;
        uint32_t nextb = (d / kSbChunk + 1) * kSbChunk;  // the next multiple of 64 KiB above d
        while (e < x1) {
            if (bb == ~0u || e + 64 + 8 > bb + kSbBuf) sb_stage(buf, T, bb = e, lane);
            const uint32_t lim = min(64u, x1 - e);
            const SbWin W = sb_window(buf, bb, e, lim, T.slen, T.dlen, lane);
            const uint32_t wx = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.nx);
            const uint32_t ws = (uint32_t)__builtin_amdgcn_readfirstlane((int)W.sm);
            if (wx >= kSbBad) break;  // (cannot happen: the stitch walked this chain)
            if (d + ws < nextb) {
                d += ws;
                e += wx;
                continue;
            }
            uint32_t q = 0;
            while (q < lim) {
                const uint32_t el = (uint32_t)__builtin_amdgcn_readlane((int)W.elen, (int)q);
                const uint32_t ol = (uint32_t)__builtin_amdgcn_readlane((int)W.olen, (int)q);
                if (el == 0) break;  // (cannot happen, as above)
                d += ol;
                q += el;
                for (; nextb <= d && nextb / kSbChunk <= m_last; nextb += kSbChunk) {
                    const uint32_t m = nextb / kSbChunk;
                    if (lane == 0) ent[B.b0 + m] = SbEnt{B.i, e + q, d, m == m_last ? 1u : 0u};
                }
            }
            if (q < lim) break;
            e += q;
        }
    }
}

__global__ __launch_bounds__(256) void k_sb_walk(const uint8_t *__restrict__ src, uint64_t src_len,
                                                 const bhg_handle *__restrict__ handles, bhg_desc *__restrict__ out,
                                                 uint8_t *__restrict__ out_vals, uint64_t out_cap,
                                                 const uint64_t *__restrict__ val_off, uint32_t *__restrict__ ctr,
                                                 const SbEnt *__restrict__ ent, uint64_t cap, uint32_t *__restrict__ blk,
                                                 uint32_t *__restrict__ ser, uint32_t lpw) {
    const uint64_t base = (uint64_t)src, end = base + src_len, oend = (uint64_t)out_vals + out_cap;
    const uint64_t total = *ctr < cap ? *ctr : cap;
    const uint32_t lane = threadIdx.x & 63;
    if (lane >= lpw) return;
    const uint64_t wv = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwv = (uint64_t)gridDim.x * blockDim.x / 64;
    for (uint64_t g = wv * lpw + lane; g < total; g += nwv * lpw) {
        const SbEnt E = ent[g];
        if (E.i == ~0u) continue;
        const uint32_t i = E.i;
        uint32_t *dw = reinterpret_cast<uint32_t *>(out + i);
        const uint32_t cpos = dw[2], dlen = dw[3];
        const bhg_handle hh = handles[i];
        const uint64_t cp = base + hh.offset + cpos;
        const uint32_t clen = hh.length - cpos;
        uint32_t hdr = 0;
        while (hdr < 10 && gld<uint8_t>(cp + hdr) >= 0x80) hdr++;
        hdr++;
        uint32_t s_end = clen - hdr, d_end = dlen;
        if (!E.last) {
            const SbEnt N = ent[g + 1];
            s_end = N.s0;
            d_end = N.d0;
        }
        const bool ok = snappy_decode_chunk(cp + hdr, E.s0, s_end, (uint64_t)out_vals + val_off[i], E.d0, d_end, end, oend);
        if (!ok) atomicOr(blk + 2 * i + 1, 1u);
        __threadfence();
        if (atomicSub(blk + 2 * i, 1u) == 1u) {  // the block's last chunk
            __threadfence();
            if (atomicOr(blk + 2 * i + 1, 0u) == 0u) {
                dw[2] = 0;  // the value's offset in out_vals is out_val_off[i]; status stays OK / CRC_MISMATCH
                dw[3] = dlen;
            } else {
                ser[atomicAdd(ctr + 1, 1u)] = i;
            }
        }
    }
}

hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off,
                         uint32_t *list, void *big) {
    if (src_len >= 64 && list) {
        // the lists the header pass filled (launch_decode with the same pointer; layout in
        // bhg_internal.h): the <= 1-KiB class, the 1-4 KiB class, and the global-memory list
        const uint32_t cap = (uint32_t)snappy_sub_cap(n);
        uint32_t *c_small = list, *c_rt = list + kSnapRtCount;
        uint32_t *e_small = list + kSnapListHdr, *e_rt = list + kSnapListHdr + (size_t)kSnapSubs * cap;
        // lanes per block: 2 in tier 1, 4 in tier 2 (snappy_walk_lds).  One lane per block in both:
        // C3 589.5 / mixdec 251.3 GiB/s; 2 / 4: 594.0 / 286.3; 1 / 4: 591.1 / 286.6; 2 / 2: 576 / 263.6
        // (2 alternating runs each, profiles/r6/slg/)
        constexpr int kG1 = 2;
        constexpr int kG2 = 4;
        {
            static const uint32_t per_cu =
                resident_per_cu((const void *)k_snappy_lds_nat<kG1>, 64, (160u * 1024u) / (kSlBpw * kSlSlot + 64));
            const uint32_t groups = (n + kSlBpw - 1) / kSlBpw, lim = (uint32_t)L.num_cus * (per_cu ? per_cu : 1u);
            const uint32_t grid = groups < lim ? (groups ? groups : 1u) : lim;
            hipLaunchKernelGGL(k_snappy_lds_nat<kG1>, dim3(grid), dim3(64), 0, L.stream, src, src_len, h, n, out, out_vals,
                               out_cap, val_off, c_small, e_small, cap, c_rt, e_rt);
            if (hipError_t e = hipGetLastError()) return e;
        }
        {
            static const uint32_t per_cu =
                resident_per_cu((const void *)k_snappy_lds_multi<kG1, kG2>, 64, (160u * 1024u) / kMultiLds);
            const uint32_t groups = (n + 3) / 4, lim = (uint32_t)L.num_cus * (per_cu ? per_cu : 1u);
            const uint32_t grid = groups < lim ? (groups ? groups : 1u) : lim;
            hipLaunchKernelGGL((k_snappy_lds_multi<kG1, kG2>), dim3(grid), dim3(64), 0, L.stream, src, src_len, h, n, out,
                               out_vals, out_cap, val_off, list, cap);
            if (hipError_t e = hipGetLastError()) return e;
        }
        // then the blocks the tiers handed on (too big for a slot, or an in-place spill): chunk-parallel
        // (k_sb_parse, k_sb_walk), and lane per block from global memory for the ones that need it
        const SbScratch B0 = sb_layout(big, n, out_cap);
        // the big path's 4 counters live in the list header, which launch_decode zeroes before the
        // header pass: one memset launch fewer per decode (C3 paid ~3 us for it)
        static_assert(kSnapRtCount + 1 <= kSnapBigCtr && kSnapBigCtr + 4 <= kSnapListHdr && kSnapBigCtr % 4 == 0,
                      "counters in the zeroed list header");
        SbScratch B = B0;
        B.ctr = list + kSnapBigCtr;
        hipLaunchKernelGGL(k_sb_parse, dim3(L.num_cus * 4), dim3(256), 0, L.stream, src, src_len, h, n, out, out_cap,
                           val_off, (const uint32_t *)c_rt, (const uint32_t *)e_rt, B.ctr, B.ent, B.cap, B.blk, B.ser,
                           B.bigs, B.segblk, B.segcap);
        // 8 workgroups of 4 waves per CU for the segment parse and the emit (window steps are
        // latency-bound: 4 per CU measured 11.36 vs 10.77 ms per bigval step, profiles/r6/bigval/)
        constexpr uint32_t sbw = 8;
        hipLaunchKernelGGL(k_sb_seg, dim3(L.num_cus * sbw), dim3(256), 0, L.stream, src, h, (const bhg_desc *)out, B.ctr,
                           B.bigs, B.segblk, B.segcap, B.res, B.ck);
        hipLaunchKernelGGL(k_sb_stitch, dim3(L.num_cus), dim3(256), 0, L.stream, src, h, (const bhg_desc *)out, B.ctr,
                           B.ent, B.blk, B.ser, B.bigs, B.segcap, B.segent, B.res, (const uint2 *)B.ck);
        hipLaunchKernelGGL(k_sb_emit, dim3(L.num_cus * sbw), dim3(256), 0, L.stream, src, h, (const bhg_desc *)out, B.ctr,
                           B.ent, B.blk, B.bigs, B.segblk, B.segcap, B.segent);
        // 8 chunks per wave (the lanes of a wave walk different chunks, each element step runs every
        // lane's path): 64 / 16 / 8 / 4 measured 25.8 / 24.8 / 24.2 / 26.8 ms per bigval step
        // (profiles/r6/bigval/walk_lanes.txt)
        hipLaunchKernelGGL(k_sb_walk, dim3(L.num_cus * 8), dim3(256), 0, L.stream, src, src_len, h, out, out_vals, out_cap,
                           val_off, B.ctr, B.ent, B.cap, B.blk, B.ser, kSbLanes);
        hipLaunchKernelGGL(k_snappy_rt, dim3(L.num_cus), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals,
                           out_cap, val_off, (const uint32_t *)(B.ctr + 1), (const uint32_t *)B.ser);
        return hipGetLastError();
    }
    uint32_t grid = (n + 255) / 256;
    const uint32_t cap = (uint32_t)L.num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_snappy_rt, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals, out_cap,
                       val_off, (const uint32_t *)nullptr, (const uint32_t *)nullptr);
    return hipGetLastError();
}

}  // namespace bhg
