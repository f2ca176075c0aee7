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
#include "bhg_snappy_parse.h"

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

// list: null (every block) or {count, block indices...} (the blocks k_snappy_lds left)
__global__ __launch_bounds__(256) void k_snappy_rt(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                   uint64_t out_cap, const uint64_t *__restrict__ val_off,
                                                   const uint32_t *__restrict__ list) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t oend = (uint64_t)out_vals + out_cap;
    const uint32_t cnt = list ? list[0] : n;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
        const uint32_t i = list ? list[1 + j] : j;
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
// k_snappy_mat: the value bytes of the blocks k_snappy_front parsed, in LDS.
//
// A workgroup is one wave and owns kSnapBPW slots of kSnapSlot bytes, lane b
// = block b of a group of kSnapBPW consecutive blocks.  A block decodes IN
// PLACE in its slot: the compressed stream staged at the slot end (P =
// slot_stream_pos(clen)), the output growing from the slot start.  The tag
// walk is already done (bhg_snappy_parse.h): the lane replays the block's ops,
// each one 16-B LDS read + one 16-B LDS write, read from the op scratch 8 at a
// time (two 16-B chunks in flight).  Per group:
//   1. the group's streams (prefetched into VGPRs, one 16-B chunk per lane per
//      block) are written into the slots;
//   2. the NEXT group's streams are requested (loads in flight during 3-5),
//      and the descriptors of the group after it;
//   3. lane b replays block b's ops (status TOO_LARGE / a corrupt stream: no ops);
//   4. the wave stores each decoded block with contiguous 16-B stores;
//   5. the descriptors are finalised.
// 8 waves per CU (two per SIMD) x 18 slots of 1,088 B fill the 160 KiB of LDS.
// Blocks the front pass could not take (oversize, in-place spill, op cap) were
// listed for k_snappy_rt, launched after this kernel.
// ---------------------------------------------------------------------------
typedef u32x4 u32x4_lds_u __attribute__((aligned(1), may_alias));

namespace {

// mode of a block in k_snappy_mat
enum : uint32_t { SM_SKIP = 0, SM_LDS = 1, SM_FINAL = 2 };

struct MatInfo {
    uint64_t cp, o0;  // stream (absolute, varint header included), output offset in out_vals
    uint32_t clen, dlen, status, mode, nops;
};

// All loads first and unconditional (index clamped to n - 1), so the caller can
// issue them ahead of the stream prefetch and wait for them alone.
__device__ __forceinline__ MatInfo mat_info(uint32_t i, uint32_t n, const bhg_desc *out, const bhg_handle *handles,
                                            const uint64_t *val_off, const uint32_t *meta, uint64_t base,
                                            uint64_t out_cap) {
    const uint32_t ii = i < n ? i : n - 1;
    const uint32_t *dw = reinterpret_cast<const uint32_t *>(out + ii);
    const uint32_t st = dw[9];
    const uint32_t cpos = dw[2], dlen = dw[3];  // provisional (front pass): value position in the record, decoded length
    const bhg_handle h = handles[ii];
    const uint64_t o0 = val_off[ii], o1 = val_off[ii + 1];
    const uint32_t m = meta[ii];
    MatInfo r;
    r.cp = base + h.offset + cpos;
    r.o0 = o0;
    r.clen = h.length - cpos;
    r.dlen = dlen;
    r.nops = m >> 8;
    r.status = st;
    r.mode = SM_SKIP;
    if (i < n && (m & 3u) == SNAP_LDS && (st == BHG_ST_OK || st == BHG_ST_CRC_MISMATCH)) {
        // snappy.Decode's order: the output capacity first, then the stream (decode_other.go)
        if (o1 > out_cap || o1 - o0 < dlen) {
            r.status = BHG_ST_SNAPPY_TOO_LARGE;
            r.mode = SM_FINAL;
        } else if (m & 4u) {
            r.status = BHG_ST_SNAPPY_CORRUPT;
            r.mode = SM_FINAL;
        } else {
            r.mode = SM_LDS;
        }
    }
    return r;
}

}  // namespace

// Op replay with dword-aligned LDS accesses only: a 16-B (or 8-B) LDS access
// off its natural alignment is replayed at 64 cycles per instruction on gfx950,
// and op sources / destinations sit at any byte.  An op reads the 5 dwords
// around its source and assembles the 16 bytes with v_perm; it writes 5 dwords
// from its destination's dword, the first merged with the lane's copy of that
// dword's final bytes (pend) -- so nothing is read back.  Writes reach 20 B past
// the cursor (k_snappy_front's in-place margin).
typedef uint32_t u32_lds __attribute__((may_alias));

template <int BPW, int SLOT>
__device__ __forceinline__ void mat_replay_op(uint8_t *lds, uint32_t op, bool act, uint32_t slot0, uint32_t trash,
                                              uint32_t &d, uint32_t &pend) {
    u32_lds *L = reinterpret_cast<u32_lds *>(lds);
    const uint32_t src = act ? slot0 + (op & 0x7ffu) : slot0;
    const uint32_t len = (op >> 11) + 1u;
    const uint32_t as = src >> 2, sr = src & 3u;
    const uint32_t r0 = L[as], r1 = L[as + 1], r2 = L[as + 2], r3 = L[as + 3], r4 = L[as + 4];
    const uint32_t selr = 0x03020100u + sr * 0x01010101u;
    const uint32_t b0 = __builtin_amdgcn_perm(r1, r0, selr), b1 = __builtin_amdgcn_perm(r2, r1, selr);
    const uint32_t b2 = __builtin_amdgcn_perm(r3, r2, selr), b3 = __builtin_amdgcn_perm(r4, r3, selr);
    const uint32_t sh = d & 3u;                                    // slot0 is 16-B aligned
    const uint32_t selw = 0x07060504u - sh * 0x01010101u;          // bytes [4 - sh, 8 - sh) of (hi:lo)
    const uint32_t m = (1u << (8u * sh)) - 1u;                     // the sh final bytes of pend
    const uint32_t sel0 = (0x03020100u & m) | (selw & ~m);
    const uint32_t q0 = __builtin_amdgcn_perm(b0, pend, sel0), q1 = __builtin_amdgcn_perm(b1, b0, selw);
    const uint32_t q2 = __builtin_amdgcn_perm(b2, b1, selw), q3 = __builtin_amdgcn_perm(b3, b2, selw);
    const uint32_t q4 = __builtin_amdgcn_perm(b3, b3, selw);
    const uint32_t D = (act ? slot0 + d : trash) >> 2;
    L[D] = q0; L[D + 1] = q1; L[D + 2] = q2; L[D + 3] = q3; L[D + 4] = q4;
    const uint32_t jn = (sh + len) >> 2;                           // the dword holding the new cursor
    const uint32_t pn = jn == 0 ? q0 : jn == 1 ? q1 : jn == 2 ? q2 : jn == 3 ? q3 : q4;
    pend = act ? pn : pend;
    d += act ? len : 0u;
}

template <int BPW, int SLOT>
__global__ __launch_bounds__(64) void k_snappy_mat(const uint8_t *__restrict__ src, uint64_t src_len,
                                                   const bhg_handle *__restrict__ handles, uint32_t n,
                                                   bhg_desc *__restrict__ out, uint8_t *__restrict__ out_vals,
                                                   uint64_t out_cap, const uint64_t *__restrict__ val_off,
                                                   const uint32_t *__restrict__ meta,
                                                   const uint16_t *__restrict__ ops) {
    static_assert(SLOT % 16 == 0 && BPW <= 64, "16-B aligned slots, a lane per block");
    constexpr uint32_t kChunks = kSnapOpCap / 8, kRegChunks = 12;  // 16-B op chunks; the first 96 ops ride in VGPRs
    __shared__ __attribute__((aligned(16))) uint8_t lds[BPW * SLOT + 64];  // + 64: literal reads past the last slot
    const uint32_t lane = threadIdx.x;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ngroups = (n + BPW - 1) / BPW;
    const uint32_t G = gridDim.x;
    uint32_t g = blockIdx.x;
    if (g >= ngroups) return;
    auto info = [&](uint32_t grp) -> MatInfo {
        const uint32_t i = grp * BPW + lane;
        return mat_info(lane < BPW && grp < ngroups ? i : n, n, out, handles, val_off, meta, base, out_cap);
    };
    auto op_chunks = [&](uint32_t grp) -> const u32x4 * {
        const uint32_t i = grp * BPW + (lane < BPW ? lane : 0u);
        return reinterpret_cast<const u32x4 *>(ops + (uint64_t)(i < n ? i : n - 1) * kSnapOpCap);
    };
    u32x4 v[BPW];
    u32x4 opc[kRegChunks], opn[kRegChunks];
    // One 16-B chunk per lane per staged block, loaded unconditionally (lanes
    // past the stream load src + 0; the dump drops them) and clamped to end
    // src (a chunk that would cross the end is loaded from end - 16 and
    // shifted into place at the dump), so no branch and no wait is tied to the
    // loads until the next dump.  (The launcher sends src_len < 64 elsewhere.)
    auto chunk_addr = [&](const MatInfo &I, int b, uint32_t &clb) -> uint64_t {
        clb = __builtin_amdgcn_readlane(I.mode == SM_LDS ? I.clen : 0u, b);
        const uint64_t cpb = readlane_u64(I.cp, b);
        return 16 * lane < clb ? cpb + 16 * lane : base;
    };
    auto prefetch = [&](const MatInfo &I) {
#pragma unroll
        for (int b = 0; b < BPW; b++) {
            uint32_t clb;
            const uint64_t a = chunk_addr(I, b, clb);
            v[b] = gld<u32x4u>(a + 16 <= end ? a : end - 16);
        }
    };
    auto load_ops = [&](u32x4 (&dst)[kRegChunks], uint32_t grp) {
        const u32x4 *oc = op_chunks(grp < ngroups ? grp : g);
#pragma unroll
        for (uint32_t c = 0; c < kRegChunks; c++) dst[c] = oc[c];
    };
    MatInfo cur = info(g);
    load_ops(opc, g);
    prefetch(cur);
    MatInfo nxt = info(g + G);
    for (; g < ngroups; g += G) {
        // 1. this group's streams -> slots (the wait here also covers this group's op chunks,
        //    loaded before the streams)
#pragma unroll
        for (int b = 0; b < BPW; b++) {
            uint32_t clb;
            const uint64_t a = chunk_addr(cur, b, clb);
            u32x4 c = v[b];
            if (a + 16 > end) {  // the chunk was loaded from end - 16: its bytes start at a - (end - 16)
                const uint32_t sh = (uint32_t)(a - (end - 16));
                unsigned __int128 x = (unsigned __int128)c.x | ((unsigned __int128)c.y << 32) |
                                      ((unsigned __int128)c.z << 64) | ((unsigned __int128)c.w << 96);
                x >>= 8 * sh;
                c = u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)};
            }
            if (16 * lane < clb)
                *reinterpret_cast<u32x4_lds_u *>(lds + b * SLOT + slot_stream_pos(SLOT, clb) + 16 * lane) = c;
        }
        lds_wave_sync();
        // 2. descriptors of the group after next; the next group's op chunks, then its streams, in flight
        const MatInfo nn = info(g + 2 * G);
        load_ops(opn, g + G);
        prefetch(nxt);
        // 3. replay the ops (8 per 16-B chunk): the first kRegChunks chunks from VGPRs, the rest loaded here
        const uint32_t nops = cur.mode == SM_LDS ? cur.nops : 0u;
        const uint32_t nch = (nops + 7) >> 3;
        const uint32_t maxc = __builtin_amdgcn_readlane(wave_incl_max(nch), 63);
        if (lane < BPW && maxc) {
            const uint32_t slot0 = lane * SLOT, trash = slot0 + SLOT - 32;
            uint32_t d = 0, pend = 0;
            auto replay8 = [&](const u32x4 &w, uint32_t c) {
#pragma unroll
                for (uint32_t j = 0; j < 8; j++) {
                    const uint32_t word = j < 2 ? w.x : j < 4 ? w.y : j < 6 ? w.z : w.w;
                    mat_replay_op<BPW, SLOT>(lds, (word >> (16 * (j & 1))) & 0xffffu, 8 * c + j < nops, slot0, trash,
                                             d, pend);
                }
            };
#pragma unroll
            for (uint32_t c = 0; c < kRegChunks; c++)
                if (c < maxc) replay8(opc[c], c);
            if (maxc > kRegChunks) {
                const u32x4 *oc = op_chunks(g);
                for (uint32_t c = kRegChunks; c < maxc && c < kChunks; c++) replay8(oc[c], c);
            }
        }
        // 4. decoded blocks -> out_vals
        lds_wave_sync();
        {
            const uint32_t dl = cur.mode == SM_LDS ? cur.dlen : 0u;
#pragma unroll
            for (int b = 0; b < BPW; b++) {
                const uint32_t dlb = __builtin_amdgcn_readlane(dl, b);
                if (16 * lane < dlb) {
                    const uint64_t ob = (uint64_t)out_vals + readlane_u64(cur.o0, b);
                    st16_clip(ob + 16 * lane, *reinterpret_cast<const u32x4_lds_u *>(lds + b * SLOT + 16 * lane),
                              ob + dlb);
                }
            }
        }
        lds_wave_sync();
        // 5. descriptors
        if (cur.mode != SM_SKIP) {
            uint32_t *dw = reinterpret_cast<uint32_t *>(out + g * BPW + lane);
            const bool ok = cur.status == BHG_ST_OK || cur.status == BHG_ST_CRC_MISMATCH;
            dw[2] = 0;
            dw[3] = ok ? cur.dlen : 0u;
            dw[9] = cur.status;
        }
        cur = nxt;
        nxt = nn;
#pragma unroll
        for (uint32_t c = 0; c < kRegChunks; c++) opc[c] = opn[c];
    }
}

hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off,
                         const uint32_t *meta, const uint16_t *ops, const uint32_t *list) {
    if (src_len >= 64 && meta && ops && list) {
        constexpr uint32_t BPW = kSnapBPW, SLOT = kSnapSlot;
        // resident workgroups per CU (LDS-bound: 8 at 18 x 1,088 B); a grid past that would
        // start its extra workgroups only when the first ones finish
        static const uint32_t per_cu =
            resident_per_cu((const void *)k_snappy_mat<BPW, SLOT>, 64, (160u * 1024u) / (BPW * SLOT + 64));
        const uint32_t groups = (n + BPW - 1) / BPW;
        const uint32_t cap = (uint32_t)L.num_cus * (per_cu ? per_cu : 1u);
        uint32_t grid = groups < cap ? groups : cap;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL((k_snappy_mat<BPW, SLOT>), dim3(grid), dim3(64), 0, L.stream, src, src_len, h, n, out,
                           out_vals, out_cap, val_off, meta, ops);
        if (hipError_t e = hipGetLastError()) return e;
        // then the blocks the front pass listed (too big for a slot, spill, op cap), lane per block from global memory
        hipLaunchKernelGGL(k_snappy_rt, dim3(L.num_cus), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals,
                           out_cap, val_off, list);
        return hipGetLastError();
    }
    uint32_t grid = (n + 255) / 256;
    const uint32_t cap = (uint32_t)L.num_cus * 8;
    if (grid > cap) grid = cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_snappy_rt, dim3(grid), dim3(256), 0, L.stream, src, src_len, h, n, out, out_vals, out_cap,
                       val_off, (const uint32_t *)nullptr);
    return hipGetLastError();
}

}  // namespace bhg
