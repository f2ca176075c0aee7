// bhg_snappy_parse.h -- golang/snappy v0.0.4 block parse (decode_other.go
// `decode`, called by internal/compress/compress.go:83-85) into 16-byte
// copy OPS for the LDS materialiser (k_snappy_mat, bhg_snappy_dec.hip).
//
// The decode is split in two kernels.  k_snappy_front (bhg_snappy_front.hip)
// stages a tile of records in LDS, CRCs them and walks each block's tag
// stream, lane per block, 64 blocks per wave, writing for every element the
// ops that produce it; k_snappy_mat later replays the ops of 18 blocks per
// wave in their LDS slots, where nothing is left to decode.
//
// The slot (SLOT bytes per block in k_snappy_mat) holds the block in place:
// the compressed stream staged at P = slot_stream_pos(clen), the output
// growing from offset 0.  An op is
//     src | (len - 1) << 11       (src: slot offset < 2048, len 1..16)
// and means: read the 16 bytes at slot offset src, write them at the output
// cursor, advance the cursor by len (the replay writes up to 20 bytes).  Only the first len bytes written are
// final; the rest are overwritten by the next ops in program order (LDS runs a
// wave's accesses in order).  Per element:
//   literal of n bytes at stream position q:   ops (P + q + 16 j, <= 16)
//   copy (offset o, length n), o >= min(n, 16): ops (d - o + 16 j, <= 16)
//   copy with a short period o < min(n, 16): the first op copies o bytes from
//     d - o, and while the period e < 16 every op copies e bytes from e bytes
//     back and doubles e (the bytes [d - o, cursor) are periodic, so e bytes
//     back is always the right phase); then 16 bytes per op from e back.
// The checks are decode_other.go's, check for check: literal length bytes
// past the input, literal longer than the remaining input or output, copy
// offset 0 or beyond the bytes written, copy past dlen, d == dlen at the end.
// A block whose 16-B writes would reach its own unread stream bytes (in
// place), or that needs more than kSnapOpCap ops, is handed to the
// global-memory decoder (k_snappy_rt).
// tests/test_snappy_walk_host.py compiles this file for the host and checks
// parse + op replay against the restated decoder.
#pragma once
#include <stdint.h>

namespace bhg {

typedef uint64_t snap_u64_a __attribute__((aligned(8), may_alias));

constexpr uint32_t kSnapOpCap = 192;  // ops per block (u16 each) in the op scratch
constexpr uint32_t kSnapSlot = 1088;  // k_snappy_mat slot bytes per block (the 1 KiB value + stream room)
constexpr uint32_t kSnapBPW = 18;     // k_snappy_mat blocks per wave (8 waves x 18 slots fill 160 KiB)

// how a block's value is decoded (k_snappy_front -> meta)
enum : uint32_t { SNAP_SKIP = 0, SNAP_LDS = 1, SNAP_GLOBAL = 2 };

// slot offset of a stream of clen bytes (16-B aligned, 8 B of tag over-read room after it)
__device__ __forceinline__ uint32_t slot_stream_pos(uint32_t slot, uint32_t clen) {
    return (slot - 8u - ((clen + 15u) & ~15u)) & ~15u;
}

// one block's parse state; LDS byte offsets into the staging arena
struct SnapParse {
    uint32_t s;      // next tag
    uint32_t se;     // end of the stream
    uint32_t lit0;   // slot offset of arena offset 0 (mod 2^32): slot(x) = lit0 + x
    uint32_t d;      // output bytes so far
    uint32_t dlen;   // decoded length (from the varint header)
    uint32_t nops;   // ops emitted
    uint32_t res;    // 0 ok so far, 1 snappy.ErrCorrupt, 2 hand over to the global-memory decoder
    uint64_t t8;     // the tag at s and the bytes after it
};

__device__ __forceinline__ uint32_t snap_op(uint32_t src, uint32_t len) { return src | ((len - 1u) << 11); }

// The 8 bytes at LDS offset p from two 8-aligned 8-byte reads (misaligned
// 8- and 16-byte LDS accesses are replayed at 64 cycles per instruction on
// gfx950; aligned ones take 2).
__device__ __forceinline__ uint64_t snap_ld8(const uint8_t *lds, uint32_t p) {
    const uint32_t a = p & ~7u, s = p & 7u;
    const uint64_t x0 = *reinterpret_cast<const snap_u64_a *>(lds + a);
    const uint64_t x1 = *reinterpret_cast<const snap_u64_a *>(lds + a + 8);
    return s ? (x0 >> (8u * s)) | (x1 << (64u - 8u * s)) : x0;
}

// One element.  emit(k, op) receives op k of the block.  Returns true while
// more elements follow.  The tag decode is straight-line (selects, no per-type
// branches); the next tag is read before the ops are emitted.
template <class Emit>
__device__ __forceinline__ bool snap_parse_step(const uint8_t *lds, SnapParse &S, Emit &&emit) {
    const uint64_t t8 = S.t8;
    const uint32_t s = S.s, d = S.d;
    const uint32_t tag = (uint32_t)t8 & 0xffu, ty = tag & 3u, x = tag >> 2;
    const uint32_t b14 = (uint32_t)(t8 >> 8);  // the 4 bytes after the tag
    //   adv: literal 1, copy-1 2, copy-2 3, copy-4 5;  offset mask: ~0 >> {-, 24, 16, 0}
    const uint32_t mlit = 0u - (uint32_t)(ty == 0u), m1 = 0u - (uint32_t)(ty == 1u);
    uint32_t n = (m1 & (4u + (x & 7u))) | (~m1 & (x + 1u));
    uint32_t adv = (0x5321u >> (4u * ty)) & 0xfu;
    const uint32_t off = (b14 & (0xffffffffu >> ((0x00101800u >> (8u * ty)) & 0xffu))) | (m1 & ((tag >> 5) << 8));
    if (ty == 0u && x >= 60u) {  // long literal: 1-4 length bytes
        const uint32_t nb = x - 59u;
        const uint32_t lmask = nb >= 4u ? 0xffffffffu : ((1u << (8u * nb)) - 1u);
        n = (b14 & lmask) + 1u;
        adv = 1u + nb;
    }
    const uint32_t rem = S.se - s;  // >= 1
    // n == 0 only for a 4-byte literal length of 2^32 - 1: too long
    const uint32_t bad_lit = (uint32_t)(n > rem - adv), bad_cp = (uint32_t)(off == 0u) | (uint32_t)(off > d);
    const bool bad = ((uint32_t)(adv > rem) | (uint32_t)(n > S.dlen - d) | (uint32_t)(n == 0u) | (mlit & bad_lit) |
                      (~mlit & bad_cp)) != 0u;
    const uint32_t sn = s + adv + (mlit & n);
    // in place: the element's writes (5 dwords from the cursor's dword) end below d + n + 20, the
    // next unread stream byte is at slot(sn)
    const bool spill = d + n + 20u > S.lit0 + sn;
    if (bad | spill) {
        S.res = bad ? 1u : 2u;
        return false;
    }
    S.t8 = snap_ld8(lds, sn);  // next tag, in flight while the ops go out
    const bool lit = mlit != 0u;
    const uint32_t lsrc = S.lit0 + s + adv;
    uint32_t e = lit ? 16u : off;
    // first op (every element has one), then the rest (elements over 16 B, short periods)
    uint32_t cap = e < 16u ? e : 16u;
    uint32_t len = n < cap ? n : cap;
    emit(S.nops, snap_op(lit ? lsrc : d - e, len));
    uint32_t k = S.nops + 1u, w = len;
    if (!lit && e < 16u) e <<= 1;
    while (w < n) {
        cap = e < 16u ? e : 16u;
        len = n - w < cap ? n - w : cap;
        emit(k, snap_op(lit ? lsrc + w : d + w - e, len));
        k++;
        w += len;
        if (!lit && e < 16u) e <<= 1;
    }
    S.nops = k;
    S.d = d + n;
    S.s = sn;
    return sn < S.se;
}

}  // namespace bhg
