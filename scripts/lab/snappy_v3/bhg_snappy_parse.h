// bhg_snappy_parse.h -- golang/snappy v0.0.4 block parse (decode_other.go
// `decode`, called by internal/compress/compress.go:83-85) into 16-byte
// copy OPS for the materialiser (k_snappy_mat, bhg_snappy_dec.hip).
//
// The decode is split in two kernels.  k_snappy_front (bhg_snappy_front.hip)
// stages a tile of records in LDS, CRCs them and walks each block's tag
// stream, lane per block, 64 blocks per wave, writing for every element the
// ops that produce it; k_snappy_mat later replays the ops of 64 blocks per
// wave, the output in LDS, where nothing is left to decode.
//
// An op is a u16:
//     src | (len - 1) << 11 | lit << 15      (src < 2048, len 1..16)
// lit: the len bytes at stream offset src (the value's bytes, varint header
// included) are output bytes; copy: the len bytes at output offset src are.
// The replay reads 16 bytes from the source and writes them at the output
// cursor (5 dwords from the cursor's dword), then advances the cursor by len:
// only the first len bytes are final, the rest are rewritten by the following
// ops in program order.  Per element:
//   literal of n bytes at stream offset q:           ops (q + 16 j, <= 16)
//   copy (offset o, length n), o >= min(n, 16):      ops (d - o + 16 j, <= 16)
//   copy with a short period o < min(n, 16): the first op copies o bytes from
//     d - o, and while the period e < 16 every op copies e bytes from e bytes
//     back and doubles e (the bytes [d - o, cursor) are periodic, so e bytes
//     back is always the right phase); then 16 bytes per op from e back.
// The first four ops of an element are emitted straight-line (every C3 element
// needs at most four); longer elements loop.  The checks are
// decode_other.go's, check for check: literal length bytes past the input,
// literal longer than the remaining input or output, copy offset 0 or beyond
// the bytes written, copy past dlen, d == dlen at the end.  A block that needs
// kSnapOpCap ops or more is handed to the global-memory decoder (k_snappy_rt).
// tests/test_snappy_walk_host.py compiles this file for the host and checks
// parse + op replay against the restated decoder.
#pragma once
#include <stdint.h>

namespace bhg {

typedef uint64_t snap_u64_a __attribute__((aligned(8), may_alias));

constexpr uint32_t kSnapOpCap = 192;     // u16 op slots per block in the op scratch; the last is a dump slot
constexpr uint32_t kSnapMaxOut = 1024;   // decoded lengths the op path takes (larger: k_snappy_rt)
constexpr uint32_t kSnapMaxStream = 2047;  // stream lengths the op path takes (op src is 11 bits)

// how a block's value is decoded (k_snappy_front -> meta)
enum : uint32_t { SNAP_SKIP = 0, SNAP_OPS = 1, SNAP_GLOBAL = 2 };

// one block's parse state; LDS byte offsets into the staging arena
struct SnapParse {
    uint32_t s;      // next tag
    uint32_t se;     // end of the stream
    uint32_t sb;     // the stream's first byte (stream offset 0)
    uint32_t d;      // output bytes so far
    uint32_t dlen;   // decoded length (from the varint header)
    uint32_t nops;   // ops emitted
    uint32_t res;    // 0 ok so far, 1 snappy.ErrCorrupt
    uint64_t t8;     // the tag at s and the bytes after it
};

__device__ __forceinline__ uint32_t snap_op(uint32_t src, uint32_t len, uint32_t lit) {
    return src | ((len - 1u) << 11) | (lit << 15);
}

// The 8 bytes at LDS offset p from two 8-aligned 8-byte reads (misaligned
// 8- and 16-byte LDS accesses are replayed at 64 cycles per instruction on
// gfx950; aligned ones take 2).
__device__ __forceinline__ uint64_t snap_ld8(const uint8_t *lds, uint32_t p) {
    const uint32_t a = p & ~7u, s = p & 7u;
    const uint64_t x0 = *reinterpret_cast<const snap_u64_a *>(lds + a);
    const uint64_t x1 = *reinterpret_cast<const snap_u64_a *>(lds + a + 8);
    return s ? (x0 >> (8u * s)) | (x1 << (64u - 8u * s)) : x0;
}

// One element.  emit(k, op, on) stores op k of the block when `on` (a slot the
// element does not use may be stored anywhere harmless).  Returns true while
// more elements follow.  The tag decode is straight-line (selects, no
// per-type branches); the next tag is read before the ops are emitted.
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
    if (bad) {
        S.res = 1u;
        return false;
    }
    const uint32_t sn = s + adv + (mlit & n);
    S.t8 = snap_ld8(lds, sn);  // next tag, in flight while the ops go out
    const uint32_t lit = mlit & 1u;
    const uint32_t lsrc = s + adv - S.sb;
    // ops 0..3 straight-line: e = how far back a copy op reads (a literal's ops step by 16)
    uint32_t e = lit ? 16u : off, w = 0, k = S.nops;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t cap = e < 16u ? e : 16u;
        const uint32_t left = n - w;  // 0 once the element is done
        const uint32_t len = left < cap ? left : cap;
        const bool on = len != 0u;
        emit(k, snap_op(lit ? lsrc + w : d + w - e, on ? len : 1u, lit), on);
        k += on ? 1u : 0u;
        w += len;
        if (!lit && e < 16u) e <<= 1;
    }
    while (w < n) {  // literals over 64 bytes, short-period copies over four ops
        const uint32_t cap = e < 16u ? e : 16u;
        const uint32_t len = n - w < cap ? n - w : cap;
        emit(k, snap_op(lit ? lsrc + w : d + w - e, len, lit), true);
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
