// bhg_device.h -- device-side building blocks for the gfx950 bithash codec.
//
// Everything here is integer byte work: no MFMA.  The CRC-32C is table
// driven out of LDS with the 1 KiB byte table replicated 32x so that lane l
// always reads bank (l & 31): a random-index lookup by all 64 lanes is then
// bank-conflict free (ds_read_b32 services lanes in two 32-lane groups, bank
// = dword address mod 32).  32 KiB of LDS per workgroup.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bithashgpu.h"

#define BHG_CRC_POLY 0x82F63B78u      // Castagnoli, reflected (hash/crc32.Castagnoli)
#define BHG_FNV_OFFSET 2166136261u    // hash/fnv offset32
#define BHG_FNV_PRIME 16777619u       // hash/fnv prime32
#define BHG_CRC_LDS_WORDS (256 * 32)  // replicated table size in dwords

namespace bhg {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// 16-byte vector that is only promised 4-byte alignment: records are packed
// back to back at arbitrary offsets, and dword alignment is enough for a
// global_load_dwordx4 on gfx950.
typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

// Global-address-space accessors for absolute (integer) addresses: keeps the
// compiler on global_load_* instead of flat_load_* (flat also counts against
// lgkmcnt and is issued through the LDS/flat arbiter).
#define BHG_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(uint64_t a) {
    return *reinterpret_cast<const BHG_GLOBAL T *>(a);
}
template <class T>
__device__ __forceinline__ void gst(uint64_t a, T v) {
    *reinterpret_cast<BHG_GLOBAL T *>(a) = v;
}

__device__ __forceinline__ uint32_t crc_table_entry(uint32_t i) {
    uint32_t c = i;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ BHG_CRC_POLY : (c >> 1);
    return c;
}

// Fill the replicated table: dword (i*32 + r) = T[i] for r in 0..31.
__device__ __forceinline__ void crc_lds_fill(uint32_t *T) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
        uint32_t v = crc_table_entry(i);
        u32x4 v4 = {v, v, v, v};
        u32x4 *dst = reinterpret_cast<u32x4 *>(T + i * 32);
#pragma unroll
        for (int r = 0; r < 8; r++) dst[r] = v4;
    }
}

// Per-lane view of the replicated table.
struct CrcLds {
    const uint32_t *t;  // T + (lane & 31)
    __device__ __forceinline__ explicit CrcLds(const uint32_t *T) : t(T + (threadIdx.x & 31)) {}
    __device__ __forceinline__ uint32_t step(uint32_t c) const { return (c >> 8) ^ t[(c & 0xffu) << 5]; }
    // absorb one full little-endian word (4 byte steps)
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        c ^= w;
        c = step(c); c = step(c); c = step(c); c = step(c);
        return c;
    }
    // absorb the low `nb` (0..4) bytes of x
    __device__ __forceinline__ uint32_t partial(uint32_t c, uint32_t x, uint32_t nb) const {
        uint32_t m = nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
        c ^= x & m;
#pragma unroll
        for (uint32_t s = 0; s < 4; s++) {
            uint32_t n = step(c);
            c = s < nb ? n : c;
        }
        return c;
    }
};

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) {  // crc.go:31-33
    return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// Aligned dword load at absolute address a (4-aligned) that never touches a
// byte at or past `end`: the last partial word is assembled from bytes.
__device__ __forceinline__ uint32_t ld32_safe(uint64_t a, uint64_t end) {
    if (a + 4 <= end) return gld<uint32_t>(a);
    uint32_t w = 0;
    for (uint32_t j = 0; j < 4; j++)
        if (a + j < end) w |= (uint32_t)gld<uint8_t>(a + j) << (8 * j);
    return w;
}

// Unaligned little-endian u32 at absolute address p; [p, p+4) must lie inside
// [.., end).  Two aligned dword loads + one v_alignbyte.
__device__ __forceinline__ uint32_t ldu32(uint64_t p, uint64_t end) {
    uint64_t a = p & ~3ull;
    uint32_t sh = (uint32_t)(p & 3);
    uint32_t lo = ld32_safe(a, end);
    if (sh == 0) return lo;
    uint32_t hi = ld32_safe(a + 4, end);
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

__device__ __forceinline__ uint64_t ldu64(uint64_t p, uint64_t end) {
    return (uint64_t)ldu32(p, end) | ((uint64_t)ldu32(p + 4, end) << 32);
}

// Raw CRC-32C chain (Go crc32.Update internals: state already inverted) over
// the absolute byte range [p, p+len), every load kept below `end`.
// One lane walks its own range; 64 B per iteration via 4 dword-aligned
// dwordx4 loads, next window prefetched while the current one is absorbed.
__device__ __forceinline__ uint32_t crc_range(const CrcLds &T, uint32_t c, uint64_t p, uint64_t len, uint64_t end) {
    if (len == 0) return c;
    // head: bytes up to the next 4-aligned address
    uint64_t a0 = p & ~3ull;
    uint32_t z = (uint32_t)(p & 3);
    if (z) {
        uint32_t nb = 4 - z;
        if ((uint64_t)nb > len) nb = (uint32_t)len;
        uint32_t w = ld32_safe(a0, end) >> (8 * z);
        c = T.partial(c, w, nb);
        p += nb;
        len -= nb;
        if (len == 0) return c;
    }
    // p is 4-aligned now
    uint64_t nw = len >> 2;
    uint32_t tail = (uint32_t)(len & 3);
    uint64_t a = p;
    if (nw) {
        const bool fast0 = a + 64 <= end;
        u32x4 cur[4], nxt[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (fast0) cur[q] = gld<u32x4_a4>(a + 16 * q);
            else cur[q] = u32x4{ld32_safe(a + 16 * q, end), ld32_safe(a + 16 * q + 4, end),
                                ld32_safe(a + 16 * q + 8, end), ld32_safe(a + 16 * q + 12, end)};
        }
        for (uint64_t base = 0; base < nw; base += 16) {
            const uint64_t an = a + 64 * (base / 16 + 1);
            const bool more = base + 16 < nw;
            if (more) {
                const bool fast = an + 64 <= end;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (fast) nxt[q] = gld<u32x4_a4>(an + 16 * q);
                    else nxt[q] = u32x4{ld32_safe(an + 16 * q, end), ld32_safe(an + 16 * q + 4, end),
                                        ld32_safe(an + 16 * q + 8, end), ld32_safe(an + 16 * q + 12, end)};
                }
            }
            const uint64_t rem = nw - base;
            if (rem >= 16) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    c = T.word(c, cur[q].x); c = T.word(c, cur[q].y);
                    c = T.word(c, cur[q].z); c = T.word(c, cur[q].w);
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if ((uint64_t)(4 * q + 0) < rem) c = T.word(c, cur[q].x);
                    if ((uint64_t)(4 * q + 1) < rem) c = T.word(c, cur[q].y);
                    if ((uint64_t)(4 * q + 2) < rem) c = T.word(c, cur[q].z);
                    if ((uint64_t)(4 * q + 3) < rem) c = T.word(c, cur[q].w);
                }
            }
            if (more) {
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nxt[q];
            }
        }
    }
    if (tail) c = T.partial(c, ld32_safe(a + 4 * nw, end), tail);
    return c;
}

// FNV-1 (hash/fnv New32: multiply, then xor) over [p, p+len).
__device__ __forceinline__ uint32_t fnv1_range(uint64_t p, uint64_t len, uint64_t end) {
    uint32_t h = BHG_FNV_OFFSET;
    uint64_t a = p & ~3ull;
    uint32_t skip = (uint32_t)(p & 3);
    uint64_t stop = p + len;
    for (; a < stop; a += 4) {
        uint32_t w = ld32_safe(a, end);
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            uint64_t b = a + j;
            uint32_t hn = (h * BHG_FNV_PRIME) ^ ((w >> (8 * j)) & 0xffu);
            h = (b >= p && b < stop) ? hn : h;
        }
        (void)skip;
    }
    return h;
}

}  // namespace bhg
