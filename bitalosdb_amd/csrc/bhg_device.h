// bhg_device.h -- device-side building blocks for the gfx950 bithash codec.
//
// Everything here is integer byte work: no MFMA.  The CRC-32C is table
// driven out of LDS: slice-by-4 tables replicated R times so that lanes read
// different banks (ds_read_b32 services lanes in two 32-lane groups, bank =
// dword address mod 32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bithashgpu.h"

#define BHG_CRC_POLY 0x82F63B78u      // Castagnoli, reflected (hash/crc32.Castagnoli)
#define BHG_FNV_OFFSET 2166136261u    // hash/fnv offset32
#define BHG_FNV_PRIME 16777619u       // hash/fnv prime32

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

// s_waitcnt vmcnt(0) as a real S_WAITCNT the compiler's wait-insertion pass
// understands (expcnt / lgkmcnt left at their maxima; gfx9 encoding).  Placed
// before a wave's descriptor stores at the end of a tile: every load is
// complete there anyway, and the pass then knows nothing loaded is pending at
// the loop latch -- otherwise it merges the back edge conservatively and waits
// vmcnt(0) after the stores, exposing a full store round trip per tile.
__device__ __forceinline__ void wait_loads_done() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Lane `src`'s 64-bit value, wave-uniform (two v_readlane_b32), and lane 0's
// (v_readfirstlane_b32).  The builtins return int: each half goes through
// uint32_t before widening, or a low word with bit 31 set sign-extends into the
// high word -- the cause of round 2's intermittent snappy-decoder faults.
// tests/test_addr_host.py compiles these for the host and checks that case.
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t readfirstlane_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Wave-wide inclusive scans through DPP (row_shr 1/2/4/8, then row_bcast 15 /
// 31): no lane-address registers, unlike __shfl_up / ds_bpermute.
#define BHG_DPP(x, ctrl, rmask) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), ctrl, rmask, 0xf, false))
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
    x += BHG_DPP(x, 0x111, 0xf);
    x += BHG_DPP(x, 0x112, 0xf);
    x += BHG_DPP(x, 0x114, 0xf);
    x += BHG_DPP(x, 0x118, 0xf);
    x += BHG_DPP(x, 0x142, 0xa);
    x += BHG_DPP(x, 0x143, 0xc);
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {  // values >= 0: 0 is the identity
    uint32_t y;
    y = BHG_DPP(x, 0x111, 0xf); x = y > x ? y : x;
    y = BHG_DPP(x, 0x112, 0xf); x = y > x ? y : x;
    y = BHG_DPP(x, 0x114, 0xf); x = y > x ? y : x;
    y = BHG_DPP(x, 0x118, 0xf); x = y > x ? y : x;
    y = BHG_DPP(x, 0x142, 0xa); x = y > x ? y : x;
    y = BHG_DPP(x, 0x143, 0xc); x = y > x ? y : x;
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_or(uint32_t x) {
    x |= BHG_DPP(x, 0x111, 0xf);
    x |= BHG_DPP(x, 0x112, 0xf);
    x |= BHG_DPP(x, 0x114, 0xf);
    x |= BHG_DPP(x, 0x118, 0xf);
    x |= BHG_DPP(x, 0x142, 0xa);
    x |= BHG_DPP(x, 0x143, 0xc);
    return x;
}
#undef BHG_DPP

// Lanes of a wave hand LDS bytes to each other (one lane writes, another
// reads): LDS runs a wave's accesses in program order, but the compiler sees
// one thread and could move a read above another lane's write, so each
// hand-over is a wavefront-scope fence (LDS types that cross it are may_alias).
__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t crc_table_entry(uint32_t i) {
    uint32_t c = i;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ BHG_CRC_POLY : (c >> 1);
    return c;
}

// Slice-by-4 tables T0..T3 (T_{k+1}[i] = T_k[i] >> 8 ^ T0[T_k[i] & 0xff]),
// each replicated R times and interleaved so that lane l reads copy (l % R):
// dword index = k*256*R + i*R + (l % R).  R = 32 is bank-conflict free for
// ds_read_b32 (128 KiB); smaller R trades LDS for bank conflicts among the
// 32/R lanes that share a copy.  One word costs 4 independent lookups, so
// the dependent LDS chain is one round trip per 4 bytes instead of 4.
template <int R>
struct Crc4Lds {
    static constexpr int kLog = R == 32 ? 5 : R == 16 ? 4 : R == 8 ? 3 : R == 4 ? 2 : R == 2 ? 1 : 0;
    static constexpr uint32_t kWords = 4u * 256u * R;
    static constexpr uint32_t kShift = 2 + kLog;  // idx -> byte offset
    const uint8_t *base;
    uint32_t lb0, lb1, lb2, lb3;  // per-table lane base byte offsets
    __device__ __forceinline__ explicit Crc4Lds(const uint32_t *T) : base(reinterpret_cast<const uint8_t *>(T)) {
        const uint32_t lo = (threadIdx.x & (R - 1)) * 4;
        lb0 = lo;
        lb1 = lo + 1u * 1024u * R;
        lb2 = lo + 2u * 1024u * R;
        lb3 = lo + 3u * 1024u * R;
    }
    __device__ __forceinline__ uint32_t ld(uint32_t off) const {
        return *reinterpret_cast<const uint32_t *>(base + off);
    }
    // lookup table k at byte (x >> sh) & 0xff; offsets of (idx << kShift) never overlap the lane bits
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        const uint32_t x = c ^ w;
        const uint32_t m = 0xffu << kShift;
        const uint32_t a3 = ((x << kShift) & m) | lb3;
        const uint32_t a2 = ((x >> (8 - kShift)) & m) | lb2;
        const uint32_t a1 = ((x >> (16 - kShift)) & m) | lb1;
        const uint32_t a0 = ((x >> (24 - kShift)) & m) | lb0;
        return ld(a3) ^ ld(a2) ^ ld(a1) ^ ld(a0);
    }
    __device__ __forceinline__ uint32_t step(uint32_t c) const {  // one byte via T0
        return (c >> 8) ^ ld(((c & 0xffu) << kShift) | lb0);
    }
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
    // fill all 4 tables (whole workgroup)
    static __device__ __forceinline__ void fill(uint32_t *T) {
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
            uint32_t t[4];
            t[0] = crc_table_entry(i);
#pragma unroll
            for (int k = 1; k < 4; k++) t[k] = (t[k - 1] >> 8) ^ crc_table_entry(t[k - 1] & 0xffu);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t *dst = T + (uint32_t)k * 256u * R + i * R;
#pragma unroll
                for (int r = 0; r < R; r++) dst[r] = t[k];
            }
        }
    }
};

// LDS by byte address: kernels that keep all their LDS in one __shared__ array (so that hipcc sees
// a single object) address tables and staging areas as byte offsets into it.
template <class T>
__device__ __forceinline__ uint32_t lds_addr(T *p) {
    return (uint32_t)(size_t)(__attribute__((address_space(3))) T *)p;
}
__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) {
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>((size_t)a);
}
template <class V>
__device__ __forceinline__ void lds_st(uint32_t a, V v) {
    *reinterpret_cast<__attribute__((address_space(3))) V *>((size_t)a) = v;
}

// Slice-by-4 tables T0..T3 with 8 replicas in 32 KiB of LDS: byte address (b << 7) | (k << 5) |
// (r << 2) for T_k[b], replica r.  Lane l reads replica l % 8, and the four lane octets of a 32-lane
// half take the four tables in rotated order (octet g's i-th lookup of a word is table (i + g) % 4),
// so one ds_read_b32 of a half touches banks (k << 3) | r -- 32 different banks for any data:
// conflict free like Crc4Perm at a quarter of its LDS.  One word = 4 x (bfe + shift-add + ds_read)
// + xors.
struct CrcR8 {
    static constexpr uint32_t kBytes = 32768;
    uint32_t tb;     // LDS byte address of the tables
    uint32_t sh[4];  // byte position of x that lookup i takes (8 * (3 - k))
    uint32_t ko[4];  // tb + table / replica offset of lookup i
    __device__ __forceinline__ explicit CrcR8(uint32_t tbase) : tb(tbase) {
        const uint32_t lane = threadIdx.x & 63, r = lane & 7, g = (lane >> 3) & 3;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t k = (i + g) & 3;
            sh[i] = 8 * (3 - k);
            ko[i] = tbase + ((k << 5) | (r << 2));
        }
    }
    __device__ __forceinline__ uint32_t look(uint32_t x, int i) const {
        return lds_ld32((__builtin_amdgcn_ubfe(x, sh[i], 8) << 7) + ko[i]);
    }
    // absorb one little-endian word (Go's crc32 slicing-by-4 step): c' = T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3]
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        const uint32_t x = c ^ w;
        return look(x, 0) ^ look(x, 1) ^ look(x, 2) ^ look(x, 3);
    }
    __device__ __forceinline__ uint32_t step(uint32_t c) const {  // one byte through T0 (k = 0)
        return (c >> 8) ^ lds_ld32(((c & 0xffu) << 7) + tb + ((threadIdx.x & 7u) << 2));
    }
    // absorb the low nb (0..4) bytes of x
    __device__ __forceinline__ uint32_t partial(uint32_t c, uint32_t x, uint32_t nb) const {
        if (nb >= 4) return word(c, x);
        c ^= x & ((1u << (8 * nb)) - 1u);
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t nx = step(c);
            c = s < nb ? nx : c;
        }
        return c;
    }
    // fill the 32 KiB at tbase (whole workgroup)
    static __device__ __forceinline__ void fill(uint32_t tbase) {
        typedef uint32_t v4 __attribute__((ext_vector_type(4)));
        for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) {
            const uint32_t k = t >> 8, b = t & 255;
            uint32_t v = crc_table_entry(b);
            for (uint32_t q = 0; q < k; q++) v = (v >> 8) ^ crc_table_entry(v & 0xffu);
            const uint32_t a = tbase + ((b << 7) | (k << 5));
            lds_st(a, v4{v, v, v, v});
            lds_st(a + 16, v4{v, v, v, v});
        }
    }
};

// Z_n(c) from an LDS shift table at byte address zt (4 x 256 words, S[k][i] = Z_n(i << 8k),
// bhg_crc_tables.h): the CRC state after n more zero bytes
__device__ __forceinline__ uint32_t zshift(uint32_t zt, uint32_t c) {
    return lds_ld32(zt + ((c & 0xffu) << 2)) ^ lds_ld32(zt + 1024 + (((c >> 8) & 0xffu) << 2)) ^
           lds_ld32(zt + 2048 + (((c >> 16) & 0xffu) << 2)) ^ lds_ld32(zt + 3072 + ((c >> 24) << 2));
}

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
// One lane walks its own range in windows of WIN x 16 B, loaded by WIN
// dword-aligned dwordx4 loads issued back to back so that a lane consumes
// whole cache lines while they are L1-resident (lanes of a wave walk
// different records: a 16 B-per-lane burst would cost one L2 request per
// 16 B).  PREFETCH keeps the next window in flight while absorbing.
template <int WIN, bool PREFETCH, class Tab>
__device__ __forceinline__ uint32_t crc_range_w(const Tab &T, uint32_t c, uint64_t p, uint64_t len, uint64_t end) {
    if (len == 0) return c;
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
    const uint64_t nw = len >> 2;
    const uint32_t tail = (uint32_t)(len & 3);
    const uint64_t a = p;
    constexpr uint32_t WW = 4 * WIN;  // words per window
    if (nw) {
        u32x4 cur[WIN], nxt[PREFETCH ? WIN : 1];
        auto load_win = [&](u32x4 *dst, uint64_t at) {
            if (at + 16 * WIN <= end) {
#pragma unroll
                for (int q = 0; q < WIN; q++) dst[q] = gld<u32x4_a4>(at + 16 * q);
            } else {
#pragma unroll
                for (int q = 0; q < WIN; q++)
                    dst[q] = u32x4{ld32_safe(at + 16 * q, end), ld32_safe(at + 16 * q + 4, end),
                                   ld32_safe(at + 16 * q + 8, end), ld32_safe(at + 16 * q + 12, end)};
            }
        };
        load_win(cur, a);
        for (uint64_t base = 0; base < nw; base += WW) {
            const bool more = base + WW < nw;
            if (PREFETCH && more) load_win(nxt, a + 4 * (base + WW));
            const uint64_t rem = nw - base;
            if (rem >= WW) {
#pragma unroll
                for (int q = 0; q < WIN; q++) {
                    c = T.word(c, cur[q].x); c = T.word(c, cur[q].y);
                    c = T.word(c, cur[q].z); c = T.word(c, cur[q].w);
                }
            } else {
#pragma unroll
                for (int q = 0; q < WIN; q++) {
                    if ((uint64_t)(4 * q + 0) < rem) c = T.word(c, cur[q].x);
                    if ((uint64_t)(4 * q + 1) < rem) c = T.word(c, cur[q].y);
                    if ((uint64_t)(4 * q + 2) < rem) c = T.word(c, cur[q].z);
                    if ((uint64_t)(4 * q + 3) < rem) c = T.word(c, cur[q].w);
                }
            }
            if (more) {
                if (PREFETCH) {
#pragma unroll
                    for (int q = 0; q < WIN; q++) cur[q] = nxt[q];
                } else {
                    load_win(cur, a + 4 * (base + WW));
                }
            }
        }
    }
    if (tail) c = T.partial(c, ld32_safe(a + 4 * nw, end), tail);
    return c;
}

// Same chain with windows aligned to 128 B lines: the WIN x 16 B window
// k covers [a0 + 16*WIN*k, +16*WIN) with a0 = (4-aligned start) & ~127, so a
// cache line is requested by exactly one window of one lane (an unaligned
// window straddles lines that are evicted before the next window asks for
// them: 2x HBM over-fetch measured).  Words outside [pa, pe) are masked off;
// the unaligned head/tail bytes are absorbed before/after the walk.
template <int WIN, class Tab, bool PF = false>
__device__ __forceinline__ uint32_t crc_range_a(const Tab &T, uint32_t c, uint64_t p, uint64_t len, uint64_t end) {
    if (len == 0) return c;
    const uint64_t pe_all = p + len;
    const uint64_t pa = (p + 3) & ~3ull;
    if (pa >= pe_all || pa + 4 > pe_all) {              // fewer than one aligned word: byte path
        uint64_t q = p;
        while (q < pe_all) {
            const uint64_t a = q & ~3ull;
            const uint32_t z = (uint32_t)(q & 3);
            uint32_t nb = 4 - z;
            if ((uint64_t)nb > pe_all - q) nb = (uint32_t)(pe_all - q);
            c = T.partial(c, ld32_safe(a, end) >> (8 * z), nb);
            q += nb;
        }
        return c;
    }
    if (pa != p) c = T.partial(c, ld32_safe(p & ~3ull, end) >> (8 * (uint32_t)(p & 3)), (uint32_t)(pa - p));
    const uint64_t pe = pe_all & ~3ull;                // end of full words
    constexpr uint32_t WB = 16 * WIN;
    auto load_win = [&](u32x4 *cur, uint64_t w) {
        if (w + WB <= end) {
#pragma unroll
            for (int q = 0; q < WIN; q++) cur[q] = gld<u32x4_a4>(w + 16 * q);
        } else {
#pragma unroll
            for (int q = 0; q < WIN; q++)
                cur[q] = u32x4{ld32_safe(w + 16 * q, end), ld32_safe(w + 16 * q + 4, end),
                               ld32_safe(w + 16 * q + 8, end), ld32_safe(w + 16 * q + 12, end)};
        }
    };
    const uint64_t w0 = pa & ~127ull;
    u32x4 cur[WIN], nxt[PF ? WIN : 1];
    if (w0 < pe) load_win(cur, w0);
    for (uint64_t w = w0; w < pe; w += WB) {
        const bool more = w + WB < pe;
        if (PF && more) load_win(nxt, w + WB);
        if (w >= pa && w + WB <= pe) {
#pragma unroll
            for (int q = 0; q < WIN; q++) {
                c = T.word(c, cur[q].x); c = T.word(c, cur[q].y);
                c = T.word(c, cur[q].z); c = T.word(c, cur[q].w);
            }
        } else {
#pragma unroll
            for (int q = 0; q < WIN; q++) {
                const uint64_t b = w + 16 * q;
                if (b + 0 >= pa && b + 0 < pe) c = T.word(c, cur[q].x);
                if (b + 4 >= pa && b + 4 < pe) c = T.word(c, cur[q].y);
                if (b + 8 >= pa && b + 8 < pe) c = T.word(c, cur[q].z);
                if (b + 12 >= pa && b + 12 < pe) c = T.word(c, cur[q].w);
            }
        }
        if (more) {
            if (PF) {
#pragma unroll
                for (int q = 0; q < WIN; q++) cur[q] = nxt[q];
            } else {
                load_win(cur, w + WB);
            }
        }
    }
    if (pe != pe_all) c = T.partial(c, ld32_safe(pe, end), (uint32_t)(pe_all - pe));
    return c;
}

template <class Tab>
__device__ __forceinline__ uint32_t crc_range(const Tab &T, uint32_t c, uint64_t p, uint64_t len, uint64_t end) {
    return crc_range_w<4, true>(T, c, p, len, end);
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
