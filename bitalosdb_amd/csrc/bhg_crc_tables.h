// bhg_crc_tables.h -- CRC-32C (Castagnoli, reflected 0x82F63B78) table math
// for the gfx950 decode kernels: the slice-by-4 lookup table laid out for
// one-VALU address generation, and "shift by n zero bytes" tables used to
// combine per-chunk CRCs of one record (the GF(2) linearity of the CRC:
// crc(A||B) = shift(crc(A), |B|) xor crc_0(B)).
//
// Reference semantics: internal/crc/crc.go:19-33 (Go hash/crc32 Castagnoli,
// state inverted on entry/exit, then masked).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bhg {

#define BHG_CRC32C_POLY 0x82F63B78u

__host__ __device__ __forceinline__ uint32_t crc32c_t0(uint32_t i) {
    uint32_t c = i;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ BHG_CRC32C_POLY : (c >> 1);
    return c;
}

// slice-by-4 table k (T_{k+1}[i] = T_k[i] >> 8 ^ T0[T_k[i] & 0xff])
__host__ __device__ __forceinline__ uint32_t crc32c_tk(uint32_t k, uint32_t i) {
    uint32_t t = crc32c_t0(i);
    for (uint32_t j = 0; j < k; j++) t = (t >> 8) ^ crc32c_t0(t & 0xffu);
    return t;
}

// ---------------------------------------------------------------------------
// Crc4Perm: slice-by-4 tables T0..T3, each replicated 32x, 128 KiB of LDS.
// Byte address of replica r of T_k[b]:
//     ((k >> 1) << 16) | (b << 8) | ((k & 1) << 7) | (r << 2)
// so one v_perm_b32 builds a lookup address: byte 1 <- the index byte of x,
// bytes 0 and 2 <- a per-lane constant holding (k & 1, r) and k >> 1.  Lane l
// reads replica l % 32: ds_read_b32 serves lanes in two groups of 32 with
// bank = (addr / 4) % 32 = r, so a random-index lookup is conflict free.
// One 4-byte step = 4 v_perm + 4 ds_read_b32 + xors.
// ---------------------------------------------------------------------------
struct Crc4Perm {
    static constexpr uint32_t kBytes = 128u * 1024u;
    static constexpr uint32_t kWords = kBytes / 4;
    const char *base;
    uint32_t lb[4];
    __device__ __forceinline__ explicit Crc4Perm(const uint32_t *T) : base(reinterpret_cast<const char *>(T)) {
        const uint32_t r = threadIdx.x & 31u;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) lb[k] = ((k >> 1) << 16) | ((k & 1u) << 7) | (r << 2);
    }
    // T_k[(x >> 8*byte) & 0xff]
    template <int K, int BYTE>
    __device__ __forceinline__ uint32_t look(uint32_t x) const {
        const uint32_t a = __builtin_amdgcn_perm(x, lb[K], 0x0c020000u | ((4u + BYTE) << 8));
        return *reinterpret_cast<const uint32_t *>(base + a);
    }
    // absorb one little-endian word: c' = T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3], x = c ^ w
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        const uint32_t x = c ^ w;
        return look<3, 0>(x) ^ look<2, 1>(x) ^ look<1, 2>(x) ^ look<0, 3>(x);
    }
    // word() on (w & keep), keep = 0 or ~0 per lane, with the state zeroed with it: one
    // 3-input bit op instead of the xor (the stream kernel's head-window padding)
    __device__ __forceinline__ uint32_t word_and(uint32_t c, uint32_t w, uint32_t keep) const {
        const uint32_t x = (c ^ w) & keep;
        return look<3, 0>(x) ^ look<2, 1>(x) ^ look<1, 2>(x) ^ look<0, 3>(x);
    }
    // absorb the low nb (0..3) bytes of x in ONE round of independent lookups
    // (slice-by-nb: T_{nb-1-i} for byte i of c ^ x)
    __device__ __forceinline__ uint32_t absorb_upto3(uint32_t c, uint32_t x, uint32_t nb) const {
        const uint32_t m = (1u << (8 * nb)) - 1u;  // nb <= 3
        const uint32_t y = c ^ (x & m);
        uint32_t r = nb ? (y >> (8 * nb)) : y;
#pragma unroll
        for (uint32_t i = 0; i < 3; i++) {
            const uint32_t k = nb > i ? nb - 1 - i : 0u;
            const uint32_t lbk = ((k >> 1) << 16) | ((k & 1u) << 7) | (lb[0] & 0x7cu);  // lb[0] & 0x7c = replica
            const uint32_t a = __builtin_amdgcn_perm(y, lbk, 0x0c020000u | ((4u + i) << 8));
            const uint32_t v = *reinterpret_cast<const uint32_t *>(base + a);
            r ^= nb > i ? v : 0u;
        }
        return r;
    }
    __device__ __forceinline__ uint32_t step(uint32_t c) const { return (c >> 8) ^ look<0, 0>(c); }
    // absorb the low nb (0..4) bytes of x
    __device__ __forceinline__ uint32_t partial(uint32_t c, uint32_t x, uint32_t nb) const {
        const uint32_t m = nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
        c ^= x & m;
#pragma unroll
        for (uint32_t s = 0; s < 4; s++) {
            const uint32_t nx = step(c);
            c = s < nb ? nx : c;
        }
        return c;
    }
    // whole workgroup fills the 128 KiB (1 (k, b) pair per thread and pass);
    // src (nullable, 1024 words k*256+b) replaces the plain slice tables,
    // e.g. with braid tables
    static __device__ __forceinline__ void fill(uint32_t *T, const uint32_t *src = nullptr) {
        for (uint32_t t = threadIdx.x; t < 1024u; t += blockDim.x) {
            const uint32_t k = t >> 8, b = t & 255u;
            const uint32_t v = src ? src[t] : crc32c_tk(k, b);
            const uint32_t a = ((k >> 1) << 16) | (b << 8) | ((k & 1u) << 7);
            typedef uint32_t v4 __attribute__((ext_vector_type(4)));
            v4 *d = reinterpret_cast<v4 *>(reinterpret_cast<char *>(T) + a);
            const v4 vv = {v, v, v, v};
#pragma unroll
            for (int j = 0; j < 8; j++) d[j] = vv;
        }
    }
};

// ---------------------------------------------------------------------------
// Zero-byte shift tables.  Z_n = the linear map "absorb n zero bytes" on the
// (inverted) CRC state.  Stored as 4 x 256 words: S[k][i] = Z_n(i << 8k), so
// Z_n(c) = S[0][c&255] ^ S[1][c>>8&255] ^ S[2][c>>16&255] ^ S[3][c>>24].
// Built on the host (matrix squaring) and copied into LDS by the kernels.
// ---------------------------------------------------------------------------
struct Gf2Mat {
    uint32_t col[32];  // image of bit i
};
inline uint32_t gf2_apply(const Gf2Mat &m, uint32_t v) {
    uint32_t r = 0;
    for (int i = 0; i < 32; i++)
        if (v >> i & 1u) r ^= m.col[i];
    return r;
}
inline Gf2Mat gf2_mul(const Gf2Mat &a, const Gf2Mat &b) {  // a after b
    Gf2Mat r;
    for (int i = 0; i < 32; i++) r.col[i] = gf2_apply(a, b.col[i]);
    return r;
}
inline Gf2Mat crc32c_zero_bytes(uint64_t n) {
    Gf2Mat one, acc;
    for (int i = 0; i < 32; i++) {
        const uint32_t v = 1u << i;
        one.col[i] = (v >> 8) ^ crc32c_t0(v & 0xffu);
        acc.col[i] = v;
    }
    while (n) {
        if (n & 1) acc = gf2_mul(one, acc);
        one = gf2_mul(one, one);
        n >>= 1;
    }
    return acc;
}
// Z_{-n}: the inverse map ("un-absorb n zero bytes").  The top byte of
// T0[i] is a bijection of i, which inverts one zero-byte step directly.
inline Gf2Mat crc32c_unzero_bytes(uint64_t n) {
    uint32_t top[256];
    for (uint32_t i = 0; i < 256; i++) top[crc32c_t0(i) >> 24] = i;
    Gf2Mat one, acc;
    for (int b = 0; b < 32; b++) {
        const uint32_t c1 = 1u << b;  // c1 = (c >> 8) ^ T0[c & 255]  ->  c
        const uint32_t idx = top[c1 >> 24];
        one.col[b] = ((c1 ^ crc32c_t0(idx)) << 8) | idx;
        acc.col[b] = c1;
    }
    while (n) {
        if (n & 1) acc = gf2_mul(one, acc);
        one = gf2_mul(one, one);
        n >>= 1;
    }
    return acc;
}
// out[1024]: the S table of a linear map
inline void gf2_table(const Gf2Mat &z, uint32_t *out) {
    for (uint32_t k = 0; k < 4; k++)
        for (uint32_t i = 0; i < 256; i++) out[k * 256 + i] = gf2_apply(z, i << (8 * k));
}
// out[1024]: the S table of Z_n
inline void crc32c_shift_table(uint64_t n, uint32_t *out) { gf2_table(crc32c_zero_bytes(n), out); }
// Braid table of stride F: T'_k[b] = Z_F(T_k[b]), k = 0..3, out[k*256 + b]
inline void crc32c_braid_table(uint64_t fold, uint32_t *out) {
    const Gf2Mat z = crc32c_zero_bytes(fold);
    for (uint32_t k = 0; k < 4; k++)
        for (uint32_t i = 0; i < 256; i++) out[k * 256 + i] = gf2_apply(z, crc32c_tk(k, i));
}

// Shift tables of the tile decode kernel (bhg_decode_tile.hip), in this order:
// Z_1024 (Horner step over 8 windows; also k_crc_long's base), Z_128, Z_256,
// Z_512 (window distance to the record end), Z_32 / Z_64 (fold of 4 / 2
// interleaved window chains).  Device copy owned by the context.
constexpr uint32_t kZTabWords = 6 * 1024;
inline void build_tile_ztab(uint32_t *out) {
    const uint64_t zs[6] = {1024, 128, 256, 512, 32, 64};
    for (uint32_t k = 0; k < 6; k++) crc32c_shift_table(zs[k], out + 1024 * k);
}

// Shift tables of the kernels built on CrcR8 (bhg_device.h): the pack kernel's chunk combine
// (Z_16 .. Z_1024, powers of two).  One device array owned by the context, 1024 words per table
// in this order.
enum XTab : uint32_t { XZ16, XZ32, XZ64, XZ128, XZ256, XZ512, XZ1024, XTAB_N };
constexpr uint64_t kXTabLen[XTAB_N] = {16, 32, 64, 128, 256, 512, 1024};
// then the long-range checksum's chain folds and span combine (k_crc_long_part / _join,
// bhg_decode.hip): Z_{2^(kXLongLo + j)}, j = 0 .. kXLongN - 1 (64 B .. 2 GiB), from word kXLong on
constexpr uint32_t kXLongLo = 6, kXLongN = 26;
constexpr uint32_t kXLong = XTAB_N * 1024;
constexpr uint32_t kXTabWords = kXLong + kXLongN * 1024;
inline void build_xtab(uint32_t *out) {
    for (uint32_t k = 0; k < XTAB_N; k++) crc32c_shift_table(kXTabLen[k], out + 1024 * k);
    for (uint32_t j = 0; j < kXLongN; j++) crc32c_shift_table(1ull << (kXLongLo + j), out + kXLong + 1024 * j);
}

// Shift tables of the LDS-DMA ring decode (lab: scripts/lab/c2_r5/decode_ring.hip), in this order: Z_32 and Z_68 (the
// folds of a 136-B window's four chains), then Z_{136 * 2^k}, k = 0..3 (136 .. 1,088 B): a lane's
// distance to the record end (k = 0..2), the Horner step over 8 windows (Z_1088), and the head's
// shift past m - 1 windows by the bits of m - 1 (bits above 3 as repeated Z_1088).
constexpr uint32_t kRingZN = 6;
inline void build_ring_ztab(uint32_t *out) {
    crc32c_shift_table(32, out);
    crc32c_shift_table(68, out + 1024);
    for (uint32_t k = 0; k < 4; k++) crc32c_shift_table(136ull << k, out + 1024 * (k + 2));
}

}  // namespace bhg
