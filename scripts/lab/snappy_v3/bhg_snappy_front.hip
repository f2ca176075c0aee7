// bhg_snappy_front.hip -- first pass of the SnappyCompressor batch decode:
// everything but the value bytes, reading each record from HBM once.
//
// Per block: readRecordHeader / readRecord / readKV + FNV-1 (bithash/
// block2.go:31-66, internal/hash/fnv.go:19-23), the masked CRC-32C of the
// whole record (internal/crc/crc.go:19-33), snappy's
// decodedLen (the sizes the output-offset scan needs), and the tag walk of
// golang/snappy's decode (compress.go:83-85), which turns the block into the
// 16-byte copy ops k_snappy_mat replays (bhg_snappy_parse.h).
//
// A wave takes tiles of 64 consecutive handles, lane = record (the next
// tile's handles and expected CRCs are loaded while a tile is processed):
//   1. the record -> the wave's LDS arena, regions 16-B aligned and laid out
//      by a wave prefix sum of the record sizes (a tile whose records do not
//      fit in one arena runs in several rounds; a record larger than the
//      arena takes the slow path below);
//   2. header, key and trailer from the region's first 64 bytes; decodedLen;
//   3. one loop runs two independent chains per lane: the CRC (8 bytes per
//      iteration, slice-by-8 tables in LDS) and the tag walk (one element per
//      iteration), so each chain's LDS latency hides behind the other's work;
//   4. descriptor, decoded size, op count / mode, ops.
// Every LDS access is aligned to its width (a misaligned 8- or 16-byte access
// is replayed at 64 cycles per instruction).  Slow path (record > arena):
// header and CRC from global memory, no walk; k_snappy_rt decodes the value.
//
// LDS: 8 KiB of tables + 4 x 37.5 KiB arenas per workgroup of 4 waves, one
// workgroup per CU.  At C3 (578-B records) a tile is 64 x ~592 B = 37 KiB.
#include "bhg_device.h"
#include "bhg_internal.h"
#include "bhg_snappy_parse.h"

namespace bhg {

namespace {

constexpr uint32_t kFrontWaves = 4;
constexpr uint32_t kFrontArena = 38400;  // bytes per wave: 64 C3 records (578 B, regions rounded to 16 B)
constexpr uint32_t kFrontBatch = 24;     // 16-B staging loads in flight per lane

// slice-by-8 CRC-32C (reflected Castagnoli) tables, one copy in LDS: T_0 is the
// byte table, T_{k+1}[i] = T_k[i] >> 8 ^ T_0[T_k[i] & 0xff]
struct Crc8Lds {
    const uint32_t *T;
    __device__ __forceinline__ explicit Crc8Lds(const uint32_t *t) : T(t) {}
    static __device__ __forceinline__ void fill(uint32_t *T) {  // whole workgroup, ends with a barrier
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) T[i] = crc_table_entry(i);
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
            uint32_t t = T[i];
#pragma unroll
            for (int k = 1; k < 8; k++) {
                t = (t >> 8) ^ T[t & 0xffu];
                T[k * 256 + i] = t;
            }
        }
        __syncthreads();
    }
    __device__ __forceinline__ uint32_t dword2(uint32_t c, uint32_t w0, uint32_t w1) const {
        const uint32_t x = c ^ w0;
        return T[7 * 256 + (x & 255u)] ^ T[6 * 256 + ((x >> 8) & 255u)] ^ T[5 * 256 + ((x >> 16) & 255u)] ^
               T[4 * 256 + (x >> 24)] ^ T[3 * 256 + (w1 & 255u)] ^ T[2 * 256 + ((w1 >> 8) & 255u)] ^
               T[256 + ((w1 >> 16) & 255u)] ^ T[w1 >> 24];
    }
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        const uint32_t x = c ^ w;
        return T[3 * 256 + (x & 255u)] ^ T[2 * 256 + ((x >> 8) & 255u)] ^ T[256 + ((x >> 16) & 255u)] ^ T[x >> 24];
    }
    __device__ __forceinline__ uint32_t byte(uint32_t c, uint32_t b) const { return (c >> 8) ^ T[(c ^ b) & 255u]; }
};

typedef u32x4 u32x4u __attribute__((aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef u32x2 u32x2u __attribute__((aligned(1)));
typedef u32x4 u32x4_lds __attribute__((aligned(16), may_alias));
typedef uint64_t u64_lds __attribute__((aligned(8), may_alias));
typedef uint32_t u32_lds __attribute__((may_alias));

// 16 bytes at a, bytes at or past `end` read as 0
__device__ __forceinline__ u32x4 ld16_end(uint64_t a, uint64_t end) {
    if (a + 16 <= end) return gld<u32x4u>(a);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < 16; b++)
        if (a + b < end) w[b >> 2] |= (uint32_t)gld<uint8_t>(a + b) << (8 * (b & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

// masked-CRC chain over [a, a + len) straight from global memory (the slow path)
__device__ __forceinline__ uint32_t crc_global(const Crc8Lds &T, uint32_t c, uint64_t a, uint32_t len) {
    uint32_t q = 0;
    for (; q + 8 <= len; q += 8) {
        const u32x2 w = gld<u32x2u>(a + q);
        c = T.dword2(c, w.x, w.y);
    }
    for (; q < len; q++) c = T.byte(c, gld<uint8_t>(a + q));
    return c;
}

}  // namespace

// meta[i]: mode (bits 0-1), body corrupt (bit 2), op count (bits 8-31)
__global__ __launch_bounds__(64 * kFrontWaves) void k_snappy_front(
    const uint8_t *__restrict__ src, uint64_t src_len, const bhg_handle *__restrict__ handles, uint32_t n,
    const uint32_t *__restrict__ expected_crc, bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes,
    uint32_t *__restrict__ meta, uint16_t *__restrict__ ops, uint32_t *__restrict__ list) {
    __shared__ __attribute__((aligned(16))) uint32_t T[8 * 256];
    __shared__ __attribute__((aligned(16))) uint8_t arenas[kFrontWaves][kFrontArena + 64];  // + 64: over-reads
    Crc8Lds::fill(T);
    const Crc8Lds crc(T);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t *const arena = arenas[wv];
    const u32_lds *const A32 = reinterpret_cast<const u32_lds *>(arena);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const bool walk = ops != nullptr;
    const bool tiny = src_len < 16;  // (uniform) staging loads assembled from bytes
    const uint32_t tstride = gridDim.x * kFrontWaves;
    uint32_t tile = blockIdx.x * kFrontWaves + wv;
    // the next tile's handle and expected CRC are in flight while a tile is processed
    // (unconditional loads, index clamped: no branch for the compiler to wait at)
    bhg_handle hn;
    uint32_t en;
    auto fetch = [&](uint32_t t) {
        const uint32_t j = t * 64 + lane, jc = t < ntiles && j < n ? j : n - 1;
        hn = handles[jc];
        en = expected_crc != nullptr ? expected_crc[jc] : 0u;
    };
    fetch(tile);
    for (; tile < ntiles; tile += tstride) {
        const bhg_handle h = hn;
        const uint32_t e0 = en;
        fetch(tile + tstride < ntiles ? tile + tstride : tile);
        const uint32_t i = tile * 64 + lane;
        const bool valid = i < n;
        uint32_t st = BHG_ST_OK;
        bool inb = false;
        if (valid) {
            if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;                    // reader.go:234-236
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset)
                st = BHG_ST_INCOMPLETE;                                       // reader.go:251-258
            else inb = true;
        }
        const uint32_t L = inb ? h.length : 0u;
        const uint64_t p = base + (inb ? h.offset : 0ull);
        const uint32_t ecrc = valid ? e0 : 0u;
        const uint32_t need = (L + 15u) & ~15u;
        const bool slow = inb && need > kFrontArena;
        bool pend = inb && !slow;
        uint32_t rw[16];  // the record's first 64 bytes (rw[t] = bytes 4t..4t+3; bytes past L are unused)
#pragma unroll
        for (int t = 0; t < 16; t++) rw[t] = 0;
        uint32_t c = 0xffffffffu;  // crc.New: Go starts from ^0
        uint64_t dsize = 0;
        uint32_t mode = SNAP_SKIP, corrupt = 0, nops = 0;
        bool dl_ok = false;
        // ---- staging rounds: a lane's record at a 16-B aligned region of the arena
        while (__ballot(pend) != 0) {
            const uint32_t x = pend ? need : 0u;
            const uint32_t R = wave_incl_add(x) - x;
            const bool go = pend && R + need <= kFrontArena;
            const uint32_t nch = go ? need >> 4 : 0u;
            const uint32_t maxch = __builtin_amdgcn_readlane(wave_incl_max(nch), 63);
            for (uint32_t t0 = 0; t0 < maxch; t0 += kFrontBatch) {
                u32x4 buf[kFrontBatch];
#pragma unroll
                for (uint32_t j = 0; j < kFrontBatch; j++) {  // all loads first, unconditional (clamped into src)
                    const uint64_t a = t0 + j < nch ? p + 16 * (t0 + j) : base;
                    buf[j] = tiny ? ld16_end(a, end) : gld<u32x4u>(a + 16 <= end ? a : end - 16);
                }
#pragma unroll
                for (uint32_t j = 0; j < kFrontBatch; j++) {
                    if (t0 + j < nch) {
                        const uint64_t a = p + 16 * (t0 + j);
                        u32x4 cv = buf[j];
                        if (!tiny && a + 16 > end) {  // loaded from end - 16: its bytes start at a - (end - 16)
                            const uint32_t sh = (uint32_t)(a - (end - 16));
                            unsigned __int128 y = (unsigned __int128)cv.x | ((unsigned __int128)cv.y << 32) |
                                                  ((unsigned __int128)cv.z << 64) | ((unsigned __int128)cv.w << 96);
                            y >>= 8 * sh;
                            cv = u32x4{(uint32_t)y, (uint32_t)(y >> 32), (uint32_t)(y >> 64), (uint32_t)(y >> 96)};
                        }
                        *reinterpret_cast<u32x4_lds *>(arena + R + 16 * (t0 + j)) = cv;
                    }
                }
            }
            lds_wave_sync();
            // head words, the walk set-up (decodedLen), then the CRC and the tag walk in one loop
            SnapParse S;
            S.s = S.se = S.sb = 0; S.d = 0; S.dlen = 0; S.nops = 0; S.res = 0; S.t8 = 0;
            bool par = false;
            if (go) {
#pragma unroll
                for (int t = 0; t < 16; t++) rw[t] = A32[(R >> 2) + t];
                const uint32_t k = L >= 12 ? rw[0] : 0u, v = L >= 12 ? rw[1] : 0u;
                const bool rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
                if (rvalid) {  // snappy decodedLen (golang/snappy decode.go, binary.Uvarint)
                    const uint32_t vb = R + 12u + k;
                    uint64_t xx = 0;
                    uint32_t sh = 0, hdr = 0;
                    for (uint32_t b = 0; b < 10 && b < v; b++) {
                        const uint32_t cb = arena[vb + b];
                        if (cb < 0x80) {
                            dl_ok = !(b == 9 && cb > 1);
                            xx |= (uint64_t)cb << sh;
                            dl_ok = dl_ok && xx <= 0xffffffffull;
                            hdr = b + 1;
                            break;
                        }
                        xx |= (uint64_t)(cb & 0x7f) << sh;
                        sh += 7;
                    }
                    // a stream cannot expand more than 64/3 x (a 3-byte copy emits 64 bytes)
                    dl_ok = dl_ok && xx * 3 <= (uint64_t)(v - hdr) * 64;
                    dsize = dl_ok ? xx : 0;
                    if (dl_ok) {
                        mode = SNAP_GLOBAL;
                        if (walk && xx <= kSnapMaxOut && v <= kSnapMaxStream) {
                            S.s = vb + hdr;
                            S.se = vb + v;
                            S.sb = vb;
                            S.dlen = (uint32_t)xx;
                            S.t8 = snap_ld8(arena, S.s);
                            par = S.s < S.se;
                            mode = SNAP_OPS;
                        }
                    }
                }
            }
            const uint32_t nw = go ? L >> 2 : 0u;
            uint32_t cw = 0;
            bool crc_on = go;
            uint16_t *const opp = walk ? ops + (uint64_t)i * kSnapOpCap : nullptr;
            while (__ballot(crc_on || par) != 0) {
                if (crc_on) {
                    if (cw + 2 <= nw) {
                        const uint64_t y = *reinterpret_cast<const u64_lds *>(arena + R + 4 * cw);
                        c = crc.dword2(c, (uint32_t)y, (uint32_t)(y >> 32));
                        cw += 2;
                    } else {
                        if (cw < nw) c = crc.word(c, A32[(R >> 2) + cw]);
                        for (uint32_t b = nw * 4; b < L; b++) c = crc.byte(c, arena[R + b]);
                        crc_on = false;
                    }
                }
                if (par)
                    par = snap_parse_step(arena, S, [&](uint32_t q, uint32_t op, bool on) {
                        if (on && q < kSnapOpCap) opp[q] = (uint16_t)op;
                    });
            }
            if (go && mode == SNAP_OPS) {
                const uint32_t r = S.res ? S.res : (S.d == S.dlen ? 0u : 1u);
                if (r == 0 && S.nops > kSnapOpCap) mode = SNAP_GLOBAL;  // too many ops: k_snappy_rt
                else if (r == 1) corrupt = 1;
                nops = S.nops;
            }
            lds_wave_sync();
            pend = pend && !go;
        }
        const uint32_t k = L >= 12 ? rw[0] : 0u, v = L >= 12 ? rw[1] : 0u, fn = L >= 12 ? rw[2] : 0u;
        const bool rvalid = inb && L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;  // block2.go:57-66
        const uint32_t cpos = 12u + k;
        if (slow) {  // a record larger than the arena: from global memory, decoded by k_snappy_rt
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = ld16_end(p + 16 * q, end);
                rw[4 * q] = x.x; rw[4 * q + 1] = x.y; rw[4 * q + 2] = x.z; rw[4 * q + 3] = x.w;
            }
            c = crc_global(crc, c, p, L);
        }
        const uint32_t ks = slow ? rw[0] : k, vs = slow ? rw[1] : v;
        const bool rv = slow ? (L >= 12 && ks != 0 && vs != 0 && (uint64_t)12 + ks + vs == (uint64_t)L) : rvalid;
        if (slow && rv) {  // decodedLen from global memory
            uint64_t xx = 0;
            uint32_t sh = 0, hdr = 0;
            const uint64_t vp = p + 12 + ks;
            for (uint32_t b = 0; b < 10 && b < vs; b++) {
                const uint32_t cb = gld<uint8_t>(vp + b);
                if (cb < 0x80) {
                    dl_ok = !(b == 9 && cb > 1);
                    xx |= (uint64_t)cb << sh;
                    dl_ok = dl_ok && xx <= 0xffffffffull;
                    hdr = b + 1;
                    break;
                }
                xx |= (uint64_t)(cb & 0x7f) << sh;
                sh += 7;
            }
            dl_ok = dl_ok && xx * 3 <= (uint64_t)(vs - hdr) * 64;
            dsize = dl_ok ? xx : 0;
            mode = dl_ok ? SNAP_GLOBAL : SNAP_SKIP;
        }
        (void)cpos;
        if (!valid) continue;
        // ---- readRecord / readKV (block2.go:38-66) + descriptor
        const uint32_t kk = slow ? ks : k, fnn = slow ? rw[2] : fn;
        uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = st;
        uint64_t dtr = 0;
        if (inb) {
            dcrc = crc_mask(~c);  // crc.go:31-33
            if (rv) {
                uint32_t key_len = 0, fnv = BHG_FNV_OFFSET;
                uint64_t trailer = 255;  // InternalKeyKindInvalid when ikeySize < 8
                if (kk >= 8) {           // readKV / DecodeInternalKey
                    key_len = kk - 8;
                    if (key_len <= 36) {
                        uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                        for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                            for (uint32_t b = 0; b < 4; b++) {
                                const uint32_t h2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * b)) & 0xffu);
                                hh = 4 * (t - 3) + b < key_len ? h2 : hh;
                            }
                        fnv = hh;
                        const uint32_t tb = 12 + key_len, tw = tb >> 2, ts = tb & 3;
                        uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                        for (uint32_t u = 3; u <= 12; u++) {  // tb <= 48: the trailer ends by byte 56
                            a0 = tw == u ? rw[u] : a0;
                            a1 = tw == u ? rw[u + 1] : a1;
                            a2 = tw == u ? rw[u + 2] : a2;
                        }
                        trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                                  ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                    } else {
                        fnv = fnv1_range(p + 12, key_len, end);
                        trailer = ldu64(p + 12 + kk - 8, end);
                    }
                }
                dk = 12; dkl = key_len; dtr = trailer; dfn = fnn; dfnv = fnv;
                if (!dl_ok) {
                    dst = BHG_ST_SNAPPY_CORRUPT;
                    mode = SNAP_SKIP;
                    dsize = 0;
                } else {
                    dvl = (uint32_t)dsize;  // provisional: the materialiser finalises
                    dvo = 12 + kk;          // provisional: compressed payload offset
                }
                if (expected_crc != nullptr && dst == BHG_ST_OK && ecrc != dcrc) dst = BHG_ST_CRC_MISMATCH;
            } else {
                dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil (reader.go:260-264)
                mode = SNAP_SKIP;
            }
        }
        uint2 *o = reinterpret_cast<uint2 *>(out + i);
        o[0] = make_uint2(dk, dkl);
        o[1] = make_uint2(dvo, dvl);
        o[2] = make_uint2((uint32_t)dtr, (uint32_t)(dtr >> 32));
        o[3] = make_uint2(dfn, dfnv);
        o[4] = make_uint2(dcrc, dst);
        sizes[i] = dsize;
        if (walk) {
            meta[i] = mode | (corrupt << 2) | (nops << 8);
            if (mode == SNAP_GLOBAL && list != nullptr) {
                const uint32_t q = atomicAdd(list, 1u);
                list[1 + q] = i;
            }
        }
    }
}

hipError_t launch_snappy_front(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                               const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes, uint32_t *meta,
                               uint16_t *ops, uint32_t *list) {
    const uint32_t tiles = (n + 63) / 64;
    const uint32_t groups = (tiles + kFrontWaves - 1) / kFrontWaves;
    static const uint32_t per_cu = resident_per_cu((const void *)k_snappy_front, 64 * kFrontWaves, 1);
    const uint32_t cap = (uint32_t)L.num_cus * (per_cu ? per_cu : 1u);
    uint32_t grid = groups < cap ? groups : cap;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_snappy_front), dim3(grid), dim3(64 * kFrontWaves), 0, L.stream, src, src_len, h, n,
                       expected_crc, out, sizes, meta, ops, list);
    return hipGetLastError();
}

}  // namespace bhg
