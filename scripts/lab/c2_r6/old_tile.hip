// bhg_decode_tile.hip -- default uncompressed decode kernel for gfx950.
//
// k_decode_tile: the NoCompressor batch decode (readRecord + readKV + FNV-1 +
// masked CRC-32C; bithash/block2.go:31-66, compress.go:57-59,
// internal/hash/fnv.go:19-23, internal/crc/crc.go:19-33) with the record
// bytes read as 128-B windows, eight lanes per record, so that a wave's
// loads in one round are one contiguous ~8.6 KB run of the table (the
// lane-per-record walk of k_decode_lane reads 64 records' 1 KB strides at
// once; its misaligned per-lane windows cost 1.17x HBM over-fetch and a
// 0.22 ms load floor at C2).
//
// A wave takes tiles of 64 consecutive handles:
//   phase 1, lane = record: handle, status, the record head [0, hl) with
//     hl = L - 128 (m-1) in 1..128 (m = ceil(L / 128)), the 12-B header,
//     UserKey, trailer.  All 64 lanes compute the head CRC (from
//     0xFFFFFFFF), the readRecord checks, FNV-1 and the trailer.
//   phase 2, 8 rounds of 8 records: lane (r, j) = (lane / 8, lane % 8) CRCs
//     the full windows q = m-1-j, m-1-j-8, ... (>= 1) of record 8s + r --
//     132-B loads from a 4-aligned address, the next round's loads issued
//     before this round is absorbed.  A window's CRC (from state 0) runs as
//     four interleaved 32-B chains folded with Z_32; windows are
//     Horner-folded with Z_1024 (8 windows), starting from the head CRC on
//     lane j == (m-1) % 8.  Linearity of CRC over GF(2):
//         crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B),
//     so record state = sum_j Z_{128 j}(acc_j): three conditional table
//     steps (Z_128, Z_256, Z_512) and a 3-step xor butterfly over the 8 lanes.
//
// The CRC tables are Crc4Perm (slice-by-4, replicated 32x: conflict free,
// v_perm addressing) plus five 4-KiB Z tables copied from the context.
// 148 KiB of LDS -> one 512-thread workgroup per CU, 2 waves per SIMD.
#include "../../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../../bitalosdb_amd/csrc/bhg_device.h"
#include "../../../bitalosdb_amd/csrc/bhg_internal.h"

// bit 0 / bit 1: the next tile's head words 0..15 / round-0 windows loaded in round 7 of the
// current tile.  Measured on the C2 layout (profiles/r4/pf_lab_tile_prefetch.txt, medians of
// 2 x 60): PF 0 / 1 / 2 / 3 = 0.254 / 0.366 / 0.251 / 0.346 ms -- bit 1 reuses the free window
// buffer (189 VGPRs), bit 0 keeps 16 more words live across the loop and spills (256 + scratch).
constexpr int kTilePfOld = 2;

constexpr int kTileNchOld = 2;  // CRC chains per window, measured: 1 / 2 / 4 chains 0.2455 / 0.2413 / 0.2445 ms (scripts/lab/run_tilevar.sh)

namespace bhg_old {
using namespace bhg;

namespace {

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint32_t zapply(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

}  // namespace

// NCH: interleaved CRC chains per 128-B window (1, 2 or 4), folded with Z_{128/NCH}.  With
// 2 waves per SIMD and a round's loads in flight, one chain's 32 dependent steps hide behind
// memory; every fold costs a conflicted shift-table lookup.
// NB: window buffers per wave -- 2: round s+1's loads in flight while round s is absorbed (the
// product, 8 waves per CU); 1: round s+1 is requested after round s is absorbed, the latency hidden
// by more waves per CU instead (lab: scripts/lab/c2_r6/, no gain).
// LONG: records longer than kLongRec get no CRC here -- their descriptors are written with crc 0
// and an unchecked status, and the long-record pass (bhg_longcrc.hip) computes the CRC with the
// whole chip and completes them.  The dispatch picks LONG = 1 for batches of long records only
// (launch_decode_tile), so the C2 instantiation is the same code as before.
template <int WPB, int NCH, int PF, int NB = 2, int LONG = 0>
__global__ __launch_bounds__(64 * WPB) void k_decode_tile(const uint8_t *__restrict__ src, uint64_t src_len,
                                                          const bhg_handle *__restrict__ handles, uint32_t n,
                                                          const uint32_t *__restrict__ expected_crc,
                                                          bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Z[kZTabWords];  // Z1024, Z128, Z256, Z512, Z32, Z64
    static_assert(NCH == 1 || NCH == 2 || NCH == 4, "chains per window");
    const uint32_t *Zf = Z + (NCH == 4 ? 4096 : 5120);  // fold table Z_{128 / NCH}
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63, rr = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    // wave-major tile index: the waves that take one tile more than the others
    // (ntiles mod tstride of them) are spread over every CU, not packed on the first ones
    uint32_t tile = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    bhg_handle hn = {0, 0, 0};
    if (tile < ntiles && tile * 64 + lane < n) hn = handles[tile * 64 + lane];
    // a record's geometry from its handle: Reader.readData's checks (reader.go:234-258), the
    // window count m = ceil(L / 128) and the head length hl = L - 128 (m-1) in 1..128
    struct Geo {
        uint64_t p;
        uint32_t st, L, m, hl;
        bool inb;
    };
    auto geo = [&](const bhg_handle &h, bool valid) {
        Geo g;
        g.st = BHG_ST_OK;
        g.inb = false;
        if (valid) {
            if (h.length == 0) g.st = BHG_ST_ILLEGAL_LENGTH;                  // reader.go:234-236
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset)
                g.st = BHG_ST_INCOMPLETE;                                     // reader.go:251-258
            else g.inb = true;
        }
        g.L = g.inb ? h.length : 0u;
        g.p = base + h.offset;
        g.m = g.inb ? (g.L + 127) / 128 : 1u;
        g.hl = g.L - 128 * (g.m - 1);
        return g;
    };
    // the record head [p & ~3, +132): words 0..15, then 16..32 when hl > 60
    auto load_head_lo = [&](uint32_t *hw, const Geo &g) {
        const uint64_t ha = g.p & ~3ull;
        if (!g.inb) return;
        if (ha + 132 <= end) {
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; t++) hw[t] = ld32_safe(ha + 4 * t, end);
        }
    };
    auto load_head_hi = [&](uint32_t *hw, const Geo &g) {
        const uint64_t ha = g.p & ~3ull;
        if (!g.inb) return;
        if (g.hl > 60) {
            if (ha + 132 <= end) {
#pragma unroll
                for (int t = 4; t < 8; t++) {
                    const u32x4 v = gld<u32x4_a4>(ha + 16 * t);
                    hw[4 * t] = v.x; hw[4 * t + 1] = v.y; hw[4 * t + 2] = v.z; hw[4 * t + 3] = v.w;
                }
                hw[32] = gld<uint32_t>(ha + 128);
            } else {
#pragma unroll
                for (int t = 16; t < 33; t++) hw[t] = ld32_safe(ha + 4 * t, end);
            }
        } else {
#pragma unroll
            for (int t = 16; t < 33; t++) hw[t] = 0;
        }
    };
    // round s's window plan for lane (rr, j): record 8s + rr of the tile whose geometry the lanes hold
    auto rinfo = [&](uint32_t s, const Geo &g, uint64_t &wb, uint32_t &mm, int32_t &qf, int32_t &q0, bool &hasw) {
        const uint32_t sl = 8 * s + rr;
        const uint32_t Lr = __shfl(g.L, sl, 64);
        const uint64_t pr = shfl_u64(g.p, sl);
        mm = __shfl(g.m, sl, 64);
        wb = pr + (Lr - 128 * (mm - 1));  // start of window 1
        q0 = (int32_t)(mm - 1) - (int32_t)j;
        hasw = Lr != 0 && q0 >= 1 && !(LONG && Lr > kLongRec);
        qf = q0 >= 1 ? (int32_t)(((uint32_t)q0 - 1) % 8 + 1) : 0;
    };
    auto load_win = [&](uint32_t *w, uint64_t wb, int32_t q) {
        const uint64_t a = (wb + 128ull * (uint32_t)(q - 1)) & ~3ull;
        if (a + 132 <= end) {
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const u32x4 x = gld<u32x4_a4>(a + 16 * t);
                w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
            }
            w[32] = gld<uint32_t>(a + 128);
        } else {
#pragma unroll
            for (int t = 0; t < 33; t++) w[t] = ld32_safe(a + 4 * t, end);
        }
    };
    uint32_t hw[33];
    uint32_t fw[NB][33];
    uint64_t wb = 0;
    uint32_t mm = 1;
    int32_t qf = 0, q0 = 0;
    bool hasw = false;
    if (PF != 0 && tile < ntiles) {  // the first tile's prefetched part; later tiles' come from round 7
        const Geo g0 = geo(hn, tile * 64 + lane < n);
        if (PF & 1) load_head_lo(hw, g0);
        if (PF & 2) {
            rinfo(0, g0, wb, mm, qf, q0, hasw);
            if (hasw) load_win(fw[0], wb, qf);
        }
    }
    // the LDS tables are built while the first tile's handles and round-0 windows are in flight
    // (kernel frac 0.6021 vs 0.5989 with the tables first, 3 alternating runs each,
    // profiles/r4/early_lab_table_fill.txt)
    Crc4Perm::fill(T);
    {  // all loads issued before the first LDS store (one memory round trip)
        constexpr uint32_t NT = 64 * WPB, NZ = (kZTabWords + NT - 1) / NT;
        uint32_t v[NZ];
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++) v[r] = threadIdx.x + r * NT < kZTabWords ? gz[threadIdx.x + r * NT] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++)
            if (threadIdx.x + r * NT < kZTabWords) Z[threadIdx.x + r * NT] = v[r];
    }
    __syncthreads();
    for (; tile < ntiles; tile += tstride) {
        // ---------------- phase 1: lane = record (Reader.readData's checks, readRecord, readKV)
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        const uint32_t tn = tile + tstride;
        if (tn < ntiles && tn * 64 + lane < n) hn = handles[tn * 64 + lane];
        const bool valid = i < n;
        // requested here, used after phase 2: a load issued at the end would expose its latency per tile
        const uint32_t ecrc = (expected_crc != nullptr && valid) ? expected_crc[i] : 0u;
        const Geo g = geo(h, valid);
        const uint32_t st = g.st, L = g.L, m = g.m, hl = g.hl;
        const uint64_t p = g.p;
        const bool inb = g.inb;
        const uint32_t hsh = (uint32_t)(p & 3);
        uint32_t mycrc = 0;
        if (!(PF & 1)) load_head_lo(hw, g);
        load_head_hi(hw, g);
        if (!(PF & 2)) {
            // round 0's windows are requested here, before phase 1's CRC / FNV-1 work, so that
            // work overlaps their memory latency
            rinfo(0, g, wb, mm, qf, q0, hasw);
            if (hasw) load_win(fw[0], wb, qf);
        }
        uint32_t hcrc = 0xffffffffu;  // crc.New: Go's crc32.Update starts from ^0
        uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
        uint64_t trailer = 255;       // InternalKeyKindInvalid when ikeySize < 8
        bool rvalid = false;
        if (inb) {
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 32; u++)
                if (u < nw) hcrc = crc.word(hcrc, __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh));
            if (hl & 3) {
                uint32_t wv = 0, wn = 0;
#pragma unroll
                for (uint32_t u = 0; u < 32; u++) {
                    wv = nw == u ? hw[u] : wv;
                    wn = nw == u ? hw[u + 1] : wn;
                }
                hcrc = crc.partial(hcrc, __builtin_amdgcn_alignbyte(wn, wv, hsh), hl & 3);
            }
            uint32_t rw[14];
#pragma unroll
            for (int u = 0; u < 14; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            // readRecordHeader (block2.go:31-36) + readRecord's length check (:57-66)
            k = L >= 12 ? rw[0] : 0u;
            v = L >= 12 ? rw[1] : 0u;
            fn = L >= 12 ? rw[2] : 0u;
            rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
            if (rvalid && k >= 8) {  // readKV / DecodeInternalKey (block2.go:38-55)
                key_len = k - 8;
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
                    for (uint32_t u = 3; u <= 12; u++) {  // tb <= 48: the trailer ends by byte 56 = rw[13]
                        a0 = tw == u ? rw[u] : a0;
                        a1 = tw == u ? rw[u + 1] : a1;
                        if (u + 2 < 14) a2 = tw == u ? rw[u + 2] : a2;  // tw == 12 only with ts == 0
                    }
                    trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                              ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                } else {
                    fnv = fnv1_range(p + 12, key_len, end);
                    trailer = ldu64(p + 12 + k - 8, end);
                }
            }
        }
        // the head lane of phase 2 (j == (m-1) % 8) owns windows iff m >= 9; its first Horner step
        // applies Z_1024 to the head CRC, done here once per record
        const uint32_t hz = m >= 9 ? zapply(Z, hcrc) : hcrc;
        // ---------------- phase 2: 8 rounds; lane (rr, j) on record 8s + rr
#pragma unroll
        for (uint32_t s = 0; s < 8; s++) {
            const uint32_t cb = NB == 2 ? (s & 1) : 0u;
            const uint64_t wb_c = wb;
            const uint32_t mm_c = mm;
            const int32_t qf_c = qf, q0_c = q0;
            const bool hasw_c = hasw;
            // the next round's loads: before this round's absorb (NB 2, into the other buffer) or
            // after it (NB 1, into the same buffer)
            auto next_loads = [&]() {
                if (s + 1 < 8) {
                    rinfo(s + 1, g, wb, mm, qf, q0, hasw);
                    if (hasw) load_win(fw[NB - 1 - cb], wb, qf);
                } else if (PF != 0 && tn < ntiles) {
                    // the next tile's record heads (into hw, dead since phase 1) and / or its round-0
                    // windows (into the free buffer), in flight across this round and the stores
                    const Geo gn = geo(hn, tn * 64 + lane < n);
                    if (PF & 1) load_head_lo(hw, gn);
                    if (PF & 2) {
                        rinfo(0, gn, wb, mm, qf, q0, hasw);
                        if (hasw) load_win(fw[NB - 1 - cb], wb, qf);
                    }
                }
            };
            if (NB == 2) next_loads();
            const uint32_t hc = __shfl(hz, 8 * s + rr, 64);
            uint32_t acc = (j == ((mm_c - 1) & 7)) ? hc : 0u;
            // every window of the round dword-aligned (records at 4-aligned offsets): no byte shifts
            const bool wal = __ballot(hasw_c && (wb_c & 3) != 0) == 0;
            if (hasw_c) {
                const uint32_t wsh = (uint32_t)(wb_c & 3);
                for (int32_t q = qf_c;; q += 8) {
                    constexpr uint32_t CW = 32 / NCH;  // words per chain
                    uint32_t c[NCH];
#pragma unroll
                    for (int kk = 0; kk < NCH; kk++) c[kk] = 0;
                    if (wal) {
#pragma unroll
                        for (uint32_t t = 0; t < CW; t++)
#pragma unroll
                            for (uint32_t kk = 0; kk < NCH; kk++) c[kk] = crc.word(c[kk], fw[cb][CW * kk + t]);
                    } else {
#pragma unroll
                        for (uint32_t t = 0; t < CW; t++)
#pragma unroll
                            for (uint32_t kk = 0; kk < NCH; kk++) {
                                const uint32_t wi = CW * kk + t;
                                c[kk] = crc.word(c[kk], __builtin_amdgcn_alignbyte(fw[cb][wi + 1], fw[cb][wi], wsh));
                            }
                    }
                    uint32_t V = c[0];
#pragma unroll
                    for (int kk = 1; kk < NCH; kk++) V = zapply(Zf, V) ^ c[kk];
                    // Horner over this lane's windows; the first step's Z_1024 of the head CRC was
                    // applied per record in phase 1 (hz)
                    acc = (q == qf_c ? acc : zapply(Z, acc)) ^ V;
                    if (q + 8 > q0_c) break;
                    load_win(fw[cb], wb_c, q + 8);  // records longer than 9 windows (synchronous)
                }
            }
            if (j & 1) acc = zapply(Z + 1024, acc);
            if (j & 2) acc = zapply(Z + 2048, acc);
            if (j & 4) acc = zapply(Z + 3072, acc);
            acc ^= __shfl_xor(acc, 1, 64);
            acc ^= __shfl_xor(acc, 2, 64);
            acc ^= __shfl_xor(acc, 4, 64);
            const uint32_t got = __shfl(acc, 8 * (lane & 7), 64);  // record 8s + r sits on lane 8r
            if ((lane >> 3) == s) mycrc = got;
            if (NB == 1) next_loads();
        }
        if (PF == 0) wait_loads_done();  // unconditional: see bhg_device.h
        if (valid) {
            uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = st;
            uint64_t dtr = 0;
            if (inb) {
                dcrc = (LONG && L > kLongRec) ? 0u : crc_mask(~mycrc);  // crc.go:31-33 (long: the pass's)
                if (rvalid) {
                    dk = 12; dkl = key_len; dvo = 12 + k; dvl = v;  // noCompressor.Decode: zero-copy view
                    dtr = trailer; dfn = fn; dfnv = fnv;
                    if (expected_crc != nullptr && ecrc != dcrc && !(LONG && L > kLongRec)) dst = BHG_ST_CRC_MISMATCH;
                } else {
                    dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil
                }
            }
            // non-temporal: descriptor writes mixed into the read stream cost ~0.03 ms per 40 MB
            // as plain stores on most boxes, ~0.013 less as nt (probe_lab tile9r_st / _st_nt);
            // staging them through LDS into contiguous 16-B stores changes nothing
            uint64_t *o = reinterpret_cast<uint64_t *>(out + i);
            __builtin_nontemporal_store((uint64_t)dk | ((uint64_t)dkl << 32), o);
            __builtin_nontemporal_store((uint64_t)dvo | ((uint64_t)dvl << 32), o + 1);
            __builtin_nontemporal_store(dtr, o + 2);
            __builtin_nontemporal_store((uint64_t)dfn | ((uint64_t)dfnv << 32), o + 3);
            __builtin_nontemporal_store((uint64_t)dcrc | ((uint64_t)dst << 32), o + 4);
        }
    }
}

hipError_t launch_decode_tile(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              const uint32_t *expected_crc, bhg_desc *out, void *long_scratch) {
    constexpr int WPB = 8;  // measured: 12 waves/CU (3 per SIMD) 0.293 ms vs 0.285; non-temporal window loads 0.58 ms
    const uint64_t tiles = (n + 63) / 64;
    uint64_t need = (tiles + WPB - 1) / WPB;
    uint64_t cap = (uint64_t)L.num_cus;  // 148 KiB of LDS: one workgroup per CU
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    if (long_scratch == nullptr) {
        hipLaunchKernelGGL((k_decode_tile<WPB, kTileNchOld, kTilePfOld>), dim3(grid), dim3(64 * WPB), 0, L.stream, src, src_len,
                           h, n, expected_crc, out, L.ztab);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_decode_tile<WPB, kTileNchOld, kTilePfOld, 2, 1>), dim3(grid), dim3(64 * WPB), 0, L.stream, src,
                       src_len, h, n, expected_crc, out, L.ztab);
    if (hipError_t e = hipGetLastError()) return e;
    return launch_long_crc(L, src, src_len, h, n, expected_crc, out, long_scratch);
}

}  // namespace bhg
