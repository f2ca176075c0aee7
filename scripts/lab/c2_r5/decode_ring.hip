// decode_ring.hip (lab, round 5; not built into the product) -- NoCompressor batch decode as an LDS-DMA loader / consumer ring (gfx950).
//
// Same outputs as k_decode_tile (readRecord + readKV + FNV-1 + masked CRC-32C per handle;
// bithash/block2.go:31-66, reader.go:233-272, compress.go:57-59, internal/hash/fnv.go:19-23,
// internal/crc/crc.go:19-33), built for handles that walk a table in offset order (table scans,
// compaction, rebuild, the C2 / C5 batches): every record byte goes HBM -> LDS once, by
// global_load_lds_dwordx4 (1 KiB contiguous per wave instruction, no VGPR staging), issued by ONE
// dedicated loader wave per CU, and is read from LDS by the consumer waves.
//
// Workgroup = one per CU, 1 loader wave + kNC consumer waves.  The CU takes a contiguous range of
// handles; consumer c owns a contiguous sub-range of it, walked in batches of 64 handles (lane =
// handle for the handle loads, the record parse and the 40-B descriptor stores: one contiguous
// 2.5 KB store burst per batch).
//   Tiles.  The consumer cuts each batch into tiles of <= kMaxR consecutive records whose bytes
//     lie in one 16-B aligned window [B, B + kSB) (B = the first record's offset rounded down
//     to 16); a record that is out of offset order or too far ahead starts a new tile, so ANY
//     handle order is decoded correctly -- sorted handles just pack 8 C2 records per tile.  A
//     record larger than a slot is a "big" tile of its own, read from global memory.
//   Loader.  Consumers post tile requests {B, bytes} into per-consumer request rings in LDS (a
//     few tiles ahead).  The loader serves them round robin into kNS ring slots of kSB bytes,
//     always kNI wave instructions per tile (instructions past the image load one 16-B piece
//     into the unused end of the slot), keeps kD tiles in flight behind a compile-time
//     s_waitcnt vmcnt(kNI * (kD - 1)), and then mails the landed tile's slot to its consumer.
//     Consumers add to the slot's FREE word when done; the loader waits for it before reuse.
//     Loads are non-temporal (the stream is read once).
//   Consumer, per tile: lane (r, j) = record r of the tile, 8 lanes per record: the record's
//     full 136-B windows counted from its end, window d on lane d % 8 (four chains of 36 + 32 +
//     36 + 32 B folded with Z_32 and Z_68; Horner over a lane's windows with Z_1088; lane j
//     shifted by Z_{136 j}; xor over the 8 lanes) -> crc_0 of the record minus its head (hl = L - 136 (m-1) bytes, 1..136).
//     The head's 35 words are copied from LDS into the registers of the record's batch lane.
//   Consumer, per batch (lane = record): head CRC from crc.New's ~0, shifted past the m-1 full
//     windows (Z_{136 (m-1)} by the bits of m-1) and xored with the windows' part;
//     readRecordHeader / readRecord / readKV / FNV-1 / trailer from the head words; expected
//     CRC check; descriptor.  CRC linearity over GF(2): crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B).
// CRC tables: CrcR8 (slice-by-4, 8 replicas, 32 KiB, conflict free) + 6 shift tables (24 KiB);
// the ring (11 x 9 KiB) beside them: 156 KiB of LDS, one workgroup per CU.
#include "../../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../../bitalosdb_amd/csrc/bhg_device.h"
#include "../../../bitalosdb_amd/csrc/bhg_internal.h"

namespace bhg {
namespace ring {

constexpr uint32_t kNI = 9;                 // DMA wave instructions (1 KiB each) per tile
constexpr uint32_t kSB = kNI * 1024;        // slot bytes
constexpr uint32_t kNS = 11;                // ring slots
constexpr uint32_t kD = 4;                  // tiles in flight behind the loader
constexpr uint32_t kNC = 7;                 // consumer waves
constexpr uint32_t kMaxR = 8;               // records per tile
constexpr uint32_t kW = 136;                // CRC window bytes
constexpr uint32_t kQR = 8;                 // request ring entries per consumer
constexpr uint32_t kQM = 8;                 // mail entries per consumer
constexpr uint32_t kLA = 4;                 // tiles a consumer keeps requested ahead
static_assert(kNI * (kD - 1) <= 63, "vmcnt field");
static_assert(kD - 1 <= 4, "outstanding tiles fit the 64-bit FIFO");
static_assert(kNS <= 16 && kNC <= 8, "FIFO entry fields");
static_assert(kLA < kQR && kLA < kQM, "rings hold the look-ahead");
// LDS byte layout
constexpr uint32_t kOffZ = CrcR8::kBytes;
constexpr uint32_t kOffRing = kOffZ + kRingZN * 4096;
constexpr uint32_t kOffReq = kOffRing + kNS * kSB;
constexpr uint32_t kOffMail = kOffReq + kNC * kQR * 8;
constexpr uint32_t kOffFree = kOffMail + kNC * kQM * 4;
constexpr uint32_t kOffErr = kOffFree + kNS * 4;
constexpr uint32_t kLds = kOffErr + 16;
static_assert(kLds <= 160 * 1024, "one workgroup per CU");
constexpr uint32_t kSpin = 1u << 20;        // bounded waits: a protocol error ends the kernel

// request word: [0, 44) B >> 4 | [44, 54) bytes >> 4 | [54] terminal | [56, 64) sequence
constexpr uint64_t kReqTerm = 1ull << 54;

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t shfl_u64_(uint64_t v, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, (int)src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// ---- LDS protocol words (inline asm: ordered against everything by the "memory" clobber) ----
__device__ __forceinline__ uint32_t poll32(uint32_t a) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    return uni(v);
}
__device__ __forceinline__ void put32(uint32_t a, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void put64(uint32_t a, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
// every LDS read of this wave has returned, then FREE += 1 (lane 0 adds 1, the others 0)
__device__ __forceinline__ void release(uint32_t a) {
    const uint32_t one = (threadIdx.x & 63) == 0 ? 1u : 0u;
    asm volatile("s_waitcnt lgkmcnt(0)\n\tds_add_u32 %0, %1" ::"v"(a), "v"(one) : "memory");
}

// ---- the loader's DMA ----
// one 1-KiB piece per wave instruction: LDS byte lds + 16 lane <- global [g, g + 16)
__device__ __forceinline__ void glds1(uint64_t g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
// four pieces from one address and one M0: the instruction offset moves both addresses
__device__ __forceinline__ void glds4(uint64_t g, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off nt\n\t"
                 "global_load_lds_dwordx4 %1, off offset:1024 nt\n\t"
                 "global_load_lds_dwordx4 %1, off offset:2048 nt\n\t"
                 "global_load_lds_dwordx4 %1, off offset:3072 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// crc_0 of a 136-B window at LDS byte address a (4-aligned) as four chains: words 0-8, 9-16, 17-25,
// 26-33 (36 + 32 + 36 + 32 B), folded as Z_68(Z_32(cA) ^ cB) ^ (Z_32(cC) ^ cD): 9 dependent steps
__device__ __forceinline__ uint32_t win_crc(const CrcR8 &crc, uint32_t z32, uint32_t z68, uint32_t a) {
    uint32_t cA = 0, cB = 0, cC = 0, cD = 0;
#pragma unroll
    for (uint32_t t = 0; t < 9; t++) {
        cA = crc.word(cA, lds_ld32(a + 4 * t));
        if (t < 8) cB = crc.word(cB, lds_ld32(a + 36 + 4 * t));
        cC = crc.word(cC, lds_ld32(a + 68 + 4 * t));
        if (t < 8) cD = crc.word(cD, lds_ld32(a + 104 + 4 * t));
    }
    return zshift(z68, zshift(z32, cA) ^ cB) ^ (zshift(z32, cC) ^ cD);
}
// the same at a byte address with a != 0 mod 4 (s = a & 3), from aligned words
__device__ __forceinline__ uint32_t win_crc_u(const CrcR8 &crc, uint32_t z32, uint32_t z68, uint32_t a) {
    const uint32_t aa = a & ~3u, s = a & 3u;
    uint32_t w[35];
#pragma unroll
    for (uint32_t t = 0; t < 35; t++) w[t] = lds_ld32(aa + 4 * t);
    uint32_t cA = 0, cB = 0, cC = 0, cD = 0;
#pragma unroll
    for (uint32_t t = 0; t < 9; t++) {
        cA = crc.word(cA, __builtin_amdgcn_alignbyte(w[t + 1], w[t], s));
        if (t < 8) cB = crc.word(cB, __builtin_amdgcn_alignbyte(w[t + 10], w[t + 9], s));
        cC = crc.word(cC, __builtin_amdgcn_alignbyte(w[t + 18], w[t + 17], s));
        if (t < 8) cD = crc.word(cD, __builtin_amdgcn_alignbyte(w[t + 27], w[t + 26], s));
    }
    return zshift(z68, zshift(z32, cA) ^ cB) ^ (zshift(z32, cC) ^ cD);
}
// crc_0 of a 136-B window at an absolute global address (big records), any alignment
__device__ __forceinline__ uint32_t win_crc_g(const CrcR8 &crc, uint32_t z68, uint64_t a, uint64_t end) {
    uint32_t cA = 0, cB = 0;
#pragma unroll
    for (uint32_t t = 0; t < 17; t++) {
        cA = crc.word(cA, ldu32(a + 4 * t, end));
        cB = crc.word(cB, ldu32(a + 68 + 4 * t, end));
    }
    return zshift(z68, cA) ^ cB;
}

// KO: timing-only knock-outs for the lab (0 in the product): 1 window CRCs, 2 head copies,
// 4 the batch parse, 8 all tile work
template <int KO = 0>
__global__ __launch_bounds__(64 * (kNC + 1)) void k_decode_ring(const uint8_t *__restrict__ src, uint64_t src_len,
                                                                const bhg_handle *__restrict__ handles, uint32_t n,
                                                                const uint32_t *__restrict__ expected_crc,
                                                                bhg_desc *__restrict__ out,
                                                                const uint32_t *__restrict__ rz,
                                                                uint32_t *__restrict__ err,
                                                                unsigned long long *__restrict__ prof = nullptr) {
    // KO & 16 (lab): per-phase shader-clock totals, prof[0..3] loader, prof[4..7] consumers
    unsigned long long pt[4] = {0, 0, 0, 0};
    auto clk = [&]() -> unsigned long long { return (KO & 16) ? (unsigned long long)__builtin_amdgcn_s_memtime() : 0ull; };
    const unsigned long long t_start = clk();
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    const uint32_t lb = lds_addr(lds);
    const uint32_t zb = lb + kOffZ;
    const uint32_t Z32 = zb, Z68 = zb + 4096, Z136 = zb + 2 * 4096, Z1088 = zb + 5 * 4096;
    // Z_{136 * 2^bt}: a table for bt <= 3, repeated Z_1088 above
    auto zwin = [&](uint32_t bt, uint32_t c) {
        if (bt <= 3) return zshift(Z136 + bt * 4096, c);
        for (uint32_t q = 0; q < (1u << (bt - 3)); q++) c = zshift(Z1088, c);
        return c;
    };
    const uint32_t ring = lb + kOffRing, reqb = lb + kOffReq, mailb = lb + kOffMail, freeb = lb + kOffFree;
    const uint32_t lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);
    const uint64_t base = (uint64_t)src, end = base + src_len;

    // ---- prologue: tables and protocol words (all waves)
    CrcR8::fill(lb);
    {
        constexpr uint32_t NT = 64 * (kNC + 1), NZ = (kRingZN * 1024 + NT - 1) / NT;
        uint32_t v[NZ];
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++) v[r] = threadIdx.x + r * NT < kRingZN * 1024 ? rz[threadIdx.x + r * NT] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++)
            if (threadIdx.x + r * NT < kRingZN * 1024) lds_st(zb + 4 * (threadIdx.x + r * NT), v[r]);
        for (uint32_t t = threadIdx.x; t < (kOffErr + 16 - kOffReq) / 4; t += NT) lds_st(reqb + 4 * t, 0u);
    }
    __syncthreads();

    // the CU's handle range, then consumer c's sub-range
    const uint32_t per = n / gridDim.x, rem = n % gridDim.x;
    const uint32_t h0 = blockIdx.x * per + (blockIdx.x < rem ? blockIdx.x : rem);
    const uint32_t hn = per + (blockIdx.x < rem ? 1u : 0u);

    if (wv == 0) {
        // =========================== loader ===========================
        uint32_t kreq[kNC];
#pragma unroll
        for (uint32_t c = 0; c < kNC; c++) kreq[c] = 0;
        uint32_t live = (1u << kNC) - 1, T = 0, nout = 0, idle = 0;
        uint64_t fifo = 0;  // outstanding tiles, newest in the low 16 bits: c | slot << 3 | seq << 8
        const uint64_t dummy = (uint64_t)handles;  // a readable address for the pad instructions
        auto publish = [&](uint32_t e) {
            const uint32_t c = e & 7, s = (e >> 3) & 15, sq = e >> 8;
            put32(mailb + 4 * (c * kQM + ((sq - 1) & (kQM - 1))), (sq << 8) | s);
        };
        static_assert(kNC * kQR <= 64, "one request word per loader lane");
        while (live != 0 || nout != 0) {
            bool prog = false;
            // every request word at once: lane c * kQR + q holds consumer c's entry q
            uint64_t ev;
            const uint32_t ra = reqb + 8 * (lane < kNC * kQR ? lane : 0u);
            asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(ev) : "v"(ra) : "memory");
#pragma unroll
            for (uint32_t c = 0; c < kNC; c++) {
                if (!((live >> c) & 1)) continue;
                const uint64_t e = readlane_u64(ev, (int)(c * kQR + (kreq[c] & (kQR - 1))));
                const uint32_t sq = (uint32_t)(e >> 56);
                if (sq != ((kreq[c] + 1) & 0xff)) continue;
                kreq[c]++;
                if (e & kReqTerm) {
                    live &= ~(1u << c);
                    continue;
                }
                // a free slot (FIFO order): tile T - kNS released
                const uint32_t s = T % kNS;
                if (T >= kNS) {
                    uint32_t sp = 0;
                    const unsigned long long t0 = clk();
                    while (poll32(freeb + 4 * s) < T / kNS) {
                        if (poll32(lb + kOffErr) != 0) break;
                        __builtin_amdgcn_s_sleep(1);
                        if (++sp >= kSpin) {
                            put32(lb + kOffErr, 1u);
                            break;
                        }
                    }
                    pt[0] += clk() - t0;
                }
                const uint64_t B = (e & ((1ull << 44) - 1)) << 4;
                const uint32_t np = (uint32_t)((e >> 44) & 1023) << 0;  // pieces (bytes >> 4)
                const uint32_t sl = ring + s * kSB;
#pragma unroll
                for (uint32_t k = 0; k < kNI; k += 4) {
                    if (k + 4 <= kNI && 64 * (k + 4) <= np) {
                        glds4(B + 1024ull * k + 16ull * lane, uni(sl + 1024 * k));
                    } else {
#pragma unroll
                        for (uint32_t q = k; q < k + 4 && q < kNI; q++) {
                            const uint32_t pc = 64 * q + lane;
                            const bool act = pc < np || lane == 0;
                            const uint64_t g = pc < np ? B + 16ull * pc : (np ? B : dummy);
                            if (act) glds1(g, uni(sl + 1024 * q));
                        }
                    }
                }
                // kD tiles in flight: the oldest has landed once all but the newest kNI * (kD - 1)
                // loads are done; at most kD - 1 = 4 entries live in the 64-bit FIFO
                if (nout == kD - 1) {
                    const unsigned long long t0 = clk();
                    wait_vm<kNI * (kD - 1)>();
                    pt[1] += clk() - t0;
                    publish((uint32_t)(fifo >> (16 * (kD - 2))) & 0xffffu);
                    nout--;
                }
                fifo = (fifo << 16) | (uint64_t)(c | (s << 3) | ((kreq[c] & 0xff) << 8));
                nout++;
                T++;
                prog = true;
            }
            if (prog) {
                idle = 0;
            } else if (nout != 0) {  // no request waiting: land and mail everything in flight
                const unsigned long long t0 = clk();
                wait_vm<0>();
                pt[2] += clk() - t0;
                for (uint32_t q = nout; q > 0; q--) publish((uint32_t)(fifo >> (16 * (q - 1))) & 0xffffu);
                nout = 0;
            } else {
                pt[3] += 1;
                __builtin_amdgcn_s_sleep(2);
                if (++idle >= kSpin || poll32(lb + kOffErr) != 0) {
                    put32(lb + kOffErr, 2u);
                    break;
                }
            }
        }
        wait_vm<0>();
    } else {
        // =========================== consumer ===========================
        const uint32_t c = wv - 1;
        const uint32_t sper = hn / kNC, srem = hn % kNC;
        const uint32_t r0 = h0 + c * sper + (c < srem ? c : srem);
        const uint32_t rn = sper + (c < srem ? 1u : 0u);
        const uint32_t r1 = r0 + rn;
        const CrcR8 crc(lb);
        const uint32_t rr = lane >> 3, j = lane & 7;
        const uint32_t myreq = reqb + 8 * c * kQR, mymail = mailb + 4 * c * kQM;

        // a batch's handles on its lanes: absolute record address, length (0 when the handle is
        // not readable: Reader.readData's checks, reader.go:234-258), status
        struct Bat {
            uint64_t p;
            uint32_t L, st;
        };
        auto load_bat = [&](uint32_t b0) {
            Bat q;
            const uint32_t i = b0 + lane;
            bhg_handle h = {0, 0, 0};
            if (b0 < r1 && i < r1) h = handles[i];
            q.st = BHG_ST_OK;
            q.L = 0;
            if (!(b0 < r1 && i < r1)) q.st = 0xffffffffu;
            else if (h.length == 0) q.st = BHG_ST_ILLEGAL_LENGTH;
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) q.st = BHG_ST_INCOMPLETE;
            else q.L = h.length;
            q.p = base + (q.st == BHG_ST_INCOMPLETE ? 0ull : h.offset);  // tile images stay inside src's pages
            return q;
        };
        // tile starts of a batch (bit i: record i starts a tile)
        auto plan = [&](const Bat &q, uint32_t cnt) {
            uint64_t pm = 0;
            uint32_t s = 0;
            const uint64_t e16 = (q.p + q.L + 15) & ~15ull;
            while (s < cnt) {
                pm |= 1ull << s;
                const uint64_t B = readlane_u64(q.p, (int)s) & ~15ull;
                const uint32_t Ls = (uint32_t)__builtin_amdgcn_readlane((int)q.L, (int)s);
                const uint64_t es = readlane_u64(e16, (int)s);
                const uint32_t lim = s + kMaxR < cnt ? s + kMaxR : cnt;
                if (Ls != 0 && es - B > kSB) {  // a big record: a tile of its own
                    s++;
                    continue;
                }
                const bool fits = q.L == 0 || (q.p >= B && e16 - B <= kSB);
                const uint64_t bad = __ballot(lane > s && lane < lim && !fits);
                s = bad ? (uint32_t)__builtin_ctzll(bad) : lim;
            }
            return pm;
        };
        // request word of the tile [ts, te) of a batch; sq = the consumer's tile number + 1
        auto tile_req = [&](const Bat &q, uint32_t ts, uint32_t te, uint32_t sq) {
            const uint64_t B = readlane_u64(q.p, (int)ts) & ~15ull;
            const uint64_t e16 = (q.p + q.L + 15) & ~15ull;
            const uint32_t v = (lane >= ts && lane < te && q.L != 0) ? (uint32_t)(e16 - B) : 0u;
            uint32_t nb = uni(__builtin_amdgcn_readlane((int)wave_incl_max(v), 63));
            if (nb > kSB) nb = 0;  // big record: no DMA, read from global memory
            return ((B >> 4) & ((1ull << 44) - 1)) | ((uint64_t)(nb >> 4) << 44) | ((uint64_t)(sq & 0xff) << 56);
        };

        // per-batch lane state (lane = record)
        uint32_t hw[35];
#pragma unroll
        for (int u = 0; u < 35; u++) hw[u] = 0;
        uint32_t wpart = 0;     // crc_0 of the record's full windows (or the whole CRC for big records)
        bool bigdone = false;   // the lane's record was a big record: wpart is its final CRC state

        const uint32_t nb = (rn + 63) / 64;
        Bat cur = load_bat(r0), nxt = load_bat(r0 + 64);
        uint32_t ecur = (expected_crc != nullptr && lane < rn) ? expected_crc[r0 + lane] : 0u;
        uint64_t pmc = rn ? plan(cur, rn < 64 ? rn : 64) : 0ull;
        uint64_t pmn = rn > 64 ? plan(nxt, rn - 64 < 64 ? rn - 64 : 64) : 0ull;
        // tiles are numbered per consumer from 0: kpost = the next tile to request, kproc = the
        // next to process; requests come from the current batch's plan, then the next batch's
        uint32_t kpost = 0, kproc = 0;
        bool term = false;
        // Simple explicit posting over (current batch, next batch) masks.
        uint64_t cur_rem_post = pmc, nxt_rem_post = pmn;  // tile starts not yet requested
        auto post_one = [&](uint32_t bidx) -> bool {      // request the next tile; false if none left
            const bool fc = cur_rem_post != 0;              // from the current batch, else the next
            if (!fc && nxt_rem_post == 0) return false;
            uint64_t rm = fc ? cur_rem_post : nxt_rem_post;
            const uint32_t bq = fc ? bidx : bidx + 1;
            const uint32_t cnt = rn - 64 * bq < 64 ? rn - 64 * bq : 64;
            const uint32_t ts = (uint32_t)__builtin_ctzll(rm);
            rm &= rm - 1;
            const uint32_t te = rm ? (uint32_t)__builtin_ctzll(rm) : cnt;
            if (fc) cur_rem_post = rm;
            else nxt_rem_post = rm;
            Bat q;
            q.p = fc ? cur.p : nxt.p;
            q.L = fc ? cur.L : nxt.L;
            q.st = 0;
            put64(myreq + 8 * (kpost & (kQR - 1)), tile_req(q, ts, te, kpost + 1));
            kpost++;
            return true;
        };

        for (uint32_t b = 0; b < nb; b++) {
            const uint32_t b0 = r0 + 64 * b;
            const uint32_t cnt = rn - 64 * b < 64 ? rn - 64 * b : 64;
            // the batch after next: handles and expected CRCs in flight during this batch
            const Bat nn = load_bat(b0 + 128);
            const uint32_t enxt = (expected_crc != nullptr && 64 * (b + 1) + lane < rn) ? expected_crc[b0 + 64 + lane] : 0u;
            bigdone = false;
            wpart = 0;
            uint64_t proc_rem = pmc;
            while (proc_rem) {
                // keep kLA tiles requested ahead of the one processed next
                while (kpost < kproc + 1 + kLA && post_one(b)) {
                }
                if (!term && !cur_rem_post && !nxt_rem_post && b + 2 >= nb) {  // every tile requested
                    put64(myreq + 8 * (kpost & (kQR - 1)), kReqTerm | ((uint64_t)((kpost + 1) & 0xff) << 56));
                    term = true;
                }
                const uint32_t ts = (uint32_t)__builtin_ctzll(proc_rem);
                proc_rem &= proc_rem - 1;
                const uint32_t te = proc_rem ? (uint32_t)__builtin_ctzll(proc_rem) : cnt;
                // the tile's slot
                const uint32_t want = (kproc + 1) & 0xff;
                uint32_t m = 0, sp = 0;
                const unsigned long long tm0 = clk();
                while (((m = poll32(mymail + 4 * (kproc & (kQM - 1)))) >> 8) != want) {
                    if (poll32(lb + kOffErr) != 0) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++sp >= kSpin) {
                        put32(lb + kOffErr, 3u);
                        break;
                    }
                }
                const unsigned long long tm1 = clk();
                pt[0] += tm1 - tm0;
                const uint32_t s = m & 15;
                const uint32_t sl = ring + s * kSB;
                const uint64_t B = readlane_u64(cur.p, (int)ts) & ~15ull;
                const uint32_t Lts = (uint32_t)__builtin_amdgcn_readlane((int)cur.L, (int)ts);
                const uint64_t e16ts = readlane_u64((cur.p + cur.L + 15) & ~15ull, (int)ts);
                const bool big = Lts != 0 && e16ts - B > kSB;
                if (KO & 8) {
                } else if (!big) {
                    // ---- window CRCs, lane (rr, j) on record ts + rr
                    const uint32_t ri = ts + rr;
                    const bool act = ri < te;
                    const uint32_t Lsh = (uint32_t)__shfl((int)cur.L, (int)(ri & 63), 64);  // every lane
                    const uint32_t Lr = act ? Lsh : 0u;
                    const uint64_t pr = shfl_u64_(cur.p, ri & 63);
                    const uint32_t A = sl + (uint32_t)(pr - B);  // LDS byte address of the record
                    const uint32_t E = A + Lr;
                    const uint32_t mw = Lr ? (Lr + kW - 1) / kW : 1u;
                    const int32_t nfull = (int32_t)mw - 1;
                    int32_t d = nfull > (int32_t)j ? (int32_t)j + 8 * ((nfull - 1 - (int32_t)j) / 8) : -1;
                    const bool wal = __ballot(d >= 0 && (E & 3) != 0) == 0;
                    uint32_t acc = 0;
                    bool first = true;
                    if (KO & 1) d = -1;
                    while (__ballot(d >= 0)) {
                        if (d >= 0) {
                            const uint32_t a = E - kW * (uint32_t)(d + 1);
                            const uint32_t V = wal ? win_crc(crc, Z32, Z68, a) : win_crc_u(crc, Z32, Z68, a);
                            acc = first ? V : (zshift(Z1088, acc) ^ V);
                            first = false;
                            d -= 8;
                        }
                    }
                    if (j & 1) acc = zshift(Z136, acc);
                    if (j & 2) acc = zshift(Z136 + 4096, acc);
                    if (j & 4) acc = zshift(Z136 + 2 * 4096, acc);
                    acc ^= __shfl_xor(acc, 1, 64);
                    acc ^= __shfl_xor(acc, 2, 64);
                    acc ^= __shfl_xor(acc, 4, 64);
                    // ---- hand the tile's records to their batch lanes: window part + head words
                    const int srcl = (int)(8 * (lane - ts));
                    const uint32_t got = __shfl(acc, srcl & 63, 64);
                    if (lane >= ts && lane < te) {
                        wpart = got;
                        if (cur.L != 0 && !(KO & 2)) {
                            const uint32_t ha = (sl + (uint32_t)(cur.p - B)) & ~3u;
#pragma unroll
                            for (uint32_t u = 0; u < 35; u++) hw[u] = lds_ld32(ha + 4 * u);
                        }
                    }
                } else {
                    // ---- a big record (one per tile), from global memory: all 64 lanes, window d on
                    // lane d % 64 (Horner with Z_8704), head from ~0 in lane (m-1) % 64's chain
                    const uint64_t pr = readlane_u64(cur.p, (int)ts);
                    const uint32_t Lr = Lts;
                    const uint32_t mw = (Lr + kW - 1) / kW, hl = Lr - kW * (mw - 1);
                    const uint64_t eb = pr + Lr;
                    int32_t d = (int32_t)lane <= (int32_t)mw - 1
                                    ? (int32_t)lane + 64 * (((int32_t)mw - 1 - (int32_t)lane) / 64) : -1;
                    uint32_t acc = 0;
                    bool first = true;
                    while (__ballot(d >= 0)) {
                        if (d >= 0) {
                            uint32_t V;
                            if (d == (int32_t)mw - 1) {  // the head, from crc.New's ~0
                                V = crc_range_w<2, false>(crc, 0xffffffffu, pr, hl, end);
                            } else {
                                V = win_crc_g(crc, Z68, eb - kW * (uint64_t)(d + 1), end);
                            }
                            if (!first) acc = zwin(6, acc);  // Z_8704: 64 windows
                            acc = first ? V : (acc ^ V);
                            first = false;
                            d -= 64;
                        }
                    }
#pragma unroll
                    for (uint32_t bt = 0; bt < 6; bt++)
                        if ((lane >> bt) & 1) acc = zwin(bt, acc);
#pragma unroll
                    for (uint32_t o = 1; o < 64; o <<= 1) acc ^= __shfl_xor(acc, o, 64);
                    if (lane == ts) {
                        wpart = acc;
                        bigdone = true;
                        const uint64_t ha = pr & ~3ull;
#pragma unroll
                        for (uint32_t u = 0; u < 35; u++) hw[u] = ld32_safe(ha + 4 * u, end);
                    }
                }
                release(freeb + 4 * s);
                pt[1] += clk() - tm1;
                kproc++;
            }
            // ---- batch end: lane = record b0 + lane
            const unsigned long long tp0 = clk();
            {
                const bool valid = lane < cnt;
                const uint32_t L = cur.L, st = cur.st;
                const bool inb = valid && L != 0;
                const uint32_t hsh = (uint32_t)(cur.p & 3);
                uint32_t rw[34];
#pragma unroll
                for (int u = 0; u < 34; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
                uint32_t fullc = 0;
                if (inb && !(KO & 4)) {
                    if (bigdone) {
                        fullc = wpart;
                    } else {
                        const uint32_t mw = (L + kW - 1) / kW, hl = L - kW * (mw - 1);
                        uint32_t hc = 0xffffffffu;  // crc.New: Go's crc32.Update starts from ^0
                        const uint32_t nw = hl >> 2;
#pragma unroll
                        for (uint32_t u = 0; u < 34; u++)
                            if (u < nw) hc = crc.word(hc, rw[u]);
                        if (hl & 3) {
                            uint32_t wv2 = 0;
#pragma unroll
                            for (uint32_t u = 0; u < 34; u++) wv2 = nw == u ? rw[u] : wv2;
                            hc = crc.partial(hc, wv2, hl & 3);
                        }
                        const uint32_t sft = mw - 1;  // <= 67 for records that fit a slot
#pragma unroll
                        for (uint32_t bt = 0; bt < 7; bt++)
                            if ((sft >> bt) & 1) hc = zwin(bt, hc);
                        fullc = hc ^ wpart;
                    }
                }
                // readRecordHeader / readRecord / readKV (block2.go:31-66)
                uint32_t k = 0, v = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
                uint64_t trailer = 255;  // InternalKeyKindInvalid when ikeySize < 8
                bool rvalid = false;
                if (inb && !(KO & 4)) {
                    k = L >= 12 ? rw[0] : 0u;
                    v = L >= 12 ? rw[1] : 0u;
                    fn = L >= 12 ? rw[2] : 0u;
                    rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;
                    if (rvalid && k >= 8) {
                        key_len = k - 8;
                        if (key_len <= 36) {
                            uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                            for (uint32_t t = 3; t < 12; t++)
#pragma unroll
                                for (uint32_t bq = 0; bq < 4; bq++) {
                                    const uint32_t h2 = (hh * BHG_FNV_PRIME) ^ ((rw[t] >> (8 * bq)) & 0xffu);
                                    hh = 4 * (t - 3) + bq < key_len ? h2 : hh;
                                }
                            fnv = hh;
                            const uint32_t tb = 12 + key_len, tw = tb >> 2, ts2 = tb & 3;
                            uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                            for (uint32_t u = 3; u <= 12; u++) {
                                a0 = tw == u ? rw[u] : a0;
                                a1 = tw == u ? rw[u + 1] : a1;
                                a2 = tw == u ? rw[u + 2] : a2;
                            }
                            trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts2) |
                                      ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts2) << 32);
                        } else {
                            fnv = fnv1_range(cur.p + 12, key_len, end);
                            trailer = ldu64(cur.p + 12 + k - 8, end);
                        }
                    }
                }
                if (valid) {
                    uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = st;
                    uint64_t dtr = 0;
                    if (inb) {
                        dcrc = crc_mask(~fullc);  // crc.go:31-33
                        if (rvalid) {
                            dk = 12; dkl = key_len; dvo = 12 + k; dvl = v;  // noCompressor.Decode: zero-copy view
                            dtr = trailer; dfn = fn; dfnv = fnv;
                            if (expected_crc != nullptr && ecur != dcrc) dst = BHG_ST_CRC_MISMATCH;
                        } else {
                            dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil
                        }
                    }
                    uint64_t *o = reinterpret_cast<uint64_t *>(out + b0 + lane);
                    __builtin_nontemporal_store((uint64_t)dk | ((uint64_t)dkl << 32), o);
                    __builtin_nontemporal_store((uint64_t)dvo | ((uint64_t)dvl << 32), o + 1);
                    __builtin_nontemporal_store(dtr, o + 2);
                    __builtin_nontemporal_store((uint64_t)dfn | ((uint64_t)dfnv << 32), o + 3);
                    __builtin_nontemporal_store((uint64_t)dcrc | ((uint64_t)dst << 32), o + 4);
                }
            }
            pt[2] += clk() - tp0;
            // advance: the next batch becomes current (its unposted tiles stay unposted)
            cur = nxt;
            nxt = nn;
            ecur = enxt;
            pmc = pmn;
            cur_rem_post = nxt_rem_post;
            const uint32_t b2 = b + 2;
            pmn = b2 < nb ? plan(nxt, rn - 64 * b2 < 64 ? rn - 64 * b2 : 64) : 0ull;
            nxt_rem_post = pmn;
        }
        if (!term) put64(myreq + 8 * (kpost & (kQR - 1)), kReqTerm | ((uint64_t)((kpost + 1) & 0xff) << 56));
    }
    if ((KO & 16) && prof != nullptr && lane == 0) {
        const uint32_t o = wv == 0 ? 0u : 4u;
        for (int q = 0; q < 4; q++) atomicAdd(prof + o + q, pt[q]);
        atomicAdd(prof + 8 + (wv == 0 ? 0 : 1), clk() - t_start);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t e = lds_ld32(lb + kOffErr);
        if (e != 0 && err != nullptr) atomicOr(err, e);
    }
}

}  // namespace ring
}  // namespace bhg
