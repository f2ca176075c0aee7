// dma_lab.hip -- development harness (not product code): the C2 decode as an
// LDS-DMA streaming kernel, checked against and timed beside the product
// bhg_decode_batch (k_decode_tile) on the C2 layout (1M x 1076 B records in
// 128 MiB tables, expected CRCs, 40-B descriptors).
//
// Per wave: a contiguous range of handles, groups of 4 records; each group's
// record bytes go HBM -> LDS by global_load_lds_dwordx4 (no VGPR staging) into
// a ring of D slots, D-1 groups in flight while one is computed.  Every VMEM
// instruction of the loop is inline asm with exact vmcnt bookkeeping (hipcc's
// own waits would drain the ring, cdna_hip_programming.md §5); handles and
// expected CRCs come through the scalar cache (lgkmcnt).
//   group compute, lane (r, j) = (lane / 16, lane % 16): record r's full
//     68-B windows e = j, j+16, ... counted from the record end (Horner with
//     Z_1088), each as 2 chains (36 + 32 B, fold Z_32); a 4-level tree over
//     the 16 lanes (Z_68, Z_136, Z_272, Z_544) gives sum_e Z_{68e}(crc0(win e));
//   parse, lane = record of a 64-record batch: the head [0, hl) (hl = L - 68
//     (m-1)) copied from LDS at group time, readRecord / readKV / FNV-1 /
//     trailer, head CRC from ~0 shifted by Z_{68(m-1)}, descriptor stores.
// CRC tables: slice-by-4 x 8 replicas (32 KiB) with the 4 tables rotated over
// the 4 lane octets of a 32-lane half, so one ds_read_b32 of 32 lanes touches
// 32 different banks: conflict free at a quarter of Crc4Perm's LDS.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../../bitalosdb_amd/csrc/bhg_device.h"
#include "../../../include/bithashgpu.h"
#include "decode_dma_kernel.hip"
#include "tile_nb3.hip"  // the product-shaped DMA kernel (lab), timed beside the product tile kernel
#include "../../../bitalosdb_amd/csrc/bhg_decode_tile.hip"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace bhg;

namespace dl {

constexpr uint32_t G = 4;                   // records per group
constexpr uint32_t WB = 68;                 // window bytes (17 words)
constexpr uint32_t SLOT = 4416;             // ring slot bytes (276 pieces: 4 x 69)
constexpr uint32_t SLOT_PIECES = SLOT / 16;
constexpr uint32_t TBYTES = 32768;
constexpr uint32_t NZ = 6;                  // Z32, Z68, Z136, Z272, Z544, Z1088
constexpr uint32_t ZBYTES = NZ * 4096;
constexpr uint32_t MAXW = 64;               // staged records: m - 1 <= 63 full windows (L <= 4352)

__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {  // LDS dword at byte address a
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>((size_t)a);
}

// slice-by-4, 8 replicas, byte address (b << 7) | (k << 5) | (r << 2); lane octet g reads table (i + g) & 3
// in its i-th lookup, so the 32 lanes of a half hit banks (k << 3) | r: all different
struct CrcRot8 {
    uint32_t tb;     // LDS byte address of the table
    uint32_t sh[4];  // byte position of x each lookup takes
    uint32_t ko[4];  // table / replica offset
    __device__ __forceinline__ explicit CrcRot8(uint32_t tbase) : tb(tbase) {
        const uint32_t lane = threadIdx.x & 63, r = lane & 7, g = (lane >> 3) & 3;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t k = (i + g) & 3;
            sh[i] = 8 * (3 - k);
            ko[i] = tbase + ((k << 5) | (r << 2));
        }
    }
    __device__ __forceinline__ uint32_t look(uint32_t x, int i) const {
        return lds_ld((__builtin_amdgcn_ubfe(x, sh[i], 8) << 7) + ko[i]);
    }
    __device__ __forceinline__ uint32_t word(uint32_t c, uint32_t w) const {
        const uint32_t x = c ^ w;
        return look(x, 0) ^ look(x, 1) ^ look(x, 2) ^ look(x, 3);
    }
    __device__ __forceinline__ uint32_t step(uint32_t c) const {  // one byte: (c >> 8) ^ T0[c & 0xff]
        // T0 sits at k = 0: byte address (b << 7) | (r << 2) with this lane's replica
        return (c >> 8) ^ lds_ld(((c & 0xffu) << 7) + tb + ((threadIdx.x & 7u) << 2));
    }
    __device__ __forceinline__ uint32_t partial(uint32_t c, uint32_t x, uint32_t nb) const {
        const uint32_t m = nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
        c ^= x & m;
#pragma unroll
        for (uint32_t s = 0; s < 3; s++) {
            const uint32_t nx = step(c);
            c = s < nb ? nx : c;
        }
        return c;
    }
    static __device__ void fill(uint32_t tbase) {
        for (uint32_t t = threadIdx.x; t < 1024; t += blockDim.x) {
            const uint32_t k = t >> 8, b = t & 255, v = crc32c_tk(k, b);
            const uint32_t a = tbase + ((b << 7) | (k << 5));
            typedef uint32_t v4 __attribute__((ext_vector_type(4)));
            auto *p = reinterpret_cast<__attribute__((address_space(3))) v4 *>((size_t)a);
            p[0] = v4{v, v, v, v};
            p[1] = v4{v, v, v, v};
        }
    }
};

// Z_n tables (4 x 256 words each, S[k][i] = Z_n(i << 8k)) at zb + 4096 * idx
__device__ __forceinline__ uint32_t zap(uint32_t zt, uint32_t c) {
    return lds_ld(zt + ((c & 0xffu) << 2)) ^ lds_ld(zt + 1024 + (((c >> 8) & 0xffu) << 2)) ^
           lds_ld(zt + 2048 + (((c >> 16) & 0xffu) << 2)) ^ lds_ld(zt + 3072 + ((c >> 24) << 2));
}

// ---- VMEM through inline asm (exact vmcnt bookkeeping) ----
__device__ __forceinline__ void glds16(uint64_t gaddr, uint32_t lds_byte) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gaddr), "s"(lds_byte)
                 : "memory", "m0");
}
__device__ __forceinline__ void gst64_nt(uint64_t a, uint64_t v) {
    asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(a), "v"(v) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (clamped to 63)
__device__ __forceinline__ void wait_vm(uint32_t n) {
#define W_(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n < 63 ? n : 63) {
        W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
        W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29)
        W_(30) W_(31) W_(32) W_(33) W_(34) W_(35) W_(36) W_(37) W_(38) W_(39) W_(40) W_(41) W_(42) W_(43)
        W_(44) W_(45) W_(46) W_(47) W_(48) W_(49) W_(50) W_(51) W_(52) W_(53) W_(54) W_(55) W_(56) W_(57)
        W_(58) W_(59) W_(60) W_(61) W_(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
    }
#undef W_
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) { return readfirstlane_u64(x); }

template <int NW, int D, int WORK = 1>
__global__ __launch_bounds__(64 * NW) void k_decode_dma(const uint8_t *__restrict__ src, uint64_t src_len,
                                                       const bhg_handle *__restrict__ handles, uint32_t n,
                                                       const uint32_t *__restrict__ expected_crc,
                                                       bhg_desc *__restrict__ out, const uint32_t *__restrict__ gz) {
    constexpr uint32_t RING = NW * D * SLOT;
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[(TBYTES + ZBYTES + RING) / 4];
    const uint32_t lbase = (uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t *)(lds_all);
    const uint32_t tb = lbase, zb = lbase + TBYTES, rb = lbase + TBYTES + ZBYTES;
    CrcRot8::fill(tb);
    // shift tables from the context: Z32 (ztab 4), Z68.. built by the host into gz (6 x 1024 words, this order)
    for (uint32_t t = threadIdx.x; t < NZ * 1024; t += blockDim.x) lds_all[(TBYTES / 4) + t] = gz[t];
    __syncthreads();
    const CrcRot8 crc(tb);
    const uint32_t Z32 = zb, Z68 = zb + 4096, Z136 = zb + 8192, Z272 = zb + 12288, Z544 = zb + 16384,
                   Z1088 = zb + 20480;

    const uint32_t lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);  // wave-uniform for the compiler
    const uint32_t r4 = lane >> 4, j = lane & 15;
    const uint32_t gw = blockIdx.x * NW + wv, nwt = gridDim.x * NW;
    const uint32_t per = n / nwt, rem = n % nwt;
    const uint32_t r0 = gw * per + (gw < rem ? gw : rem);
    const uint32_t cnt = per + (gw < rem ? 1u : 0u);
    const uint32_t ngroups = (cnt + G - 1) / G;
    const uint32_t ring = rb + wv * D * SLOT;
    const uint64_t base = (uint64_t)src, end = base + src_len;

    // per-group record info (wave-uniform; scalar registers, reloaded through the scalar cache
    // when needed instead of being carried for every group in flight: SGPR pressure)
    struct GInfo {
        uint64_t a[G];   // absolute record address
        uint32_t L[G];   // length (0: no record / not in bounds)
        uint32_t st[G];  // status before decode (0xffffffff: no record)
        uint32_t ec[G];  // expected CRC
    };
    auto ginfo = [&](uint32_t g, bool want_ec) {
        GInfo q;
        // every scalar load of the group first (index clamped into the range), then one lgkmcnt wait
        // -- loads interleaved with each record's checks were waited for record by record
        bhg_handle hh[G];
        uint32_t ee[G];
#pragma unroll
        for (uint32_t r = 0; r < G; r++) {
            const uint32_t i = G * g + r;
            const uint32_t ic = r0 + (i < cnt ? i : (cnt ? cnt - 1 : 0u));
            hh[r] = handles[ic];
            ee[r] = (want_ec && expected_crc != nullptr) ? expected_crc[ic] : 0u;
        }
#pragma unroll
        for (uint32_t r = 0; r < G; r++) {
            const uint32_t i = G * g + r;
            const bhg_handle h = i < cnt ? hh[r] : bhg_handle{0, 0, 0};
            const uint32_t e = i < cnt ? ee[r] : 0u;
            uint32_t st = BHG_ST_OK, L = 0;
            if (i >= cnt) st = 0xffffffffu;
            else if (h.length == 0) st = BHG_ST_ILLEGAL_LENGTH;                                      // reader.go:234-236
            else if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset) st = BHG_ST_INCOMPLETE;  // :251-258
            else L = h.length;
            q.a[r] = base + h.offset;
            q.L[r] = L;
            q.st[r] = st;
            q.ec[r] = e;
        }
        return q;
    };
    // slot layout of a group: record r at byte pc_r * 16 + (a_r & 15), pieces = its 16-B aligned global lines
    auto layout = [&](const GInfo &q, uint32_t *off, uint32_t *pc) {
        pc[0] = 0;
#pragma unroll
        for (uint32_t r = 0; r < G; r++) {
            const uint32_t np = q.L[r] ? (uint32_t)(((q.a[r] + q.L[r] + 15) >> 4) - (q.a[r] >> 4)) : 0u;
            off[r] = pc[r] * 16 + (uint32_t)(q.a[r] & 15);
            pc[r + 1] = pc[r] + np;
        }
    };
    // issue group g's DMA into slot g % D; returns the VM-op count after it
    uint32_t ops = 0;
    auto issue = [&](uint32_t g, const GInfo &q) {
        const uint32_t slot = ring + (g % D) * SLOT;
        uint32_t off[G], pc[G + 1];
        layout(q, off, pc);
        const uint32_t np = pc[G];  // <= SLOT_PIECES for C2-shaped records (checked on the host in this lab)
        for (uint32_t x0 = 0; x0 < np; x0 += 64) {
            const uint32_t x = x0 + lane;
            uint64_t s = (q.a[0] & ~15ull) + 16ull * x;
#pragma unroll
            for (uint32_t r = 1; r < G; r++)
                if (x >= pc[r]) s = (q.a[r] & ~15ull) + 16ull * (x - pc[r]);
            if (x < np) glds16(s, uni(slot + 16 * x0));   // lane 0 always active: never a skipped op
            ops++;
        }
        return ops;
    };

    // per-lane batch state (lane = record 64 b + lane of this wave's range)
    uint32_t hw[18];
#pragma unroll
    for (int u = 0; u < 18; u++) hw[u] = 0;
    uint32_t b_st = 0, b_L = 0, b_ec = 0, b_wc = 0;
    uint64_t b_a = 0;

    static_assert(D == 3, "ring rotation below is written for 3 slots");
    uint32_t o0 = 0, o1 = 0, o2 = 0;   // VM-op counts after groups g, g+1, g+2 were issued
    if (ngroups > 0) o0 = issue(0, ginfo(0, false));
    if (ngroups > 1) o1 = issue(1, ginfo(1, false));
    GInfo qd = ginfo(2, false);         // the next DMA group's info, loaded one iteration ahead
    GInfo qc = ginfo(0, true);          // group g's info, loaded one iteration ahead
    for (uint32_t g = 0; g < ngroups; g++) {
        if (g + 2 < ngroups) o2 = issue(g + 2, qd);
        if (g + 3 < ngroups) qd = ginfo(g + 3, false);
        wait_vm(ops - o0);
        const GInfo q = qc;
        if (g + 1 < ngroups) qc = ginfo(g + 1, true);
        uint32_t qoff[G], qpc[G + 1];
        layout(q, qoff, qpc);
        const uint32_t slot = ring + (g % D) * SLOT;
        // ---- this lane's record r4
        uint32_t L = q.L[0], off = qoff[0];
#pragma unroll
        for (uint32_t r = 1; r < G; r++)
            if (r4 == r) { L = q.L[r]; off = qoff[r]; }
        const uint32_t R0 = slot + off;
        const uint32_t m = L ? (L + WB - 1) / WB : 0u;  // windows; the head is window m-1
        // full windows e = j, j + 16, ... <= m - 2, from the highest (Horner with Z_1088)
        int32_t e = (int32_t)m - 2 < (int32_t)j ? -1 : (int32_t)j + 16 * (((int32_t)m - 2 - (int32_t)j) / 16);
        uint32_t acc = 0;
        const uint32_t Lal = L;  // (aligned path: (R0 + L) % 4 == 0 for every record of the wave)
        bool firstw = true;
        if (!WORK) e = -1;  // floor probe: the DMA ring, parse and stores without the window CRCs
        while (__ballot(e >= 0)) {
            if (e >= 0) {
                const uint32_t A = R0 + Lal - WB * (uint32_t)(e + 1);
                uint32_t cA = 0, cB = 0;
                if (((R0 + L) & 3) == 0) {
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++) {
                        cA = crc.word(cA, lds_ld(A + 4 * t));
                        cB = crc.word(cB, lds_ld(A + 36 + 4 * t));
                    }
                    cA = crc.word(cA, lds_ld(A + 32));
                } else {
                    const uint32_t Aa = A & ~3u, s = A & 3u;
                    uint32_t w[18];
#pragma unroll
                    for (uint32_t t = 0; t < 18; t++) w[t] = lds_ld(Aa + 4 * t);
#pragma unroll
                    for (uint32_t t = 0; t < 8; t++) {
                        cA = crc.word(cA, __builtin_amdgcn_alignbyte(w[t + 1], w[t], s));
                        cB = crc.word(cB, __builtin_amdgcn_alignbyte(w[t + 10], w[t + 9], s));
                    }
                    cA = crc.word(cA, __builtin_amdgcn_alignbyte(w[9], w[8], s));
                }
                const uint32_t c = zap(Z32, cA) ^ cB;
                acc = firstw ? c : (zap(Z1088, acc) ^ c);
                firstw = false;
                e -= 16;
            }
        }
        // tree over the 16 lanes of the record: sum_j Z_{68 j}(acc_j)
        uint32_t v = acc, z;
        z = zap(Z68, v);  v = (j & 1) ? z : v;  v ^= __shfl_xor(v, 1, 64);
        z = zap(Z136, v); v = (j & 2) ? z : v;  v ^= __shfl_xor(v, 2, 64);
        z = zap(Z272, v); v = (j & 4) ? z : v;  v ^= __shfl_xor(v, 4, 64);
        z = zap(Z544, v); v = (j & 8) ? z : v;  v ^= __shfl_xor(v, 8, 64);
        // ---- hand the group's records to their batch lanes 4 (g % 16) + r
        const uint32_t gb = g & 15;
        const uint32_t wc = __shfl(v, (int)(16 * (lane & 3)), 64);
        if ((lane >> 2) == gb) {
            const uint32_t r = lane & 3;
            uint32_t sL = q.L[0], so = qoff[0], sst = q.st[0], sec = q.ec[0];
            uint64_t sa = q.a[0];
#pragma unroll
            for (uint32_t rr = 1; rr < G; rr++)
                if (r == rr) { sL = q.L[rr]; so = qoff[rr]; sst = q.st[rr]; sec = q.ec[rr]; sa = q.a[rr]; }
            b_L = sL; b_st = sst; b_ec = sec; b_wc = wc; b_a = sa;
            if (sL) {
                const uint32_t ha = (slot + so) & ~3u;
#pragma unroll
                for (uint32_t u = 0; u < 18; u++) hw[u] = lds_ld(ha + 4 * u);
            }
        }
        // ---- batch end: parse, lane = record
        if (gb == 15 || g + 1 == ngroups) {
            const uint32_t i = (g & ~15u) * G + lane;  // record index in this wave's range
            const bool valid = i < cnt;
            const bool inb = valid && b_st == BHG_ST_OK;
            const uint32_t Lr = inb ? b_L : 0u;
            const uint32_t hsh = (uint32_t)(b_a & 3);
            uint32_t rw[17];
#pragma unroll
            for (int u = 0; u < 17; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            const uint32_t mr = Lr ? (Lr + WB - 1) / WB : 1u;
            const uint32_t hl = Lr - WB * (mr - 1);
            // head CRC from ~0 over [0, hl), shifted past the m-1 full windows
            uint32_t hc = 0xffffffffu;
            const uint32_t nw = hl >> 2;
#pragma unroll
            for (uint32_t u = 0; u < 17; u++)
                if (u < nw) hc = crc.word(hc, rw[u]);
            if (hl & 3) {
                uint32_t wv2 = 0;
#pragma unroll
                for (uint32_t u = 0; u < 17; u++) wv2 = nw == u ? rw[u] : wv2;
                hc = crc.partial(hc, wv2, hl & 3);
            }
            const uint32_t sft = mr - 1;
            if (sft & 1) hc = zap(Z68, hc);
            if (sft & 2) hc = zap(Z136, hc);
            if (sft & 4) hc = zap(Z272, hc);
            if (sft & 8) hc = zap(Z544, hc);
            if (sft & 16) hc = zap(Z1088, hc);
            if (sft & 32) { hc = zap(Z1088, hc); hc = zap(Z1088, hc); }
            const uint32_t fullc = hc ^ b_wc;
            // readRecordHeader / readRecord / readKV (block2.go:31-66)
            uint32_t k = 0, vv = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
            uint64_t trailer = 255;
            bool rvalid = false;
            if (inb) {
                k = Lr >= 12 ? rw[0] : 0u;
                vv = Lr >= 12 ? rw[1] : 0u;
                fn = Lr >= 12 ? rw[2] : 0u;
                rvalid = Lr >= 12 && k != 0 && vv != 0 && (uint64_t)12 + k + vv == (uint64_t)Lr;
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
                        const uint32_t tbq = 12 + key_len, tw = tbq >> 2, ts = tbq & 3;
                        uint32_t a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
                        for (uint32_t u = 3; u <= 12; u++) {
                            a0 = tw == u ? rw[u] : a0;
                            a1 = tw == u ? rw[u + 1] : a1;
                            a2 = tw == u ? rw[u + 2] : a2;
                        }
                        trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                                  ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                    } else {
                        fnv = 0xdeadbeefu;  // lab: long keys not handled
                    }
                }
            }
            if (valid) {
                uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = b_st;
                uint64_t dtr = 0;
                if (inb) {
                    dcrc = crc_mask(~fullc);
                    if (rvalid) {
                        dk = 12; dkl = key_len; dvo = 12 + k; dvl = vv;
                        dtr = trailer; dfn = fn; dfnv = fnv;
                        if (expected_crc != nullptr && b_ec != dcrc) dst = BHG_ST_CRC_MISMATCH;
                    } else {
                        dst = BHG_ST_RECORD_NIL;
                    }
                }
                const uint64_t o = (uint64_t)(out + r0 + i);
                gst64_nt(o, (uint64_t)dk | ((uint64_t)dkl << 32));
                gst64_nt(o + 8, (uint64_t)dvo | ((uint64_t)dvl << 32));
                gst64_nt(o + 16, dtr);
                gst64_nt(o + 24, (uint64_t)dfn | ((uint64_t)dfnv << 32));
                gst64_nt(o + 32, (uint64_t)dcrc | ((uint64_t)dst << 32));
            }
            ops += 5;
        }
        o0 = o1;
        o1 = o2;
    }
    wait_vm(0);
}

}  // namespace dl

// ---- harness ----
static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static inline uint64_t rnd() {
    rng_state ^= rng_state << 13; rng_state ^= rng_state >> 7; rng_state ^= rng_state << 17;
    return rng_state;
}

template <int NW, int D, int WORK = 1>
static void launch(const uint8_t *src, uint64_t len, const bhg_handle *h, uint32_t n, const uint32_t *ec, bhg_desc *out,
                   const uint32_t *gz, int cus, hipStream_t s) {
    hipLaunchKernelGGL((dl::k_decode_dma<NW, D, WORK>), dim3(cus), dim3(64 * NW), 0, s, src, len, h, n, ec, out, gz);
}

static uint32_t *g_xtab = nullptr;
static void launch_product(const uint8_t *src, uint64_t len, const bhg_handle *h, uint32_t n, const uint32_t *ec,
                           bhg_desc *out, const uint32_t *, int cus, hipStream_t s) {
    bhg::Launch L;
    L.stream = s; L.num_cus = cus; L.ztab = nullptr; L.stab = nullptr; L.xtab = g_xtab;
    CK(bhg::launch_decode_dma(L, src, len, h, n, 0, ec, out, nullptr));
}

static uint32_t *g_ztab = nullptr;
static void launch_nb3(const uint8_t *src, uint64_t len, const bhg_handle *h, uint32_t n, const uint32_t *ec,
                       bhg_desc *out, const uint32_t *, int cus, hipStream_t s) {
    const uint64_t tiles = (n + 63) / 64;
    uint64_t need = (tiles + 7) / 8;
    uint32_t grid = (uint32_t)(need < (uint64_t)cus ? need : cus);
    hipLaunchKernelGGL((bhg::nb3::k_decode_tile_nb3<8, 2, 0>), dim3(grid), dim3(512), 0, s, src, len, h, n, ec, out, g_ztab);
}
template <int PF, int WPB = 8, int NCH = 2>
static void launch_tile(const uint8_t *src, uint64_t len, const bhg_handle *h, uint32_t n, const uint32_t *ec,
                        bhg_desc *out, const uint32_t *, int cus, hipStream_t s) {
    const uint64_t tiles = (n + 63) / 64;
    uint64_t need = (tiles + WPB - 1) / WPB;
    uint32_t grid = (uint32_t)(need < (uint64_t)cus ? need : cus);
    hipLaunchKernelGGL((bhg::k_decode_tile<WPB, NCH, PF>), dim3(grid), dim3(64 * WPB), 0, s, src, len, h, n, ec, out, g_ztab);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 30;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000000u;
    const uint32_t L = 1076, R = (128u << 20) / L + 1, TB = R * L + 12;
    const uint32_t ntab = (n + R - 1) / R;
    const uint64_t len = (uint64_t)ntab * TB;
    std::vector<uint8_t> host(len, 0);
    std::vector<bhg_handle> hh(n);
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t off = (uint64_t)(i / R) * TB + (uint64_t)(i % R) * L;
        uint8_t *p = &host[off];
        const uint32_t hdr[3] = {40, 1024, 1 + i / R};
        memcpy(p, hdr, 12);
        for (uint32_t b = 12; b < 44; b++) p[b] = (uint8_t)('a' + rnd() % 26);
        const uint64_t tr = ((uint64_t)(i + 1) << 8) | 1;
        memcpy(p + 44, &tr, 8);
        for (uint32_t b = 52; b < L; b += 8) { uint64_t x = rnd(); memcpy(p + b, &x, 8); }
        hh[i] = bhg_handle{off, L, 0};
    }
    if (n > 10) hh[7].length = 0;                                   // ILLEGAL_LENGTH
    if (n > 20) hh[13].length = L - 1;                              // RECORD_NIL
    bhg_ctx *ctx = bhg_create(0, 0);
    if (!ctx) { fprintf(stderr, "no ctx\n"); return 1; }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint8_t *src; bhg_handle *dh; uint32_t *ec; bhg_desc *o1, *o2; uint32_t *gz;
    CK(hipMalloc(&src, len + 64)); CK(hipMalloc(&dh, n * 16ull)); CK(hipMalloc(&ec, n * 4ull));
    CK(hipMalloc(&o1, n * 40ull)); CK(hipMalloc(&o2, n * 40ull)); CK(hipMalloc(&gz, dl::NZ * 4096));
    CK(hipMemcpy(src, host.data(), len, hipMemcpyHostToDevice));
    CK(hipMemcpy(dh, hh.data(), n * 16ull, hipMemcpyHostToDevice));
    std::vector<uint32_t> z(dl::NZ * 1024);
    const uint64_t zs[dl::NZ] = {32, 68, 136, 272, 544, 1088};
    for (uint32_t k = 0; k < dl::NZ; k++) crc32c_shift_table(zs[k], z.data() + 1024 * k);
    CK(hipMemcpy(gz, z.data(), z.size() * 4, hipMemcpyHostToDevice));
    hipStream_t s = (hipStream_t)bhg_stream(ctx);
    if (bhg_crc32c_masked_batch(ctx, src, len, dh, n, ec, s) != 0) { fprintf(stderr, "crc batch\n"); return 1; }
    CK(hipStreamSynchronize(s));
    // corrupt one expected CRC -> CRC_MISMATCH
    if (n > 30) { uint32_t x; CK(hipMemcpy(&x, ec + 29, 4, hipMemcpyDeviceToHost)); x ^= 1; CK(hipMemcpy(ec + 29, &x, 4, hipMemcpyHostToDevice)); }
    typedef void (*lfn)(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *, int, hipStream_t);
    struct V { const char *name; lfn fn; };
    static uint32_t *xt = nullptr;
    if (!xt) {
        std::vector<uint32_t> x(1024u * 6);
        const uint64_t zl[6] = {32, 68, 136, 272, 544, 1088};
        for (int k = 0; k < 6; k++) crc32c_shift_table(zl[k], x.data() + 1024 * k);
        CK(hipMalloc(&xt, x.size() * 4));
        CK(hipMemcpy(xt, x.data(), x.size() * 4, hipMemcpyHostToDevice));
    }
    g_xtab = xt;
    if (!g_ztab) {
        std::vector<uint32_t> zt(kZTabWords);
        build_tile_ztab(zt.data());
        CK(hipMalloc(&g_ztab, zt.size() * 4));
        CK(hipMemcpy(g_ztab, zt.data(), zt.size() * 4, hipMemcpyHostToDevice));
    }
    const V vs[] = {{"tile_pf2", launch_tile<2>}, {"tile_nb3", launch_nb3}, {"tile_pf0", launch_tile<0>},
                    {"tile_pf2_b", launch_tile<2>}, {"tile_nb3_b", launch_nb3}, {"tile_pf0_b", launch_tile<0>}};
    auto prod = [&]() { if (bhg_decode_batch(ctx, src, len, dh, n, 0, ec, o1, nullptr, 0, nullptr, s)) { fprintf(stderr, "prod\n"); exit(1); } };
    for (int it = 0; it < 200; it++) prod();  // clocks
    CK(hipStreamSynchronize(s));
    std::vector<bhg_desc> d1(n), d2(n);
    CK(hipMemcpy(d1.data(), o1, n * 40ull, hipMemcpyDeviceToHost));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](auto fn) {
        std::vector<float> ts;
        for (int it = 0; it < iters; it++) {
            CK(hipEventRecord(a, s)); fn(); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return std::make_pair(ts[ts.size() / 2], ts[0]);
    };
    const double alg = (double)n * 1136;
    auto tp = timeit(prod);
    printf("%-14s median %.4f ms best %.4f  frac %.4f\n", "product", tp.first, tp.second, alg / (tp.first * 1e-3) / 8e12);
    for (const V &v : vs) {
        CK(hipMemset(o2, 0xee, n * 40ull));
        v.fn(src, len, dh, n, ec, o2, gz, cus, s);
        CK(hipStreamSynchronize(s));
        CK(hipGetLastError());
        CK(hipMemcpy(d2.data(), o2, n * 40ull, hipMemcpyDeviceToHost));
        uint32_t bad = 0, first = 0xffffffffu;
        for (uint32_t i = 0; i < n; i++)
            if (memcmp(&d1[i], &d2[i], 40) != 0) { if (!bad) first = i; bad++; }
        auto t = timeit([&]() { v.fn(src, len, dh, n, ec, o2, gz, cus, s); });
        printf("%-14s median %.4f ms best %.4f  frac %.4f  mismatches %u (first %u)\n", v.name, t.first, t.second,
               alg / (t.first * 1e-3) / 8e12, bad, first);
        if (bad) {
            const uint32_t i = first;
            printf("  prod: crc %08x st %u fnv %08x tr %llx | lab: crc %08x st %u fnv %08x tr %llx\n", d1[i].crc,
                   d1[i].status, d1[i].fnv1, (unsigned long long)d1[i].trailer, d2[i].crc, d2[i].status, d2[i].fnv1,
                   (unsigned long long)d2[i].trailer);
        }
        fflush(stdout);
    }
    bhg_destroy(ctx);
    return 0;
}
