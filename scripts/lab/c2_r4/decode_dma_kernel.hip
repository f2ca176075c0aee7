// decode_dma_kernel.hip -- LAB (not product code; included by dma_lab.hip): the record decode
// as an LDS-DMA stream (gfx950).  Bit-exact against the product on the C2 batch, but 0.59-0.62 ms
// against the register-staged k_decode_tile's 0.25-0.27 on the same boxes (its no-CRC floor:
// 0.40-0.47 ms), so the product keeps k_decode_tile (profiles/r4/).
//
// k_decode_dma: readRecord + readKV + FNV-1 + masked CRC-32C (bithash/block2.go:31-66,
// compress.go:57-59, internal/hash/fnv.go:19-23, internal/crc/crc.go:19-33) for a batch of
// handles; MODE 0 is the NoCompressor decode, MODE 1 the snappy header pass (the same record
// checks and CRC plus snappy's decodedLen; bhg_snappy_dec.hip decodes the values after it).
//
// Each wave owns a contiguous range of handles and walks it in groups of 4 records.  A group's
// record bytes go HBM -> LDS with global_load_lds_dwordx4 (no VGPR staging, 16-B pieces of the
// 16-B aligned lines each record covers) into a ring of 3 slots per wave: while group g is
// computed, groups g+1 and g+2 are in flight (~8.6 KB per wave, ~69 KB per CU).  Every VMEM
// instruction of the loop is inline asm with exact vmcnt bookkeeping -- hipcc waits vmcnt(0)
// for an LDS-DMA at the next use of any ordinary load result (cdna_hip_programming.md §5),
// which would drain the ring every group -- and the handles / expected CRCs come through the
// scalar cache (lgkmcnt).
//   group compute, lane (r, j) = (lane / 16, lane % 16), record r of the group: the record's
//     full 68-B windows e = j, j+16, ... counted from the record end (Horner with Z_1088), each
//     as 2 chains (36 + 32 B, folded with Z_32); a 4-level tree over the 16 lanes (Z_68, Z_136,
//     Z_272, Z_544) gives W = sum_e Z_{68 e}(crc_0(window e)).  CRC linearity over GF(2):
//     crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B).
//   batch parse, lane = record of a 64-record batch (16 groups): the record head [0, hl),
//     hl = L - 68 (m - 1) in 1..68, copied from LDS at group time, gives readRecordHeader /
//     readRecord / readKV / FNV-1 / trailer, and the head CRC from crc.New's ~0, shifted past
//     the m - 1 full windows (Z_{68 (m-1)} by the bits of m - 1) and xored with W; then the
//     40-B descriptor (non-temporal stores).
// A record that is too long for a slot (> 4,352 B or the group's slot full) is read from
// global memory by its 16 lanes in the same window structure ("global mode"; correct for any
// length, slower).  CRC tables: CrcR8 (32 KiB, conflict free) + six 4-KiB shift tables, so the
// ring (8 waves x 3 x 4,416 B) fits beside them in one 160-KiB workgroup per CU.
#include "../../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../../bitalosdb_amd/csrc/bhg_device.h"
#include "../../../bitalosdb_amd/csrc/bhg_internal.h"

namespace bhg {

namespace {

constexpr uint32_t DG = 4;                    // records per group
constexpr uint32_t DWB = 68;                  // window bytes (17 words)
constexpr uint32_t DSLOT = 4416;              // ring slot bytes: 276 pieces (4 C2 records at any alignment)
constexpr uint32_t DSLOT_PIECES = DSLOT / 16;
constexpr uint32_t DSTAGE_MAX = 64 * DWB;     // staged records: at most 63 full windows (head shift bits 0..5)
constexpr uint32_t DNW = 8;                   // waves per workgroup
constexpr uint32_t DD = 3;                    // ring slots per wave
constexpr uint32_t DNZ = 6;                   // Z_32, Z_68, Z_136, Z_272, Z_544, Z_1088
constexpr uint32_t DLDS = CrcR8::kBytes + DNZ * 4096 + DNW * DD * DSLOT;
static_assert(DLDS <= 160 * 1024, "one workgroup per CU");

// ---- VMEM through inline asm ----
__device__ __forceinline__ void glds16(uint64_t gaddr, uint32_t lds_byte) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gaddr), "s"(lds_byte)
                 : "memory", "m0");
}
__device__ __forceinline__ void gst64_nt(uint64_t a, uint64_t v) {
    asm volatile("global_store_dwordx2 %0, %1, off nt" ::"v"(a), "v"(v) : "memory");
}
// s_waitcnt vmcnt(n), n wave-uniform at run time (a wave never has more than 63 outstanding)
__device__ __forceinline__ void wait_vm(uint32_t n) {
#define W_(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
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

// crc_0 of one 68-B window whose first byte is at LDS byte address A (2 chains: 36 + 32 B)
__device__ __forceinline__ uint32_t win_lds(const CrcR8 &crc, uint32_t Z32, uint32_t A) {
    uint32_t cA = 0, cB = 0;
    if ((A & 3) == 0) {
#pragma unroll
        for (uint32_t t = 0; t < 8; t++) {
            cA = crc.word(cA, lds_ld32(A + 4 * t));
            cB = crc.word(cB, lds_ld32(A + 36 + 4 * t));
        }
        cA = crc.word(cA, lds_ld32(A + 32));
    } else {
        const uint32_t Aa = A & ~3u, s = A & 3u;
        uint32_t w[18];
#pragma unroll
        for (uint32_t t = 0; t < 18; t++) w[t] = lds_ld32(Aa + 4 * t);
#pragma unroll
        for (uint32_t t = 0; t < 8; t++) {
            cA = crc.word(cA, __builtin_amdgcn_alignbyte(w[t + 1], w[t], s));
            cB = crc.word(cB, __builtin_amdgcn_alignbyte(w[t + 10], w[t + 9], s));
        }
        cA = crc.word(cA, __builtin_amdgcn_alignbyte(w[9], w[8], s));
    }
    return zshift(Z32, cA) ^ cB;
}

// the same from global memory (global-mode records; [a, a + 68) inside [.., end))
__device__ __forceinline__ uint32_t win_global(const CrcR8 &crc, uint32_t Z32, uint64_t a, uint64_t end) {
    uint32_t cA = 0, cB = 0;
#pragma unroll
    for (uint32_t t = 0; t < 8; t++) {
        cA = crc.word(cA, ldu32(a + 4 * t, end));
        cB = crc.word(cB, ldu32(a + 36 + 4 * t, end));
    }
    cA = crc.word(cA, ldu32(a + 32, end));
    return zshift(Z32, cA) ^ cB;
}

}  // namespace

template <int MODE>
__global__ __launch_bounds__(64 * DNW) void k_decode_dma(const uint8_t *__restrict__ src, uint64_t src_len,
                                                        const bhg_handle *__restrict__ handles, uint32_t n,
                                                        const uint32_t *__restrict__ expected_crc,
                                                        bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes,
                                                        const uint32_t *__restrict__ xtab) {
    // ALL of the kernel's LDS in one array (a second __shared__ object can make hipcc wait for the
    // DMA before every LDS read): CrcR8 | Z tables | ring
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[DLDS / 4];
    const uint32_t tb = lds_addr(lds_all), zb = tb + CrcR8::kBytes, rb = zb + DNZ * 4096;
    CrcR8::fill(tb);
    {
        // xtab: the lab's Z_32, Z_68, Z_136, Z_272, Z_544, Z_1088 (1024 words each, this order)
        for (uint32_t t = threadIdx.x; t < DNZ * 1024; t += blockDim.x) lds_all[CrcR8::kBytes / 4 + t] = xtab[t];
    }
    __syncthreads();
    const CrcR8 crc(tb);
    const uint32_t Z32 = zb, Z68 = zb + 4096, Z136 = zb + 8192, Z272 = zb + 12288, Z544 = zb + 16384,
                   Z1088 = zb + 20480;

    const uint32_t lane = threadIdx.x & 63, wv = uni(threadIdx.x >> 6);  // wave-uniform for the compiler
    const uint32_t r4 = lane >> 4, j = lane & 15;
    const uint32_t gw = blockIdx.x * DNW + wv, nwt = gridDim.x * DNW;
    const uint32_t per = n / nwt, rem = n % nwt;
    const uint32_t r0 = gw * per + (gw < rem ? gw : rem);
    const uint32_t cnt = per + (gw < rem ? 1u : 0u);
    const uint32_t ngroups = (cnt + DG - 1) / DG;
    const uint32_t ring = rb + wv * DD * DSLOT;
    const uint64_t base = (uint64_t)src, end = base + src_len;

    // a group's records (wave-uniform, scalar registers; re-read through the scalar cache)
    struct GInfo {
        uint64_t a[DG];   // absolute record address
        uint32_t L[DG];   // length (0: no record / out of range)
        uint32_t st[DG];  // status before decode (0xffffffff: past the wave's range)
        uint32_t ec[DG];  // expected CRC
    };
    auto ginfo = [&](uint32_t g, bool want_ec) {
        GInfo q;
        // every scalar load of the group first (index clamped into the range), then one lgkmcnt wait
        // -- loads interleaved with each record's checks were waited for record by record
        bhg_handle hh[DG];
        uint32_t ee[DG];
#pragma unroll
        for (uint32_t r = 0; r < DG; r++) {
            const uint32_t i = DG * g + r;
            const uint32_t ic = r0 + (i < cnt ? i : (cnt ? cnt - 1 : 0u));
            hh[r] = handles[ic];
            ee[r] = (want_ec && expected_crc != nullptr) ? expected_crc[ic] : 0u;
        }
#pragma unroll
        for (uint32_t r = 0; r < DG; r++) {
            const uint32_t i = DG * g + r;
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
    // slot layout: staged record r at byte pc_r * 16 + (a_r & 15), its 16-B aligned lines as pieces;
    // a record that does not fit (or is longer than DSTAGE_MAX) is not staged (off = ~0)
    auto layout = [&](const GInfo &q, uint32_t *off, uint32_t *pc) {
        pc[0] = 0;
#pragma unroll
        for (uint32_t r = 0; r < DG; r++) {
            uint32_t np = q.L[r] ? (uint32_t)(((q.a[r] + q.L[r] + 15) >> 4) - (q.a[r] >> 4)) : 0u;
            const bool fit = q.L[r] <= DSTAGE_MAX && pc[r] + np <= DSLOT_PIECES;
            if (!fit) np = 0;
            off[r] = fit ? pc[r] * 16 + (uint32_t)(q.a[r] & 15) : 0xffffffffu;
            pc[r + 1] = pc[r] + np;
        }
    };
    uint32_t ops = 0;  // VM instructions this wave has issued (DMAs + descriptor stores)
    auto issue = [&](uint32_t g) {
        const GInfo q = ginfo(g, false);
        const uint32_t slot = ring + (g % DD) * DSLOT;
        uint32_t off[DG], pc[DG + 1];
        layout(q, off, pc);
        const uint32_t np = pc[DG];
        for (uint32_t x0 = 0; x0 < np; x0 += 64) {
            const uint32_t x = x0 + lane;
            uint64_t s = (q.a[0] & ~15ull) + 16ull * x;
#pragma unroll
            for (uint32_t r = 1; r < DG; r++)
                if (x >= pc[r]) s = (q.a[r] & ~15ull) + 16ull * (x - pc[r]);
            // a 16-B aligned line that holds a byte of [a, a + L) never crosses a page, so the
            // pieces past src_len (at most 15 B) cannot fault; lane 0 is always active (no op skipped)
            if (x < np) glds16(s, uni(slot + 16 * x0));
            ops++;
        }
        return ops;
    };

    // per-lane batch state: lane = record 64 b + lane of this wave's range
    uint32_t hw[18];
#pragma unroll
    for (int u = 0; u < 18; u++) hw[u] = 0;
    uint32_t b_st = 0, b_L = 0, b_ec = 0, b_wc = 0;
    uint64_t b_a = 0;

    uint32_t o0 = 0, o1 = 0, o2 = 0;  // VM-op counts after groups g, g+1, g+2 were issued
    if (ngroups > 0) o0 = issue(0);
    if (ngroups > 1) o1 = issue(1);
    GInfo qc = ginfo(0, true);        // group g's info, loaded one iteration ahead
    for (uint32_t g = 0; g < ngroups; g++) {
        if (g + 2 < ngroups) o2 = issue(g + 2);
        wait_vm(ops - o0);
        const GInfo q = qc;
        if (g + 1 < ngroups) qc = ginfo(g + 1, true);
        uint32_t qoff[DG], qpc[DG + 1];
        layout(q, qoff, qpc);
        const uint32_t slot = ring + (g % DD) * DSLOT;
        // ---- lane (r4, j): record r4's full windows e = j, j + 16, ... <= m - 2
        uint32_t L = q.L[0], off = qoff[0];
        uint64_t ra = q.a[0];
#pragma unroll
        for (uint32_t r = 1; r < DG; r++)
            if (r4 == r) { L = q.L[r]; off = qoff[r]; ra = q.a[r]; }
        const bool staged = off != 0xffffffffu;
        const uint32_t R0 = slot + off;
        const uint32_t m = L ? (L + DWB - 1) / DWB : 0u;  // windows; the head is window m - 1
        int32_t e = (int32_t)m - 2 < (int32_t)j ? -1 : (int32_t)j + 16 * (((int32_t)m - 2 - (int32_t)j) / 16);
        uint32_t acc = 0;
        while (__ballot(e >= 0)) {
            if (e >= 0) {
                const uint32_t wo = L - DWB * (uint32_t)(e + 1);  // record offset of the window
                const uint32_t c = staged ? win_lds(crc, Z32, R0 + wo) : win_global(crc, Z32, ra + wo, end);
                acc = zshift(Z1088, acc) ^ c;  // Horner (Z(0) = 0: the first window needs no case)
                e -= 16;
            }
        }
        // tree over the 16 lanes of the record: sum_j Z_{68 j}(acc_j)
        uint32_t v = acc, z;
        z = zshift(Z68, v);  v = (j & 1) ? z : v;  v ^= __shfl_xor(v, 1, 64);
        z = zshift(Z136, v); v = (j & 2) ? z : v;  v ^= __shfl_xor(v, 2, 64);
        z = zshift(Z272, v); v = (j & 4) ? z : v;  v ^= __shfl_xor(v, 4, 64);
        z = zshift(Z544, v); v = (j & 8) ? z : v;  v ^= __shfl_xor(v, 8, 64);
        // ---- hand the group's records to their batch lanes 4 (g % 16) + r, with the record head
        const uint32_t gb = g & 15;
        const uint32_t wc = __shfl(v, (int)(16 * (lane & 3)), 64);
        if ((lane >> 2) == gb) {
            const uint32_t r = lane & 3;
            uint32_t sL = q.L[0], so = qoff[0], sst = q.st[0], sec = q.ec[0];
            uint64_t sa = q.a[0];
#pragma unroll
            for (uint32_t rr = 1; rr < DG; rr++)
                if (r == rr) { sL = q.L[rr]; so = qoff[rr]; sst = q.st[rr]; sec = q.ec[rr]; sa = q.a[rr]; }
            b_L = sL; b_st = sst; b_ec = sec; b_wc = wc; b_a = sa;
            if (sL && so != 0xffffffffu) {
                const uint32_t ha = (slot + so) & ~3u;
#pragma unroll
                for (uint32_t u = 0; u < 18; u++) hw[u] = lds_ld32(ha + 4 * u);
            } else if (sL) {  // global mode: the head from memory
                const uint64_t ga = sa & ~3ull;
#pragma unroll
                for (uint32_t u = 0; u < 18; u++) hw[u] = ld32_safe(ga + 4 * u, end);
            }
        }
        // ---- batch end: lane = record
        if (gb == 15 || g + 1 == ngroups) {
            const uint32_t i = (g & ~15u) * DG + lane;  // record index in this wave's range
            const bool valid = i < cnt;
            const bool inb = valid && b_st == BHG_ST_OK;
            const uint32_t Lr = inb ? b_L : 0u;
            const uint32_t hsh = (uint32_t)(b_a & 3);
            uint32_t rw[17];
#pragma unroll
            for (int u = 0; u < 17; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
            const uint32_t mr = Lr ? (Lr + DWB - 1) / DWB : 1u;
            const uint32_t hl = Lr - DWB * (mr - 1);
            // head CRC from crc.New's ~0 over [0, hl), then past the m - 1 full windows
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
            uint32_t sft = mr - 1;
            if (sft & 1) hc = zshift(Z68, hc);
            if (sft & 2) hc = zshift(Z136, hc);
            if (sft & 4) hc = zshift(Z272, hc);
            if (sft & 8) hc = zshift(Z544, hc);
            for (sft >>= 4; sft; sft--) hc = zshift(Z1088, hc);  // 16 windows per Z_1088 (global mode: any length)
            const uint32_t fullc = hc ^ b_wc;
            // readRecordHeader / readRecord / readKV (block2.go:31-66)
            const uint64_t p = b_a;
            uint32_t k = 0, vv = 0, fn = 0, key_len = 0, fnv = BHG_FNV_OFFSET;
            uint64_t trailer = 255;  // InternalKeyKindInvalid when ikeySize < 8
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
                        for (uint32_t u = 3; u <= 12; u++) {  // tb <= 48: the trailer ends by byte 56
                            a0 = tw == u ? rw[u] : a0;
                            a1 = tw == u ? rw[u + 1] : a1;
                            a2 = tw == u ? rw[u + 2] : a2;
                        }
                        trailer = (uint64_t)__builtin_amdgcn_alignbyte(a1, a0, ts) |
                                  ((uint64_t)__builtin_amdgcn_alignbyte(a2, a1, ts) << 32);
                    } else {
                        fnv = fnv1_range(p + 12, key_len, end);
                        trailer = ldu64(p + 12 + k - 8, end);
                    }
                }
            }
            if (valid) {
                uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = b_st;
                uint64_t dtr = 0, dsize = 0;
                if (inb) {
                    dcrc = crc_mask(~fullc);  // crc.go:31-33
                    dst = BHG_ST_OK;
                    if (rvalid) {
                        dk = 12; dkl = key_len; dtr = trailer; dfn = fn; dfnv = fnv;
                        if (MODE == 0) {
                            dvo = 12 + k; dvl = vv;  // noCompressor.Decode: zero-copy view (compress.go:57-59)
                        } else {
                            // snappy decodedLen (golang/snappy decode.go): the uvarint at the value start
                            uint64_t x = 0;
                            uint32_t s = 0, hdr = 0;
                            bool ok = false;
                            const uint64_t vp = p + 12 + k;
                            const bool inw = k <= 43;  // its first 5 bytes inside the head words (< 60 B)
                            for (uint32_t b = 0; b < 10 && b < vv; b++) {
                                uint32_t c;
                                if (inw && b < 5) {
                                    const uint32_t o = 12 + k + b;
                                    uint32_t wd = 0;
#pragma unroll
                                    for (uint32_t u = 0; u < 15; u++) wd = (o >> 2) == u ? rw[u] : wd;
                                    c = (wd >> (8 * (o & 3))) & 0xffu;
                                } else {
                                    c = gld<uint8_t>(vp + b);
                                }
                                if (c < 0x80) {
                                    ok = !(b == 9 && c > 1);
                                    x |= (uint64_t)c << s;
                                    ok = ok && x <= 0xffffffffull;
                                    hdr = b + 1;
                                    break;
                                }
                                x |= (uint64_t)(c & 0x7f) << s;
                                s += 7;
                            }
                            // a stream cannot expand more than 64/3 x (a 3-byte copy emits 64 bytes)
                            if (!ok || x * 3 > (uint64_t)(vv - hdr) * 64) {
                                dst = BHG_ST_SNAPPY_CORRUPT;
                            } else {
                                dsize = x;
                                dvl = (uint32_t)x;  // provisional: the snappy kernel finalises
                                dvo = 12 + k;       // provisional: compressed payload offset
                            }
                        }
                        if (expected_crc != nullptr && dst == BHG_ST_OK && b_ec != dcrc) dst = BHG_ST_CRC_MISMATCH;
                    } else {
                        dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil (reader.go:260-264)
                    }
                }
                const uint64_t o = (uint64_t)(out + r0 + i);
                gst64_nt(o, (uint64_t)dk | ((uint64_t)dkl << 32));
                gst64_nt(o + 8, (uint64_t)dvo | ((uint64_t)dvl << 32));
                gst64_nt(o + 16, dtr);
                gst64_nt(o + 24, (uint64_t)dfn | ((uint64_t)dfnv << 32));
                gst64_nt(o + 32, (uint64_t)dcrc | ((uint64_t)dst << 32));
                if (MODE == 1) gst64_nt((uint64_t)(sizes + r0 + i), dsize);
            }
            ops += MODE == 1 ? 6 : 5;
#pragma unroll
            for (int u = 0; u < 18; u++) hw[u] = 0;
        }
        o0 = o1;
        o1 = o2;
    }
    wait_vm(0);
}

hipError_t launch_decode_dma(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             int mode, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes) {
    // one 8-wave workgroup per CU (LDS-bound); each wave takes an equal contiguous share of the handles
    uint32_t grid = (uint32_t)L.num_cus;
    const uint32_t need = (n + 64 * DNW - 1) / (64 * DNW);  // at least 64 records per wave when n is small
    if (need < grid) grid = need ? need : 1;
    if (mode == 0)
        hipLaunchKernelGGL(k_decode_dma<0>, dim3(grid), dim3(64 * DNW), 0, L.stream, src, src_len, h, n, expected_crc,
                           out, sizes, L.xtab);
    else
        hipLaunchKernelGGL(k_decode_dma<1>, dim3(grid), dim3(64 * DNW), 0, L.stream, src, src_len, h, n, expected_crc,
                           out, sizes, L.xtab);
    return hipGetLastError();
}

}  // namespace bhg
