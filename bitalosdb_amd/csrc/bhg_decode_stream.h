// bhg_decode_stream.h -- the NoCompressor batch decode for gfx950 (and the
// header / CRC pass of the snappy decode): readRecordHeader + readRecord +
// readKV + FNV-1 + masked CRC-32C per block (bithash/block2.go:31-66,
// compress.go:57-59, internal/hash/fnv.go:19-23, internal/crc/crc.go:19-33).
//
// A wave takes tiles of 64 consecutive handles (lane r = record r of the
// tile).  Each record of length L is cut into m = ceil(L / 128) windows of
// 128 B aligned to the record END: windows 1..m-1 are full, window 0 (the
// head) holds the first hl = L - 128 (m-1) bytes, left-padded with 128 - hl
// zero bytes.  The tile's windows are numbered record-major (M_r = exclusive
// prefix of m over the tile) and streamed in passes of 64: lane l of pass p
// takes window 64 p + l.  Consecutive lanes therefore read consecutive
// 128-B windows: a pass reads ~8 KiB of the table nearly contiguously, every
// byte once (the previous tile kernel read each record head twice, 13 % HBM
// over-fetch).
//
// Per window (lane): NCH interleaved slice-by-4 chains of 32/NCH words from
// state 0, folded with Z_{128/NCH} -> crc_0(window).  For the head window the
// pad bytes are zeroed (leading zeros leave a state-0 CRC unchanged) and Go's
// initial state ^0 enters as E[hl] = Z_hl(0xFFFFFFFF), by linearity:
//     crc_{~0}(R) = crc_0(R) ^ Z_|R|(~0),   crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B).
// The record state is the Horner sum S_q = Z_128(S_{q-1}) ^ c_q over its
// windows: a SEGMENTED inclusive scan across the wave (Hillis-Steele, level
// j adds Z_{128 2^j}(v_{k-2^j}) when lane k-2^j is in the same record;
// segments start at head windows), with the state of a record that runs past
// the pass carried into lane 0 of the next pass.  Only ceil(log2(max m))
// levels run.  The record lane pulls its state from the lane that holds its
// last window.  Header / UserKey / trailer words (64 B at the record start)
// are loaded by the record lane in the pass that streams the record's head
// (same lines, L2-hot) and parsed once per tile.
//
// LDS: Crc4Perm (slice-by-4 replicated 32x, 128 KiB, conflict free) + the
// fold table + six scan tables + E = 156.5 KiB -> one workgroup per CU.
#pragma once
#include "bhg_crc_tables.h"
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

// Global table set of one (window, chains) configuration (words), built on the
// host, owned by the context and copied into LDS by the kernel:
//   Zf = Z_{win / nch} (chain fold), Zs[j] = Z_{win * 2^j}, j = 0..5 (scan
//   levels), E[k] = Z_{4k}(~0), k = 0..win/4 (head init state).
constexpr uint32_t kStreamZf = 0, kStreamZs = 1024, kStreamE = 1024 + 6 * 1024;
constexpr uint32_t kStreamTabWords = kStreamE + 128;
inline void build_stream_tab(uint32_t *out, uint32_t win, uint32_t nch) {
    crc32c_shift_table(win / nch, out + kStreamZf);
    for (uint32_t j = 0; j < 6; j++) crc32c_shift_table((uint64_t)win << j, out + kStreamZs + 1024 * j);
    for (uint32_t k = 0; k < 128; k++)
        out[kStreamE + k] = k <= win / 4 ? gf2_apply(crc32c_zero_bytes(4 * k), 0xffffffffu) : 0;
}

namespace stream_detail {

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = __shfl((uint32_t)v, src, 64), hi = __shfl((uint32_t)(v >> 32), src, 64);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Z_n(c) from a 4 x 256-word shift table
__device__ __forceinline__ uint32_t zapply(const uint32_t *Zt, uint32_t c) {
    return Zt[c & 255u] ^ Zt[256 + ((c >> 8) & 255u)] ^ Zt[512 + ((c >> 16) & 255u)] ^ Zt[768 + (c >> 24)];
}

// dword at the 4-aligned address a, or -- when that dword holds no byte of
// the source range -- the nearest one that does (lo4 / hi4: the first / last
// dword holding a byte of the range).  Never faults (a dword with a byte of
// the range lies on the range's pages) and keeps every loaded byte that is
// used: bytes outside the range are only ever the head's zero padding (masked)
// or the unused tail of a window's 33rd dword.
__device__ __forceinline__ uint32_t ld32_clamp(uint64_t a, uint64_t lo4, uint64_t hi4) {
    return gld<uint32_t>(a < lo4 ? lo4 : (a > hi4 ? hi4 : a));
}

// wave_incl_add / wave_incl_max: bhg_device.h

}  // namespace stream_detail

// MODE 0: NoCompressor.  MODE 1: snappy header pass (CRC + header +
// decodedLen varint -> sizes[i]; the value is decoded by the snappy kernel).
// KO (lab only, knock-outs for timing; outputs are then wrong): bit 0 no CRC
// chains, 1 no scan, 2 no header loads, 3 no chain fold, 4 uniform-m locate,
// 5 no head init / tail, 6 no descriptor stores, 7 no shift-table loads in the prologue.
// LONG: records longer than kLongRec own no windows (the header words are loaded on their own); their
// CRC and CRC status are left to the long-record pass (launch_long_crc), run right after this one
template <int MODE, int NCH, int WPB, int WIN = 128, int PIPE = 0, int KO = 0, int LONG = 0>
__global__ __launch_bounds__(64 * WPB) void k_decode_stream(const uint8_t *__restrict__ src, uint64_t src_len,
                                                            const bhg_handle *__restrict__ handles, uint32_t n,
                                                            const uint32_t *__restrict__ expected_crc,
                                                            bhg_desc *__restrict__ out, uint64_t *__restrict__ sizes,
                                                            const uint32_t *__restrict__ gtab,
                                                            uint32_t *__restrict__ lists, uint32_t sub_cap) {
    using namespace stream_detail;
    static_assert(WIN == 128 || WIN == 256, "128- or 256-byte windows");
    constexpr int NW = WIN / 4;   // words per window
    constexpr int CW = NW / NCH;  // words per chain
    static_assert(CW * NCH == NW && CW >= 4, "chain split");
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t Zf[1024];
    __shared__ __attribute__((aligned(16))) uint32_t Zs[6 * 1024];
    __shared__ uint32_t E[128];
    const Crc4Perm crc(T);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint64_t lo4 = base & ~3ull, hi4 = (end - 1) & ~3ull;  // first / last dword holding source bytes
    const uint64_t safe = (base + 3) & ~3ull;                     // stand-in load address (interior tiles)
    const uint64_t lowmask = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint32_t ntiles = (n + 63) / 64;
    const uint32_t tstride = gridDim.x * WPB;
    // wave-major tile index: waves that take one tile more than the others are spread over every CU
    uint32_t tile = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    // the next tile's handles and the expected CRCs are loaded with no branch around them
    // (index clamped; see fetch below for why)
    auto hidx = [&](uint32_t t) { const uint32_t x = t * 64 + lane; return x < n ? x : n - 1; };
    const uint32_t *ecp = expected_crc != nullptr ? expected_crc : gtab;
    const uint32_t emask = expected_crc != nullptr ? 0xffffffffu : 0u;
    bhg_handle hn = handles[hidx(tile < ntiles ? tile : 0)];
    // (the first tile's handles are in flight while the LDS tables are built: C3 step 0.9383 vs
    // 0.9406 ms, 3 alternating runs each, profiles/r4/early_lab_stream_handles.txt)
    Crc4Perm::fill(T);
    if (!(KO & 128)) {  // all loads issued before the first LDS store (one memory round trip)
        constexpr uint32_t NT = 64 * WPB, NZ = (7 * 1024 + NT - 1) / NT;
        uint32_t v[NZ];
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++) {
            const uint32_t t = threadIdx.x + r * NT;
            v[r] = t < 7 * 1024 ? gtab[kStreamZf + t] : 0u;  // Zf and Zs are contiguous in gtab
        }
        const uint32_t e = threadIdx.x < 128 ? gtab[kStreamE + threadIdx.x] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < NZ; r++) {
            const uint32_t t = threadIdx.x + r * NT;
            if (t < 1024) Zf[t] = v[r];
            else if (t < 7 * 1024) Zs[t - 1024] = v[r];
        }
        if (threadIdx.x < 128) E[threadIdx.x] = e;
    }
    __syncthreads();
    for (; tile < ntiles; tile += tstride) {
        const bhg_handle h = hn;
        const uint32_t i = tile * 64 + lane;
        {
            const uint32_t tn = tile + tstride;
            hn = handles[hidx(tn < ntiles ? tn : tile)];
        }
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
        const bool lrec = LONG && L > kLongRec;
        const uint32_t m = lrec ? 0u : (uint32_t)(((uint64_t)L + WIN - 1) / WIN);
        const uint32_t pad = (uint32_t)WIN * m - L;  // 0..WIN-1 (head left padding)
        const uint32_t ecrc = ecp[(i < n ? i : n - 1) & emask];
        // record-major window numbering: M = exclusive prefix of m over the tile
        const uint32_t incl = wave_incl_add(m);
        const uint32_t M = incl - m;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t mx = __builtin_amdgcn_readlane(wave_incl_max(m < 64 ? m : 64u), 63);
        const uint32_t levels = __builtin_amdgcn_readfirstlane(mx <= 1 ? 0u : 32u - __builtin_clz(mx - 1));
        // window g of this record starts at Bw + WIN g (mod 2^64); see the head rule in window_crc
        const uint64_t Bw = p + L - (uint64_t)WIN * ((uint64_t)m + M);
        // records owning windows; "dense" = they are lanes 0..k-1 (rank of a record = its lane)
        const uint64_t vmask = __ballot(m != 0);
        const bool dense = (vmask & (vmask + 1)) == 0;
        // interior tile: every window and header load of the tile stays inside the source, so
        // windows are fetched with plain 16-B loads (else: clamped dword loads)
        const bool edge_rec = inb && !(h.offset >= WIN && h.offset + (L > 56 ? L : 56u) + 8 <= src_len);
        const bool interior = __ballot(edge_rec) == 0 && src_len >= WIN + 64;
        uint32_t rcrc = 0;
        uint32_t hw[16];
#pragma unroll
        for (int t = 0; t < 16; t++) hw[t] = 0;
        uint32_t carry = 0, hb = 0;  // carried record state; heads seen in earlier passes
        const uint32_t npass = (total + 63) >> 6;

        struct PassIn {
            uint64_t A;     // window start (absolute)
            uint32_t padr;  // head padding of the window's record
            bool head, act;
        };
        // window -> record: the pass's head windows form a bit mask (OR-reduced from the record
        // lanes); a window's record has rank hb + (heads at or before it) - 1 among the
        // records that own windows
        auto locate = [&](uint32_t ps) {
            PassIn pi;
            if (KO & 256) {  // probe addressing (lab): the tile's first record start + 8 KB per pass
                const uint64_t b0 = readfirstlane_u64(p);
                pi.act = ps * 64 + lane < total;
                pi.head = false;
                pi.padr = 0;
                const uint64_t a = b0 + 8192ull * ps + (uint64_t)WIN * lane, amax = end - WIN - 64;
                pi.A = a < amax ? a : amax;  // the tile's last pass may run past the source
                return pi;
            }
            if (KO & 16) {  // uniform m, dense tile (lab data): r = g / m
                const uint32_t mu = __builtin_amdgcn_readfirstlane(m);
                const uint32_t g = ps * 64 + lane;
                const uint32_t r = (g / mu) & 63;
                pi.act = g < total;
                pi.head = pi.act && (g % mu) == 0;
                const uint32_t padr = __shfl(pad, (int)r, 64);
                pi.padr = padr;
                pi.A = shfl64(Bw, (int)r) + (uint64_t)WIN * g - (pi.head ? (((uint32_t)WIN - padr) & 3u) : 0u);
                return pi;
            }
            const uint32_t g0 = ps * 64, g = g0 + lane;
            const bool hp = m != 0 && M >= g0 && M < g0 + 64;
            const uint64_t bit = hp ? (1ull << (M - g0)) : 0ull;
            const uint32_t hlo = __builtin_amdgcn_readlane(wave_incl_or((uint32_t)bit), 63);
            const uint32_t hhi = __builtin_amdgcn_readlane(wave_incl_or((uint32_t)(bit >> 32)), 63);
            const uint64_t hmask = (uint64_t)hlo | ((uint64_t)hhi << 32);
            pi.act = g < total;
            pi.head = pi.act && ((hmask >> lane) & 1ull);
            const uint32_t rank = hb + (uint32_t)__builtin_popcountll(hmask & lowmask) - 1u;
            uint32_t r = rank;
            if (!dense) {  // rank -> lane: position of the rank-th set bit of vmask
                uint32_t pos = 0;
#pragma unroll
                for (uint32_t step = 32; step; step >>= 1) {
                    const uint32_t t = pos + step;
                    const uint64_t below = t >= 64 ? vmask : (vmask & ((1ull << t) - 1ull));
                    if ((uint32_t)__builtin_popcountll(below) <= rank) pos = t;
                }
                r = pos;
            }
            r &= 63;
            hb += (uint32_t)__builtin_popcountll(hmask);
            const uint32_t padr = __shfl(pad, (int)r, 64);
            pi.padr = padr;
            // head window: ends at record byte hl' = hl & ~3 (hl = WIN - pad), the hl & 3 tail
            // bytes after it are absorbed byte-wise (window_crc)
            pi.A = shfl64(Bw, (int)r) + (uint64_t)WIN * g - (pi.head ? (((uint32_t)WIN - padr) & 3u) : 0u);
            return pi;
        };
        // Loads are issued with no branch around them (a branch would make the compiler's
        // count of outstanding loads at the merge assume the fewer, and wait for the next
        // pass's loads too early): lanes with nothing to load read `safe`.  Every load of a
        // pass targets that pass's own buffers (a load into a register another pass's load
        // may still write waits for it).
        auto fetch = [&](const PassIn &pi, uint32_t ps, uint32_t (&w)[NW + 2], uint32_t (&hwt)[16], bool inter) {
            const uint32_t g0 = ps * 64;
            const uint64_t a = pi.A & ~3ull;
            if (inter) {
                const uint64_t la = pi.act ? a : safe;
#pragma unroll
                for (int t = 0; t < NW / 4; t++) {
                    const u32x4 x = gld<u32x4_a4>(la + 16 * t);
                    w[4 * t] = x.x; w[4 * t + 1] = x.y; w[4 * t + 2] = x.z; w[4 * t + 3] = x.w;
                }
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                typedef u32x2 u32x2_a4 __attribute__((aligned(4)));
                const u32x2 y = gld<u32x2_a4>(la + WIN);
                w[NW] = y.x; w[NW + 1] = y.y;
            } else {
#pragma unroll
                for (int t = 0; t < NW + 2; t++) w[t] = ld32_clamp(a + 4 * t, lo4, hi4);
            }
            // the record lane fetches its header words in the pass that streams its head (L2-hot)
            const bool hp = m != 0 && M >= g0 && M < g0 + 64;
            const uint64_t ha = p & ~3ull;
            if (KO & 4) {
            } else if (inter) {
                const uint64_t lh = hp ? ha : safe;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const u32x4 x = gld<u32x4_a4>(lh + 16 * t);
                    hwt[4 * t] = x.x; hwt[4 * t + 1] = x.y; hwt[4 * t + 2] = x.z; hwt[4 * t + 3] = x.w;
                }
            } else {
#pragma unroll
                for (int t = 0; t < 16; t++) hwt[t] = ld32_clamp(ha + 4 * t, lo4, hi4);
            }
        };
        // crc_0 of a window.  Head: words before the record start are zeroed (one bfe per word:
        // the head window ends on a whole word), Go's initial ^0 enters as E[hl'/4] =
        // Z_hl'(~0), then the hl & 3 tail bytes are absorbed (slice-by-<=3, one round).
        auto window_crc = [&](const PassIn &pi, const uint32_t (&w)[NW + 2]) {
            const uint32_t sh = (uint32_t)(pi.A & 3);
            uint32_t V;
            if (KO & 1) {
                uint32_t v4[4] = {0, 0, 0, 0};
#pragma unroll
                for (int t = 0; t < NW; t++) v4[t & 3] ^= __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                V = v4[0] ^ v4[1] ^ v4[2] ^ v4[3];
                return pi.act ? V : 0u;
            }
            const uint32_t hl = (uint32_t)WIN - pi.padr, hlp = hl & ~3u, tl = hl & 3u;
            const uint32_t uA = pi.head ? (uint32_t)NW - (hlp >> 2) : 0u;  // first record word
            // keep word t iff t >= uA (bits of words 0..31 / 32..63)
            const uint32_t kb0 = uA >= 32 ? 0u : (0xffffffffu << uA);
            const uint32_t kb1 = uA >= 64 ? 0u : (uA <= 32 ? 0xffffffffu : (0xffffffffu << (uA - 32)));
            uint32_t cc[NCH];
#pragma unroll
            for (int c = 0; c < NCH; c++) cc[c] = 0;
#pragma unroll
            for (int u = 0; u < CW; u++)
#pragma unroll
                for (int c = 0; c < NCH; c++) {
                    const int t = c * CW + u;
                    const uint32_t x = __builtin_amdgcn_alignbyte(w[t + 1], w[t], sh);
                    const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int)(t < 32 ? kb0 : kb1), t & 31, 1);  // 0/~0
                    cc[c] = crc.word_and(cc[c], x, keep);
                }
            V = cc[0];
#pragma unroll
            for (int c = 1; c < NCH; c++) V = (KO & 8) ? (V ^ cc[c]) : (zapply(Zf, V) ^ cc[c]);
            if (pi.head && !(KO & 32)) {
                V ^= E[hlp >> 2];
                // absorb record bytes [hl', hl): the low tl bytes of the word after the window
                const uint32_t xt = __builtin_amdgcn_alignbyte(w[NW + 1], w[NW], sh);
                V = crc.absorb_upto3(V, xt, tl);
            }
            return pi.act ? V : 0u;
        };
        auto absorb = [&](const PassIn &pi, uint32_t ps, const uint32_t (&w)[NW + 2], const uint32_t (&hwt)[16]) {
            if (KO & 512) {  // lab: fold the words into rcrc, nothing else
#pragma unroll
                for (int t = 0; t < NW + 2; t++) rcrc ^= w[t];
                if (!(KO & 4)) {
#pragma unroll
                    for (int t = 0; t < 16; t++) rcrc += hwt[t];
                }
                return;
            }
            const uint32_t g0 = ps * 64;
            const bool hp = m != 0 && M >= g0 && M < g0 + 64;
            if (!(KO & 4)) {
#pragma unroll
                for (int t = 0; t < 16; t++) hw[t] = hp ? hwt[t] : hw[t];
            }
            uint32_t V = window_crc(pi, w);
            // continuation of the record carried out of the previous pass
            if (lane == 0 && pi.act && !pi.head) V ^= zapply(Zs, carry);
            // segmented inclusive scan (segments start at head windows and at lane 0)
            const uint64_t hm = __ballot(pi.head) | 1ull;
            const int32_t sk = 63 - __builtin_clzll(hm & lowmask);
            for (uint32_t j = 0; j < ((KO & 2) ? 0u : levels); j++) {
                const uint32_t d = 1u << j;
                const uint32_t y = __shfl_up(V, d, 64);
                const uint32_t zy = zapply(Zs + 1024 * j, y);
                if ((int32_t)lane - (int32_t)d >= sk) V ^= zy;
            }
            carry = __builtin_amdgcn_readlane(V, 63);
            // the record lane takes its state from the lane holding its last window
            const uint32_t gl = M + m - 1;
            const uint32_t vv = __shfl(V, (int)((gl - g0) & 63), 64);
            if (m != 0 && gl >= g0 && gl < g0 + 64) rcrc = vv;
        };
        // PIPE: two buffers, pass ps+1 in flight while pass ps is absorbed; else one pass at a
        // time (loads of one pass never outlive its loop iteration) with more waves per CU
        auto run = [&](bool inter) {
            if (PIPE == 2) {  // software pipeline: pass ps+1's loads in flight while ps is absorbed
                uint32_t wa[NW + 2], wb[NW + 2], ha[16], hb2[16];
                PassIn pa = locate(0);
                fetch(pa, 0, wa, ha, inter);
                for (uint32_t ps = 0; ps < npass; ps++) {
                    const PassIn pb = locate(ps + 1);  // past the last pass: every lane loads `safe`
                    fetch(pb, ps + 1, wb, hb2, inter);
                    absorb(pa, ps, wa, ha);
                    pa = pb;
#pragma unroll
                    for (int t = 0; t < NW + 2; t++) wa[t] = wb[t];
#pragma unroll
                    for (int t = 0; t < 16; t++) ha[t] = hb2[t];
                }
            } else if (PIPE) {
                uint32_t wa[NW + 2], wb[NW + 2], ha[16], hb[16];
                for (uint32_t ps = 0; ps < npass; ps += 2) {
                    const PassIn pa = locate(ps);
                    fetch(pa, ps, wa, ha, inter);
                    const PassIn pb = locate(ps + 1);
                    fetch(pb, ps + 1, wb, hb, inter);
                    absorb(pa, ps, wa, ha);
                    absorb(pb, ps + 1, wb, hb);  // past the last pass: an empty pass, no effect
                }
            } else {
                uint32_t wa[NW + 2], ha[16];
                for (uint32_t ps = 0; ps < npass; ps++) {
                    const PassIn pa = locate(ps);
                    fetch(pa, ps, wa, ha, inter);
                    absorb(pa, ps, wa, ha);
                }
            }
        };
        if (npass != 0) {
            if (interior) run(true);
            else run(false);
        }
        if (LONG && lrec) {
#pragma unroll
            for (int t = 0; t < 16; t++) hw[t] = ld32_clamp((p & ~3ull) + 4 * t, lo4, hi4);
        }
        wait_loads_done();  // unconditional: see bhg_device.h
        if (KO & 1024) {  // lab: no record section
            if (rcrc == 0x9e3779b9u) out[i].crc = rcrc;
            continue;
        }
        uint32_t cls = ~0u;  // MODE 1: the decode list this lane's block joins (0 small, 1.. large buckets)
        if (valid) {
            // ---- readRecordHeader / readRecord / readKV from the record's first 60 bytes
            uint32_t dk = 0, dkl = 0, dvo = 0, dvl = 0, dfn = 0, dfnv = 0, dcrc = 0, dst = st;
            uint64_t dtr = 0, dsize = 0;
            uint32_t vlen = 0;  // MODE 1: the stored (compressed) value length
            if (inb) {
                const uint32_t hsh = (uint32_t)(p & 3);
                uint32_t rw[15];
#pragma unroll
                for (int u = 0; u < 15; u++) rw[u] = __builtin_amdgcn_alignbyte(hw[u + 1], hw[u], hsh);
                const uint32_t k = L >= 12 ? rw[0] : 0u, v = L >= 12 ? rw[1] : 0u, fn = L >= 12 ? rw[2] : 0u;
                const bool rvalid = L >= 12 && k != 0 && v != 0 && (uint64_t)12 + k + v == (uint64_t)L;  // block2.go:57-66
                dcrc = lrec ? 0u : crc_mask(~rcrc);                                                        // crc.go:31-33
                if (rvalid) {
                    uint32_t key_len = 0, fnv = BHG_FNV_OFFSET;
                    uint64_t trailer = 255;  // InternalKeyKindInvalid when ikeySize < 8
                    if (k >= 8) {            // readKV / DecodeInternalKey (block2.go:38-55)
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
                    dk = 12; dkl = key_len; dtr = trailer; dfn = fn; dfnv = fnv;
                    if (MODE == 0) {
                        dvo = 12 + k; dvl = v;  // noCompressor.Decode: zero-copy view (compress.go:57-59)
                    } else {
                        // snappy decodedLen (golang/snappy decode.go decodedLen); the value is decoded later.
                        // Its bytes come from the header words when they lie in the first 60 B (k <= 43:
                        // a varint of <= 5 bytes), else from memory.
                        uint64_t x = 0;
                        uint32_t s = 0, hdr = 0;
                        bool ok = false;
                        const uint64_t vp = p + 12 + k;
                        const bool inw = k <= 43;
                        for (uint32_t b = 0; b < 10 && b < v; b++) {
                            uint32_t c;
                            if (inw && b < 5) {
                                const uint32_t o = 12 + k + b;  // < 60
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
                        if (!ok || x * 3 > (uint64_t)(v - hdr) * 64) {
                            dst = BHG_ST_SNAPPY_CORRUPT;
                        } else {
                            dsize = x;
                            dvl = (uint32_t)x;  // provisional: the snappy kernel finalises
                            dvo = 12 + k;       // provisional: compressed payload offset
                            vlen = v;
                        }
                    }
                    if (expected_crc != nullptr && dst == BHG_ST_OK && ecrc != dcrc && !lrec) dst = BHG_ST_CRC_MISMATCH;
                } else {
                    dst = BHG_ST_RECORD_NIL;  // ErrBhReadRecordNil (reader.go:260-264)
                }
            }
            uint2 *o = reinterpret_cast<uint2 *>(out + i);
            if (KO & 64) {
                if (dcrc == 0x9e3779b9u) o[4] = make_uint2(dcrc, dst);
                continue;
            }
            o[0] = make_uint2(dk, dkl);
            o[1] = make_uint2(dvo, dvl);
            o[2] = make_uint2((uint32_t)dtr, (uint32_t)(dtr >> 32));
            o[3] = make_uint2(dfn, dfnv);
            o[4] = make_uint2(dcrc, dst);
            if (MODE == 1) sizes[i] = dsize;
            if (MODE == 1 && (dst == BHG_ST_OK || dst == BHG_ST_CRC_MISMATCH)) {
                // the block's decode list: the 1-KiB LDS slots (a value of <= 1 KiB whose stream fits
                // beside it), else the 4-KiB tier's bucket of its decoded size, largest first
                // (appended below, with the wave converged)
                const bool small = dsize <= kSnapSmallMax && vlen + 24u <= kSnapSmallSlot;
                const uint32_t b = dsize <= kSnapSmallMax ? 0u : (uint32_t)((dsize - kSnapSmallMax - 1) / kSnapBucketBytes);
                cls = small ? 0u : 1u + (kSnapBuckets - 1) - (b < kSnapBuckets - 1 ? b : kSnapBuckets - 1);
            }
        }
        if (MODE == 1 && lists != nullptr) {
            // one atomic per wave and list on sub-list (tile mod 64) of each class present, all
            // issued before any result is used, then each lane's rank among the wave's blocks of
            // its class (per-lane atomics on the counters: C3 5.5 ms)
            const uint32_t sub = (uint32_t)__builtin_amdgcn_readfirstlane((int)tile) & 63u;
            const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            uint64_t cm[1 + kSnapBuckets];
            uint32_t cb[1 + kSnapBuckets];
#pragma unroll
            for (uint32_t q = 0; q <= kSnapBuckets; q++) {
                cm[q] = __ballot(cls == q);
                cb[q] = 0;
            }
            if (lane == 0) {
#pragma unroll
                for (uint32_t q = 0; q <= kSnapBuckets; q++)
                    if (cm[q]) cb[q] = atomicAdd(lists + 64 * q + sub, (uint32_t)__builtin_popcountll(cm[q]));
            }
#pragma unroll
            for (uint32_t q = 0; q <= kSnapBuckets; q++) {
                const uint32_t bq = (uint32_t)__builtin_amdgcn_readfirstlane((int)cb[q]);
                if (cls == q)
                    lists[kSnapListHdr + (64 * q + sub) * sub_cap + bq + (uint32_t)__builtin_popcountll(cm[q] & below)] = i;
            }
        }
    }
}

}  // namespace bhg
