// bhg_tscan.hip -- the sequential data-region scan of a .bht table on gfx950:
// TableIterator.findEntry (bithash/table.go:358-395, mode 0) and
// Writer.rebuild (bithash/writer.go:539-583, mode 1).
//
// A record's start depends on the previous header, so each
// table is one dependency chain.  Stages: the uniform prefix of every table,
// grid-wide (k_tscan_uni); speculative segment walks from guessed entries and
// their stitch (k_tscan_seg / k_tscan_stitch, below), which resolve a table
// whenever the true chain meets every segment walk it enters; for any other
// table, the serial walk of one 1024-thread workgroup (k_tscan), in which two
// moves alternate:
//  * speculation (uniform record lengths -- the common bulk-load case):
//    from a known start `off` with the last record length G, thread i reads
//    the header at off + i*G.  Threads up to the first one whose length is
//    not G (or that hits a stop rule) are all true record starts, and that
//    first different one is a true start too: up to 1025 records per
//    global-memory round trip.
//  * window chase (mixed lengths): the workgroup stages the next 128 KiB of
//    the table in LDS with coalesced loads (all in flight at once) and thread
//    0 follows the headers at LDS latency.  Windows follow each other with no
//    speculation step between them until the chase sees a run of 16 equal
//    lengths.
// The scan runs twice: count per table -> exclusive scan (out_first) ->
// the same walk again writing the handles.
//
// Before the walk, k_tscan_uni finds each table's UNIFORM PREFIX with every CU
// at once: the first F records from offset 0 whose length is the first record's
// G0 (record i at i * G0; the first record that is not -- a different length or
// a stop rule -- is F, a true record start, since records 0..F-1 are).  A
// bulk-loaded table is one uniform prefix ended by its terminating stop, so the
// one-workgroup walk only starts at record F; the F handles are written by a
// grid-wide pass (k_tscan_uni<true>).
//
// The count walk logs its steps (start offset, record count, and for a
// speculation step its guess, run and break record); the write pass then
// replays every logged step at once, a wave per step (k_tscan_logw: a window is
// re-chased from global memory by one lane), instead of walking each table
// again.  A table with more than TS_LOG_CAP steps is written by the serial walk.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

constexpr int TS_THREADS = 1024;
constexpr int TS_WAVES = TS_THREADS / 64;
constexpr uint32_t TS_WIN = 128 * 1024;  // one workgroup per table and CU: most of the LDS
constexpr uint32_t TS_LOG_CAP = 4096;     // logged walk steps per table (128 KiB)

// one step of the count walk: a speculation step found `a` records of length G at off + i G
// (x = a << 32, plus bit 62 and the u32 length when record a followed with another length), or a
// window chase started at off (x bit 63)
struct TsLog {
    uint64_t off, cnt, G, x;
};
constexpr uint64_t TS_LOG_WIN = 1ull << 63, TS_LOG_BRK = 1ull << 62;

struct Hdr {
    bool stop;
    uint64_t adv;  // bytes to the next record; the handle length is (uint32)adv
};

// Stop rules of bho_scan_region / the reference loops, given the remaining
// table bytes `rem` at the record start and its header words k, v.
__device__ __forceinline__ Hdr hdr_rule(uint64_t rem, uint32_t k, uint32_t v, int mode) {
    Hdr h = {true, 0};
    if (mode == 0) {
        if (k == 0 || v == 0) return h;                     // table.go:373-375: end of data
        const uint32_t kv = k + v;                          // uint32 arithmetic, table.go:377
        if (rem - 12 < kv) return h;                        // short ReadAt of key+value -> error
        h.stop = false;
        h.adv = 12 + (uint64_t)kv;
    } else {
        if (k == 0) return h;                               // writer.go:558
        if (rem - 12 < k) return h;                         // short key read
        h.stop = false;
        h.adv = 12 + (uint64_t)(uint32_t)(k + v);           // value may run past the end (writer.go:566-572)
    }
    return h;
}

__device__ __forceinline__ Hdr read_hdr_global(uint64_t t0, uint64_t tlen, uint64_t off, int mode) {
    const uint64_t rem = tlen > off ? tlen - off : 0;
    if (rem < 12) return Hdr{true, 0};                      // short header read
    const uint64_t p = t0 + off, end = t0 + tlen;
    return hdr_rule(rem, ldu32(p, end), ldu32(p + 4, end), mode);
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t *s) {
    return (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
}

// uniform prefix per table: uni[t] = F (atomic min over the failing record indices; the
// caller sets uni to ~0 first).  WRITE: the F handles of every table at out[first[t] + i].
constexpr int TU_THREADS = 256, TU_PARTS = 64;  // workgroups per table
template <bool WRITE>
__global__ __launch_bounds__(TU_THREADS) void k_tscan_uni(const uint8_t *__restrict__ src,
                                                          const uint64_t *__restrict__ table_off, int mode,
                                                          unsigned long long *__restrict__ uni,
                                                          bhg_handle *__restrict__ out, uint64_t max_out,
                                                          const uint64_t *__restrict__ first) {
    const uint32_t t = blockIdx.y, lane = threadIdx.x & 63;
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase;
    const Hdr h0 = read_hdr_global(t0, tlen, 0, mode);
    const uint64_t G = h0.stop ? 0 : h0.adv;
    const uint64_t step = (uint64_t)TU_PARTS * TU_THREADS;
    const uint64_t i0 = (uint64_t)blockIdx.x * TU_THREADS + threadIdx.x;
    if (WRITE) {
        const uint64_t F = uni[t], w0 = first[t];
        for (uint64_t i = i0; i < F && w0 + i < max_out; i += step) out[w0 + i] = bhg_handle{tbase + i * G, (uint32_t)G, 0};
        return;
    }
    if (G == 0) {  // record 0 ends the scan: no prefix
        if (i0 == 0) atomicMin(uni + t, 0ull);
        return;
    }
    // record tlen / G + 1 starts past the table's end and stops, so F <= tlen / G + 1 (in mode 1 a
    // record of length G may start at tlen / G: its value may run past the end, writer.go:566-572)
    const uint64_t last = tlen / G + 1;
    for (uint64_t i = i0; i - lane <= last; i += step) {  // whole waves iterate together
        bool bad = false;
        if (i <= last) {
            const Hdr h = read_hdr_global(t0, tlen, i * G, mode);
            bad = h.stop || h.adv != G;
        }
        const uint64_t m = __ballot(bad);
        if (m) {
            if (lane == (uint32_t)__builtin_ctzll(m)) atomicMin(uni + t, (unsigned long long)i);
            break;  // the wave's later records lie past a failure
        }
    }
}

template <bool WRITE>
__global__ __launch_bounds__(TS_THREADS) void k_tscan(const uint8_t *__restrict__ src,
                                                      const uint64_t *__restrict__ table_off, int mode,
                                                      bhg_handle *__restrict__ out, uint64_t max_out,
                                                      uint64_t *__restrict__ first, uint64_t *__restrict__ out_end,
                                                      const unsigned long long *__restrict__ uni,
                                                      TsLog *__restrict__ logs, uint32_t *__restrict__ log_n) {
    // WRITE: only the tables whose walk overflowed the log (the others are replayed by k_tscan_logw)
    // count: not the tables the segment walks resolved (log_n = ~0); write: only the tables whose
    // serial walk overflowed the log (the others are replayed by k_tscan_logw / k_tscan_segw)
    if (!WRITE && log_n[blockIdx.x] == ~0u) return;
    if (WRITE && (log_n[blockIdx.x] <= TS_LOG_CAP || log_n[blockIdx.x] == ~0u)) return;
    __shared__ alignas(16) uint8_t win[TS_WIN];
    __shared__ uint32_t s_brk[2][TS_WAVES];
    __shared__ uint64_t s_adv[2][TS_WAVES];
    __shared__ uint64_t s_off, s_cnt, s_G;
    __shared__ int s_done, s_chase;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t t = blockIdx.x;
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase;
    const uint64_t w0 = WRITE ? first[t] : 0;

    uint64_t off = 0, cnt = 0, G = 0;
    {  // start after the table's uniform prefix (k_tscan_uni): records 0..F-1 of length G0
        const uint64_t F = uni[t];
        if (F != 0) {
            G = read_hdr_global(t0, tlen, 0, mode).adv;
            off = F * G;
            cnt = F;
        }
    }
    int par = 0;
    bool chase = false;  // the last window's lengths were mixed: the next step is a window again
    uint32_t nlog = 0;   // count walk: steps logged (the same on every thread)
    auto log_step = [&](uint64_t o, uint64_t c, uint64_t g, uint64_t x) {
        if (!WRITE) {
            if (tid == 0 && nlog < TS_LOG_CAP) logs[(uint64_t)t * TS_LOG_CAP + nlog] = TsLog{o, c, g, x};
            nlog++;
        }
    };
    for (;;) {
      if (!chase) {
        // ---- speculation step ----
        const uint64_t po = off + (uint64_t)tid * G;
        Hdr h = {true, 0};
        if (tid == 0 || G != 0) h = read_hdr_global(t0, tlen, po, mode);
        const bool same = G != 0 && !h.stop && h.adv == G;
        const uint64_t brk = __ballot(!same);
        const uint32_t wb = brk ? (uint32_t)__builtin_ctzll(brk) : 64u;
        if (lane == 0) s_brk[par][wv] = wb;
        if (wb < 64 && lane == wb) s_adv[par][wv] = h.stop ? ~0ull : h.adv;
        __syncthreads();
        uint32_t a = TS_THREADS;
        uint64_t adv_a = ~0ull;
        for (int q = 0; q < TS_WAVES; q++) {
            const uint32_t b = s_brk[par][q];
            if (b < 64) {
                a = 64 * q + b;
                adv_a = s_adv[par][q];
                break;
            }
        }
        par ^= 1;  // the next step writes the other slot: no second barrier needed
        log_step(off, cnt, G, ((uint64_t)a << 32) |
                                  (a < TS_THREADS && adv_a != ~0ull ? TS_LOG_BRK | (uint32_t)adv_a : 0ull));
        if (WRITE && tid < a && w0 + cnt + tid < max_out)
            out[w0 + cnt + tid] = bhg_handle{tbase + po, (uint32_t)G, 0};
        cnt += a;
        off += (uint64_t)a * G;
        if (a == TS_THREADS) continue;
        if (adv_a == ~0ull) break;  // record a hits a stop rule: the scan ends at its start
        if (WRITE && tid == 0 && w0 + cnt < max_out) out[w0 + cnt] = bhg_handle{tbase + off, (uint32_t)adv_a, 0};
        cnt += 1;
        const uint64_t G_prev = G;
        off += adv_a;
        G = adv_a;
        if (a >= 32 || G_prev == 0) continue;  // speculation still pays (or had no guess yet)
      }

        // ---- window chase: stage [off, off + TS_WIN) in LDS, thread 0 follows headers ----
        const uint64_t wbeg = off;
        const uint64_t wend = tlen > off ? (tlen - off < TS_WIN ? tlen : off + TS_WIN) : off;
        const uint32_t wlen = (uint32_t)(wend - wbeg);
        log_step(wbeg, cnt, 0, TS_LOG_WIN);
        if (wlen == TS_WIN) {  // a whole window: every load in flight before the first store
            constexpr uint32_t PER = TS_WIN / (TS_THREADS * 16);
            u32x4 r[PER];
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) r[q] = gld<u32x4_a4>(t0 + wbeg + 16 * (q * TS_THREADS + tid));
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) *reinterpret_cast<u32x4_a4 *>(win + 16 * (q * TS_THREADS + tid)) = r[q];
        } else {
            for (uint32_t b = tid * 16; b < wlen; b += TS_THREADS * 16) {
                if (b + 16 <= wlen) {
                    *reinterpret_cast<u32x4_a4 *>(win + b) = gld<u32x4_a4>(t0 + wbeg + b);
                } else {
                    for (uint32_t j = b; j < wlen; j++) win[j] = gld<uint8_t>(t0 + wbeg + j);
                }
            }
        }
        __syncthreads();
        if (tid == 0) {
            int done = 0;
            uint32_t run = 0;  // records in a row of the same length
            for (;;) {
                const uint64_t rem = tlen > off ? tlen - off : 0;
                if (rem < 12) { done = 1; break; }
                if (off + 8 > wend) break;  // header not staged: next step
                const uint8_t *s = win + (off - wbeg);
                const Hdr hh = hdr_rule(rem, lds_u32(s), lds_u32(s + 4), mode);
                if (hh.stop) { done = 1; break; }
                if (WRITE && w0 + cnt < max_out) out[w0 + cnt] = bhg_handle{tbase + off, (uint32_t)hh.adv, 0};
                cnt += 1;
                off += hh.adv;
                run = hh.adv == G ? run + 1 : 0;
                G = hh.adv;
            }
            s_off = off;
            s_cnt = cnt;
            s_G = G;
            s_done = done;
            s_chase = run < 16;
        }
        __syncthreads();
        off = s_off;
        cnt = s_cnt;
        G = s_G;
        chase = s_chase != 0;
        if (s_done) break;
        // the next chase overwrites win / s_*: every reader passes the speculation barrier first
    }
    if (tid == 0) {
        if (!WRITE) {
            first[t] = cnt;
            log_n[t] = nlog;
        }
        if (out_end) out_end[t] = off;
    }
}

// the write pass of the logged walks: one wave per logged step, handles at out[first[t] + cnt ...]
constexpr int TL_THREADS = 256, TL_PARTS = 64;  // workgroups per table
__global__ __launch_bounds__(TL_THREADS) void k_tscan_logw(const uint8_t *__restrict__ src,
                                                           const uint64_t *__restrict__ table_off, int mode,
                                                           bhg_handle *__restrict__ out, uint64_t max_out,
                                                           const uint64_t *__restrict__ first,
                                                           const TsLog *__restrict__ logs,
                                                           const uint32_t *__restrict__ log_n) {
    const uint32_t t = blockIdx.y, lane = threadIdx.x & 63;
    const uint32_t n = log_n[t];
    if (n > TS_LOG_CAP) return;  // written by the serial walk
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase, tend = t0 + tlen;
    const uint64_t w0 = first[t];
    constexpr uint32_t WPT = TL_PARTS * (TL_THREADS / 64);
    for (uint32_t k = blockIdx.x * (TL_THREADS / 64) + (threadIdx.x >> 6); k < n; k += WPT) {
        const TsLog e = logs[(uint64_t)t * TS_LOG_CAP + k];
        if (!(e.x & TS_LOG_WIN)) {  // speculation step: a records of length G, then maybe record a
            const uint32_t a = (uint32_t)(e.x >> 32) & 0x7ffu;
            for (uint32_t i = lane; i < a; i += 64)
                if (w0 + e.cnt + i < max_out) out[w0 + e.cnt + i] = bhg_handle{tbase + e.off + i * e.G, (uint32_t)e.G, 0};
            if ((e.x & TS_LOG_BRK) && lane == 0 && w0 + e.cnt + a < max_out)
                out[w0 + e.cnt + a] = bhg_handle{tbase + e.off + (uint64_t)a * e.G, (uint32_t)e.x, 0};
        } else if (lane == 0) {  // window: the count walk's chase, from global memory
            uint64_t off = e.off, cnt = e.cnt;
            const uint64_t wend = tlen > off ? (tlen - off < TS_WIN ? tlen : off + TS_WIN) : off;
            for (;;) {
                const uint64_t rem = tlen > off ? tlen - off : 0;
                if (rem < 12 || off + 8 > wend) break;
                const Hdr hh = hdr_rule(rem, ldu32(t0 + off, tend), ldu32(t0 + off + 4, tend), mode);
                if (hh.stop) break;
                if (w0 + cnt < max_out) out[w0 + cnt] = bhg_handle{tbase + off, (uint32_t)hh.adv, 0};
                cnt += 1;
                off += hh.adv;
            }
        }
    }
}

// ---- speculative segment walks (mixed lengths) ----
// After the uniform prefix (end P) a table's region [P, tlen) is cut into TS_SEGS segments.
// k_tscan_seg: segment j's workgroup guesses where the record chain enters it (j = 0: P itself;
// else the first of its first 32 KiB of positions whose chain survives TS_SURVIVE headers, or 3
// before it leaves the staged window, or ends in a terminator or exactly at the data's end), walks the chain from there to the first node at or past the segment's end, and logs its
// windows.  k_tscan_stitch then follows the true chain: where it enters segment j at e, e must
// be a node of that walk (re-chased from the logged window holding e), and the walk's records
// from e on are the table's.  A miss (no guess, a wrong guess, a log overflow) sends the table
// to the serial walk (k_tscan), so a guess never decides a result.
#ifndef BHG_SEG_WIN_KB
#define BHG_SEG_WIN_KB 64
#endif
// segment walks: 512-thread workgroups with 64-KiB windows, two per CU (a CU's two walks hide each
// other's window loads); guesses probed in the window's first half
constexpr int SG_THREADS = BHG_SEG_WIN_KB == 128 ? 1024 : 512;
constexpr uint32_t SG_WIN = BHG_SEG_WIN_KB * 1024u;
constexpr uint32_t TS_SEGS = 64, TS_SEG_LOG = 512, TS_PROBE = SG_WIN / 2, TS_SURVIVE = 8;
constexpr uint32_t TS_SEG_GROUP = 32;  // a log entry every 32 records too: the replay's unit of work
constexpr uint64_t TS_SEG_MIN = 1ull << 20;
struct TsSeg {
    uint64_t g, cnt, x;  // guessed entry; records walked in [g, segment end); where the walk stopped
    uint32_t nlog, flags;
    uint64_t base, r;    // (stitch) out index of the walk's record 0 within the table; first record used
};
constexpr uint32_t TSF_WALKED = 1, TSF_END = 2, TSF_FAIL = 4;
struct TsWin {
    uint64_t off, cnt, we;  // a logged window: chase start, records before it, staged window end
};

__device__ __forceinline__ uint64_t prefix_end(uint64_t t0, uint64_t tlen, int mode, uint64_t F) {
    return F ? F * read_hdr_global(t0, tlen, 0, mode).adv : 0ull;
}
__device__ __forceinline__ void seg_geo(uint64_t P, uint64_t tlen, uint32_t j, uint64_t &s0, uint64_t &s1) {
    const uint64_t span = tlen > P ? tlen - P : 0;
    uint64_t S = (span + TS_SEGS - 1) / TS_SEGS;
    if (S < TS_SEG_MIN) S = TS_SEG_MIN;
    s0 = P + (uint64_t)j * S;
    s1 = s0 + S;
    if (s0 > tlen) s0 = tlen;
    if (s1 > tlen || j == TS_SEGS - 1) s1 = tlen;
}
// one step of the chase inside a window: the shared rules of the walk, its log replay and the
// stitch's membership check.  0: record (adv), 1: at / past the segment end, 2: table end or stop,
// 3: header not inside the window
__device__ __forceinline__ int seg_step(uint64_t off, uint64_t s1, uint64_t tlen, uint64_t we, uint32_t k, uint32_t v,
                                        int mode, uint64_t &adv) {
    if (off >= s1) return 1;
    const uint64_t rem = tlen > off ? tlen - off : 0;
    if (rem < 12) return 2;
    if (off + 8 > we) return 3;
    const Hdr hh = hdr_rule(rem, k, v, mode);
    if (hh.stop) return 2;
    adv = hh.adv;
    return 0;
}

__global__ __launch_bounds__(SG_THREADS) void k_tscan_seg(const uint8_t *__restrict__ src,
                                                          const uint64_t *__restrict__ table_off, int mode,
                                                          const unsigned long long *__restrict__ uni,
                                                          TsSeg *__restrict__ segs, TsWin *__restrict__ wins) {
    __shared__ alignas(16) uint8_t win[SG_WIN];
    __shared__ uint32_t s_best, s_nlog;
    __shared__ uint64_t s_off, s_cnt;
    __shared__ int s_state;
    const uint32_t tid = threadIdx.x, j = blockIdx.x, t = blockIdx.y;
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase;
    const uint64_t P = prefix_end(t0, tlen, mode, uni[t]);
    uint64_t s0, s1;
    seg_geo(P, tlen, j, s0, s1);
    TsSeg *sg = segs + (uint64_t)t * TS_SEGS + j;
    TsWin *wl = wins + ((uint64_t)t * TS_SEGS + j) * TS_SEG_LOG;
    if (s0 >= s1) {
        if (tid == 0) *sg = TsSeg{s0, 0, s0, 0, 0, 0, ~0ull};
        return;
    }
    auto stage = [&](uint64_t wbeg) -> uint64_t {  // [wbeg, we) into LDS; returns we
        const uint64_t we = tlen - wbeg < SG_WIN ? tlen : wbeg + SG_WIN;
        const uint32_t wlen = (uint32_t)(we - wbeg);
        if (wlen == SG_WIN) {
            constexpr uint32_t PER = SG_WIN / (SG_THREADS * 16);
            u32x4 r[PER];
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) r[q] = gld<u32x4_a4>(t0 + wbeg + 16 * (q * SG_THREADS + tid));
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) *reinterpret_cast<u32x4_a4 *>(win + 16 * (q * SG_THREADS + tid)) = r[q];
        } else {
            for (uint32_t b = tid * 16; b < wlen; b += SG_THREADS * 16) {
                if (b + 16 <= wlen) *reinterpret_cast<u32x4_a4 *>(win + b) = gld<u32x4_a4>(t0 + wbeg + b);
                else for (uint32_t q = b; q < wlen; q++) win[q] = gld<uint8_t>(t0 + wbeg + q);
            }
        }
        return we;
    };
    auto hdr_lds = [&](uint64_t off, uint64_t wb, uint32_t &k, uint32_t &v) {
        const uint8_t *h = win + (off - wb);
        k = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
        v = (uint32_t)h[4] | ((uint32_t)h[5] << 8) | ((uint32_t)h[6] << 16) | ((uint32_t)h[7] << 24);
    };
    uint64_t wb = s0, we = stage(s0);
    if (tid == 0) s_best = j == 0 ? 0u : ~0u;
    __syncthreads();
    if (j > 0) {  // the guess: the first probed position whose chain survives TS_SURVIVE headers
        const uint64_t lim = s1 - s0 < TS_PROBE ? s1 - s0 : TS_PROBE;
        for (uint32_t c = tid; c < lim; c += SG_THREADS) {
            uint64_t q = s0 + c;
            uint32_t n = 0;
            bool acc = false;
            for (;;) {
                // the data's end after a record: landing inside the table's last 12 bytes (a false
                // chain's jump past the end -- a rebuild-mode value running out -- does not count)
                if (q > tlen) break;
                const uint64_t rem = tlen - q;
                if (rem < 12) { acc = n > 0; break; }
                // a chain that leaves the staged window counts only after 3 records inside it:
                // false headers jump anywhere up to 4 GB, and one landing on a true record later
                // merges with the true chain (taking any chain that left: 3 of 16 scanmix tables
                // missed); three in-window steps of a false chain are ~1e-14 likely
                if (q + 8 > we) { acc = n >= 3; break; }
                uint32_t k, v;
                hdr_lds(q, wb, k, v);
                const Hdr hh = hdr_rule(rem, k, v, mode);
                if (hh.stop) { acc = n > 0 && k == 0 && v == 0; break; }  // a terminator after a record
                if (++n == TS_SURVIVE) { acc = true; break; }
                q += hh.adv;
            }
            if (acc) {
                atomicMin(&s_best, c);
                break;  // this thread's later positions are larger
            }
        }
        __syncthreads();
    }
    if (s_best == ~0u) {
        if (tid == 0) *sg = TsSeg{s0, 0, s0, 0, TSF_FAIL, 0, ~0ull};
        return;
    }
    const uint64_t g = s0 + s_best;
    uint64_t off = g, cnt = 0;
    uint32_t nlog = 0;
    int state = 0;
    for (;;) {
        if (tid == 0) {  // chase inside the staged window
            if (nlog < TS_SEG_LOG) wl[nlog] = TsWin{off, cnt, we};
            nlog++;
            for (;;) {
                uint32_t k = 0, v = 0;
                if (off < s1 && off + 8 <= we && off + 12 <= tlen) hdr_lds(off, wb, k, v);
                uint64_t adv = 0;
                const int r = seg_step(off, s1, tlen, we, k, v, mode, adv);
                if (r == 3) break;
                if (r != 0) { state = r; break; }
                cnt++;
                off += adv;
                if (cnt % TS_SEG_GROUP == 0) {
                    if (nlog < TS_SEG_LOG) wl[nlog] = TsWin{off, cnt, we};
                    nlog++;
                }
            }
            s_off = off;
            s_cnt = cnt;
            s_nlog = nlog;
            s_state = state;
        }
        __syncthreads();
        off = s_off;
        cnt = s_cnt;
        nlog = s_nlog;
        state = s_state;
        if (state != 0) break;
        wb = off;
        we = stage(wb);
        __syncthreads();
    }
    if (tid == 0)
        *sg = TsSeg{g, cnt, off, nlog, TSF_WALKED | (state == 2 ? TSF_END : 0u) | (nlog > TS_SEG_LOG ? TSF_FAIL : 0u), 0,
                    ~0ull};  // r: set by the stitch for the segments the chain uses
}

// one lane per table: follow the true chain through the segment walks (see above)
__global__ __launch_bounds__(64) void k_tscan_stitch(const uint8_t *__restrict__ src,
                                                     const uint64_t *__restrict__ table_off, int mode,
                                                     const unsigned long long *__restrict__ uni,
                                                     TsSeg *__restrict__ segs, const TsWin *__restrict__ wins,
                                                     uint64_t *__restrict__ first, uint64_t *__restrict__ out_end,
                                                     uint32_t *__restrict__ log_n) {
    if (threadIdx.x != 0) return;
    const uint32_t t = blockIdx.x;
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase, tend = t0 + tlen;
    const uint64_t F = uni[t];
    const uint64_t P = prefix_end(t0, tlen, mode, F);
    uint64_t e = P, cnt = F;
    bool ok = true;
    for (uint32_t j = 0; j < TS_SEGS && ok; j++) {
        uint64_t s0, s1;
        seg_geo(P, tlen, j, s0, s1);
        if (s0 >= s1) break;
        TsSeg &sg = segs[(uint64_t)t * TS_SEGS + j];
        if (e >= s1) continue;  // the chain jumped over this segment (r stays ~0: nothing written)
        if (!(sg.flags & TSF_WALKED) || (sg.flags & TSF_FAIL) || e < sg.g) { ok = false; break; }
        uint64_t off = e, c = 0, we = 0;
        if (e != sg.g) {  // (the guess is the entry: record 0, nothing to check)
            // the logged window holding e: the last one starting at or before e
            const TsWin *wl = wins + ((uint64_t)t * TS_SEGS + j) * TS_SEG_LOG;
            uint32_t lo = 0, hi = sg.nlog;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (wl[mid].off <= e) lo = mid; else hi = mid;
            }
            off = wl[lo].off;
            c = wl[lo].cnt;
            we = wl[lo].we;
        }
        while (off < e) {
            uint64_t adv = 0;
            uint32_t k = 0, v = 0;
            if (off + 12 <= tlen) { k = ldu32(t0 + off, tend); v = ldu32(t0 + off + 4, tend); }
            if (seg_step(off, s1, tlen, we, k, v, mode, adv) != 0) break;
            off += adv;
            c++;
        }
        if (off != e) { ok = false; break; }
        sg.r = c;
        sg.base = cnt - c;
        cnt += sg.cnt - c;
        e = sg.x;
        if (sg.flags & TSF_END) break;
    }
    if (ok) {
        first[t] = cnt;
        if (out_end) out_end[t] = e;
        log_n[t] = ~0u;
    } else {
        log_n[t] = 0;  // the serial walk counts this table
    }
}

// the write pass of the segment walks: one lane per logged entry (a window start or every 32nd
// record), records from the stitch's r on
__global__ __launch_bounds__(TS_THREADS) void k_tscan_segw(const uint8_t *__restrict__ src,
                                                           const uint64_t *__restrict__ table_off, int mode,
                                                           const unsigned long long *__restrict__ uni,
                                                           const TsSeg *__restrict__ segs, const TsWin *__restrict__ wins,
                                                           const uint32_t *__restrict__ log_n,
                                                           const uint64_t *__restrict__ first,
                                                           bhg_handle *__restrict__ out, uint64_t max_out) {
    const uint32_t j = blockIdx.x, t = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (log_n[t] != ~0u) return;
    const TsSeg sg = segs[(uint64_t)t * TS_SEGS + j];
    if (!(sg.flags & TSF_WALKED) || sg.r == ~0ull) return;
    const uint64_t tbase = table_off[t], tlen = table_off[t + 1] - tbase;
    const uint64_t t0 = (uint64_t)src + tbase, tend = t0 + tlen;
    const uint64_t P = prefix_end(t0, tlen, mode, uni[t]);
    uint64_t s0, s1;
    seg_geo(P, tlen, j, s0, s1);
    const TsWin *wl = wins + ((uint64_t)t * TS_SEGS + j) * TS_SEG_LOG;
    const uint64_t w0 = first[t] + sg.base;
    const uint32_t nl = sg.nlog;
    for (uint32_t q = wv * 64 + lane; q < nl; q += TS_THREADS) {  // a lane per logged entry
        const TsWin w = wl[q];
        const uint64_t cend = q + 1 < nl ? wl[q + 1].cnt : sg.cnt;  // the entry's records: [w.cnt, cend)
        uint64_t off = w.off, c = w.cnt;
        while (c < cend) {
            uint32_t k = 0, v = 0;
            if (off + 12 <= tlen) { k = ldu32(t0 + off, tend); v = ldu32(t0 + off + 4, tend); }
            uint64_t adv = 0;
            if (seg_step(off, s1, tlen, w.we, k, v, mode, adv) != 0) break;
            if (c >= sg.r && w0 + c < max_out) out[w0 + c] = bhg_handle{tbase + off, (uint32_t)adv, 0};
            off += adv;
            c++;
        }
    }
}

// Writer.rebuild's per-record work after the header chase (writer.go:569-575):
// bh = {offset inside the table, recordLen}, khash = hash.Fnv32(UserKey) of
// base.DecodeInternalKey(key) (UserKey empty when ikeySize < 8), table index.
// Entries past the scanned count get table = UINT32_MAX.
__global__ __launch_bounds__(256) void k_rebuild_recs(const uint8_t *src, const uint64_t *table_off, uint32_t ntables,
                                                      const bhg_handle *h, uint64_t max_out, const uint64_t *first,
                                                      uint32_t *khash, uint32_t *bh_off, uint32_t *table) {
    const uint64_t total = first[ntables];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < max_out;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (i >= total) {
            table[i] = 0xffffffffu;
            khash[i] = 0;
            bh_off[i] = 0;
            continue;
        }
        uint32_t lo = 0, hi = ntables;  // last t with first[t] <= i
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (first[mid] <= i) lo = mid; else hi = mid;
        }
        const bhg_handle r = h[i];
        const uint64_t p = (uint64_t)src + r.offset, tend = (uint64_t)src + table_off[lo + 1];
        const uint32_t k = ldu32(p, tend);  // the chase read this header and its key inside the table
        table[i] = lo;
        bh_off[i] = (uint32_t)(r.offset - table_off[lo]);
        khash[i] = fnv1_range(p + 12, k >= 8 ? k - 8 : 0, tend);
    }
}

}  // namespace

hipError_t launch_rebuild_recs(const Launch &L, const uint8_t *src, const uint64_t *table_off, uint32_t ntables,
                               const bhg_handle *h, uint64_t max_out, const uint64_t *first, uint32_t *khash,
                               uint32_t *bh_off, uint32_t *table) {
    if (max_out == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rebuild_recs, dim3(lane_grid(L, max_out, 256)), dim3(256), 0, L.stream, src, table_off,
                       ntables, h, max_out, first, khash, bh_off, table);
    return hipGetLastError();
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// The walk's scratch (uniform prefixes, step logs, segment walks and their window logs) is ~0.9 MiB
// per table; tables are scanned TS_CHUNK at a time through one scratch area, so a call over any
// number of tables needs at most TS_CHUNK tables' worth (~230 MiB), and only the 12 B per table
// that are read before they are written (uni, log_n) are filled.
constexpr uint32_t TS_CHUNK = 256;

// first[0..m] holds a chunk's exclusive scan (first[m] = the chunk's total): add the record
// count of the tables before the chunk (*carry) and advance *carry past the chunk.
__global__ __launch_bounds__(256) void k_tscan_carry(uint64_t *first, uint32_t m, uint64_t *carry, int first_chunk) {
    const uint64_t c = first_chunk ? 0ull : *carry;
    const uint64_t tot = first[m];
    __syncthreads();  // every read above happens before first[m] or *carry is rewritten
    for (uint32_t i = threadIdx.x; i <= m; i += blockDim.x) first[i] += c;
    if (threadIdx.x == 0) *carry = c + tot;
}

// per table: which pass wrote its handles (BHG_SCAN_PATH_*: segment walks, log replay, serial walk)
__global__ __launch_bounds__(256) void k_tscan_path(const uint32_t *log_n, uint32_t m, uint32_t *path) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
        path[i] = log_n[i] == ~0u ? 0u : (log_n[i] <= TS_LOG_CAP ? 1u : 2u);
}

size_t tscan_uni_bytes(uint32_t ntables) {
    const size_t m = ntables < TS_CHUNK ? ntables : TS_CHUNK;
    return 256 + al256(m * 8) + al256(m * 4) + al256(m * TS_LOG_CAP * sizeof(TsLog)) +
           al256(m * TS_SEGS * sizeof(TsSeg)) + m * TS_SEGS * TS_SEG_LOG * sizeof(TsWin);
}

hipError_t launch_tscan(const Launch &L, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                        bhg_handle *out, uint64_t max_out, uint64_t *first, uint64_t *out_end, void *scan_scratch,
                        void *uni_scratch, uint32_t *out_path) {
    const uint32_t M = ntables < TS_CHUNK ? ntables : TS_CHUNK;
    uint8_t *sp = static_cast<uint8_t *>(uni_scratch);
    uint64_t *carry = reinterpret_cast<uint64_t *>(sp);
    sp += 256;
    unsigned long long *uni = reinterpret_cast<unsigned long long *>(sp);
    sp += al256((size_t)M * 8);
    uint32_t *log_n = reinterpret_cast<uint32_t *>(sp);
    sp += al256((size_t)M * 4);
    TsLog *logs = reinterpret_cast<TsLog *>(sp);
    sp += al256((size_t)M * TS_LOG_CAP * sizeof(TsLog));
    TsSeg *segs = reinterpret_cast<TsSeg *>(sp);
    sp += al256((size_t)M * TS_SEGS * sizeof(TsSeg));
    TsWin *wins = reinterpret_cast<TsWin *>(sp);
    hipError_t e = hipSuccess;
    for (uint32_t c0 = 0; c0 < ntables; c0 += M) {
        const uint32_t m = ntables - c0 < M ? ntables - c0 : M;
        const uint64_t *toff = table_off + c0;
        uint64_t *fst = first + c0;
        uint64_t *oend = out_end ? out_end + c0 : nullptr;
        // uni starts at ~0 (atomic min); log_n is written by the stitch for every table, filled anyway.
        // Segments, logs and windows are written before they are read.
        if ((e = hipMemsetAsync(uni, 0xff, al256((size_t)M * 8) + (size_t)m * 4, L.stream)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_tscan_uni<false>), dim3(TU_PARTS, m), dim3(TU_THREADS), 0, L.stream, src, toff, mode, uni,
                           out, max_out, fst);
        // segment walks, then the stitch per table
        hipLaunchKernelGGL(k_tscan_seg, dim3(TS_SEGS, m), dim3(SG_THREADS), 0, L.stream, src, toff, mode, uni, segs, wins);
        hipLaunchKernelGGL(k_tscan_stitch, dim3(m), dim3(64), 0, L.stream, src, toff, mode, uni, segs, wins, fst, oend,
                           log_n);
        hipLaunchKernelGGL((k_tscan<false>), dim3(m), dim3(TS_THREADS), 0, L.stream, src, toff, mode, out, max_out, fst,
                           oend, uni, logs, log_n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if ((e = launch_exclusive_scan_u64(L, fst, fst, m, scan_scratch)) != hipSuccess) return e;
        if (ntables > M)
            hipLaunchKernelGGL(k_tscan_carry, dim3(1), dim3(256), 0, L.stream, fst, m, carry, c0 == 0 ? 1 : 0);
        if (out_path)
            hipLaunchKernelGGL(k_tscan_path, dim3((m + 255) / 256), dim3(256), 0, L.stream, log_n, m, out_path + c0);
        if (out == nullptr || max_out == 0) continue;  // counts and ends only
        hipLaunchKernelGGL((k_tscan_uni<true>), dim3(TU_PARTS, m), dim3(TU_THREADS), 0, L.stream, src, toff, mode, uni,
                           out, max_out, fst);
        hipLaunchKernelGGL(k_tscan_logw, dim3(TL_PARTS, m), dim3(TL_THREADS), 0, L.stream, src, toff, mode, out, max_out,
                           fst, logs, log_n);
        hipLaunchKernelGGL(k_tscan_segw, dim3(TS_SEGS, m), dim3(TS_THREADS), 0, L.stream, src, toff, mode, uni, segs,
                           wins, log_n, fst, out, max_out);
        hipLaunchKernelGGL((k_tscan<true>), dim3(m), dim3(TS_THREADS), 0, L.stream, src, toff, mode, out, max_out, fst,
                           oend, uni, logs, log_n);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipGetLastError();
}

}  // namespace bhg
