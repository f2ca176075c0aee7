// bhg_snappy_enc.hip -- golang/snappy v0.0.4 block encoder on gfx950, byte
// exact with encode.go / encode_other.go (Encode, encodeBlock, emitLiteral,
// emitCopy; restated in oracle/bithash_oracle.c).
//
// One WAVE per value.  The <= 4 KiB block and its hash table live in LDS.
// The greedy matcher is serial in its decisions but its literal-scan phase
// is not: from a scan start s the positions visited are s + F[k] (F fixed by
// the skip heuristic, skip = 32, +skip>>5 per step), so 64 consecutive scan
// iterations are evaluated at once -- hash, candidate (table value, or the
// latest earlier lane of the batch with the same bucket), 4-byte compare --
// and the first lane that matches (or runs past sLimit) ends the batch.
// Table writes use ds_max_u32: positions only grow, so max == "last write
// wins" in program order.  Match extension compares 64 bytes per step.
// Values longer than 4 KiB (golang/snappy cuts them into 64-KiB blocks) take the block path:
// every 64-KiB block of every such value is a work item of its own (k_snappy_enc_blocks: one
// wave per block, its table in LDS, the block read in place, the same matcher), written to a block slot; then
// k_snappy_concat joins each value's uvarint header and block outputs.  (Until round 6 a lane-0
// walk with its table in global memory encoded them one block after another: bench.py --config
// bigval 764 ms per step, 1.3 GiB/s, profiles/r6/bigval/.)
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

typedef u32x4 u32x4u __attribute__((aligned(1)));
// Tuning constants, each measured (lab records under profiles/r2*, r3/enc*):
constexpr uint32_t kSeDcnt = 272;  // dwords of the in-batch duplicate check: 1,024 bucket bytes + 64 lane bytes
constexpr uint32_t kSeHeads = 8;   // queue heads per class list
constexpr uint32_t kSeStatic = 75; // % of a class list handed out round-robin before the work queue takes over
constexpr int kSeWpg = 3;          // waves per workgroup of the large-value launch
constexpr int kSeMinwSmall = 4;    // waves per SIMD the small-value kernel is compiled for (VGPR budget)
constexpr uint32_t kSeWaves = 7;   // resident waves per CU the large-value launch is sized for
// the hash table holds u16 positions (blocks here are <= 4 KiB): 13 KiB of LDS per wave,
// 11 waves per CU (a u32 table: 7 waves per CU, 37.7 vs 49.4 GiB/s in round 2)
typedef uint16_t se_tab_t;

#define SE_CAP 4096                 // LDS block capacity of the large-value kernel (values past it: the block path)
#define SE_CAP_BLOCK 65536          // ... of the block path (encode.go maxBlockSize)
#define SE_CAP_SMALL 2048           // ... of the small-value kernel (values <= 2 KiB)
#define SE_MAXBLOCK 65536           // encode.go maxBlockSize
#define SE_MARGIN 15                // inputMargin
#define SE_MINNONLIT 17             // minNonLiteralBlockSize
// LDS of a wave with block capacity CAP: the block (+16 zero bytes), the table (CAP u16
// entries: tableSize <= len), the dedupe counters, and 64 scratch u16 slots (SE_DUMMY, after
// the table and the counters): lanes that must not store write there instead of being masked
// off (no exec-mask branch)
// (GSRC: the block is not staged, the matcher reads the value in place: no block words)
template <int CAP, bool GSRC = false>
struct SeLayout {
    static constexpr uint32_t kTab = CAP < 16384 ? CAP : 16384;  // tableSize <= min(len, maxTableSize)
    static constexpr uint32_t kDummy = kTab + 2 * kSeDcnt;
    static constexpr uint32_t kBlk = GSRC ? 0u : (CAP + 16) / 4;
    static constexpr uint32_t kWords = kBlk + kTab * sizeof(se_tab_t) / 4 + kSeDcnt + 32;
};

struct SkipTab {
    uint32_t f[1025];
    constexpr SkipTab() : f() {
        uint64_t off = 0, skip = 32;
        for (int k = 0; k < 1025; k++) {
            f[k] = off > 0x7fffffffull ? 0x7fffffffu : (uint32_t)off;
            const uint64_t step = skip >> 5;
            off += step;
            skip += step;
        }
    }
};
__constant__ SkipTab kSkip = SkipTab();

__device__ __forceinline__ uint32_t se_hash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

// in[p .. p + 4) from two dword-aligned LDS reads (one ds_read2_b32) and a byte funnel:
// misaligned DS accesses are replayed on gfx950 (62 % of the LDS-active cycles of the
// round-2 encoder were unaligned stalls)
__device__ __forceinline__ uint32_t ld32a(const uint32_t *in32, uint32_t p) {
    const uint32_t w = p >> 2;
    return __builtin_amdgcn_alignbyte(in32[w + 1], in32[w], p & 3);
}
// lane i's value for a wave-uniform i: v_readlane, not an LDS permute
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); }

// The block the matcher reads.  SrcLds: staged in LDS with 16 zero bytes after it (reads past
// the end land in the zero bytes or the table: never used, the matcher clips every compare to
// the block length).  SrcGlb: the value in global memory, read in place (L2-resident after the
// first touch); the copy loop's window loads near the block's end (tail: positions up to
// len + 66) clamp the address into the block instead, so nothing past the value is read.
struct SrcLds {
    const uint8_t *in;
    __device__ __forceinline__ uint32_t w(uint32_t p) const { return ld32a(reinterpret_cast<const uint32_t *>(in), p); }
    __device__ __forceinline__ uint32_t b(uint32_t p) const { return in[p]; }
    __device__ __forceinline__ uint32_t wt(uint32_t p) const { return w(p); }
    __device__ __forceinline__ uint32_t bt(uint32_t p) const { return b(p); }
};
typedef uint32_t u32_unal __attribute__((aligned(1)));
struct SrcGlb {
    const uint8_t *g;
    uint32_t len;  // >= SE_MINNONLIT
    __device__ __forceinline__ uint32_t w(uint32_t p) const { return *reinterpret_cast<const u32_unal *>(g + p); }
    __device__ __forceinline__ uint32_t b(uint32_t p) const { return g[p]; }
    // tail forms: in[p ..) exact for the bytes below len, anything above it
    __device__ __forceinline__ uint32_t wt(uint32_t p) const {
        const uint32_t q = min(p, len - 4);
        return w(q) >> (8 * min(p - q, 3u));
    }
    __device__ __forceinline__ uint32_t bt(uint32_t p) const { return g[min(p, len - 1)]; }
};

struct Out {
    uint8_t *g;   // global destination of this value's stream
    uint32_t d;   // bytes written (wave-uniform)
};

// emitLiteral (encode_other.go): tag by lane 0, bytes by all lanes
__device__ __forceinline__ void se_emit_literal(Out &o, const uint8_t *lit_lds, const uint8_t *lit_g, uint32_t len,
                                                uint32_t lane, uint32_t nl = 64) {
    const uint32_t n = len - 1;
    uint32_t hdr;
    if (lane == 0) {
        if (n < 60) { o.g[o.d] = (uint8_t)(n << 2); }
        else if (n < 256) { o.g[o.d] = 60 << 2; o.g[o.d + 1] = (uint8_t)n; }
        else { o.g[o.d] = 61 << 2; o.g[o.d + 1] = (uint8_t)n; o.g[o.d + 2] = (uint8_t)(n >> 8); }
    }
    hdr = n < 60 ? 1 : n < 256 ? 2 : 3;
    uint8_t *dst = o.g + o.d + hdr;
    if (lit_lds) {
        for (uint32_t t = lane; t < len; t += nl) dst[t] = lit_lds[t];
    } else {
        for (uint32_t t = lane; t < len; t += nl) dst[t] = lit_g[t];
    }
    o.d += hdr + len;
}

// emitCopy (encode_other.go), lane 0 writes
__device__ __forceinline__ void se_emit_copy(Out &o, uint32_t offset, uint32_t length, uint32_t lane) {
    uint32_t i = 0;
    uint8_t *dst = o.g + o.d;
    while (length >= 68) {
        if (lane == 0) { dst[i] = 63 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8); }
        i += 3;
        length -= 64;
    }
    if (length > 64) {
        if (lane == 0) { dst[i] = 59 << 2 | 2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8); }
        i += 3;
        length -= 60;
    }
    if (length >= 12 || offset >= 2048) {
        if (lane == 0) {
            dst[i] = (uint8_t)((length - 1) << 2 | 2); dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
        }
        o.d += i + 3;
        return;
    }
    if (lane == 0) { dst[i] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | 1); dst[i + 1] = (uint8_t)offset; }
    o.d += i + 2;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// ballot of a bool straight from its compare (HIP's bal(int) re-materialises the bool in a
// VGPR and compares it again: two VALU per ballot)
__device__ __forceinline__ uint64_t bal(bool b) { return __builtin_amdgcn_ballot_w64(b); }
// order LDS accesses of this wave (no instruction: LDS executes a wave's ops in order)
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }

// The matcher does not write output bytes.  Every copy it finds becomes one op --
// (copy start, copy end, candidate: the literal run before it ends where the previous op
// ended), the block's final literal an op with copy length 0 -- written into lane n of
// three VGPRs by selects.  Every 64 ops
// se_flush turns them into golang/snappy's bytes with all lanes at once: per-op sizes
// (emitLiteral header + literal + emitCopy tags), a wave prefix sum for the output
// offsets, tags written by their own lanes, literal bytes copied from the LDS block by
// the whole wave.
struct OpRing {
    uint32_t s;   // lane k: op k's copy start (the final literal: the block length)
    uint32_t e;   // lane k: op k's copy end (its literal run is [end of op k - 1, s))
    uint32_t c;   // lane k: op k's candidate (offset s - c)
    uint32_t n;   // ops held (wave-uniform)
    uint32_t e0;  // end of the op before lane 0's (wave-uniform)
};

// lane i <- lane i - 1 (DPP wave_shr:1, bound_ctrl off: lane 0, whose source is out of
// range, keeps `first`)
__device__ __forceinline__ uint32_t lane_prev(uint32_t v, uint32_t first) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)v, 0x138, 0xf, 0xf, false);
}

template <class S>
__device__ __forceinline__ void se_flush(Out &o, const S &in, OpRing &r, uint32_t lane) {
    const bool act = lane < r.n;
    // (no lane-0 select here: the compiler turned one into an exec-masked branch around the
    // DPP, and a DPP move reading an inactive lane returns `old`)
    const uint32_t prev_e = lane_prev(r.e, r.e0);
    const uint32_t base = r.s;
    const uint32_t lit = act ? base - prev_e : 0u, cl = act ? r.e - base : 0u, off = base - r.c;
    const uint32_t lh = lit == 0 ? 0u : lit <= 60 ? 1u : lit <= 256 ? 2u : 3u;  // emitLiteral: n = lit - 1
    uint32_t L = cl, n64 = 0;
    if (L >= 68) {  // emitCopy: "for length >= 68 { 64-byte copy; length -= 64 }"
        n64 = (L - 68) / 64 + 1;
        L -= 64 * n64;
    }
    const uint32_t n60 = L > 64 ? 1u : 0u;  // "if length > 64 { 60-byte copy }"
    if (n60) L -= 60;
    const bool c2 = L >= 12 || off >= 2048;
    const uint32_t ct = cl == 0 ? 0u : 3 * (n64 + n60) + (c2 ? 3u : 2u);
    const uint32_t sz = lh + lit + ct;
    const uint32_t incl = wave_incl_add(sz);
    const uint32_t total = lane_val(incl, 63);
    uint8_t *dst = o.g + o.d + (incl - sz);
    if (lh) {
        const uint32_t m = lit - 1;
        dst[0] = lh == 1 ? (uint8_t)(m << 2) : lh == 2 ? (uint8_t)(60 << 2) : (uint8_t)(61 << 2);
        if (lh >= 2) dst[1] = (uint8_t)m;
        if (lh == 3) dst[2] = (uint8_t)(m >> 8);
    }
    if (cl) {
        uint8_t *q = dst + lh + lit;
        for (uint32_t i = 0; i < n64 + n60; i++, q += 3) {
            q[0] = i < n64 ? (uint8_t)(63 << 2 | 2) : (uint8_t)(59 << 2 | 2);
            q[1] = (uint8_t)off;
            q[2] = (uint8_t)(off >> 8);
        }
        if (c2) {
            q[0] = (uint8_t)((L - 1) << 2 | 2);
            q[1] = (uint8_t)off;
            q[2] = (uint8_t)(off >> 8);
        } else {
            q[0] = (uint8_t)((off >> 8) << 5 | (L - 4) << 2 | 1);
            q[1] = (uint8_t)off;
        }
    }
    // literal bytes: one op at a time, 64 bytes per wave instruction
    uint64_t lm = bal(lit != 0);
    while (lm) {
        const uint32_t k = (uint32_t)__builtin_ctzll(lm);
        lm &= lm - 1;
        const uint32_t ll = lane_val(lit, k), s0 = lane_val(base, k) - ll;
        uint8_t *d0 = o.g + o.d + (lane_val(incl, k) - lane_val(sz, k)) + lane_val(lh, k);
        for (uint32_t t = lane; t < ll; t += 64) d0[t] = (uint8_t)in.b(s0 + t);
    }
    o.d += total;
    r.e0 = lane_val(r.e, r.n - 1);
    r.n = 0;
}

// op n of the ring (the caller flushes a full ring before the next push): three selects,
// no exec-mask branch, nothing on the matcher's dependency chain
// v with lane i := x (x, i wave-uniform): the v_writelane_b32 intrinsic (no clang builtin here)
extern "C" __device__ int bhg_llvm_writelane(int x, int i, int v) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wlane(uint32_t v, uint32_t x, uint32_t i) {
    return (uint32_t)bhg_llvm_writelane((int)x, (int)i, (int)v);
}
__device__ __forceinline__ void se_push(OpRing &r, uint32_t lane, uint32_t s, uint32_t e, uint32_t c) {
    // s, e, c, r.n are wave-uniform: one v_writelane each
    r.s = wlane(r.s, s, r.n);
    r.e = wlane(r.e, e, r.n);
    r.c = wlane(r.c, c, r.n);
    r.n = uni(r.n + 1);
}

// lane i <- lane i + 1 (DPP wave_shl:1; lane 63 gets 0)
__device__ __forceinline__ uint32_t lane_next(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

#ifdef BHG_SE_PROF
__device__ uint64_t se_prof[8];  // lab: cycles in scan / copy loop / flushes, counts
#define SE_T(x) const uint64_t x = __builtin_amdgcn_s_memtime()
#else
#define SE_T(x)
#endif

// The one LDS property se_batch's duplicate-bucket check relies on: when several lanes of ONE
// ds_write_b8 store to the same byte, the highest lane's byte is the one that stays.  This code
// cites no ISA rule for it, so bhg_create runs this probe on every device and refuses a device
// where it fails: the encoder never runs on an unchecked ordering.  64 mappings of the
// 64 lanes onto 1 .. 64 bytes; *bad counts the bytes that kept another lane's value.
__global__ __launch_bounds__(64) void k_lds_order_probe(uint32_t *bad) {
    __shared__ uint32_t words[64];
    uint8_t *const db = reinterpret_cast<uint8_t *>(words);
    const uint32_t lane = threadIdx.x;
    uint32_t errs = 0;
    for (uint32_t pat = 0; pat < 64; pat++) {
        const uint32_t nb = 1u << (pat % 7);  // 1 .. 64 distinct bytes
        const uint32_t idx = (((lane + 7 * pat) * 0x9E3779B1u) >> 20) % nb + 64 * (pat & 1);
        words[lane] = 0;
        wsync();
        db[idx] = (uint8_t)(lane + 1);
        wsync();
        const uint32_t got = db[idx];
        wsync();
        uint32_t hi = 0;
        for (uint32_t j = 0; j < 64; j++)
            if ((uint32_t)__builtin_amdgcn_readlane((int)idx, (int)j) == idx) hi = j;
        errs += got != hi + 1;
    }
    errs = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)__popcll(__ballot(errs != 0)));
    if (lane == 0) *bad = errs;
}

hipError_t launch_lds_order_probe(hipStream_t stream, uint32_t *bad) {
    hipLaunchKernelGGL(k_lds_order_probe, dim3(1), dim3(64), 0, stream, bad);
    return hipGetLastError();
}

// The end of one scan batch (lane = one iteration of encodeBlock's candidate loop, in order;
// lanes >= nl are not part of it): candidates read from the table as it was before the batch
// are corrected for buckets that two lanes share (the latest earlier lane wins -- Go stores
// every iteration's position before the next lookup), the 4-byte checks evaluated, the first
// event (a match, or an iteration past sLimit) found, and the table updated with the
// iterations up to it.  `eq` holds in[c .. c + 4) == u for the pre-batch c; lanes whose
// candidate changes are re-checked.  Returns the event lane (>= nl: none in this batch) and
// m_js, whether it is a match.
template <uint32_t DUMMY, class S>
__device__ __forceinline__ uint32_t se_batch(const S &in, se_tab_t *tab, uint32_t *dcnt, uint32_t lane,
                                             uint32_t nl, bool valid, uint64_t vmask, uint32_t pos, uint32_t u, uint32_t h,
                                             uint32_t &c, bool eq, bool &m_js, uint64_t *acc) {
    // lanes whose bucket (h mod 1024) a HIGHER lane of the batch shares: every lane writes its
    // lane number + 1 into the bucket's byte and reads it back -- in one LDS store instruction the
    // highest lane's byte is the one that stays (checked on the device by k_lds_order_probe when
    // the context is created), so exactly the lanes below another lane of their
    // bucket read a foreign byte (the highest lane of a bucket has no lane above it to hand its
    // position to, and nothing to learn from the walk: its nxt stays 64).  Invalid lanes write
    // into their own scratch bytes.  Two LDS operations, no atomics (the per-bucket counters
    // before: add, read, subtract).
    uint8_t *const db = reinterpret_cast<uint8_t *>(dcnt);
    const uint32_t bidx = valid ? (h & 1023u) : 1024u + lane;
    db[bidx] = (uint8_t)(lane + 1);
    wsync();
    const uint32_t got = db[bidx];
    wsync();
    // (lane predicates combined as 64-bit masks: a ballot of a combined bool re-materialises it
    // in a VGPR, two VALU each)
    const uint64_t vm = vmask;
    const uint64_t dm0 = vm & bal(got != lane + 1);
#ifdef BHG_SE_PROF
    acc[6] += 1;
    acc[7] += __builtin_popcountll(dm0);
#endif
    // in increasing lane order i: lanes above i with i's hash take pos_i as candidate (the
    // last such i wins), and lane i notes the first lane above it with its hash (nxt: it
    // stores into the table only if no later updating lane shares its bucket)
    const uint32_t c0 = c;
    uint32_t nxt = 64;
    uint64_t dm = dm0;
    while (dm) {
        const uint32_t i = (uint32_t)__builtin_ctzll(dm);
        dm &= dm - 1;
        const uint32_t hi = lane_val(h, i), pi = lane_val(pos, i);
        const bool same = h == hi;
        const uint64_t above = bal(same) & (~1ull << i);   // lanes > i with hash hi
        c = same && lane > i ? pi : c;
        nxt = wlane(nxt, above ? (uint32_t)__builtin_ctzll(above) : 64u, i);
    }
    uint64_t em = bal(eq);
    if (bal(c != c0)) em = bal(in.w(c) == u);
    const uint64_t mb = vm & em;  // matches
    const uint64_t ev = (nl >= 64 ? ~0ull : ((1ull << nl) - 1ull)) & (~vm | mb);
    const uint32_t js = ev ? (uint32_t)__builtin_ctzll(ev) : 64u;
    const uint32_t mj = (uint32_t)__builtin_popcountll(mb & ev & (0ull - ev));  // the event lane's match bit
    m_js = mj != 0;
    // updating iterations: the lanes before the event, and the event itself when it is a match
    const uint32_t nu = min(js + mj, nl);
    tab[lane < nu && nxt >= nu ? h : DUMMY + lane] = (se_tab_t)pos;   // others: a scratch slot each
    wsync();
    return js;
}

// encodeBlock on an LDS-staged block (len in [17, CAP]); tab zeroed by the caller.
// f0 / f0n: this lane's skip offsets F[lane] and F[lane + 1] (the block's first batch).
template <uint32_t DUMMY, class S>
__device__ void se_block_lds(Out &o, const S &in, uint32_t len, se_tab_t *tab, uint32_t *dcnt, uint32_t lane,
                             uint32_t f0, uint32_t f0n, uint64_t *acc) {
    len = uni(len);
    uint32_t shift = 24;
    for (uint32_t ts = 256; ts < 16384 && ts < len; ts *= 2) shift--;
    shift = uni(shift);
    const uint32_t tmask = 16383;
    const uint32_t sLimit = len - SE_MARGIN;
    uint32_t nextEmit = 0, s = 1;
    OpRing r;
    r.s = 0;
    r.e = 0;
    r.c = 0;
    r.n = 0;
    r.e0 = 0;
    // after a copy chain ends, the copy loop's last (failed) check leaves in[s - 1 + lane ..)
    // (U), its hash (hU) and the table entry of that hash (tU) in this lane's registers
    bool fast = false;
    uint32_t Uw = 0, hUw = 0, tUw = 0;
    for (;;) {
        // ---- scan phase: iterations k = 0,1,... at positions s + F[k] ----
        uint32_t cand = 0;
        bool remainder = false, found = false;
        SE_T(t_scan0);
        uint32_t kb = 0;
        if (fast) {
            // iterations 0..32 (F[k] = k; F[33] = 34) at s + k = lane k + 1 of the failed
            // check: u, its hash and its pre-batch table entry need no LDS read, and the
            // 4-byte check of that entry is issued with the duplicate count
            const uint32_t u = lane_next(Uw), h = lane_next(hUw);
            uint32_t c = lane_next(tUw);
            const bool inl = s + (lane < 32 ? lane + 1 : 34u) <= sLimit;
            const bool valid = lane <= 32 && inl;
            const uint64_t vmask = bal(inl) & ((2ull << 32) - 1ull);
            const uint32_t pos = s + lane;
            const bool eq = in.w(valid ? c : 0u) == u;
            bool m;
            const uint32_t js = se_batch<DUMMY>(in, tab, dcnt, lane, 33, valid, vmask, pos, u, h, c, eq, m, acc);
            if (js < 33) {
                found = true;
                if (!m) remainder = true;
                else { s = lane_val(pos, js); cand = lane_val(c, js); }
            }
            kb = 33;
        }
        for (; !found; kb += 64) {
            // skip offsets: the block's first batch from registers, later ones from the
            // constant table (a global load: it waits for the flushed output stores too)
            uint32_t fk = f0, fk1 = f0n;
            if (kb != 0) {
                // clamped, unconditional loads (F[1024] is the 2^31 - 1 sentinel; a <= 4 KiB
                // block's scan ends by k = 177)
                fk = kSkip.f[min(kb + lane, 1024u)];
                fk1 = kSkip.f[min(kb + lane + 1, 1024u)];
            }
            // s < 64 Ki and F[k] <= 2^31 - 1: the sums fit in 32 bits
            const bool valid = s + fk1 <= sLimit;
            const uint32_t pos = valid ? s + fk : 0u;
            const uint32_t u = in.w(pos);
            const uint32_t h = se_hash(u, shift) & tmask;
            uint32_t c = tab[h];  // invalid lanes hash position 0: any entry, unused
            const bool eq = in.w(c) == u;
            bool m;
            const uint32_t js = se_batch<DUMMY>(in, tab, dcnt, lane, 64, valid, bal(valid), pos, u, h, c, eq, m, acc);
            if (js < 64) {
                found = true;
                if (!m) remainder = true;
                else { s = lane_val(pos, js); cand = lane_val(c, js); }
            }
        }
#ifdef BHG_SE_PROF
        SE_T(t_scan1);
        acc[0] += t_scan1 - t_scan0;
        acc[3] += 1;
#endif
        if (remainder) break;
        // ---- copies (encode_other.go's inner loop).  Each iteration reads, at once,
        // U = in[s + lane .. + 4) and in[cand + lane] -- the byte compare both verifies the
        // 4-byte match (Go's load32 check; always true for the scan's match) and extends it
        // 64 bytes a round (Go extends from s + 4 after a verified match: the same first
        // mismatch) -- and U's hashes are the table slots of every position the copy can end
        // at below s + 64.  The table is read for all of them right away: the only
        // store between now and Go's lookup at the copy end e is tab[prevHash] = e - 1, and
        // prevHash == currHash is resolved by a compare.  So the lookup costs no LDS round
        // trip after the compare; copies ending at s + 64 or later take a serial lookup.
        for (;;) {
            // s, cand are wave-uniform; the compiler's divergence analysis cannot see it through
            // the loop's phis and kept them (and everything computed from them) in VGPRs
            s = uni(s);
            cand = uni(cand);
            const bool tail = s + 67 > len;  // (wave-uniform) the window reaches past the block
            const uint32_t U = tail ? in.wt(s + lane) : in.w(s + lane);
            const uint32_t V = tail ? in.bt(cand + lane) : in.b(cand + lane);
            const uint32_t hU = se_hash(U, shift) & tmask;
            const uint32_t tU = tab[hU];
            const uint64_t mm = bal((U & 0xffu) != V);
            // the first mismatch lane (64: none) as a scalar, so the mins stay SALU
            uint32_t f = min(uni(mm ? (uint32_t)__builtin_ctzll(mm) : 64u), len - s);
            if (f < 4u) {  // the chained candidate does not match: scanning resumes at s + 1
                Uw = U;
                hUw = hU;
                tUw = tU;
                break;
            }
            uint32_t r0 = s;  // start of the round that found the mismatch
            while (f == 64u) {
                r0 += 64;
                const bool t2 = r0 + 64 > len;
                const uint64_t m2 = bal(t2 ? in.bt(r0 + lane) != in.bt(cand + (r0 - s) + lane)
                                           : in.b(r0 + lane) != in.b(cand + (r0 - s) + lane));
                f = min(uni(m2 ? (uint32_t)__builtin_ctzll(m2) : 64u), len - r0);
            }
            const uint32_t e = r0 + f;
            se_push(r, lane, s, e, cand);
            nextEmit = e;
            const uint32_t q = e - s;
            s = e;
            if (s >= sLimit) break;
            uint32_t prevHash, currHash, tc;
            if (q < 64u) {
                prevHash = lane_val(hU, q - 1);
                currHash = lane_val(hU, q);
                tc = lane_val(tU, q);
            } else {  // x = in[s - 1 .. s + 7), then Go's lookup
                const uint32_t x0 = uni(in.w(s - 1)), x1 = uni(in.w(s + 3));
                prevHash = se_hash(x0, shift) & tmask;
                currHash = se_hash(x0 >> 8 | x1 << 24, shift) & tmask;
                tc = uni(tab[currHash]);
            }
            // tab[prevHash] = s - 1, then tab[currHash] = s: one store by lanes 0 and 1 (when
            // the slots coincide both lanes store s)
            const bool same = prevHash == currHash;
            wsync();
            // lane 0 stores s - 1 (s when the slots coincide) at prevHash, lane 1 s at currHash,
            // the others s into their scratch slots: two v_writelane per operand
            {
                const uint32_t ad = wlane(wlane(DUMMY + lane, prevHash, 0), currHash, 1);
                tab[ad] = (se_tab_t)wlane(s, same ? s : s - 1, 0);
            }
            cand = same ? s - 1 : tc;
            wsync();
            if (r.n == 64) se_flush(o, in, r, lane);
        }
#ifdef BHG_SE_PROF
        SE_T(t_cp1);
        acc[2] += t_cp1 - t_scan1;
#endif
        if (s >= sLimit) break;
        s += 1;
        fast = true;
    }
    if (nextEmit < len) {
        if (r.n == 64) se_flush(o, in, r, lane);
        se_push(r, lane, len, len, len);
    }
    if (r.n) se_flush(o, in, r, lane);
}

// one wave per value: val bytes vals[val_off[i] .. val_off[i+1]) -> scratch[soff[i] ..), clen[i],
// for the values i = list[0 .. *cnt) (*head: the work-queue head, zeroed by the caller).  CAP:
// the LDS block capacity (SE_CAP_SMALL: the values <= 2 KiB, whose 7.3 KiB of LDS lets VGPRs
// bound the waves per CU; SE_CAP: the values of 2-4 KiB, 13.2 KiB).  The class lists never hold a
// value longer than CAP (k_enc_class: longer values take the block path).
template <int CAP, int WPG, int MINW>
__global__ __launch_bounds__(64 * WPG, MINW) void k_snappy_enc(const uint8_t *__restrict__ vals, const uint64_t *__restrict__ val_off,
                                                   const uint32_t *__restrict__ list, const uint32_t *__restrict__ cnt,
                                                   uint32_t *__restrict__ head,
                                                   uint8_t *__restrict__ scratch, uint64_t scap,
                                                   const uint64_t *__restrict__ soff, uint64_t *__restrict__ clen) {
    // one LDS buffer: block (+16 zero bytes), table, dedupe counters, scratch store slots.
    // The copy loop's compares read up to 67 bytes past a position < CAP: into the
    // table, never past the buffer, and clipped to the block length.
    typedef SeLayout<CAP> LY;
    // WPG waves per workgroup, each on its own LDS slice and its own values (no barriers):
    // LDS is allocated per workgroup in 2-KiB granules, so 3 x 13.2 KiB fit 4 times in a CU's
    // 160 KiB (12 waves) where single 13.2 KiB waves fit 11 times
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[WPG][LY::kWords];
    const uint32_t wid = threadIdx.x >> 6, gw = blockIdx.x * WPG + wid, nw = gridDim.x * WPG;
    uint32_t *lds = lds_all[wid];
    uint8_t *in = reinterpret_cast<uint8_t *>(lds);
    se_tab_t *tab = reinterpret_cast<se_tab_t *>(lds + (CAP + 16) / 4);
    uint32_t *dcnt = lds + (CAP + 16) / 4 + LY::kTab * sizeof(se_tab_t) / 4;
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t j = lane; j < kSeDcnt; j += 64) dcnt[j] = 0;
    const uint32_t f0 = kSkip.f[lane], f0n = kSkip.f[lane + 1];
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef BHG_SE_PROF
    const uint64_t t_k0 = __builtin_amdgcn_s_memtime();
#endif
    // work queue: a wave's first value is list[gw] (gw: its wave index), every later one
    // list[nw + atomicAdd(head)] -- value costs vary ~30x (length, compressibility), so a
    // static round-robin split left the waves with the most work running alone at the end
    // (C4 84.5 -> 98.3 GiB/s on one box).  The next index is requested when a value starts
    // and read when it ends.  (Longest-first order within a class measured 1 % slower.)
    const uint32_t n = *cnt;
    // Positions are pipelined so that no value waits for its own bookkeeping: while value j
    // runs, the next position's list entry i1 is known and its offsets (m1) are loaded, and
    // the position after it (j2) is taken from the queue and its list entry loaded -- issued
    // once this value's bytes are staged (the staging round trip covers the queue atomic).
    // Before, every value started with three dependent round trips (list, offsets, bytes).
    struct Meta {
        uint32_t i;
        uint64_t v0, v1, s0, s1;
    };
    auto meta_of = [&](uint32_t jj, uint32_t ii) {
        Meta m = {ii, 0, 0, 0, 0};
        if (jj < n) {
            m.v0 = val_off[ii];
            m.v1 = val_off[ii + 1];
            m.s0 = soff[ii];
            m.s1 = soff[ii + 1];
        }
        return m;
    };
    // the first kSeStatic % of the list goes round-robin (position cur + nw, no atomic: a
    // queue atomic per value made every wave contend on one address), the rest through the
    // queue (positions qbase + head++), which evens out the end of the launch
    const uint32_t qbase = (uint32_t)((uint64_t)n * kSeStatic / 100 / nw * nw);
    auto need_q = [&](uint32_t cur) { return cur + nw >= qbase; };
    // kSeHeads queue heads, 128 B apart: wave gw takes from head gw mod H, whose positions are
    // qstart + h + H k (the waves of one head are an interleaved H-th of the grid, its positions
    // an interleaved H-th of the queued part: balanced, and H times fewer atomics per address)
    const uint32_t hq = gw % kSeHeads;
    uint32_t *const myhead = head + 32 * hq;
    auto take = [&](uint32_t cur, uint32_t req) {
        return need_q(cur) ? max(qbase, nw) + hq + kSeHeads * uni(req) : cur + nw;
    };
    uint32_t j = gw;
    Meta mc = meta_of(j, j < n ? list[j] : 0u);
    uint32_t r0 = 0;
    if (lane == 0 && need_q(j)) r0 = atomicAdd(myhead, 1u);
    uint32_t j1 = take(j, r0);
    uint32_t i1 = j1 < n ? list[j1] : 0u;
    while (j < n) {
        uint32_t rq = 0;
        if (lane == 0 && need_q(j1)) rq = atomicAdd(myhead, 1u);  // the position after j1
        uint32_t j2 = 0, i2 = 0;
        Meta m1 = {0, 0, 0, 0, 0};
        bool hooked = false;
        auto hook = [&]() {  // once per value, after its bytes are staged
            if (hooked) return;
            hooked = true;
            j2 = take(j1, rq);
            i2 = j2 < n ? list[j2] : 0u;
            m1 = meta_of(j1, i1);
        };
        const uint32_t i = mc.i;
        const uint64_t v0 = mc.v0, vlen = mc.v1 - mc.v0;
        if (mc.s1 > scap) {  // val_off inconsistent with the vals_len the caller passed
            if (lane == 0) clen[i] = ~0ull;
            hook();
            j = j1; j1 = j2; i1 = i2; mc = m1;
            continue;
        }
        const uint8_t *src = vals + v0;
        Out o;
        o.g = scratch + mc.s0;
        o.d = 0;
        // uvarint(len(src))
        {
            uint64_t x = vlen;
            uint32_t k = 0;
            while (x >= 0x80) {
                if (lane == 0) o.g[k] = (uint8_t)x | 0x80;
                x >>= 7;
                k++;
            }
            if (lane == 0) o.g[k] = (uint8_t)x;
            o.d = k + 1;
        }
        for (uint64_t b0 = 0; b0 < vlen; b0 += SE_MAXBLOCK) {
            const uint32_t blen = (uint32_t)(vlen - b0 < SE_MAXBLOCK ? vlen - b0 : SE_MAXBLOCK);
            const uint8_t *bs = src + b0;
            if (blen < SE_MINNONLIT) {
                se_emit_literal(o, nullptr, bs, blen, lane);
            } else {  // blen <= CAP: the class lists hold values of at most CAP bytes
                // one 16-B load per lane per 1 KiB (one memory round trip), then the 16 zero bytes
                for (uint32_t t = 16 * lane; t < blen; t += 1024) {
                    u32x4 v;
                    if (t + 16 <= blen) {
                        v = gld<u32x4u>((uint64_t)(bs + t));
                    } else {
                        uint32_t w[4] = {0, 0, 0, 0};
                        for (uint32_t b = 0; t + b < blen; b++) w[b >> 2] |= (uint32_t)bs[t + b] << (8 * (b & 3));
                        v = u32x4{w[0], w[1], w[2], w[3]};
                    }
                    *reinterpret_cast<u32x4 *>(in + t) = v;
                }
                wsync();
                for (uint32_t t = blen + lane; t < blen + 16; t += 64) in[t] = 0;
                uint32_t ts = 256;
                while (ts < 16384 && ts < blen) ts *= 2;
                for (uint32_t t = 8 * lane; t < ts; t += 512)   // 16 B per lane per store (ts >= 256)
                    *reinterpret_cast<u32x4 *>(tab + t) = u32x4{0, 0, 0, 0};
                wsync();
                hook();
                se_block_lds<LY::kDummy>(o, SrcLds{in}, blen, tab, dcnt, lane, f0, f0n, acc);
            }
        }
        hook();  // (values with no LDS block)
        if (lane == 0) clen[i] = o.d;
        acc[4] += 1;
        j = j1;
        j1 = j2;
        i1 = i2;
        mc = m1;
    }
#ifdef BHG_SE_PROF
    acc[5] = __builtin_amdgcn_s_memtime() - t_k0;
    if (lane == 0)
        for (int q = 0; q < 8; q++) atomicAdd((unsigned long long *)&se_prof[q], (unsigned long long)acc[q]);
    if ((gw & 255) == 0 && lane == 0)
        printf("se_prof cap %d wave %u: scan %llu lit %llu copy %llu phases %llu values %llu total %llu batches %llu duplanes %llu\n",
               CAP, gw,
               (unsigned long long)acc[0], (unsigned long long)acc[1], (unsigned long long)acc[2],
               (unsigned long long)acc[3], (unsigned long long)acc[4], (unsigned long long)acc[5],
               (unsigned long long)acc[6], (unsigned long long)acc[7]);
#endif
}

__global__ __launch_bounds__(256) void k_snappy_maxlen(const uint64_t *val_off, uint32_t n, uint64_t *out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t v = val_off[i + 1] - val_off[i];
        out[i] = 32 + v + v / 6;                 // MaxEncodedLen (encode.go)
    }
}

hipError_t launch_snappy_maxlen(const Launch &L, const uint64_t *val_off, uint32_t n, uint64_t *out) {
    hipLaunchKernelGGL(k_snappy_maxlen, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, val_off, n, out);
    return hipGetLastError();
}

// values <= SE_CAP_SMALL -> list[0 ..), those of (SE_CAP_SMALL, SE_CAP] -> list[n ..) (longer ones take the
// block path); counts in cnt[0], cnt[1]
// (zeroed by the caller).  A workgroup of 16 waves takes 4,096 consecutive values and makes one
// atomic per list (one per wave contended on two addresses: 0.36 ms per 1M values).  Order
// within a list only schedules the encoder's waves.
constexpr uint32_t kClassWaves = 16, kClassPer = 4;
__global__ __launch_bounds__(64 * kClassWaves) void k_enc_class(const uint64_t *__restrict__ val_off, uint32_t n,
                                                                uint32_t *__restrict__ list, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t wc[kClassWaves][2];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    const uint32_t b0 = blockIdx.x * (64 * kClassWaves * kClassPer);
    uint64_t ms[kClassPer], mb[kClassPer];
    uint32_t cs = 0, cb = 0;
#pragma unroll
    for (uint32_t it = 0; it < kClassPer; it++) {
        const uint32_t i = b0 + it * 64 * kClassWaves + threadIdx.x;
        const uint64_t vl = i < n ? val_off[i + 1] - val_off[i] : 0;
        const bool v = i < n && vl <= SE_CAP;  // longer values: the block path (k_snappy_enc_blocks)
        const bool big = v && vl > SE_CAP_SMALL;
        mb[it] = __ballot(big);
        ms[it] = __ballot(v && !big);
        cs += (uint32_t)__builtin_popcountll(ms[it]);
        cb += (uint32_t)__builtin_popcountll(mb[it]);
    }
    if (lane == 0) { wc[w][0] = cs; wc[w][1] = cb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t ts = 0, tb = 0;
        for (uint32_t k = 0; k < kClassWaves; k++) {
            const uint32_t s0 = wc[k][0], s1 = wc[k][1];
            wc[k][0] = ts; wc[k][1] = tb;  // exclusive offsets of the waves
            ts += s0; tb += s1;
        }
        const uint32_t bs = ts ? atomicAdd(&cnt[0], ts) : 0u, bb = tb ? atomicAdd(&cnt[1], tb) : 0u;
        for (uint32_t k = 0; k < kClassWaves; k++) { wc[k][0] += bs; wc[k][1] += bb; }
    }
    __syncthreads();
    uint32_t os = wc[w][0], ob = wc[w][1];
#pragma unroll
    for (uint32_t it = 0; it < kClassPer; it++) {
        const uint32_t i = b0 + it * 64 * kClassWaves + threadIdx.x;
        if ((mb[it] >> lane) & 1ull) list[n + ob + __builtin_popcountll(mb[it] & below)] = i;
        if ((ms[it] >> lane) & 1ull) list[os + __builtin_popcountll(ms[it] & below)] = i;
        os += (uint32_t)__builtin_popcountll(ms[it]);
        ob += (uint32_t)__builtin_popcountll(mb[it]);
    }
}

// workgroups: as many as are resident (LDS-bound: 3 x 13.2 KiB per workgroup at SE_CAP -> 4
// per CU with 2-KiB allocation granules; 7.3 KiB at SE_CAP_SMALL -> VGPR-bound): a grid past
// what is resident would start its extra workgroups only when the first ones finish
template <int CAP, int WPG, int MINW>
static uint32_t enc_grid(const Launch &L, uint32_t n) {
    static const uint32_t per_cu = resident_per_cu((const void *)k_snappy_enc<CAP, WPG, MINW>, 64 * WPG, kSeWaves / WPG);
    uint32_t pc = per_cu;
    uint32_t g = (uint32_t)L.num_cus * pc;
    if ((uint64_t)g * WPG > n) g = (n + WPG - 1) / WPG;
    return g ? g : 1;
}

// ---- the block path: values longer than SE_CAP ----
constexpr uint32_t kSeBlockMax = 32 + SE_MAXBLOCK + SE_MAXBLOCK / 6;  // MaxEncodedLen(64 KiB): a full block's slot

// per value: its 64-KiB blocks when it takes the block path (else 0), and the bytes of its block
// slots (full blocks kSeBlockMax apart, the last one MaxEncodedLen of its length)
// (a value past the vals_len the caller passed gets no blocks and clen ~0: NO_SPACE, as the
// value kernels' scratch check gives)
__global__ __launch_bounds__(256) void k_enc_bcount(const uint64_t *__restrict__ val_off, uint32_t n, uint64_t vals_len,
                                                    uint64_t *__restrict__ bcnt, uint64_t *__restrict__ bbytes,
                                                    uint64_t *__restrict__ clen) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t v = val_off[i + 1] - val_off[i];
        uint64_t nb = 0, by = 0;
        if (v > SE_CAP && val_off[i + 1] > vals_len) {
            clen[i] = ~0ull;
        } else if (v > SE_CAP) {
            nb = (v + SE_MAXBLOCK - 1) / SE_MAXBLOCK;
            const uint64_t last = v - (nb - 1) * SE_MAXBLOCK;
            by = (nb - 1) * kSeBlockMax + 32 + last + last / 6;
        }
        bcnt[i] = nb;
        bbytes[i] = by;
    }
}

// after the scans (bbase: first block index per value, bbase[n] blocks; bsoff: slot bytes):
// the (value, block) list
__global__ __launch_bounds__(256) void k_enc_bemit(const uint64_t *__restrict__ bbase, uint32_t n,
                                                   uint2 *__restrict__ ent) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b0 = bbase[i], b1 = bbase[i + 1];
        for (uint64_t b = b0; b < b1; b++) ent[b] = make_uint2(i, (uint32_t)(b - b0));
    }
}

// one wave per 64-KiB block, blocks taken from a queue: encodeBlock (or emitLiteral for a last
// block under 17 bytes) into the block's slot, its length into bclen.  The matcher reads the block
// in place (SrcGlb): LDS holds only the 16-K-entry table (33 KiB), so 4 waves run per CU.  With
// the block staged in LDS too (98 KiB, one wave per CU) bench.py --config bigval encoded at 20.5
// GiB/s against 40.4 (profiles/r6/bigval/enc_blocks_gsrc.txt); for the <= 4 KiB values the
// staged block wins (C4 179 vs 145 GiB/s with the value read in place, profiles/r6/c4_gsrc/):
// their limit is one wave's latency chain, not the waves per CU.
constexpr uint32_t kSeBlockWaves = 4;
__global__ __launch_bounds__(64) void k_snappy_enc_blocks(const uint8_t *__restrict__ vals,
                                                          const uint64_t *__restrict__ val_off,
                                                          const uint64_t *__restrict__ bbase, uint32_t n,
                                                          const uint2 *__restrict__ ent, uint32_t *__restrict__ head,
                                                          uint8_t *__restrict__ bscr, const uint64_t *__restrict__ bsoff,
                                                          uint32_t *__restrict__ bclen) {
    typedef SeLayout<SE_CAP_BLOCK, true> LY;
    __shared__ __attribute__((aligned(16))) uint32_t lds[LY::kWords];
    se_tab_t *tab = reinterpret_cast<se_tab_t *>(lds + LY::kBlk);
    uint32_t *dcnt = lds + LY::kBlk + LY::kTab * sizeof(se_tab_t) / 4;
    const uint32_t lane = threadIdx.x;
    for (uint32_t j = lane; j < kSeDcnt; j += 64) dcnt[j] = 0;
    const uint32_t f0 = kSkip.f[lane], f0n = kSkip.f[lane + 1];
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t total = bbase[n];
    uint32_t q = blockIdx.x;  // the first block: no queue round trip
    while (q < total) {
        const uint2 e = ent[q];
        // the next block's position, taken now (its atomic in flight while this block runs)
        uint32_t nq = 0;
        if (lane == 0) nq = atomicAdd(head, 1u) + gridDim.x;
        const uint64_t v0 = val_off[e.x], vlen = val_off[e.x + 1] - v0;
        const uint64_t b0 = (uint64_t)e.y * SE_MAXBLOCK;
        const uint32_t blen = (uint32_t)(vlen - b0 < SE_MAXBLOCK ? vlen - b0 : SE_MAXBLOCK);
        const uint8_t *bs = vals + v0 + b0;
        Out o;
        o.g = bscr + bsoff[e.x] + (uint64_t)e.y * kSeBlockMax;
        o.d = 0;
        if (blen < SE_MINNONLIT) {
            se_emit_literal(o, nullptr, bs, blen, lane);
        } else {
            uint32_t ts = 256;
            while (ts < 16384 && ts < blen) ts *= 2;
            for (uint32_t t = 8 * lane; t < ts; t += 512) *reinterpret_cast<u32x4 *>(tab + t) = u32x4{0, 0, 0, 0};
            wsync();
            se_block_lds<LY::kDummy>(o, SrcGlb{bs, blen}, blen, tab, dcnt, lane, f0, f0n, acc);
        }
        if (lane == 0) bclen[q] = o.d;
        q = uni(nq);
        wsync();  // the next block's table reset overwrites the LDS the matcher read
    }
}

// one WAVE per block of the block path (persistent grid): the block's output copied to its place in
// the value's scratch range -- after uvarint(len(src)) (encode.go Encode) and the outputs of the
// value's earlier blocks, whose lengths the wave sums -- and, by block 0's wave, the header and
// clen[i].  (A wave per VALUE copying 64 bytes per instruction took 1.54 ms of the bigval encode step
// for the longest value's 2.3 MB, and 83 us of every C4 step launching a wave per value;
// profiles/r6/final/.)
#define SE_BCOPY_WAVES 4
__global__ __launch_bounds__(64 * SE_BCOPY_WAVES) void k_snappy_bcopy(const uint64_t *__restrict__ val_off, uint32_t n,
                                                                    const uint64_t *__restrict__ bbase,
                                                                    const uint2 *__restrict__ ent,
                                                                    const uint8_t *__restrict__ bscr,
                                                                    const uint64_t *__restrict__ bsoff,
                                                                    const uint32_t *__restrict__ bclen,
                                                                    uint8_t *__restrict__ scratch, uint64_t scap,
                                                                    const uint64_t *__restrict__ soff,
                                                                    uint64_t *__restrict__ clen) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t total = bbase[n];
    const uint64_t nw = (uint64_t)gridDim.x * SE_BCOPY_WAVES, w0 = (uint64_t)blockIdx.x * SE_BCOPY_WAVES + (threadIdx.x >> 6);
    for (uint64_t q = w0; q < total; q += nw) {
        const uint2 e = ent[q];
        const uint32_t i = e.x, b = e.y;
        const uint64_t b0 = bbase[i], b1 = bbase[i + 1];
        if (soff[i + 1] > scap) {  // val_off inconsistent with the vals_len the caller passed
            if (b == 0 && lane == 0) clen[i] = ~0ull;
            continue;
        }
        const uint64_t x = val_off[i + 1] - val_off[i];
        uint32_t hdr = 1;
        for (uint64_t y = x; y >= 0x80; y >>= 7) hdr++;
        // the outputs before this block (all of them, for block 0's clen)
        const uint32_t upto = b == 0 ? (uint32_t)(b1 - b0) : b;
        uint64_t before = 0;
        for (uint32_t k = lane; k < upto; k += 64) before += bclen[b0 + k];
        for (int m = 1; m < 64; m <<= 1) before += (uint64_t)__shfl_xor((long long)before, m, 64);
        uint8_t *d0 = scratch + soff[i];
        if (b == 0) {
            if (lane < hdr) d0[lane] = (uint8_t)((x >> (7 * lane)) & 0x7f) | (lane + 1 < hdr ? 0x80 : 0);
            if (lane == 0) clen[i] = hdr + before;
            before = 0;
        }
        const uint64_t dst = (uint64_t)d0 + hdr + before, len = bclen[q];
        const uint64_t src = (uint64_t)bscr + bsoff[i] + (uint64_t)b * kSeBlockMax;
        // bytes up to the first 4-aligned output address, then 16-B output chunks from 20-B source
        // windows (the slot is MaxEncodedLen long, the buffer 64 B longer: the windows stay inside)
        const uint64_t head = ((4u - (uint32_t)(dst & 3)) & 3u) < len ? ((4u - (uint32_t)(dst & 3)) & 3u) : len;
        if (lane < head) reinterpret_cast<uint8_t *>(dst)[lane] = reinterpret_cast<const uint8_t *>(src)[lane];
        const uint64_t qd = dst + head, qend = dst + len, sd = src + head;
        const uint32_t nc = (uint32_t)((qend - qd + 15) >> 4);
        for (uint32_t c0 = 0; c0 < nc; c0 += 256) {
            u32x4 wx[4];
            uint32_t w4[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t c = c0 + lane + 64 * k;
                const uint64_t sa = (sd + 16ull * (c < nc ? c : 0u)) & ~3ull;
                wx[k] = gld<u32x4_a4>(sa);
                w4[k] = gld<uint32_t>(sa + 16);
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t c = c0 + lane + 64 * k;
                if (c >= nc) continue;
                const uint32_t f = (uint32_t)((sd + 16ull * c) & 3);
                const u32x4 y = {__builtin_amdgcn_alignbyte(wx[k].y, wx[k].x, f), __builtin_amdgcn_alignbyte(wx[k].z, wx[k].y, f),
                                 __builtin_amdgcn_alignbyte(wx[k].w, wx[k].z, f), __builtin_amdgcn_alignbyte(w4[k], wx[k].w, f)};
                const uint64_t o = qd + 16ull * c;
                if (o + 16 <= qend) {
                    gst<u32x4_a4>(o, y);
                } else {
                    const uint32_t yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                    for (int z = 0; z < 4; z++) {
                        const uint64_t oz = o + 4 * z;
                        if (oz + 4 <= qend) {
                            gst<uint32_t>(oz, yy[z]);
                        } else {
#pragma unroll
                            for (int t = 0; t < 4; t++)
                                if (oz + t < qend) gst<uint8_t>(oz + t, (uint8_t)(yy[z] >> (8 * t)));
                        }
                    }
                }
            }
        }
    }
}

// class lists (2n), class counts (4 words), then 2 x kSeHeads queue heads of 32 words each, then
// the block queue's head
constexpr uint32_t kQueueWords = 4 + 2 * kSeHeads * 32 + 32;
size_t snappy_enc_list_bytes(uint32_t n) { return ((size_t)2 * n + kQueueWords) * 4; }

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
static uint64_t max_blocks(uint32_t n, uint64_t vals_len) { return vals_len / SE_MAXBLOCK + n + 1; }
size_t snappy_block_scratch_bytes(uint32_t n, uint64_t vals_len) {
    const uint64_t mb = max_blocks(n, vals_len);
    return 2 * al256(((size_t)n + 1) * 8) + al256(scan_scratch_bytes(n)) + al256(mb * 8) + al256(mb * 4) +
           al256(32 * mb + vals_len + vals_len / 6 + 64);
}

hipError_t launch_snappy_enc(const Launch &L, const uint8_t *vals, const uint64_t *val_off, uint32_t n, uint64_t vals_len,
                             uint8_t *scratch, uint64_t scap, const uint64_t *soff, uint64_t *clen, uint32_t *lists,
                             void *block_scratch) {
    uint32_t *cnt = lists + 2 * (size_t)n;  // class counts cnt[0..1], queue heads from cnt + 4
    uint32_t *bhead = cnt + 4 + 2 * kSeHeads * 32;
    if (hipError_t e = hipMemsetAsync(cnt, 0, kQueueWords * 4, L.stream)) return e;
    const uint32_t per = 64 * kClassWaves * kClassPer;
    hipLaunchKernelGGL(k_enc_class, dim3((n + per - 1) / per), dim3(64 * kClassWaves), 0, L.stream, val_off, n, lists,
                       cnt);
    if (hipError_t e = hipGetLastError()) return e;
    static_assert(SE_CAP_SMALL <= SE_CAP, "small-value class must fit the LDS block");
    hipLaunchKernelGGL((k_snappy_enc<SE_CAP_SMALL, 1, kSeMinwSmall>), dim3(enc_grid<SE_CAP_SMALL, 1, kSeMinwSmall>(L, n)), dim3(64), 0, L.stream, vals,
                       val_off, (const uint32_t *)lists, cnt, cnt + 4, scratch, scap, soff, clen);
    if (hipError_t e = hipGetLastError()) return e;
    hipLaunchKernelGGL((k_snappy_enc<SE_CAP, kSeWpg, 3>), dim3(enc_grid<SE_CAP, kSeWpg, 3>(L, n)), dim3(64 * kSeWpg), 0,
                       L.stream, vals, val_off, (const uint32_t *)lists + n, cnt + 1, cnt + 4 + 32 * kSeHeads, scratch, scap, soff, clen);
    if (hipError_t e = hipGetLastError()) return e;
    // the block path (values > SE_CAP): block counts -> scans -> (value, block) list -> blocks -> concat
    uint8_t *sp = static_cast<uint8_t *>(block_scratch);
    uint64_t *bbase = reinterpret_cast<uint64_t *>(sp);
    sp += al256(((size_t)n + 1) * 8);
    uint64_t *bsoff = reinterpret_cast<uint64_t *>(sp);
    sp += al256(((size_t)n + 1) * 8);
    void *scan = sp;
    sp += al256(scan_scratch_bytes(n));
    const uint64_t mb = max_blocks(n, vals_len);
    uint2 *ent = reinterpret_cast<uint2 *>(sp);
    sp += al256(mb * 8);
    uint32_t *bclen = reinterpret_cast<uint32_t *>(sp);
    sp += al256(mb * 4);
    uint8_t *bscr = sp;
    hipLaunchKernelGGL(k_enc_bcount, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, val_off, n, vals_len, bbase,
                       bsoff, clen);
    if (hipError_t e = hipGetLastError()) return e;
    if (hipError_t e = launch_exclusive_scan_u64(L, bbase, bbase, n, scan)) return e;
    if (hipError_t e = launch_exclusive_scan_u64(L, bsoff, bsoff, n, scan)) return e;
    hipLaunchKernelGGL(k_enc_bemit, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, bbase, n, ent);
    hipLaunchKernelGGL(k_snappy_enc_blocks, dim3(L.num_cus * kSeBlockWaves), dim3(64), 0, L.stream, vals, val_off, bbase,
                       n, ent, bhead, bscr, bsoff, bclen);
    hipLaunchKernelGGL(k_snappy_bcopy, dim3(L.num_cus * 8), dim3(64 * SE_BCOPY_WAVES), 0, L.stream, val_off, n, bbase,
                       (const uint2 *)ent, bscr, bsoff, bclen, scratch, scap, soff, clen);
    return hipGetLastError();
}

}  // namespace bhg
