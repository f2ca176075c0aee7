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
// Blocks longer than 4 KiB (values > 4 KiB are cut in 64 KiB blocks) use a
// lane-0 walk with the table in global scratch.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

typedef u32x4 u32x4u __attribute__((aligned(1)));
#ifndef BHG_SE_U16
#define BHG_SE_U16 1  // measured with the register skip offsets: 49.4 GiB/s (11 waves/CU) vs 37.7 (u32, 7)
#endif
#ifndef BHG_SE_STAGE16
#define BHG_SE_STAGE16 1  // measured: C4 30.7 vs 30.0 GiB/s (u16 table: 28.1 at 7 waves, 26.5 at 12)
#endif
#ifndef BHG_SE_DCNT
#define BHG_SE_DCNT 256  // dwords of byte counters for the in-batch duplicate check (4 buckets each)
#endif
#ifndef BHG_SE_WAVES
#define BHG_SE_WAVES 7
#endif
#if BHG_SE_U16
typedef uint16_t se_tab_t;
#else
typedef uint32_t se_tab_t;
#endif

#define SE_CAP 4096                 // LDS block capacity
#define SE_TAB 4096                 // LDS table entries (tableSize <= 4096 when len <= 4096)
#define SE_MAXBLOCK 65536           // encode.go maxBlockSize
#define SE_MARGIN 15                // inputMargin
#define SE_MINNONLIT 17             // minNonLiteralBlockSize

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

// one (unaligned) ds_read_b32: gfx950 LDS takes unaligned dword reads
typedef uint32_t u32_lds_u __attribute__((aligned(1), may_alias));
// (4 byte reads measured 5 % slower, two aligned dwords + a funnel shift the same)
__device__ __forceinline__ uint32_t lds_ld32(const uint8_t *b, uint32_t i) {
    return *reinterpret_cast<const u32_lds_u *>(b + i);
}
// lane i's value for a wave-uniform i: v_readlane, not an LDS permute
__device__ __forceinline__ uint32_t lane_val(uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); }

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
// order LDS accesses of this wave (no instruction: LDS executes a wave's ops in order)
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }

// encodeBlock on an LDS-staged block (len in [17, SE_CAP]); tab zeroed by the caller.
// this lane's skip offsets F[64 j + lane] and F[64 j + lane + 1], j < 16 (k < 1024)
struct LaneSkip {
    uint32_t f[16], f1[16];
};

#ifdef BHG_SE_PROF
__device__ uint64_t se_prof[8];  // lab: cycles in scan / literal emit / copy loop, counts
#define SE_T(x) const uint64_t x = __builtin_amdgcn_s_memtime()
#else
#define SE_T(x)
#endif
__device__ void se_block_lds(Out &o, const uint8_t *in, uint32_t len, se_tab_t *tab, uint32_t *dcnt, uint32_t lane,
                             const LaneSkip &F, uint64_t *acc) {
    uint32_t shift = 24;
    for (uint32_t ts = 256; ts < 16384 && ts < len; ts *= 2) shift--;
    const uint32_t tmask = 16383;
    const uint32_t sLimit = len - SE_MARGIN;
    uint32_t nextEmit = 0, s = 1;
    for (;;) {
        // ---- scan phase: iterations k = 0,1,... at positions s + F[k] ----
        uint32_t cand = 0;
        bool remainder = false;
        SE_T(t_scan0);
        for (uint32_t kb = 0;; kb += 64) {
            // skip offsets from registers: a global load here would make the wave wait
            // (vmcnt counts stores on gfx950) for every byte of output emitted so far
            uint32_t fk = F.f[0], fk1 = F.f1[0];
            if (kb != 0) {  // wave-uniform; the first batch is by far the most common
                fk = 0x7fffffffu;
                fk1 = 0x7fffffffu;
#pragma unroll
                for (uint32_t j = 1; j < 16; j++)
                    if (kb == 64 * j) {
                        fk = F.f[j];
                        fk1 = F.f1[j];
                    }
            }
            // s < 64 Ki and F[k] <= 2^31 - 1: the sums fit in 32 bits
            const bool valid = s + fk1 <= sLimit;
            const uint32_t pos = valid ? s + fk : 0u;
            const uint32_t u = lds_ld32(in, pos);
            const uint32_t h = se_hash(u, shift) & tmask;
            // bucket duplicates inside the batch (latest earlier lane wins): per-bucket counts
            // of h mod 1024, one byte per bucket (<= 64 adds per byte)
            const uint32_t slot = (h >> 2) & (BHG_SE_DCNT - 1u), sh8 = 8 * (h & 3);
            atomicAdd(&dcnt[slot], valid ? 1u << sh8 : 0u);  // unconditional: no exec-mask branch
            wsync();
            const bool maybe_dup = valid && ((dcnt[slot] >> sh8) & 0xffu) > 1;
            const uint64_t dm0 = __ballot(maybe_dup);
            uint64_t dm = dm0;
            uint32_t c = tab[h];  // invalid lanes hash position 0: any entry, unused
            while (dm) {
                const uint32_t i = __builtin_ctzll(dm);
                dm &= dm - 1;
                const uint32_t hi = lane_val(h, i), pi = lane_val(pos, i);
                if (valid && lane > i && hi == h) c = pi;   // lanes visited in increasing i: last wins
            }
            atomicSub(&dcnt[slot], valid ? 1u << sh8 : 0u);
            wsync();
            const bool eq = lds_ld32(in, c) == u;
            const bool m = valid && eq;
            const uint64_t ev = __ballot(!valid || m);
            const uint32_t js = ev ? (uint32_t)__builtin_ctzll(ev) : 64u;
            // table updates: iterations before the event, plus the event itself when it is a match
            const bool upd = valid && (lane < js || (lane == js && m));
#if BHG_SE_U16
            // of the updating lanes with one bucket only the last one stores (plain u16 store)
            bool last = upd;
            dm = dm0 & __ballot(upd);
            while (dm) {
                const uint32_t i = __builtin_ctzll(dm);
                dm &= dm - 1;
                if (lane_val(h, i) == h && i > lane) last = false;
            }
            if (last) tab[h] = (se_tab_t)pos;
#else
            if (upd) atomicMax(&tab[h], pos);
#endif
            wsync();
            if (js < 64) {
                const bool is_match = lane_val((uint32_t)m, js) != 0;
                if (!is_match) { remainder = true; break; }
                s = lane_val(pos, js);
                cand = lane_val(c, js);
                break;
            }
        }
#ifdef BHG_SE_PROF
        SE_T(t_scan1);
        acc[0] += t_scan1 - t_scan0;
        acc[3] += 1;
#endif
        if (remainder) break;
        se_emit_literal(o, in + nextEmit, nullptr, s - nextEmit, lane);
#ifdef BHG_SE_PROF
        SE_T(t_lit1);
        acc[1] += t_lit1 - t_scan1;
#endif
        // ---- copies: emit, then check for an immediate next match ----
        // encode_other.go's inner loop with two LDS round trips per copy: the table
        // read for currHash (its hash input comes from the lanes' registers), then one
        // compare of in[cand + t] with in[s + t] for t < 64 that both verifies the
        // 4-byte match and extends it (Go's extension starts at s + 4 after a verified
        // 4-byte match: the same first mismatch).
        bool to_rem = false;
        uint32_t f;  // first mismatch of in[cand + t] vs in[s + t] (t < 64 per round)
        uint32_t bt; // this lane's in[r0 + lane .. + 4) of the round that found f
        {
            const uint32_t t = lane;
            const uint32_t bw = lds_ld32(in, s + t), a = in[cand + t], b = bw & 0xffu;  // past len: forced mismatch
            bt = bw;
            const uint64_t mm = __ballot(s + t >= len || a != b);
            f = mm ? (uint32_t)__builtin_ctzll(mm) : 64u;
        }
        for (;;) {
            const uint32_t base = s;
            uint32_t fb = f;  // mismatch relative to the round's start
            uint32_t r0 = s;  // start of the round that found fb
            while (fb == 64u) {  // all 64 equal: next round
                r0 += 64;
                const uint32_t t = lane;
                const uint32_t bw = lds_ld32(in, r0 + t), a = in[cand + (r0 - base) + t], b = bw & 0xffu;
                bt = bw;
                const uint64_t mm = __ballot(r0 + t >= len || a != b);
                fb = mm ? (uint32_t)__builtin_ctzll(mm) : 64u;
            }
            s = r0 + fb;
            se_emit_copy(o, base - cand, s - base, lane);
            nextEmit = s;
            if (s >= sLimit) { to_rem = true; break; }
            // x = in[s - 1 .. s + 7): lane t of the last round holds in[r0 + t .. r0 + t + 4)
            uint64_t x;
            const uint32_t k = s - 1 - r0;  // lane holding in[s - 1]
            if (s - 1 >= r0 && k + 4 < 64u) {
                x = (uint64_t)lane_val(bt, k) | ((uint64_t)lane_val(bt, k + 4) << 32);
            } else {
                x = (uint64_t)lds_ld32(in, s - 1) | ((uint64_t)lds_ld32(in, s + 3) << 32);
            }
            const uint32_t prevHash = se_hash((uint32_t)x, shift) & tmask;
            const uint32_t currHash = se_hash((uint32_t)(x >> 8), shift) & tmask;
            const uint32_t tc = tab[currHash];  // read before the two stores (program order); prevHash == currHash gives s - 1
            wsync();
            if (lane == 0) {
                tab[prevHash] = (se_tab_t)(s - 1);
                tab[currHash] = (se_tab_t)s;
            }
            const uint32_t c = uni(prevHash == currHash ? s - 1 : tc);
            wsync();
            // verify in[c .. c + 4) == in[s .. s + 4) and extend in the same compare
            {
                const uint32_t t = lane;
                const uint32_t bw = lds_ld32(in, s + t), a = in[c + t], b = bw & 0xffu;
                bt = bw;
                const uint64_t mm = __ballot(s + t >= len || a != b);
                f = mm ? (uint32_t)__builtin_ctzll(mm) : 64u;
            }
            if (f < 4u) {
                s += 1;
                break;
            }
            cand = c;
        }
#ifdef BHG_SE_PROF
        SE_T(t_cp1);
        acc[2] += t_cp1 - t_lit1;
#endif
        if (to_rem) break;
    }
    if (nextEmit < len) se_emit_literal(o, in + nextEmit, nullptr, len - nextEmit, lane);
}

// encodeBlock, lane 0 only, table of u16 in global scratch (blocks > SE_CAP)
__device__ void se_block_serial(Out &o, const uint8_t *src, uint32_t len, uint16_t *table) {
    uint32_t shift = 24;
    for (uint32_t ts = 256; ts < 16384 && ts < len; ts *= 2) shift--;
    for (uint32_t i = 0; i < 16384; i++) table[i] = 0;
    auto ld32 = [&](uint32_t i) {
        return (uint32_t)src[i] | ((uint32_t)src[i + 1] << 8) | ((uint32_t)src[i + 2] << 16) | ((uint32_t)src[i + 3] << 24);
    };
    const int sLimit = (int)len - SE_MARGIN;
    int nextEmit = 0, s = 1;
    uint32_t nextHash = se_hash(ld32(1), shift);
    for (;;) {
        int skip = 32, nextS = s, candidate = 0;
        for (;;) {
            s = nextS;
            const int b = skip >> 5;
            nextS = s + b;
            skip += b;
            if (nextS > sLimit) goto rem;
            candidate = table[nextHash & 16383];
            table[nextHash & 16383] = (uint16_t)s;
            nextHash = se_hash(ld32(nextS), shift);
            if (ld32(s) == ld32(candidate)) break;
        }
        se_emit_literal(o, nullptr, src + nextEmit, s - nextEmit, 0, 1);
        for (;;) {
            const int base = s;
            s += 4;
            for (int i = candidate + 4; s < (int)len && src[i] == src[s]; i++, s++) {}
            se_emit_copy(o, base - candidate, s - base, 0);
            nextEmit = s;
            if (s >= sLimit) goto rem;
            const uint64_t x = (uint64_t)ld32(s - 1) | ((uint64_t)ld32(s + 3) << 32);
            table[se_hash((uint32_t)x, shift) & 16383] = (uint16_t)(s - 1);
            const uint32_t ch = se_hash((uint32_t)(x >> 8), shift) & 16383;
            candidate = table[ch];
            table[ch] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != ld32(candidate)) {
                nextHash = se_hash((uint32_t)(x >> 16), shift);
                s++;
                break;
            }
        }
    }
rem:
    if (nextEmit < (int)len) se_emit_literal(o, nullptr, src + nextEmit, len - nextEmit, 0, 1);
}

// one wave per value: val bytes vals[val_off[i] .. val_off[i+1]) -> scratch[soff[i] ..), clen[i]
__global__ __launch_bounds__(64) void k_snappy_enc(const uint8_t *__restrict__ vals, const uint64_t *__restrict__ val_off,
                                                   uint32_t n, uint8_t *__restrict__ scratch, uint64_t scap,
                                                   const uint64_t *__restrict__ soff, uint64_t *__restrict__ clen,
                                                   uint16_t *__restrict__ gtables) {
    __shared__ __attribute__((aligned(16))) uint8_t in[SE_CAP + 16];
    __shared__ __attribute__((aligned(16))) se_tab_t tab[SE_TAB];
    __shared__ uint32_t dcnt[BHG_SE_DCNT];
    const uint32_t lane = threadIdx.x;
    for (uint32_t j = lane; j < BHG_SE_DCNT; j += 64) dcnt[j] = 0;
    LaneSkip F;
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
        F.f[j] = kSkip.f[64 * j + lane];
        F.f1[j] = kSkip.f[64 * j + lane + 1];
    }
    uint16_t *gt = gtables + (size_t)blockIdx.x * 16384;
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#ifdef BHG_SE_PROF
    const uint64_t t_k0 = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t v0 = val_off[i], vlen = val_off[i + 1] - v0;
        if (soff[i + 1] > scap) {  // val_off inconsistent with the vals_len the caller passed
            if (lane == 0) clen[i] = ~0ull;
            continue;
        }
        const uint8_t *src = vals + v0;
        Out o;
        o.g = scratch + soff[i];
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
            } else if (blen <= SE_CAP) {
#if BHG_SE_STAGE16
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
#else
                for (uint32_t t = lane; t < blen; t += 64) in[t] = bs[t];
#endif
                for (uint32_t t = blen + lane; t < blen + 16; t += 64) in[t] = 0;
                uint32_t ts = 256;
                while (ts < 16384 && ts < blen) ts *= 2;
                for (uint32_t t = lane; t < ts; t += 64) tab[t] = 0;
                wsync();
                se_block_lds(o, in, blen, tab, dcnt, lane, F, acc);
            } else {
                uint32_t d = o.d;
                if (lane == 0) {
                    Out ol = o;
                    se_block_serial(ol, bs, blen, gt);
                    d = ol.d;
                }
                o.d = uni(d);
            }
        }
        if (lane == 0) clen[i] = o.d;
        acc[4] += 1;
    }
#ifdef BHG_SE_PROF
    acc[5] = __builtin_amdgcn_s_memtime() - t_k0;
    if (lane == 0)
        for (int q = 0; q < 6; q++) atomicAdd((unsigned long long *)&se_prof[q], (unsigned long long)acc[q]);
    if (blockIdx.x == 0 && lane == 0)
        printf("se_prof wave0: scan %llu lit %llu copy %llu phases %llu values %llu total %llu\n",
               (unsigned long long)acc[0], (unsigned long long)acc[1], (unsigned long long)acc[2],
               (unsigned long long)acc[3], (unsigned long long)acc[4], (unsigned long long)acc[5]);
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

// one wave per resident workgroup slot (LDS: 13 KiB per wave with the u16 table, 21 KiB
// with u32 -- 11 / 7 per CU on MI355X): a grid past what is resident would start its extra
// workgroups only when the first ones finish
uint32_t snappy_enc_grid(const Launch &L, uint32_t n) {
    static const uint32_t per_cu = resident_per_cu((const void *)k_snappy_enc, 64, BHG_SE_WAVES);
    uint32_t g = (uint32_t)L.num_cus * (uint32_t)per_cu;
    if (g > n) g = n;
    return g ? g : 1;
}

hipError_t launch_snappy_enc(const Launch &L, const uint8_t *vals, const uint64_t *val_off, uint32_t n,
                             uint8_t *scratch, uint64_t scap, const uint64_t *soff, uint64_t *clen,
                             uint16_t *gtables) {
    hipLaunchKernelGGL(k_snappy_enc, dim3(snappy_enc_grid(L, n)), dim3(64), 0, L.stream, vals, val_off, n, scratch,
                       scap, soff, clen, gtables);
    return hipGetLastError();
}

}  // namespace bhg
