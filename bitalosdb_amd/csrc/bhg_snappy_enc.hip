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
#define BHG_SE_U16 0
#endif
#ifndef BHG_SE_STAGE16
#define BHG_SE_STAGE16 1  // measured: C4 30.7 vs 30.0 GiB/s (u16 table: 28.1 at 7 waves, 26.5 at 12)
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

__device__ __forceinline__ uint32_t lds_ld32(const uint8_t *b, uint32_t i) {
    return (uint32_t)b[i] | ((uint32_t)b[i + 1] << 8) | ((uint32_t)b[i + 2] << 16) | ((uint32_t)b[i + 3] << 24);
}

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
__device__ void se_block_lds(Out &o, const uint8_t *in, uint32_t len, se_tab_t *tab, uint32_t *dcnt, uint32_t lane) {
    uint32_t shift = 24;
    for (uint32_t ts = 256; ts < 16384 && ts < len; ts *= 2) shift--;
    const uint32_t tmask = 16383;
    const uint32_t sLimit = len - SE_MARGIN;
    uint32_t nextEmit = 0, s = 1;
    for (;;) {
        // ---- scan phase: iterations k = 0,1,... at positions s + F[k] ----
        uint32_t cand = 0;
        bool remainder = false;
        for (uint32_t kb = 0;; kb += 64) {
            const uint32_t k = kb + lane;
            const uint32_t fk = k < 1024 ? kSkip.f[k] : 0x7fffffffu;
            const uint32_t fk1 = k < 1024 ? kSkip.f[k + 1] : 0x7fffffffu;
            const uint64_t pos64 = (uint64_t)s + fk, nxt64 = (uint64_t)s + fk1;
            const bool valid = nxt64 <= sLimit;
            const uint32_t pos = valid ? (uint32_t)pos64 : 0u;
            const uint32_t u = lds_ld32(in, pos);
            const uint32_t h = se_hash(u, shift) & tmask;
            // bucket duplicates inside the batch (latest earlier lane wins)
            const uint32_t slot = h & 255;
            if (valid) atomicAdd(&dcnt[slot], 1u);
            wsync();
            const bool maybe_dup = valid && dcnt[slot] > 1;
            const uint64_t dm0 = __ballot(maybe_dup);
            uint64_t dm = dm0;
            uint32_t c = valid ? tab[h] : 0u;
            while (dm) {
                const uint32_t i = __builtin_ctzll(dm);
                dm &= dm - 1;
                const uint32_t hi = __shfl(h, i, 64), pi = __shfl(pos, i, 64);
                if (valid && lane > i && hi == h) c = pi;   // lanes visited in increasing i: last wins
            }
            if (valid) atomicSub(&dcnt[slot], 1u);
            wsync();
            const bool m = valid && lds_ld32(in, c) == u;
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
                if (__shfl(h, i, 64) == h && i > lane) last = false;
            }
            if (last) tab[h] = (se_tab_t)pos;
#else
            if (upd) atomicMax(&tab[h], pos);
#endif
            wsync();
            if (js < 64) {
                const bool is_match = __shfl((int)m, js, 64) != 0;
                if (!is_match) { remainder = true; break; }
                s = uni(__shfl(pos, js, 64));
                cand = uni(__shfl(c, js, 64));
                break;
            }
        }
        if (remainder) break;
        se_emit_literal(o, in + nextEmit, nullptr, s - nextEmit, lane);
        // ---- copies: emit, then check for an immediate next match ----
        bool to_rem = false;
        for (;;) {
            const uint32_t base = s;
            s += 4;
            // extend: first t with s+t == len or in[cand+4+t] != in[s+t]
            uint32_t i0 = cand + 4;
            for (;;) {
                const uint32_t t = lane;
                const bool inr = s + t < len;
                bool neq = true;
                if (inr) neq = in[i0 + t] != in[s + t];
                const uint64_t mm = __ballot(neq);
                if (mm) { const uint32_t f = (uint32_t)__builtin_ctzll(mm); s += f; break; }
                s += 64;
                i0 += 64;
            }
            se_emit_copy(o, base - cand, s - base, lane);
            nextEmit = s;
            if (s >= sLimit) { to_rem = true; break; }
            const uint32_t x0 = lds_ld32(in, s - 1), x4 = lds_ld32(in, s + 3);
            const uint64_t x = (uint64_t)x0 | ((uint64_t)x4 << 32);
            const uint32_t prevHash = se_hash((uint32_t)x, shift) & tmask;
#if BHG_SE_U16
            if (lane == 0) tab[prevHash] = (se_tab_t)(s - 1);
#else
            if (lane == 0) atomicMax(&tab[prevHash], s - 1);
#endif
            wsync();
            const uint32_t currHash = se_hash((uint32_t)(x >> 8), shift) & tmask;
            cand = uni(tab[currHash]);
            wsync();
#if BHG_SE_U16
            if (lane == 0) tab[currHash] = (se_tab_t)s;
#else
            if (lane == 0) atomicMax(&tab[currHash], s);
#endif
            wsync();
            if ((uint32_t)(x >> 8) != lds_ld32(in, cand)) {
                s += 1;
                break;
            }
        }
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
    __shared__ uint32_t dcnt[256];
    const uint32_t lane = threadIdx.x;
    for (uint32_t j = lane; j < 256; j += 64) dcnt[j] = 0;
    uint16_t *gt = gtables + (size_t)blockIdx.x * 16384;
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
                se_block_lds(o, in, blen, tab, dcnt, lane);
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
    }
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

uint32_t snappy_enc_grid(const Launch &L, uint32_t n) {
    uint32_t g = (uint32_t)L.num_cus * BHG_SE_WAVES;  // LDS: 21 KiB per wave (u32 table), 13 KiB (u16)
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
