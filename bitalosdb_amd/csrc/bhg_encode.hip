// bhg_encode.hip -- batched BithashWriter.Add for gfx950.
//
// Pipeline (one launch sequence per batch, all on the caller's stream):
//   k_enc_sizes   lane/record: key/value size checks (writer.go:258-265) and
//                 record length L = 12 + (|ukey|+8) + |value'| (block2.go:73-105)
//   scan          exclusive prefix of L -> record positions (bhg_scan.hip)
//   k_enc_split   one workgroup: table split points -- after each successful
//                 add, meta.Size >= TableMaxSize starts the next table
//                 (bithash_writer.go:38,47-67); a 1024-ary search per table
//   k_enc_pack    wave per tile of 64 records: header | ukey | trailer |
//                 value into the output stream, FNV-1 of the user key
//                 (writer.go:246) and the masked CRC-32C of each record
//                 computed from the registers the bytes are stored from (the
//                 packed output is not read back)
//   k_enc_meta    lane per record: handle / table / status outputs
// value' is the raw value (NoCompressor) or its golang/snappy encoding
// (bhg_snappy_enc.hip) staged in ctx scratch.
#include "bhg_crc_tables.h"
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

#define BHG_MAX_KEY_SIZE (33u << 10)          // writer.go:42
#define BHG_MAX_VALUE_SIZE (256u << 20)       // writer.go:43

struct EncArgs {
    const uint8_t *keys;
    const uint64_t *key_off;
    const uint64_t *trailers;
    const uint8_t *vals;          // value' bytes base (raw values or snappy scratch)
    uint64_t vals_end;            // end of the buffer vals points into (0: unknown; loads then stay in each value)
    const uint64_t *vpos;         // value' start offset per record (into vals)
    const uint64_t *vlen;         // value' length per record
    uint32_t n;
    const uint32_t *file_nums;
    const uint32_t *rec_file_nums;  // AddIkey: header fileNum per record (nullable -> file_nums[table])
    const uint8_t *live;          // compaction liveness mask (nullable -> all live)
    const uint32_t *khash;        // AddIkey: given khash per record (nullable -> FNV-1 of the key)
    const uint32_t *key_len;      // nullable: key i = keys[key_off[i] .. + key_len[i]) (else key_off[i+1] ends it)
    const uint32_t *pre_status;   // nullable: non-OK -> the record is not added (repack's record checks)
    int single_table;             // AddIkey: one table, no split, dataMaxSize checked per record
    uint32_t max_tables;
    uint32_t init_size;
    uint64_t table_max;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *lens;               // scratch: L per record, then exclusive scan -> positions (n+1)
    const uint32_t *xtab;         // the context's CrcR8 shift tables (bhg_crc_tables.h build_xtab)
    uint32_t long_min;            // 0, or kLongRec: longer records are left to k_enc_lcopy + the long CRC pass
    const uint64_t *lbase;        // long mode: segment base per record (scanned k_enc_lcount), lbase[n] total
    uint64_t lcap;                // long mode: segment list capacity (records past it stay with k_enc_pack)
    bhg_encode_out o;
};

__device__ __forceinline__ uint32_t key_len_of(const EncArgs &a, uint32_t i) {
    return a.key_len != nullptr ? a.key_len[i] : (uint32_t)(a.key_off[i + 1] - a.key_off[i]);
}

#define BHG_DATA_MAX_SIZE (0xFFFFFFFFull - (256ull << 20))  // writer.go:45

// the add of record i (status OK after k_enc_sizes, position P, length L)
// lands in the output: out_cap for every batch, dataMaxSize (writer.go:266-269)
// for the single-table AddIkey batch (the split batch rejects table_max values
// that could reach it up front)
__device__ __forceinline__ uint32_t fit_status(const EncArgs &a, uint64_t P, uint32_t L) {
    if (P + L > a.out_cap) return BHG_ST_NO_SPACE;
    if (a.single_table && (uint64_t)a.init_size + P + L > BHG_DATA_MAX_SIZE) return BHG_ST_DATA_MAX_EXCEEDED;
    return BHG_ST_OK;
}

__global__ __launch_bounds__(256) void k_enc_sizes(EncArgs a) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
        const uint64_t klen = key_len_of(a, i);
        const uint64_t vl = a.vlen[i];
        uint32_t st = BHG_ST_OK;
        uint64_t L = 0;
        if (a.live != nullptr && a.live[i] == 0) st = BHG_ST_SKIPPED;           // bitree/bithash.go:225-228
        else if (a.pre_status != nullptr && a.pre_status[i] != BHG_ST_OK) st = a.pre_status[i];
        else if (klen + 8 > BHG_MAX_KEY_SIZE) st = BHG_ST_KEY_TOO_LARGE;
        else if (vl == ~0ull) st = BHG_ST_NO_SPACE;                              // snappy scratch overflow
        else if (vl > BHG_MAX_VALUE_SIZE) st = BHG_ST_VALUE_TOO_LARGE;
        else L = 12 + klen + 8 + vl;
        a.o.status[i] = st;
        a.lens[i] = L;
    }
}

// One workgroup of 1024 threads.  pos[0..n] = exclusive scan of L.
// Table t starts at record s with start size S; it ends at the first record
// e >= s with L_e > 0 and S + pos[e+1] - pos[s] >= table_max (the add that
// reaches the limit stays in the table; a new, possibly empty, table follows).
__device__ uint32_t first_geq(const uint64_t *pos, uint32_t lo, uint32_t hi, uint64_t T, uint32_t *s_best) {
    // first e in [lo, hi) with pos[e+1] >= T, or hi; every thread returns the same value
    while (lo < hi) {
        const uint32_t span = hi - lo;
        const uint32_t stepw = (span + 1023) / 1024;
        __syncthreads();
        if (threadIdx.x == 0) *s_best = hi;
        __syncthreads();
        const uint64_t e = (uint64_t)lo + (uint64_t)threadIdx.x * stepw;
        if (e < hi && pos[e + 1] >= T) atomicMin(s_best, (uint32_t)e);
        __syncthreads();
        const uint32_t b = *s_best;
        if (stepw == 1 || b == lo) return b;
        if (b == hi) {
            const uint32_t last = lo + ((span - 1) / stepw) * stepw;   // last (false) probe
            lo = last + 1;
        } else {
            lo = b - stepw + 1;                                          // probe b - stepw was false
            hi = b;
        }
    }
    return hi;
}

__global__ __launch_bounds__(1024) void k_enc_split(EncArgs a) {
    __shared__ uint32_t s_best;
    const uint64_t *pos = a.lens;
    const uint32_t n = a.n;
    uint32_t s = 0, t = 0, fail = 0;
    uint64_t S = a.init_size;
    if (threadIdx.x == 0) a.o.table_start[0] = 0;
    // BithashWriter.AddIkey never splits (bithash_writer.go:43-45)
    while (!a.single_table && s < n) {
        const uint64_t T = a.table_max > S ? pos[s] + (a.table_max - S) : pos[s];
        uint32_t e = first_geq(pos, s, n, T, &s_best);
        while (e < n && pos[e + 1] == pos[e]) e++;     // split check runs only after a successful add
        if (e >= n) break;
        if (t + 1 >= a.max_tables) { fail = 1; break; }
        t++;
        if (threadIdx.x == 0) a.o.table_start[t] = e + 1;
        s = e + 1;
        S = 0;
    }
    if (threadIdx.x == 0) {
        a.o.summary[0] = pos[n];
        a.o.summary[1] = fail ? 0 : t + 1;
        a.o.summary[2] = 0;
        a.o.summary[3] = fail;
    }
}

// table index of record i: last t with table_start[t] <= i
__device__ __forceinline__ uint32_t table_of(const uint32_t *ts, uint32_t nt, uint32_t i) {
    uint32_t lo = 0, hi = nt;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ts[mid] <= i) lo = mid; else hi = mid;
    }
    return lo;
}

#define ENC_WAVES 8
#define ENC_PACK_K 2  // 16-B value chunks per lane per record pass (2 KiB)
// LDS of the pack kernel: CrcR8 (32 KiB) + Z_16 .. Z_1024 (7 x 4 KiB) = 60 KiB, two workgroups per CU
constexpr uint32_t kPackZ = 7;
constexpr uint32_t kPackLds = CrcR8::kBytes + kPackZ * 4096;
// One WAVE per tile of 64 records (records are back to back in `out`).
//  phase A, lane = record: metadata, FNV-1 of the user key, then the record's prefix (header |
//    ukey | trailer, <= 56 B for ukeys <= 36 B) and the value bytes up to the next 4-aligned
//    output address qa, assembled byte by byte from registers (header, trailer) and dword
//    windows of the key and the value head, and written as dwords (the first one, shared with
//    the previous record, as bytes).  Per-byte work is spread over 64 records per instruction.
//    The lane also runs the record's CRC over these dwords: P = crc_0 of the prefix with crc.New's
//    ~0 start folded into the record's first 4 bytes (crc_~0(X) = crc_0(X ^ ~0 at bytes 0..3);
//    the bytes before the record in the first dword are 0, and leading zeros leave crc_0 at 0).
//  phase B, wave per record: the value from qa on in 16-B output chunks (4-aligned dwordx4
//    stores), each from a 20-B aligned source window and a byte funnel; two records per pass
//    with all loads issued before the first store.  Chunk c (0 .. nc-1) sits on lane c % 64;
//    each lane Horner-folds the crc_0 of its full chunks (stride 64 chunks: Z_1024), lane 63
//    starting from P (the prefix ends at qa: it is chunk -1), then
//        S = sum_lanes Z_{16 d}(acc),  d = (nc - 2 - lane) mod 64 (chunks after the lane's last)
//    (six conditional shifts, a wave xor-reduce), and the lane holding the last chunk (1..16
//    bytes) absorbs it into S: the record's CRC state.  CRC linearity over GF(2):
//    crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B).
// A record with a ukey > 36 B has its prefix (header | ukey | trailer | value bytes up to qa)
// written byte by byte by its lane (rare), P bytewise; its value still goes through phase B.
// (The wave-per-record version loaded the metadata record by record: ~6 dependent memory round
// trips per record, 1.42 ms per C4 batch; the dword version of this one 1.05 ms.  The CRC used to
// be a separate lane-per-record kernel that read the 1 GB of packed records back: 0.46 ms and
// 1.27 GB of a C4 step.)
__global__ __launch_bounds__(64 * ENC_WAVES) void k_enc_pack(EncArgs a) {
    const uint32_t ntab = (uint32_t)a.o.summary[1];
    if (ntab == 0) return;  // split failed (max_tables too small): every thread leaves
    __shared__ __attribute__((aligned(16))) uint32_t lds_all[kPackLds / 4];
    const uint32_t tb = lds_addr(lds_all), zb = tb + CrcR8::kBytes;
    CrcR8::fill(tb);
    for (uint32_t t = threadIdx.x; t < kPackZ * 1024; t += blockDim.x)
        lds_all[CrcR8::kBytes / 4 + t] = a.xtab[XZ16 * 1024 + t];
    __syncthreads();
    const CrcR8 crc(tb);
    const uint32_t Z1024 = zb + 4096 * (XZ1024 - XZ16);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nwaves = gridDim.x * ENC_WAVES;
    const uint32_t ntiles = (a.n + 63) / 64;
    const uint64_t dummy = (uint64_t)a.lens;  // a valid, 16-B aligned address for loads whose result is unused
    for (uint32_t tile = blockIdx.x * ENC_WAVES + (threadIdx.x >> 6); tile < ntiles; tile += nwaves) {
        // ---------------- phase A: lane = record
        const uint32_t r = tile * 64 + lane;
        const uint32_t rr = r < a.n ? r : a.n - 1;
        const uint32_t st = a.o.status[rr];
        const uint64_t P = a.lens[rr];
        const uint32_t L = (uint32_t)(a.lens[rr + 1] - P);
        const uint32_t kl = key_len_of(a, rr);
        const uint32_t vl = (uint32_t)a.vlen[rr];
        const uint64_t kp = (uint64_t)a.keys + a.key_off[rr];
        const uint64_t tr = a.trailers[rr];
        const uint64_t vp = (uint64_t)a.vals + a.vpos[rr];
        const uint32_t t = table_of(a.o.table_start, ntab, rr);
        const uint32_t fn = a.rec_file_nums != nullptr ? a.rec_file_nums[rr] : a.file_nums[t];
        const bool ok = r < a.n && st == BHG_ST_OK && fit_status(a, P, L) == BHG_ST_OK;
        const uint64_t dst = (uint64_t)a.out + P, dend = dst + L;
        const uint32_t pre = 20 + kl;
        const bool shortk = kl <= 36;
        // output [q0, qa): the dwords holding the prefix (qa: first 4-aligned address >= the value start)
        const uint64_t q0 = dst & ~3ull, vdst = dst + pre;
        const uint64_t qa = (vdst + 3) & ~3ull;
        const uint32_t sh = (uint32_t)(dst & 3);  // record offset of output byte q0 + x is x - sh
        // key window: 10 dwords from ka (ukey <= 36 B at any alignment); value head: 2 dwords from va
        uint32_t kw[10], vw[2];
        const uint64_t ka = kp & ~3ull, va = vp & ~3ull, kend = kp + kl, vend = vp + vl;
        const bool kload = r < a.n && shortk && (ok || a.khash == nullptr);
#pragma unroll
        for (int u = 0; u < 10; u++) kw[u] = gld<uint32_t>(kload && ka + 4 * u < kend ? ka + 4 * u : dummy);
#pragma unroll
        for (int u = 0; u < 2; u++) vw[u] = gld<uint32_t>(ok && shortk && va + 4 * u < vend ? va + 4 * u : dummy);
        const uint32_t kd = (uint32_t)(kp - ka);
        // FNV-1 of the user key (writer.go:246, every record) or the caller's khash (AddIkey, :249)
        if (r < a.n) {
            uint32_t fnv;
            if (a.khash != nullptr) {
                fnv = a.khash[r];
            } else if (shortk) {
                uint32_t hh = BHG_FNV_OFFSET;
#pragma unroll
                for (uint32_t u = 0; u < 9; u++) {
                    const uint32_t kwd = __builtin_amdgcn_alignbyte(kw[u + 1], kw[u], kd);
#pragma unroll
                    for (uint32_t b = 0; b < 4; b++) {
                        const uint32_t h2 = (hh * BHG_FNV_PRIME) ^ ((kwd >> (8 * b)) & 0xffu);
                        hh = 4 * u + b < kl ? h2 : hh;
                    }
                }
                fnv = hh;
            } else {
                fnv = fnv1_range(kp, kl, kp + kl);
            }
            a.o.fnv1[r] = fnv;
        }
        uint32_t pc = 0;  // CRC of the record bytes in [dst, min(qa, dend)), ~0 start folded in
        if (ok && shortk) {
            const uint32_t vd = (uint32_t)(vp - va);
            const uint32_t nq = (uint32_t)((qa - q0) >> 2);  // <= 16
            for (uint32_t u = 0; u < nq; u++) {
                uint32_t x = 0;
#pragma unroll
                for (uint32_t b = 0; b < 4; b++) {
                    const int32_t o = (int32_t)(4 * u + b) - (int32_t)sh;  // record offset
                    uint32_t by = 0;
                    if (o >= 0 && o < 12) {
                        const uint32_t hd = o < 4 ? kl + 8 : o < 8 ? vl : fn;
                        by = (hd >> (8 * ((uint32_t)o & 3))) & 0xffu;
                    } else if (o >= 12 && o < 12 + (int32_t)kl) {
                        const uint32_t y = kd + (uint32_t)(o - 12);
                        uint32_t wd = 0;
#pragma unroll
                        for (uint32_t z = 0; z < 10; z++) wd = (y >> 2) == z ? kw[z] : wd;
                        by = (wd >> (8 * (y & 3))) & 0xffu;
                    } else if (o >= 12 + (int32_t)kl && o < (int32_t)pre) {
                        by = (uint32_t)(tr >> (8 * (uint32_t)(o - 12 - (int32_t)kl))) & 0xffu;
                    } else if (o >= (int32_t)pre) {
                        const uint32_t y = vd + (uint32_t)(o - (int32_t)pre);  // < 8
                        by = ((y < 4 ? vw[0] : vw[1]) >> (8 * (y & 3))) & 0xffu;
                    }
                    x |= by << (8 * b);
                }
                const uint64_t q = q0 + 4ull * u;
                if (q >= dst && q + 4 <= dend) {
                    gst<uint32_t>(q, x);
                } else {  // the first dword (shared with the previous record) or a record ending here
#pragma unroll
                    for (uint32_t b = 0; b < 4; b++)
                        if (q + b >= dst && q + b < dend) gst<uint8_t>(q + b, (uint8_t)(x >> (8 * b)));
                }
                // record bytes 0..3 lie in dwords 0 and 1: u == 0 holds offsets 0 .. 3 - sh at bytes
                // sh..3, u == 1 offsets 4 - sh .. 3 at bytes 0 .. sh - 1
                const uint32_t init = u == 0 ? (0xffffffffu << (8 * sh)) : u == 1 ? ((1u << (8 * sh)) - 1u) : 0u;
                if (q + 4 <= dend) pc = crc.word(pc, x ^ init);
                else if (q < dend) pc = crc.partial(pc, x ^ init, (uint32_t)(dend - q));
            }
        } else if (ok) {  // ukey > 36 B: the prefix [dst, qa) byte by byte; phase B copies the value from qa
            const uint32_t np = (uint32_t)((qa < dend ? qa : dend) - dst);
            pc = 0xffffffffu;  // crc.New: bytewise from ~0 (the same state as the folded start)
            for (uint32_t o = 0; o < np; o++) {
                uint32_t by;
                if (o < 12) by = ((o < 4 ? kl + 8 : o < 8 ? vl : fn) >> (8 * (o & 3))) & 0xffu;
                else if (o < 12 + kl) by = gld<uint8_t>(kp + (o - 12));
                else if (o < pre) by = (uint32_t)(tr >> (8 * (o - 12 - kl))) & 0xffu;
                else by = gld<uint8_t>(vp + (o - pre));
                gst<uint8_t>(dst + o, (uint8_t)by);
                pc = crc.step(pc ^ by);
            }
        }
        if (ok && qa >= dend) a.o.crc[r] = crc_mask(~pc);  // the whole record was in the prefix dwords
        // ---------------- phase B: wave per record, the value from qa on
        // long mode: records whose segments k_enc_lemit listed are k_enc_lcopy's
        const bool listed = a.lbase != nullptr && a.lbase[rr + 1] > a.lbase[rr] && a.lbase[rr + 1] <= a.lcap;
        uint64_t todo = __ballot(ok && qa < dend && !listed);
        while (todo) {
            int jr[2];
            jr[0] = __builtin_ctzll(todo);
            todo &= todo - 1;
            jr[1] = todo ? __builtin_ctzll(todo) : -1;
            if (todo) todo &= todo - 1;
            uint64_t qb[2], de[2], sb[2], ve[2];
            uint32_t nc[2], acc[2], lw[2][4], rl[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int j = jr[h] < 0 ? jr[0] : jr[h];
                qb[h] = readlane_u64(qa, j);
                de[h] = readlane_u64(dend, j);
                // source address of output byte qb: value offset qb - vdst
                sb[h] = readlane_u64(vp, j) + (qb[h] - readlane_u64(vdst, j));
                ve[h] = readlane_u64(vend, j);
                nc[h] = jr[h] < 0 ? 0u : (uint32_t)((de[h] - qb[h] + 15) >> 4);
                const uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)pc, j);
                acc[h] = lane == 63 ? pj : 0u;  // the prefix is chunk -1: lane 63's first Horner term
                lw[h][0] = lw[h][1] = lw[h][2] = lw[h][3] = 0;
                rl[h] = 0;
            }
            const uint32_t ncmax = nc[0] > nc[1] ? nc[0] : nc[1];
            for (uint32_t cb = 0; cb < ncmax; cb += 64 * ENC_PACK_K) {
                // loads: 20-B source windows (dwordx4 + dword) of both records' chunks
                u32x4 wx[2][ENC_PACK_K];
                uint32_t w4[2][ENC_PACK_K];
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int k = 0; k < ENC_PACK_K; k++) {
                        const uint32_t c = cb + lane + 64 * k;
                        const uint64_t s = sb[h] + 16ull * c, sa = s & ~3ull;
                        // a dword is loaded only if it holds a byte of the value, or lies inside the
                        // buffer the value is in (vals_end)
                        const uint64_t lim = a.vals_end > ve[h] ? a.vals_end : ((ve[h] + 3) & ~3ull);
                        const bool use = c < nc[h];
                        wx[h][k] = gld<u32x4_a4>(use && sa + 16 <= lim ? sa : dummy);
                        w4[h][k] = gld<uint32_t>(use && sa + 20 <= lim ? sa + 16 : dummy);
                    }
#pragma unroll
                for (int h = 0; h < 2; h++)
#pragma unroll
                    for (int k = 0; k < ENC_PACK_K; k++) {
                        const uint32_t c = cb + lane + 64 * k;
                        if (c >= nc[h]) continue;
                        const uint64_t s = sb[h] + 16ull * c, sa = s & ~3ull;
                        const uint64_t lim = a.vals_end > ve[h] ? a.vals_end : ((ve[h] + 3) & ~3ull);
                        uint32_t d[5] = {wx[h][k].x, wx[h][k].y, wx[h][k].z, wx[h][k].w, w4[h][k]};
                        if (sa + 20 > lim) {  // the value's last bytes at the end of its buffer: dword by dword
#pragma unroll
                            for (int z = 0; z < 5; z++) d[z] = sa + 4 * z < lim ? gld<uint32_t>(sa + 4 * z) : 0u;
                        }
                        const uint32_t f = (uint32_t)(s & 3);
                        const u32x4 y = {__builtin_amdgcn_alignbyte(d[1], d[0], f), __builtin_amdgcn_alignbyte(d[2], d[1], f),
                                         __builtin_amdgcn_alignbyte(d[3], d[2], f), __builtin_amdgcn_alignbyte(d[4], d[3], f)};
                        const uint64_t q = qb[h] + 16ull * c;
                        if (q + 16 <= de[h]) {
                            gst<u32x4_a4>(q, y);
                        } else {  // the record's last chunk: whole dwords, then the bytes of a partial one
                            const uint32_t yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                            for (int z = 0; z < 4; z++) {
                                const uint64_t qz = q + 4 * z;
                                if (qz + 4 <= de[h]) {
                                    gst<uint32_t>(qz, yy[z]);
                                } else {
#pragma unroll
                                    for (int b = 0; b < 4; b++)
                                        if (qz + b < de[h]) gst<uint8_t>(qz + b, (uint8_t)(yy[z] >> (8 * b)));
                                }
                            }
                        }
                        if (c + 1 < nc[h]) {  // a full chunk: into this lane's Horner chain
                            const uint32_t v = crc.word(crc.word(crc.word(crc.word(0u, y.x), y.y), y.z), y.w);
                            acc[h] = zshift(Z1024, acc[h]) ^ v;
                        } else {              // the last chunk (1..16 bytes): absorbed after the lane sum
                            lw[h][0] = y.x; lw[h][1] = y.y; lw[h][2] = y.z; lw[h][3] = y.w;
                            rl[h] = (uint32_t)(de[h] - q);
                        }
                    }
            }
            // S = sum over lanes of Z_{16 d}(acc), d = chunks after the lane's last full chunk
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (jr[h] < 0) continue;
                const uint32_t d = (uint32_t)((int32_t)nc[h] - 2 - (int32_t)lane) & 63u;
                uint32_t v = acc[h];
#pragma unroll
                for (uint32_t z = 0; z < 6; z++) {
                    const uint32_t sv = zshift(zb + 4096 * z, v);  // Z_{16 << z}
                    v = (d >> z) & 1u ? sv : v;
                }
#pragma unroll
                for (int m = 1; m < 64; m <<= 1) v ^= __shfl_xor(v, m, 64);
                if (lane == ((nc[h] - 1) & 63u)) {
                    const uint32_t nw = rl[h] >> 2, nb = rl[h] & 3;
#pragma unroll
                    for (uint32_t w = 0; w < 4; w++)
                        if (w < nw) v = crc.word(v, lw[h][w]);
                    if (nb) {
                        uint32_t x = lw[h][0];
#pragma unroll
                        for (uint32_t w = 1; w < 4; w++) x = nw == w ? lw[h][w] : x;
                        v = crc.partial(v, x, nb);
                    }
                    a.o.crc[tile * 64 + (uint32_t)jr[h]] = crc_mask(~v);
                }
            }
        }
    }
}

// lane per record: the outputs that need no record bytes (the CRC and FNV-1 come from k_enc_pack):
// final status, position, table-relative BlockHandle, table index, failed-add count
__global__ __launch_bounds__(256) void k_enc_meta(EncArgs a) {
    const uint32_t ntab = (uint32_t)a.o.summary[1];
    uint32_t failed = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
        const uint32_t t = ntab ? table_of(a.o.table_start, ntab, i) : 0;
        a.o.table[i] = t;
        const uint64_t P = a.lens[i];
        const uint32_t L = (uint32_t)(a.lens[i + 1] - P);
        uint32_t st = a.o.status[i];
        if (st == BHG_ST_OK) st = ntab != 0 ? fit_status(a, P, L) : BHG_ST_NO_SPACE;  // ntab 0: out of file_nums
        if (st != BHG_ST_OK) {
            if (st != a.o.status[i]) a.o.status[i] = st;
            failed += st != BHG_ST_SKIPPED;
            a.o.pos[i] = ~0ull;
            a.o.bh_off[i] = 0;
            a.o.bh_len[i] = 0;
            a.o.crc[i] = 0;
            if (a.o.rec) a.o.rec[i] = bhg_handle{~0ull, 0, 0};
            if (ntab == 0 && a.khash == nullptr) {  // k_enc_pack did not run: FNV-1 here
                const uint64_t kp = (uint64_t)a.keys + a.key_off[i];
                const uint32_t klen = key_len_of(a, i);
                a.o.fnv1[i] = fnv1_range(kp, klen, kp + klen);
            } else if (ntab == 0) {
                a.o.fnv1[i] = a.khash[i];
            }
            continue;
        }
        a.o.pos[i] = P;
        const uint64_t P0 = a.lens[a.o.table_start[t]];
        a.o.bh_off[i] = (uint32_t)((t == 0 ? (uint64_t)a.init_size : 0ull) + (P - P0));
        a.o.bh_len[i] = L;
        if (a.o.rec) a.o.rec[i] = bhg_handle{P, L, 0};
    }
    // summary[2]: failed adds (every status but OK / SKIPPED); one vector atomic per wave
    for (int d = 32; d >= 1; d >>= 1) failed += __shfl_xor(failed, d);
    if ((threadIdx.x & 63) == 0 && failed) atomicAdd(reinterpret_cast<unsigned long long *>(a.o.summary + 2),
                                                     (unsigned long long)failed);
}

// table_size[t]: the writer's currentOffset after the batch -- end of the
// table's last successful add (init_size / 0 for a table with none)
__global__ __launch_bounds__(256) void k_enc_tsize(EncArgs a) {
    const uint32_t ntab = (uint32_t)a.o.summary[1];
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < a.max_tables; t += gridDim.x * blockDim.x) {
        uint64_t size = t == 0 ? a.init_size : 0;
        if (t < ntab) {
            const uint32_t s = a.o.table_start[t], e = t + 1 < ntab ? a.o.table_start[t + 1] : a.n;
            for (uint32_t i = e; i > s; i--) {
                if (a.o.status[i - 1] == BHG_ST_OK) {
                    size = (uint64_t)a.o.bh_off[i - 1] + a.o.bh_len[i - 1];
                    break;
                }
            }
        } else {
            size = 0;
        }
        a.o.table_size[t] = size;
    }
}

// value' = raw values: vpos = val_off, vlen = val_off[i+1]-val_off[i]
__global__ __launch_bounds__(256) void k_enc_rawvals(const uint64_t *val_off, uint32_t n, uint64_t *vlen) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        vlen[i] = val_off[i + 1] - val_off[i];
}

// Compaction re-pack from stored records (bhg_repack_batch): the AddIkey
// inputs of each record read straight from its bytes -- what TableIterator
// hands compactBithashFiles (table.go:358-395: ikey, stored value, header
// fileNum).  A handle that is out of range or not a whole record
// (12 + ikeySize + valueSize != length, ikeySize == 0) -> RECORD_NIL.  A
// record with ikeySize 1..7 is what readKV returns it as (block2.go:38-55):
// an empty UserKey and trailer InternalKeyKindInvalid (255), so AddIkey
// re-writes it with ikeySize 8 -- the liveness filter decides, as in
// compactBithashFiles.
__global__ __launch_bounds__(256) void k_repack_prep(const uint8_t *src, uint64_t src_len, const bhg_handle *h,
                                                     uint32_t n, uint64_t *key_off, uint32_t *key_len,
                                                     uint64_t *trailers, uint64_t *vpos, uint64_t *vlen,
                                                     uint32_t *fns, uint32_t *pre) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const bhg_handle r = h[i];
        uint32_t st = BHG_ST_RECORD_NIL, k = 8, v = 0, fn = 0;
        uint64_t tr = 0;
        uint32_t kl = 0;
        if (r.length >= 13 && r.offset <= src_len && (uint64_t)r.length <= src_len - r.offset) {
            const uint64_t p = base + r.offset;
            k = ldu32(p, end);
            v = ldu32(p + 4, end);
            fn = ldu32(p + 8, end);
            // readRecord's nil rules (block2.go:57-66): ikeySize == 0 or valueSize == 0 is no record
            // (TableIterator.findEntry stops at valueSize <= 0, table.go:373)
            if (k >= 1 && v >= 1 && 12ull + k + v == r.length) {
                st = BHG_ST_OK;
                kl = k >= 8 ? k - 8 : 0u;
                tr = k >= 8 ? ldu64(p + 12 + k - 8, end) : 255ull;  // InternalKeyKindInvalid
            } else {
                k = 8;
                v = 0;
            }
        }
        key_off[i] = r.offset + 12;
        key_len[i] = kl;
        trailers[i] = tr;
        vpos[i] = r.offset + 12 + k;
        vlen[i] = v;
        fns[i] = fn;
        pre[i] = st;
    }
}

hipError_t launch_repack_prep(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              uint64_t *key_off, uint32_t *key_len, uint64_t *trailers, uint64_t *vpos,
                              uint64_t *vlen, uint32_t *fns, uint32_t *pre) {
    hipLaunchKernelGGL(k_repack_prep, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, src, src_len, h, n, key_off,
                       key_len, trailers, vpos, vlen, fns, pre);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Long records (a batch of long values: bhg_encode_batch picks this by long_batch, as the decode
// does).  k_enc_pack gives a record one wave, so a 1-4 MiB value was one wave's 16-B chunks plus a
// Horner CRC while the rest of the GPU idled: k_enc_pack took 4.45 of the 25.3-ms bigval encode step
// (bench.py --config bigval, profiles/r6/final/bigval_kernel_stats.csv).  Here k_enc_pack writes such
// a record's prefix dwords only (phase A), then
//   k_enc_lcount  lane per record: the 16-KiB output segments of its value part [qa, dend)
//   (scan)        segment base per record
//   k_enc_lemit   lane per record: its list entries {record, segment}
//   k_enc_lcopy   wave per segment (persistent grid): the value bytes in 16-B output chunks from
//                 20-B source windows, as phase B of k_enc_pack
// and, once k_enc_meta has written each record's handle {P, L}, the decode's long-record CRC pass
// (bhg_longcrc.hip) computes the masked CRC-32C of every record longer than kLongRec from the packed
// output, the whole chip at once (crc(A || B) = Z_|B|(crc(A)) ^ crc_0(B) over 8-KiB pieces).
constexpr uint32_t kEncSeg = 16384;  // output bytes per copy work item (16 chunks per lane)

struct EncRec {  // a record's placement, as k_enc_pack computes it
    uint64_t dst, dend, vdst, qa, vp, vend;
    bool ok;
};
__device__ __forceinline__ EncRec enc_rec(const EncArgs &a, uint32_t i, uint32_t ntab) {
    EncRec r;
    const uint64_t P = a.lens[i];
    const uint32_t L = (uint32_t)(a.lens[i + 1] - P);
    r.ok = ntab != 0 && a.o.status[i] == BHG_ST_OK && fit_status(a, P, L) == BHG_ST_OK && L > a.long_min;
    const uint32_t kl = key_len_of(a, i);
    r.dst = (uint64_t)a.out + P;
    r.dend = r.dst + L;
    r.vdst = r.dst + 20 + kl;
    r.qa = (r.vdst + 3) & ~3ull;
    r.vp = (uint64_t)a.vals + a.vpos[i];
    r.vend = r.vp + (uint32_t)a.vlen[i];
    return r;
}

__global__ __launch_bounds__(256) void k_enc_lcount(EncArgs a, uint64_t *__restrict__ cnt) {
    const uint32_t ntab = (uint32_t)a.o.summary[1];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += gridDim.x * blockDim.x) {
        const EncRec r = enc_rec(a, i, ntab);
        cnt[i] = r.ok && r.qa < r.dend ? (r.dend - r.qa + kEncSeg - 1) / kEncSeg : 0ull;
    }
}

// a record whose segments would pass the list's capacity is not listed (k_enc_pack keeps it: its
// phase B copies it); later records then are not either (base is non-decreasing)
__global__ __launch_bounds__(256) void k_enc_lemit(const uint64_t *__restrict__ base, uint32_t n, uint64_t cap,
                                                   uint2 *__restrict__ ent) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t b0 = base[i], b1 = base[i + 1];
        if (b1 > cap) {  // the list ends inside this record: its slots up to cap are marked empty
            for (uint64_t k = b0; k < cap; k++) ent[k] = make_uint2(~0u, 0u);
            continue;
        }
        for (uint64_t k = b0; k < b1; k++) ent[k] = make_uint2(i, (uint32_t)(k - b0));
    }
}

#define ENC_LCOPY_WAVES 4
__global__ __launch_bounds__(64 * ENC_LCOPY_WAVES) void k_enc_lcopy(EncArgs a, const uint64_t *__restrict__ base,
                                                                  const uint2 *__restrict__ ent) {
    const uint32_t ntab = (uint32_t)a.o.summary[1];
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t total = base[a.n] < a.lcap ? base[a.n] : a.lcap;
    const uint64_t nw = (uint64_t)gridDim.x * ENC_LCOPY_WAVES, w0 = (uint64_t)blockIdx.x * ENC_LCOPY_WAVES + (threadIdx.x >> 6);
    const uint64_t dummy = (uint64_t)a.lens;  // a valid, 16-B aligned address for loads whose result is unused
    constexpr uint32_t K = kEncSeg / 1024;   // chunks per lane per segment
    for (uint64_t g = w0; g < total; g += nw) {
        const uint2 e = ent[g];
        if (e.x == ~0u) continue;  // an empty slot (the list ended inside a record)
        const EncRec r = enc_rec(a, e.x, ntab);
        const uint64_t qs = r.qa + (uint64_t)kEncSeg * e.y;
        const uint64_t qe = qs + kEncSeg < r.dend ? qs + kEncSeg : r.dend;
        const uint32_t nc = (uint32_t)((qe - qs + 15) >> 4);
        const uint64_t sb = r.vp + (qs - r.vdst);  // source of output byte qs
        // a dword is loaded only if it holds a byte of the value, or lies inside the buffer the
        // value is in (vals_end)
        const uint64_t lim = a.vals_end > r.vend ? a.vals_end : ((r.vend + 3) & ~3ull);
#pragma unroll
        for (uint32_t k0 = 0; k0 < K; k0 += 4) {
            u32x4 wx[4];
            uint32_t w4[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t c = lane + 64 * (k0 + k);
                const uint64_t sa = (sb + 16ull * c) & ~3ull;
                const bool use = c < nc;
                wx[k] = gld<u32x4_a4>(use && sa + 16 <= lim ? sa : dummy);
                w4[k] = gld<uint32_t>(use && sa + 20 <= lim ? sa + 16 : dummy);
            }
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t c = lane + 64 * (k0 + k);
                if (c >= nc) continue;
                const uint64_t s = sb + 16ull * c, sa = s & ~3ull;
                uint32_t d[5] = {wx[k].x, wx[k].y, wx[k].z, wx[k].w, w4[k]};
                if (sa + 20 > lim) {  // the value's last bytes at the end of its buffer: dword by dword
#pragma unroll
                    for (int z = 0; z < 5; z++) d[z] = sa + 4 * z < lim ? gld<uint32_t>(sa + 4 * z) : 0u;
                }
                const uint32_t f = (uint32_t)(s & 3);
                const u32x4 y = {__builtin_amdgcn_alignbyte(d[1], d[0], f), __builtin_amdgcn_alignbyte(d[2], d[1], f),
                                 __builtin_amdgcn_alignbyte(d[3], d[2], f), __builtin_amdgcn_alignbyte(d[4], d[3], f)};
                const uint64_t q = qs + 16ull * c;
                if (q + 16 <= r.dend) {
                    gst<u32x4_a4>(q, y);
                } else {  // the record's last chunk: whole dwords, then the bytes of a partial one
                    const uint32_t yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                    for (int z = 0; z < 4; z++) {
                        const uint64_t qz = q + 4 * z;
                        if (qz + 4 <= r.dend) {
                            gst<uint32_t>(qz, yy[z]);
                        } else {
#pragma unroll
                            for (int b = 0; b < 4; b++)
                                if (qz + b < r.dend) gst<uint8_t>(qz + b, (uint8_t)(yy[z] >> (8 * b)));
                        }
                    }
                }
            }
        }
    }
}

static size_t al256e(size_t x) { return (x + 255) & ~(size_t)255; }
// List capacities from the bytes the values lie in (vbound), not from out_cap (a caller may pass any
// capacity): a record's value part is at most its value' bytes, and its header and key at most
// 12 + 33 KiB + 8 (writer.go:42), so its 8-KiB CRC pieces number at most value'/8K + 6.  (A copy list
// that overflowed would lose segments, so its bound must hold; the CRC pass walks records past its
// list with one wave each.)
static uint64_t enc_seg_cap(uint32_t n, uint64_t vbound) { return vbound / kEncSeg + n + 1; }
static uint64_t enc_piece_cap(uint32_t n, uint64_t vbound) { return vbound / 8192 + 6ull * n + 1; }
size_t enc_long_scratch_bytes(uint32_t n, uint64_t vbound) {
    return al256e(((size_t)n + 1) * 8) + al256e(scan_scratch_bytes(n)) + al256e((size_t)enc_seg_cap(n, vbound) * 8) +
           al256e((size_t)n * sizeof(bhg_handle)) + al256e(long_crc_scratch_bytes_cap(n, enc_piece_cap(n, vbound)));
}

hipError_t launch_encode(const Launch &L, const EncodeLaunch &E) {
    EncArgs a;
    a.keys = E.keys; a.key_off = E.key_off; a.trailers = E.trailers;
    a.vals = E.vbase; a.vpos = E.vpos; a.vlen = E.vlen; a.vals_end = (uint64_t)E.vend;
    a.n = E.n; a.file_nums = E.file_nums; a.rec_file_nums = E.rec_file_nums; a.live = E.live; a.khash = E.khash;
    a.key_len = E.key_len; a.pre_status = E.pre_status;
    a.single_table = E.single_table; a.max_tables = E.max_tables; a.init_size = E.init_size;
    a.table_max = E.table_max; a.out = E.out; a.out_cap = E.out_cap; a.lens = E.lens; a.o = E.o;
    a.xtab = L.xtab;
    a.long_min = E.long_scratch ? kLongRec : 0u;
    a.lbase = nullptr;
    a.lcap = 0;
    const uint32_t g = lane_grid(L, E.n, 256);
    hipLaunchKernelGGL(k_enc_sizes, dim3(g), dim3(256), 0, L.stream, a);
    hipError_t e = launch_exclusive_scan_u64(L, E.lens, E.lens, E.n, E.scan_scratch);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_enc_split, dim3(1), dim3(1024), 0, L.stream, a);
    // long mode: the long records' copy segments listed before the pack, which leaves them alone
    uint64_t *base = nullptr, vbound = 0;
    uint2 *ent = nullptr;
    bhg_handle *rec = nullptr;
    uint8_t *crc_scratch = nullptr;
    if (E.long_scratch) {
        uint8_t *sp = static_cast<uint8_t *>(E.long_scratch);
        vbound = (uint64_t)(E.vend - E.vbase);
        base = reinterpret_cast<uint64_t *>(sp);
        sp += al256e(((size_t)E.n + 1) * 8);
        void *scan = sp;
        sp += al256e(scan_scratch_bytes(E.n));
        ent = reinterpret_cast<uint2 *>(sp);
        sp += al256e((size_t)enc_seg_cap(E.n, vbound) * 8);
        rec = reinterpret_cast<bhg_handle *>(sp);
        sp += al256e((size_t)E.n * sizeof(bhg_handle));
        crc_scratch = sp;
        hipLaunchKernelGGL(k_enc_lcount, dim3(g), dim3(256), 0, L.stream, a, base);
        if ((e = launch_exclusive_scan_u64(L, base, base, E.n, scan)) != hipSuccess) return e;
        a.lbase = base;
        a.lcap = enc_seg_cap(E.n, vbound);
        hipLaunchKernelGGL(k_enc_lemit, dim3(g), dim3(256), 0, L.stream, (const uint64_t *)base, E.n, a.lcap, ent);
    }
    uint32_t gp = (E.n + 64 * ENC_WAVES - 1) / (64 * ENC_WAVES);  // a wave per 64-record tile
    static const uint32_t per_cu = resident_per_cu((const void *)k_enc_pack, 64 * ENC_WAVES, 2);
    const uint32_t capp = (uint32_t)L.num_cus * per_cu;
    if (gp > capp) gp = capp;
    if (gp == 0) gp = 1;
    hipLaunchKernelGGL(k_enc_pack, dim3(gp), dim3(64 * ENC_WAVES), 0, L.stream, a);
    if (!E.long_scratch) {
        hipLaunchKernelGGL(k_enc_meta, dim3(lane_grid(L, E.n, 256)), dim3(256), 0, L.stream, a);
    } else {
        hipLaunchKernelGGL(k_enc_lcopy, dim3(L.num_cus * 8), dim3(64 * ENC_LCOPY_WAVES), 0, L.stream, a,
                           (const uint64_t *)base, (const uint2 *)ent);
        // the records' handles {P, L} (the caller's o.rec when it asked for them), then their CRCs
        EncArgs m = a;
        if (!m.o.rec) m.o.rec = rec;
        hipLaunchKernelGGL(k_enc_meta, dim3(lane_grid(L, E.n, 256)), dim3(256), 0, L.stream, m);
        if ((e = launch_long_crc(L, E.out, E.out_cap, m.o.rec, E.n, nullptr, nullptr, crc_scratch, E.o.crc,
                                 enc_piece_cap(E.n, vbound))) != hipSuccess)
            return e;
    }
    if (E.o.table_size)
        hipLaunchKernelGGL(k_enc_tsize, dim3(lane_grid(L, E.max_tables, 256)), dim3(256), 0, L.stream, a);
    return hipGetLastError();
}

hipError_t launch_enc_rawvals(const Launch &L, const uint64_t *val_off, uint32_t n, uint64_t *vlen) {
    hipLaunchKernelGGL(k_enc_rawvals, dim3(lane_grid(L, n, 256)), dim3(256), 0, L.stream, val_off, n, vlen);
    return hipGetLastError();
}

}  // namespace bhg
