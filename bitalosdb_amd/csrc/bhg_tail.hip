// bhg_tail.hip -- the table tail of Writer.writeTable on the GPU, for many
// tables at once: writeData's empty header, writeConflict, writeIndexHash
// (HashIndex build + serialize + checksum), writeMeta and writeFooter
// (bithash/writer.go:312-338, 393-533; internal/bindex/hash_index.go:217-363;
// bithash/block.go:595-729; bithash/table.go:56-68).
//
// Input: the table's records in add order -- for each record its position
// in `recs` (bhg_handle: offset + length), its table-relative BlockHandle
// offset, khash, table index and status.  updateHash (writer.go:285-310) is
// a fold over add order; grouped by khash it is:
//   * all records of a khash carry the same user key -> one index item, the
//     LAST add's handle (ih.bh = bh);
//   * two or more distinct keys -> the item points at conflictBH and every
//     distinct key of the group lands in conflictKeys with its LAST handle.
// So the device work is a stable sort of (table, khash) -> runs, a conflict
// test per run, last-occurrence flags, then every byte of the tail:
//
//   k_tail_keys    lane/record: sort key (table << 32 | khash), invalid -> ~0
//   radix sort     bhg_sort.hip, stable (add order kept inside a run), key bits
//                  [0, 32 + bits(ntables)): invalid keys (~0) stay above every valid one
//   k_tail_heads   lane/position: run-head flags -> scan -> run index
//   k_tail_runs    lane/run: run position, key, length, conflict flag
//   k_tail_keep    lane/position: last occurrence of its key in a conflict run
//   k_tail_klist   scan of keep -> compacted kept positions
//   k_tail_dedupe  lane/kept position: a key kept by two runs of one table
//                  (the caller passed one key under two khash values) stays
//                  only where conflictKeys[key] was assigned last
//                  -> scan -> conflict list (sorted by table)
//   k_tail_tables  lane/table: run range, conflict range, tail size bound
//                  -> scan -> tail_off
//   k_conf_rank    lane/conflict key: rank by key bytes (sort.Strings) inside its table
//   k_conf_size    lane/rank: blockWriter entry size (shared prefix with the
//                  previous key, restart every 16 entries) -> scan
//   k_conf_write   lane/rank: the entry bytes, restart array, count
//   k_tail_items   lane/run: the 10-byte big-endian HashIndex item
//   k_tail_shards  lane/(table, shard): cumulative shard count (big-endian)
//   k_tail_crch    lane/table: HashIndex header, checksum range
//   k_crc_long     the indexhash_data checksum (bhg_decode.hip)
//   k_tail_finish  lane/table: block headers, checksum entry, meta block, footer
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

constexpr uint32_t kShards = 64u << 10;                 // HashIndex shards (hi16)
constexpr uint32_t kIdxHeader = 8;                      // SuccinctHeaderSize
constexpr uint32_t kIdxItemOff = kIdxHeader + kShards * 4;
constexpr uint32_t kItem = 10;                          // HashIndexItem64Size: BE u16 lo16 + BE u64
constexpr uint32_t kMetaBytes = 122;                    // 3 entries (35 + 39 + 40) + restart + count
constexpr uint32_t kFooter = 21;                        // table.go:56-68
constexpr uint32_t kRestart = 16;                       // blockRestartInterval
constexpr uint32_t kTailFixed = 12 + 2 + 5 + 22 + 39 + 8 + kMetaBytes + kFooter;

struct TailArgs {
    const uint8_t *recs;
    const bhg_handle *rec;
    const uint32_t *bh_off, *khash, *table, *status;
    uint32_t n, ntables;
    const uint64_t *data_end;
    uint8_t *tail;
    uint64_t tail_cap;
    uint64_t *tail_off, *tail_len;
    uint32_t *stats;
    // scratch
    uint64_t *sk, *sk_s;
    uint32_t *idx, *idx_s;
    uint64_t *head, *runidx;        // n+1
    uint32_t *run_pos, *run_len;    // n
    uint64_t *run_key;              // n
    uint8_t *run_conf;              // n
    uint64_t *keep, *kpos;          // n+1
    uint64_t *kscan;                // n+1: exclusive scan of keep
    uint32_t *klist;                // n: kept positions, in sorted order
    uint64_t *kpre, *kaddr;         // n: per kept entry (klist order): big-endian first 8 key bytes, key address
    uint32_t *klen, *katk;          // n: ... key length, kat of its position
    uint64_t *cpre, *caddr;         // n: the same per conflict entry (clist order)
    uint32_t *cklen;                // n
    uint32_t *kat;                  // n: when updateHash last assigned conflictKeys[key] from this run
    uint32_t *clist, *cord;         // n
    uint64_t *csz;                  // n+1: conflict entry sizes -> offsets
    uint32_t *tab_run, *tab_c;      // ntables+1
    uint64_t *cbound;               // ntables
    uint32_t *cinfo;                // ntables x 2: conflict block bytes, keys
    bhg_handle *crc_h;              // ntables
    uint32_t *crc;                  // ntables
};

__device__ __forceinline__ uint32_t ld8(uint64_t a) { return gld<uint8_t>(a); }
__device__ __forceinline__ void st8(uint64_t a, uint32_t v) { gst<uint8_t>(a, (uint8_t)v); }

// user key of record i: (address, length); ikeySize < 8 -> empty (DecodeInternalKey)
__device__ __forceinline__ void rec_key(const TailArgs &a, uint32_t i, uint64_t &kp, uint32_t &kl) {
    const uint64_t p = (uint64_t)a.recs + a.rec[i].offset;
    const uint32_t ik = ld8(p) | ld8(p + 1) << 8 | ld8(p + 2) << 16 | ld8(p + 3) << 24;
    kl = ik >= 8 ? ik - 8 : 0;
    kp = p + 12;
}

__device__ __forceinline__ bool key_eq(uint64_t a, uint32_t al, uint64_t b, uint32_t bl) {
    if (al != bl) return false;
    for (uint32_t k = 0; k < al; k++)
        if (ld8(a + k) != ld8(b + k)) return false;
    return true;
}

// bytes.Compare < 0
__device__ __forceinline__ bool key_lt(uint64_t a, uint32_t al, uint64_t b, uint32_t bl) {
    const uint32_t m = al < bl ? al : bl;
    for (uint32_t k = 0; k < m; k++) {
        const uint32_t x = ld8(a + k), y = ld8(b + k);
        if (x != y) return x < y;
    }
    return al < bl;
}

// the first 8 key bytes, big-endian, zero-padded: keys whose prefixes differ compare as their
// prefixes do (bytes.Compare); equal prefixes need the full compare
__device__ __forceinline__ uint64_t key_prefix(uint64_t kp, uint32_t kl) {
    uint64_t x = 0;
    for (uint32_t k = 0; k < 8; k++) x = (x << 8) | (k < kl ? ld8(kp + k) : 0u);
    return x;
}

// byte j of the internal key userKey || trailer(seq 1, kind SET) (MakeInternalKey(k, 1, InternalKeyKindSet))
__device__ __forceinline__ uint32_t ikey_byte(uint64_t kp, uint32_t kl, uint32_t j) {
    if (j < kl) return ld8(kp + j);
    return j - kl < 2 ? 1u : 0u;  // trailer (1 << 8 | 1) little-endian
}

__device__ __forceinline__ uint32_t varint_len(uint64_t x) {
    uint32_t n = 1;
    while (x >= 0x80) { x >>= 7; n++; }
    return n;
}

__device__ __forceinline__ uint64_t put_varint(uint64_t p, uint64_t x) {
    while (x >= 0x80) { st8(p++, (uint32_t)(x & 0x7f) | 0x80); x >>= 7; }
    st8(p++, (uint32_t)x);
    return p;
}

__device__ __forceinline__ uint64_t put_le32(uint64_t p, uint32_t v) {
    for (int b = 0; b < 4; b++) st8(p + b, v >> (8 * b));
    return p + 4;
}

__device__ __forceinline__ uint64_t put_str(uint64_t p, const char *s, uint32_t n) {
    for (uint32_t k = 0; k < n; k++) st8(p + k, (uint8_t)s[k]);
    return p + n;
}

__device__ __forceinline__ uint64_t put_trailer(uint64_t p) {
    st8(p, 1); st8(p + 1, 1);
    for (int b = 2; b < 8; b++) st8(p + b, 0);
    return p + 8;
}

// first index in [lo, hi) with key(index) >= x; key = f(index)
template <class F>
__device__ __forceinline__ uint32_t lower_bound(uint32_t lo, uint32_t hi, uint64_t x, F key) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (key(mid) < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

#define GRID_LOOP(i, n) for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
                             i += (uint64_t)gridDim.x * blockDim.x)

__global__ __launch_bounds__(256) void k_tail_keys(TailArgs a) {
    GRID_LOOP(i, a.n) {
        const uint32_t t = a.table[i];
        const bool valid = t < a.ntables && (a.status == nullptr || a.status[i] == BHG_ST_OK) && a.rec[i].length > 0;
        a.sk[i] = valid ? ((uint64_t)t << 32 | a.khash[i]) : ~0ull;
        a.idx[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void k_tail_heads(TailArgs a) {
    GRID_LOOP(j, a.n) {
        const uint64_t k = a.sk_s[j];
        a.head[j] = k != ~0ull && (j == 0 || a.sk_s[j - 1] != k) ? 1 : 0;
    }
}

// lane per sorted position: a head writes its run's record
__global__ __launch_bounds__(256) void k_tail_runs(TailArgs a) {
    GRID_LOOP(j, a.n) {
        const uint64_t k = a.sk_s[j];
        if (k == ~0ull || (j > 0 && a.sk_s[j - 1] == k)) continue;
        const uint32_t r = (uint32_t)a.runidx[j];
        uint32_t e = (uint32_t)j + 1;
        while (e < a.n && a.sk_s[e] == k) e++;
        uint64_t kp0; uint32_t kl0;
        rec_key(a, a.idx_s[j], kp0, kl0);
        bool conf = false;
        for (uint32_t q = (uint32_t)j + 1; q < e && !conf; q++) {
            uint64_t kp; uint32_t kl;
            rec_key(a, a.idx_s[q], kp, kl);
            conf = !key_eq(kp0, kl0, kp, kl);
        }
        a.run_pos[r] = (uint32_t)j;
        a.run_len[r] = e - (uint32_t)j;
        a.run_key[r] = k;
        a.run_conf[r] = conf;
    }
}

// lane per sorted position: conflictKeys member = last occurrence of its key in a conflict run
__global__ __launch_bounds__(256) void k_tail_keep(TailArgs a) {
    GRID_LOOP(j, a.n) {
        const uint64_t k = a.sk_s[j];
        uint64_t keep = 0;
        if (k != ~0ull) {
            const uint32_t r = (uint32_t)(a.runidx[j] + a.head[j] - 1);  // run of position j
            if (a.run_conf[r]) {
                const uint32_t e = a.run_pos[r] + a.run_len[r];
                uint64_t kp; uint32_t kl;
                rec_key(a, a.idx_s[j], kp, kl);
                keep = 1;
                for (uint32_t q = (uint32_t)j + 1; q < e && keep; q++) {
                    uint64_t kq; uint32_t lq;
                    rec_key(a, a.idx_s[q], kq, lq);
                    if (key_eq(kp, kl, kq, lq)) keep = 0;
                }
                if (keep) {  // blockWriter entry bound: 3 varints + ikey + 8-B handle + a restart slot
                    atomicAdd(reinterpret_cast<unsigned long long *>(a.cbound + (k >> 32)),
                              (unsigned long long)(15 + kl + 8 + 8 + 4));
                    // updateHash (writer.go:285-310) assigns conflictKeys[key] at every add of the key
                    // once the run conflicts, and the run's first key once more at the add that makes
                    // it conflict (conflictKeys[ih.userKey] = ih.bh): the assignment time is the
                    // later of this last add and, for the first key, that add
                    uint32_t at = a.idx_s[j];
                    const uint32_t p0 = a.run_pos[r];
                    uint64_t k0; uint32_t l0;
                    rec_key(a, a.idx_s[p0], k0, l0);
                    if (key_eq(kp, kl, k0, l0)) {
                        uint32_t q = p0 + 1;
                        for (; q < e; q++) {
                            uint64_t kq; uint32_t lq;
                            rec_key(a, a.idx_s[q], kq, lq);
                            if (!key_eq(k0, l0, kq, lq)) break;
                        }
                        const uint32_t tc = a.idx_s[q < e ? q : e - 1];
                        at = at > tc ? at : tc;
                    }
                    a.kat[j] = at;
                }
            }
        }
        a.keep[j] = keep;
    }
}

// kept positions, compacted: klist[kscan[j]] = j (kscan = exclusive scan of keep), with each
// kept key's prefix / address / length / kat laid out in the same order for k_tail_dedupe
__global__ __launch_bounds__(256) void k_tail_klist(TailArgs a) {
    GRID_LOOP(j, a.n) {
        if (a.kscan[j + 1] != a.kscan[j]) {
            const uint64_t g = a.kscan[j];
            uint64_t kp; uint32_t kl;
            rec_key(a, a.idx_s[j], kp, kl);
            a.klist[g] = (uint32_t)j;
            a.kpre[g] = key_prefix(kp, kl);
            a.kaddr[g] = kp;
            a.klen[g] = kl;
            a.katk[g] = a.kat[j];
        }
    }
}

// conflictKeys is one map per table, keyed by user key: a key kept by two runs (two khash
// values for one key, possible through AddIkey) keeps the run that assigned it last.  Without
// this the conflict list would hold a key twice and the rank permutation would break.  Each
// kept position compares itself with the kept positions of its own table only (klist, sorted
// by table like sk_s): O(kept_t^2) per table, over the contiguous prefix / length arrays (the
// key bytes only when both match).
__global__ __launch_bounds__(256) void k_tail_dedupe(TailArgs a) {
    const uint32_t K = (uint32_t)a.kscan[a.n];
    GRID_LOOP(j, a.n) {
        uint64_t f = a.keep[j];
        if (f) {
            const uint64_t t = a.sk_s[j] >> 32;
            const uint32_t g0 = lower_bound(0, K, t << 32, [&](uint32_t g) { return a.sk_s[a.klist[g]]; });
            const uint32_t g1 = lower_bound(g0, K, (t + 1) << 32, [&](uint32_t g) { return a.sk_s[a.klist[g]]; });
            const uint64_t gj = a.kscan[j];
            const uint64_t pre = a.kpre[gj], kp = a.kaddr[gj];
            const uint32_t kl = a.klen[gj], at = a.kat[j];
            for (uint32_t g = g0; g < g1 && f; g++) {
                if (a.kpre[g] != pre || a.klen[g] != kl || g == gj) continue;
                const uint32_t q = a.klist[g], aq = a.katk[g];
                if (aq < at || (aq == at && q < j)) continue;
                if (key_eq(kp, kl, a.kaddr[g], kl)) f = 0;
            }
        }
        a.kpos[j] = f;
    }
}

__global__ __launch_bounds__(256) void k_tail_clist(TailArgs a) {
    GRID_LOOP(j, a.n) {
        if (a.kpos[j + 1] != a.kpos[j]) {
            const uint64_t f = a.kpos[j], g = a.kscan[j];
            a.clist[f] = (uint32_t)j;
            a.cpre[f] = a.kpre[g];
            a.caddr[f] = a.kaddr[g];
            a.cklen[f] = a.klen[g];
        }
    }
}

// lane per table t <= ntables: run range, conflict range, size bound
__global__ __launch_bounds__(256) void k_tail_tables(TailArgs a) {
    const uint32_t R = (uint32_t)a.runidx[a.n];
    const uint32_t M = (uint32_t)a.kpos[a.n];
    GRID_LOOP(t, (uint64_t)a.ntables + 1) {
        const uint64_t x = t << 32;
        a.tab_run[t] = lower_bound(0, R, x, [&](uint32_t r) { return a.run_key[r]; });
        a.tab_c[t] = lower_bound(0, M, x, [&](uint32_t g) { return a.sk_s[a.clist[g]]; });
        if (t < a.ntables) {
            const uint32_t Rt = lower_bound(0, R, (t + 1) << 32, [&](uint32_t r) { return a.run_key[r]; }) -
                                a.tab_run[t];
            const uint64_t cb = a.cbound[t] ? a.cbound[t] + 8 : 0;
            a.tail_off[t] = kTailFixed + cb + (Rt ? (uint64_t)kIdxItemOff + (uint64_t)kItem * Rt : 0);
            a.cinfo[2 * t] = 0;
            a.cinfo[2 * t + 1] = 0;
        }
    }
}

__device__ __forceinline__ uint32_t table_of_pos(const TailArgs &a, uint32_t j) { return (uint32_t)(a.sk_s[j] >> 32); }

// tables whose tail slot ends past tail_cap are not written (tail_len 0)
__device__ __forceinline__ bool tail_fits(const TailArgs &a, uint32_t t) { return a.tail_off[t + 1] <= a.tail_cap; }

// lane per conflict key g: rank among its table's conflict keys by user key bytes (sort.Strings),
// over the contiguous prefix array (the key bytes only when two prefixes are equal)
__global__ __launch_bounds__(256) void k_conf_rank(TailArgs a) {
    const uint32_t M = (uint32_t)a.kpos[a.n];
    GRID_LOOP(g, M) {
        const uint32_t t = table_of_pos(a, a.clist[g]);
        const uint32_t c0 = a.tab_c[t], c1 = a.tab_c[t + 1];
        const uint64_t pre = a.cpre[g], kp = a.caddr[g];
        const uint32_t kl = a.cklen[g];
        uint32_t rank = 0;
        for (uint32_t f = c0; f < c1; f++) {
            const uint64_t pf = a.cpre[f];
            if (pf != pre) rank += pf < pre;
            else if (f != g) rank += key_lt(a.caddr[f], a.cklen[f], kp, kl);
        }
        a.cord[c0 + rank] = (uint32_t)g;  // keys of a table are distinct (k_tail_dedupe): ranks are a permutation
    }
}

// shared prefix of entry q's internal key with entry q-1's (0 at a restart)
__device__ __forceinline__ uint32_t conf_shared(const TailArgs &a, uint32_t q, uint32_t c0, uint64_t kp, uint32_t kl) {
    if ((q - c0) % kRestart == 0) return 0;
    uint64_t pp; uint32_t pl;
    rec_key(a, a.idx_s[a.clist[a.cord[q - 1]]], pp, pl);
    const uint32_t m = (kl < pl ? kl : pl) + 8;
    uint32_t s = 0;
    while (s < m && ikey_byte(kp, kl, s) == ikey_byte(pp, pl, s)) s++;
    return s;
}

__global__ __launch_bounds__(256) void k_conf_size(TailArgs a) {
    const uint32_t M = (uint32_t)a.kpos[a.n];
    GRID_LOOP(q, M) {
        const uint32_t g = a.cord[q];
        const uint32_t t = table_of_pos(a, a.clist[g]);
        uint64_t kp; uint32_t kl;
        rec_key(a, a.idx_s[a.clist[g]], kp, kl);
        const uint32_t sh = conf_shared(a, (uint32_t)q, a.tab_c[t], kp, kl);
        const uint32_t un = kl + 8 - sh;
        a.csz[q] = varint_len(sh) + varint_len(un) + 1 + un + 8;
    }
}

// lane per rank q: entry bytes at the table's conflict block (tail_off + 12)
__global__ __launch_bounds__(256) void k_conf_write(TailArgs a) {
    const uint32_t M = (uint32_t)a.kpos[a.n];
    GRID_LOOP(q, M) {
        const uint32_t g = a.cord[q];
        const uint32_t j = a.clist[g];
        const uint32_t t = table_of_pos(a, j);
        if (!tail_fits(a, t)) continue;
        const uint32_t c0 = a.tab_c[t], m = a.tab_c[t + 1] - c0, qq = (uint32_t)q - c0;
        const uint64_t ent_bytes = a.csz[a.tab_c[t + 1]] - a.csz[c0];
        const uint32_t nres = (m + kRestart - 1) / kRestart;
        const uint64_t blk = (uint64_t)a.tail + a.tail_off[t] + 12;
        const uint64_t off = a.csz[q] - a.csz[c0];
        const uint32_t i = a.idx_s[j];
        uint64_t kp; uint32_t kl;
        rec_key(a, i, kp, kl);
        const uint32_t sh = conf_shared(a, (uint32_t)q, c0, kp, kl);
        uint64_t p = blk + off;
        p = put_varint(p, sh);
        p = put_varint(p, kl + 8 - sh);
        p = put_varint(p, 8);
        for (uint32_t b = sh; b < kl + 8; b++) st8(p++, ikey_byte(kp, kl, b));
        p = put_le32(p, a.bh_off[i]);          // encodeBlockHandle(conflictKeys[k]) (block.go:26-39)
        p = put_le32(p, a.rec[i].length);
        if (qq % kRestart == 0) put_le32(blk + ent_bytes + 4ull * (qq / kRestart), (uint32_t)off);
        if (qq == 0) {
            put_le32(blk + ent_bytes + 4ull * nres, nres);
            a.cinfo[2 * t] = (uint32_t)(ent_bytes + 4ull * nres + 4);
            a.cinfo[2 * t + 1] = m;
        }
    }
}

// the indexhash_data value of table t: position inside tail, length
__device__ __forceinline__ void idx_data(const TailArgs &a, uint32_t t, uint32_t Rt, uint64_t &pos, uint64_t &len) {
    len = Rt ? (uint64_t)kIdxItemOff + (uint64_t)kItem * Rt : 0;
    pos = a.tail_off[t] + 12 + a.cinfo[2 * t] + (Rt ? 2 + varint_len(len) + 22 : 0);
}

// lane per run r: the HashIndex item (writeIndexHash's hindex.Add + writeItem64)
__global__ __launch_bounds__(256) void k_tail_items(TailArgs a) {
    const uint32_t R = (uint32_t)a.runidx[a.n];
    GRID_LOOP(r, R) {
        const uint64_t k = a.run_key[r];
        const uint32_t t = (uint32_t)(k >> 32);
        if (!tail_fits(a, t)) continue;
        const uint32_t Rt = a.tab_run[t + 1] - a.tab_run[t];
        uint64_t dpos, dlen;
        idx_data(a, t, Rt, dpos, dlen);
        uint32_t off, len;
        if (a.run_conf[r]) {  // conflictBH = {currentOffset after writeData, conflict block length}
            off = (uint32_t)(a.data_end[t] + 12);
            len = a.cinfo[2 * t];
        } else {              // the last add of the key (ih.bh = bh)
            const uint32_t i = a.idx_s[a.run_pos[r] + a.run_len[r] - 1];
            off = a.bh_off[i];
            len = a.rec[i].length;
        }
        const uint64_t v = (uint64_t)off | (uint64_t)len << 32;  // LittleEndian.Uint64(encodeBlockHandle)
        const uint64_t p = (uint64_t)a.tail + dpos + kIdxItemOff + (uint64_t)kItem * (r - a.tab_run[t]);
        st8(p, (uint32_t)(k >> 8) & 0xffu);                      // lo16, big-endian
        st8(p + 1, (uint32_t)k & 0xffu);
        for (int b = 0; b < 8; b++) st8(p + 2 + b, (uint32_t)(v >> (56 - 8 * b)) & 0xffu);
    }
}

// lane per (table, shard): writeShard(totalCount) = items in shards 0..s, big-endian
__global__ __launch_bounds__(256) void k_tail_shards(TailArgs a) {
    GRID_LOOP(x, (uint64_t)a.ntables * kShards) {
        const uint32_t t = (uint32_t)(x / kShards), s = (uint32_t)(x % kShards);
        const uint32_t r0 = a.tab_run[t], r1 = a.tab_run[t + 1];
        if (r0 == r1 || !tail_fits(a, t)) continue;
        const uint64_t lim = ((uint64_t)t << 32) + ((uint64_t)(s + 1) << 16);  // first key past shard s (s = 65535: next table)
        const uint32_t cnt = lower_bound(r0, r1, lim, [&](uint32_t r) { return a.run_key[r]; }) - r0;
        uint64_t dpos, dlen;
        idx_data(a, t, r1 - r0, dpos, dlen);
        const uint64_t p = (uint64_t)a.tail + dpos + kIdxHeader + 4ull * s;
        for (int b = 0; b < 4; b++) st8(p + b, (cnt >> (24 - 8 * b)) & 0xffu);
    }
}

__global__ __launch_bounds__(256) void k_tail_crch(TailArgs a) {
    GRID_LOOP(t, a.ntables) {
        const uint32_t Rt = a.tab_run[t + 1] - a.tab_run[t];
        uint64_t dpos, dlen;
        idx_data(a, (uint32_t)t, Rt, dpos, dlen);
        bhg_handle h;
        h.offset = dpos;
        h.length = (uint32_t)dlen;
        h.pad = 0;
        if (!tail_fits(a, (uint32_t)t)) {
            h.offset = ~0ull;  // out of range -> not computed
        } else if (Rt) {       // HashIndex header (big-endian): version 1, reserved 0, shards 65536
            const uint64_t p = (uint64_t)a.tail + dpos;
            st8(p, 0); st8(p + 1, 1); st8(p + 2, 0); st8(p + 3, 0);
            st8(p + 4, 0); st8(p + 5, 1); st8(p + 6, 0); st8(p + 7, 0);
        }
        a.crc_h[t] = h;
    }
}

// lane per table: everything but the conflict entries and the HashIndex body
__global__ __launch_bounds__(64) void k_tail_finish(TailArgs a) {
    GRID_LOOP(t, a.ntables) {
        const uint32_t Rt = a.tab_run[t + 1] - a.tab_run[t];
        const uint32_t C = a.cinfo[2 * t], nconf = a.cinfo[2 * t + 1];
        if (a.stats) {
            a.stats[4 * t] = Rt;
            a.stats[4 * t + 1] = nconf;
            a.stats[4 * t + 2] = tail_fits(a, (uint32_t)t) ? BHG_ST_OK : BHG_ST_NO_SPACE;
            a.stats[4 * t + 3] = 0;
        }
        if (!tail_fits(a, (uint32_t)t)) {
            a.tail_len[t] = 0;
            continue;
        }
        const uint64_t base = (uint64_t)a.tail + a.tail_off[t];
        const uint32_t D = (uint32_t)a.data_end[t];
        for (int b = 0; b < 12; b++) st8(base + b, 0);  // writeData: setEmptyHeader
        // writeIndexHash (writer.go:449-490)
        const uint64_t ib = base + 12 + C;
        uint64_t dpos, dlen;
        idx_data(a, (uint32_t)t, Rt, dpos, dlen);
        uint64_t p = ib;
        if (Rt) {
            p = put_varint(p, 0);
            p = put_varint(p, 22);
            p = put_varint(p, dlen);
            p = put_str(p, "indexhash_data", 14);
            p = put_trailer(p);
            p += dlen;  // header (k_tail_crch), shards, items: written before the checksum
        }
        // indexhash_checksum: strconv.FormatUint(crc.New(data).Value(), 10)
        char dig[10];
        uint32_t nd = 0, c = a.crc[t];
        do { dig[nd++] = (char)('0' + c % 10); c /= 10; } while (c);
        if (Rt) {  // shares "indexhash_" with the previous key
            p = put_varint(p, 10);
            p = put_varint(p, 16);
            p = put_varint(p, nd);
            p = put_str(p, "checksum", 8);
        } else {
            p = put_varint(p, 0);
            p = put_varint(p, 26);
            p = put_varint(p, nd);
            p = put_str(p, "indexhash_checksum", 18);
        }
        p = put_trailer(p);
        for (uint32_t k = 0; k < nd; k++) st8(p++, (uint8_t)dig[nd - 1 - k]);
        p = put_le32(p, 0);  // restarts {0}
        p = put_le32(p, 1);
        const uint32_t IB = (uint32_t)(p - ib);
        // writeMeta (writer.go:492-521): three restart-less entries, no shared prefixes
        const uint64_t mb = p;
        const uint32_t bh[3][2] = {{0, D + 12}, {D + 12, C}, {D + 12 + C, IB}};
        const char *names[3] = {"data_blockhandle", "conflict_blockhandle", "indexhash_blockhandle"};
        const uint32_t nl[3] = {16, 20, 21};
        for (int e = 0; e < 3; e++) {
            p = put_varint(p, 0);
            p = put_varint(p, nl[e] + 8);
            p = put_varint(p, 8);
            p = put_str(p, names[e], nl[e]);
            p = put_trailer(p);
            p = put_le32(p, bh[e][0]);
            p = put_le32(p, bh[e][1]);
        }
        p = put_le32(p, 0);
        p = put_le32(p, 1);
        // writeFooter (table.go:56-68): checksum type, metaBH, format version, magic
        st8(p++, 1);
        p = put_le32(p, D + 12 + C + IB);
        p = put_le32(p, kMetaBytes);
        p = put_le32(p, 2);
        const uint8_t magic[8] = {0xf7, 0xcf, 0xf4, 0x85, 0xb7, 0x41, 0xe2, 0x88};
        for (int b = 0; b < 8; b++) st8(p++, magic[b]);
        (void)mb;
        a.tail_len[t] = p - base;
    }
}

size_t sort_tmp_bytes(uint32_t n) { return radix_sort_scratch_bytes(n); }

// key bits the sort looks at: khash (32) + the table index; ntables itself fits too, so a
// truncated invalid key (~0) is above every valid key
uint32_t sort_end_bit(uint32_t ntables) {
    const uint32_t tb = ntables ? 32u - (uint32_t)__builtin_clz(ntables) : 1u;
    return 32u + tb > 64u ? 64u : 32u + tb;
}

}  // namespace

size_t tail_scratch_bytes(uint32_t n, uint32_t ntables) {
    const size_t sort_tmp = sort_tmp_bytes(n);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t N = (size_t)n + 1, T = (size_t)ntables + 1;
    return al(sort_tmp) + 2 * al(N * 8) + 2 * al(N * 4) + 2 * al(N * 8) + 2 * al(N * 4) + al(N * 8) + al(N) +
           3 * al(N * 8) + 2 * al(N * 4) + 2 * al(N * 4) + al(N * 8) + 2 * al(T * 4) + al(T * 8) + al(T * 8) +
           al(T * 16) + al(T * 4) + al(scan_scratch_bytes(N > T ? N : T)) + al(crc_long_scratch_bytes((uint32_t)T)) +
           4 * al(N * 8) + 3 * al(N * 4) + 32 * 256;
}

hipError_t launch_table_tail(const Launch &L, const TailLaunch &T, void *scratch) {
    TailArgs a;
    a.recs = T.recs; a.rec = T.rec; a.bh_off = T.bh_off; a.khash = T.khash; a.table = T.table; a.status = T.status;
    a.n = T.n; a.ntables = T.ntables; a.data_end = T.data_end; a.tail = T.tail; a.tail_cap = T.tail_cap;
    a.tail_off = T.tail_off; a.tail_len = T.tail_len; a.stats = T.stats;
    const uint32_t n = T.n, nt = T.ntables;
    size_t sort_tmp = sort_tmp_bytes(n);
    hipError_t e = hipSuccess;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    uint8_t *s = reinterpret_cast<uint8_t *>(scratch);
    auto take = [&](size_t b) { uint8_t *p = s; s += al(b); return p; };
    const size_t N = (size_t)n + 1, TT = (size_t)nt + 1;
    void *sort_buf = take(sort_tmp);
    a.sk = (uint64_t *)take(N * 8); a.sk_s = (uint64_t *)take(N * 8);
    a.idx = (uint32_t *)take(N * 4); a.idx_s = (uint32_t *)take(N * 4);
    a.head = (uint64_t *)take(N * 8); a.runidx = (uint64_t *)take(N * 8);
    a.run_pos = (uint32_t *)take(N * 4); a.run_len = (uint32_t *)take(N * 4);
    a.run_key = (uint64_t *)take(N * 8); a.run_conf = take(N);
    a.keep = (uint64_t *)take(N * 8); a.kpos = (uint64_t *)take(N * 8); a.kat = (uint32_t *)take(N * 4);
    a.kscan = (uint64_t *)take(N * 8); a.klist = (uint32_t *)take(N * 4);
    a.kpre = (uint64_t *)take(N * 8); a.kaddr = (uint64_t *)take(N * 8);
    a.klen = (uint32_t *)take(N * 4); a.katk = (uint32_t *)take(N * 4);
    a.cpre = (uint64_t *)take(N * 8); a.caddr = (uint64_t *)take(N * 8); a.cklen = (uint32_t *)take(N * 4);
    a.clist = (uint32_t *)take(N * 4); a.cord = (uint32_t *)take(N * 4);
    a.csz = (uint64_t *)take(N * 8);
    a.tab_run = (uint32_t *)take(TT * 4); a.tab_c = (uint32_t *)take(TT * 4);
    a.cbound = (uint64_t *)take(TT * 8); a.cinfo = (uint32_t *)take(TT * 8);
    a.crc_h = (bhg_handle *)take(TT * 16); a.crc = (uint32_t *)take(TT * 4);
    void *scan_s = take(scan_scratch_bytes(N > TT ? N : TT));  // also scans tail_off over the tables
    void *crc_s = take(crc_long_scratch_bytes((uint32_t)TT));

    const uint32_t g = lane_grid(L, n ? n : 1, 256);
    e = hipMemsetAsync(a.cbound, 0, TT * 8, L.stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_keys, dim3(g), dim3(256), 0, L.stream, a);
    e = launch_radix_sort_pairs(L, a.sk, a.sk_s, a.idx, a.idx_s, n, sort_end_bit(nt), sort_buf);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_heads, dim3(g), dim3(256), 0, L.stream, a);
    if ((e = launch_exclusive_scan_u64(L, a.head, a.runidx, n, scan_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_runs, dim3(g), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_keep, dim3(g), dim3(256), 0, L.stream, a);
    if ((e = launch_exclusive_scan_u64(L, a.keep, a.kscan, n, scan_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_klist, dim3(g), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_dedupe, dim3(g), dim3(256), 0, L.stream, a);
    if ((e = launch_exclusive_scan_u64(L, a.kpos, a.kpos, n, scan_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_clist, dim3(g), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_tables, dim3(lane_grid(L, (uint64_t)nt + 1, 256)), dim3(256), 0, L.stream, a);
    if ((e = launch_exclusive_scan_u64(L, a.tail_off, a.tail_off, nt, scan_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_conf_rank, dim3(g), dim3(256), 0, L.stream, a);
    // conflict entry offsets: csz[0..M] (M <= n; entries past M are never read)
    if ((e = hipMemsetAsync(a.csz, 0, N * 8, L.stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_conf_size, dim3(g), dim3(256), 0, L.stream, a);
    if ((e = launch_exclusive_scan_u64(L, a.csz, a.csz, n, scan_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_conf_write, dim3(g), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_items, dim3(g), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_shards, dim3(lane_grid(L, (uint64_t)nt * kShards, 256)), dim3(256), 0, L.stream, a);
    hipLaunchKernelGGL(k_tail_crch, dim3(lane_grid(L, nt, 256)), dim3(256), 0, L.stream, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_crc_long(L, T.tail, T.tail_cap, a.crc_h, nt, a.crc, crc_s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tail_finish, dim3((nt + 63) / 64), dim3(64), 0, L.stream, a);
    return hipGetLastError();
}

}  // namespace bhg
