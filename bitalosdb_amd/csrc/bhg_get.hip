// bhg_get.hip -- batched point lookup over .bht tables resident in HBM.
//
// k_get: one LANE per query.  Reader.Get minus the pread (bithash/reader.go:209-231):
//   khash   = hash.Fnv32(key)                                (internal/hash/fnv.go:19-23)
//   v, ok   = HashIndex.Get64(khash)                         (internal/bindex/hash_index.go:399-431)
//             shard counts and items are BIG-endian; items are {u16 lo16, u64 value} sorted by lo16
//             within the shard; findItem is a lower-bound binary search   (:487-503)
//   bh      = decodeBlockHandle(LE bytes of v)               (reader.go:215-217)
//   if conflictBH.Length != 0 && bh.Offset >= conflictBH.Offset && bh.Length <= conflictBH.Length:
//       bh = readConflict(key): blockIter.SeekGE over the conflict block  (reader.go:274-289,
//            block.go:274-350): binary search over the restart points, then a forward scan
//            of prefix-compressed entries (block.go:112-182); hit iff the entry's UserKey == key
//       miss -> {0, 0} -> ErrBhIllegalBlockLength (reader.go:224-226)
// The output handle is rebased to src (table base + bh.Offset) so that it can
// be fed straight to bhg_decode_batch: Get + readData as two launches.
//
// Lookups are latency-bound dependent reads (2 shard counts + log2(items in
// the shard) item probes, ~1.5 MB of index per table: L2/MALL-resident under
// load); the grid is sized for many queries in flight per CU.
#include "bhg_device.h"
#include "bhg_internal.h"

namespace bhg {

namespace {

__device__ __forceinline__ uint32_t ld8(uint64_t a) { return gld<uint8_t>(a); }
__device__ __forceinline__ uint32_t be16(uint64_t a) { return (ld8(a) << 8) | ld8(a + 1); }
__device__ __forceinline__ uint32_t be32(uint64_t a) {
    return (ld8(a) << 24) | (ld8(a + 1) << 16) | (ld8(a + 2) << 8) | ld8(a + 3);
}
__device__ __forceinline__ uint64_t be64(uint64_t a) { return ((uint64_t)be32(a) << 32) | be32(a + 4); }
__device__ __forceinline__ uint32_t le32(uint64_t a) {
    return ld8(a) | (ld8(a + 1) << 8) | (ld8(a + 2) << 16) | (ld8(a + 3) << 24);
}

// readEntry's varint32 (block.go:115-172): up to 5 bytes, the 5th taken whole
__device__ __forceinline__ uint32_t uvarint32(uint64_t &p) {
    uint32_t x = 0;
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t b = ld8(p + i);
        if (b < 128 || i == 4) {
            x |= b << (7 * i);
            p += i + 1;
            return x;
        }
        x |= (b & 0x7fu) << (7 * i);
    }
    return x;
}

// bytes.Compare(a[0:al], b[0:bl]) over device memory
__device__ __forceinline__ int bcmp(uint64_t a, uint32_t al, uint64_t b, uint32_t bl) {
    const uint32_t m = al < bl ? al : bl;
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t x = ld8(a + i), y = ld8(b + i);
        if (x != y) return x < y ? -1 : 1;
    }
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

constexpr uint32_t kShards = 65536;          // HashIndexShardsNum
constexpr uint32_t kHdr = 8;                 // SuccinctHeaderSize
constexpr uint32_t kItemOff = kHdr + kShards * 4;
constexpr uint32_t kItem = 10;               // HashIndexItem64Size
constexpr uint64_t kSearchTrailer = ((1ull << 56) - 1) << 8 | 18;  // MakeSearchKey: SeqNumMax, KindMax

// big-endian fields of the index by dword loads (ldu32: two aligned dwords + v_alignbyte, bytes
// only past `end`): the byte loads they replace made k_get memory-instruction bound
__device__ __forceinline__ uint32_t be32w(uint64_t a, uint64_t end) { return __builtin_bswap32(ldu32(a, end)); }
__device__ __forceinline__ uint32_t be16w(uint64_t a, uint64_t end) { return be32w(a, end) >> 16; }

// HashIndex.Get64 (hash_index.go:399-431); false = not found
__device__ bool get64(uint64_t d, uint64_t len, uint32_t key, uint64_t &val) {
    if (len <= kItemOff) return false;        // SetReader rejects len(d) <= itemOffset
    const uint64_t end = d + len;
    if (be32w(d + 4, end) == 0) return false;  // header.shards <= 0
    const uint32_t hid = key >> 16, lid = key & 0xffffu;
    const uint32_t origin = hid > 0 ? be32w(d + kHdr + (hid - 1) * 4, end) : 0u;
    const uint32_t dest = be32w(d + kHdr + hid * 4, end);
    if (dest <= origin) return false;
    const uint32_t cnt = dest - origin;
    const uint64_t cur = d + kItemOff + (uint64_t)origin * kItem;
    if ((uint64_t)kItemOff + ((uint64_t)origin + cnt) * kItem > len) return false;  // corrupt index: Go would panic
    uint32_t i = 0, j = cnt;
    while (i < j) {
        const uint32_t h = (i + j) >> 1;
        if (be16w(cur + (uint64_t)kItem * h, end) < lid) i = h + 1;
        else j = h;
    }
    if (i < cnt && be16w(cur + (uint64_t)kItem * i, end) == lid) {
        const uint64_t a = cur + (uint64_t)kItem * i + 2;
        val = ((uint64_t)be32w(a, end) << 32) | be32w(a + 4, end);
        return true;
    }
    return false;
}

// readConflict (reader.go:274-289): SeekGE(key) then UserKey == key; returns the
// entry's 8-B block handle or {0, 0}.  Keys are InternalKeys; the search key is
// MakeSearchKey(key) = (key, SeqNumMax, KindMax), ordered by InternalCompare
// (internal.go:108-119): UserKey ascending, then trailer descending.
constexpr uint32_t kMaxChain = 32;  // entries per restart interval (the writer uses 16, block.go:607)

struct Chain {  // the entries since the last restart: full key of entry e = key(e-1)[:sh[e]] || suffix(e)
    uint32_t n;
    uint32_t sh[kMaxChain];
    uint64_t sa[kMaxChain];
    __device__ uint32_t byte_at(uint32_t e, uint32_t idx) const {
        while (idx < sh[e]) e--;  // sh[0] == 0 at the restart: terminates
        return ld8(sa[e] + (idx - sh[e]));
    }
};

// sign of InternalCompare(search key, entry e's key of length kl)
__device__ int cmp_search(const Chain &C, uint32_t e, uint32_t kl, uint64_t key, uint32_t klen) {
    const uint32_t ul = kl >= 8 ? kl - 8 : 0u;  // kl < 8: UserKey nil, trailer Invalid (255)
    const uint32_t m = klen < ul ? klen : ul;
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t x = ld8(key + i), y = C.byte_at(e, i);
        if (x != y) return x < y ? -1 : 1;
    }
    if (klen != ul) return klen < ul ? -1 : 1;
    uint64_t tr = 255;
    if (kl >= 8) {
        tr = 0;
        for (uint32_t b = 0; b < 8; b++) tr |= (uint64_t)C.byte_at(e, ul + b) << (8 * b);
    }
    return kSearchTrailer > tr ? -1 : (kSearchTrailer < tr ? 1 : 0);
}

__device__ void seek_conflict(uint64_t blk, uint32_t blen, uint64_t key, uint32_t klen, uint32_t &off,
                              uint32_t &length) {
    off = 0;
    length = 0;
    if (blen < 4) return;
    const uint32_t nres = le32(blk + blen - 4);
    if (nres == 0 || (uint64_t)4 * (nres + 1) > blen) return;  // newBlockIter: no restart points
    const uint64_t restarts = blk + blen - 4ull * (nres + 1);
    const uint32_t data_end = blen - 4 * (nres + 1);
    Chain C;
    // binary search over the restart points (block.go:281-333); a restart key is stored whole
    uint32_t index = 0, upper = nres;
    while (index < upper) {
        const uint32_t h = (index + upper) >> 1;
        uint64_t p = blk + le32(restarts + 4ull * h) + 1;  // skip shared (== 0, one byte)
        const uint32_t un = uvarint32(p);
        (void)uvarint32(p);
        C.n = 1;
        C.sh[0] = 0;
        C.sa[0] = p;
        if (cmp_search(C, 0, un, key, klen) >= 0) index = h + 1;
        else upper = h;
    }
    uint32_t o = index > 0 ? le32(restarts + 4ull * (index - 1)) : 0u;
    // forward scan (readEntry + Next) until the first entry >= search key
    C.n = 0;
    while (o < data_end) {
        uint64_t p = blk + o;
        const uint32_t sh = uvarint32(p), un = uvarint32(p), vl = uvarint32(p);
        if (sh == 0) C.n = 0;
        if (C.n == kMaxChain) return;  // longer restart interval than any writer of this format emits
        C.sh[C.n] = sh;
        C.sa[C.n] = p;
        const uint32_t e = C.n++;
        const uint32_t kl = sh + un;
        if (cmp_search(C, e, kl, key, klen) <= 0) {  // entry >= search key
            // hit iff UserKey == key (bytes.Equal): same length and bytes
            if (kl >= 8 && kl - 8 == klen) {
                bool eq = true;
                for (uint32_t i = 0; i < klen && eq; i++) eq = ld8(key + i) == C.byte_at(e, i);
                if (eq && vl >= 8) {  // decodeBlockHandle (block.go:26-39)
                    off = le32(p + un);
                    length = le32(p + un + 4);
                }
            }
            return;
        }
        o = (uint32_t)(p + un + vl - blk);
    }
}

// Reader.Get's index path on one opened table: status OK / NOT_FOUND / ILLEGAL_LENGTH and the
// handle rebased to src
__device__ __forceinline__ uint32_t table_lookup(uint64_t base, uint64_t src_len, const bhg_table &t, uint64_t kp,
                                                 uint32_t klen, uint32_t kh, bhg_handle &h) {
    uint64_t v;
    const bool idx_ok = t.index_off <= src_len && t.index_len <= src_len - t.index_off;
    if (!(idx_ok && get64(base + t.index_off, t.index_len, kh, v))) return BHG_ST_NOT_FOUND;
    uint32_t bo = (uint32_t)v, bl = (uint32_t)(v >> 32);  // LE handle bytes (reader.go:215-217)
    if (t.conflict_bh_len != 0 && bo >= t.conflict_bh_off && bl <= t.conflict_bh_len) {
        const bool cf_ok = t.conflict_off <= src_len && t.conflict_bh_len <= src_len - t.conflict_off;
        if (cf_ok) seek_conflict(base + t.conflict_off, t.conflict_bh_len, kp, klen, bo, bl);
        else bo = bl = 0;
        if (bo == 0 && bl == 0) return BHG_ST_ILLEGAL_LENGTH;  // reader.go:224-226
    }
    h = bhg_handle{t.base + bo, bl, 0};
    return BHG_ST_OK;
}

// hash.Fnv32 of the query key, its bytes loaded a dword at a time
__device__ __forceinline__ uint32_t query_hash(uint64_t kp, uint32_t klen) {
    uint32_t kh = BHG_FNV_OFFSET;
    const uint64_t kend = kp + klen;
    uint32_t q = 0;
    for (; q + 16 <= klen; q += 16) {  // four dwords in flight
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < 4; u++) w[u] = ldu32(kp + q + 4 * u, kend);
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int b = 0; b < 4; b++) kh = (kh * BHG_FNV_PRIME) ^ ((w[u] >> (8 * b)) & 0xffu);
    }
    for (; q < klen; q += 4) {
        const uint32_t w = ldu32(kp + q, kend);  // bytes past kend read as 0 and not hashed
        const uint32_t nb = klen - q < 4 ? klen - q : 4u;
#pragma unroll
        for (uint32_t b = 0; b < 4; b++)
            if (b < nb) kh = (kh * BHG_FNV_PRIME) ^ ((w >> (8 * b)) & 0xffu);
    }
    return kh;
}

template <bool HAVE_HASH>
__global__ __launch_bounds__(256) void k_get(const uint8_t *__restrict__ src, uint64_t src_len,
                                             const bhg_table *__restrict__ tables, uint32_t ntables,
                                             const uint8_t *__restrict__ keys, const uint64_t *__restrict__ key_off,
                                             const uint32_t *__restrict__ table_idx, const uint32_t *__restrict__ khash,
                                             uint32_t n, bhg_handle *__restrict__ out_h, uint32_t *__restrict__ out_st) {
    const uint64_t base = (uint64_t)src;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t ti = table_idx[i];
        const uint64_t k0 = key_off[i], k1 = key_off[i + 1];
        const uint64_t kp = (uint64_t)keys + k0;
        const uint32_t klen = (uint32_t)(k1 - k0);
        bhg_handle h = {0, 0, 0};
        uint32_t st = BHG_ST_NOT_FOUND;
        if (ti < ntables) st = table_lookup(base, src_len, tables[ti], kp, klen, HAVE_HASH ? khash[i] : query_hash(kp, klen), h);
        out_h[i] = h;
        out_st[i] = st;
    }
}

// the user key of a stored record (ikeySize at +0, UserKey at +12; ikeySize < 8 -> empty)
__device__ __forceinline__ void rec_user_key(uint64_t p, uint64_t end, uint64_t &kp, uint32_t &kl) {
    const uint32_t ik = p + 4 <= end ? ldu32(p, end) : 0u;
    kl = ik >= 8 ? ik - 8 : 0u;
    kp = p + 12;
    if (kp + kl > end) kl = 0;
}

__device__ __forceinline__ bool keq(uint64_t a, uint32_t al, uint64_t b, uint32_t bl) {
    return al == bl && bcmp(a, al, b, bl) == 0;
}

// Writer.Get's index (writer.go:171-228 over the state updateHash leaves, :285-310): the khash run
// of the sorted record list; one distinct UserKey in the run -> ih.bh = the last add, whatever
// the queried key; two or more (conflict) -> conflictKeys[key] = the last add of that key, or
// nothing.  Returns true with the handle when Writer.Get would read a record.
__device__ bool writer_lookup(uint64_t base, uint64_t end, const bhg_writer_index &w, uint64_t kp, uint32_t klen,
                              uint32_t kh, bhg_handle &h) {
    const bhg_handle *rec = reinterpret_cast<const bhg_handle *>(w.rec);
    const uint32_t *sorted = reinterpret_cast<const uint32_t *>(w.sorted);
    const uint32_t *skh = reinterpret_cast<const uint32_t *>(w.sorted_kh);
    uint32_t lo = 0, hi = w.n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (skh[m] < kh) lo = m + 1; else hi = m;
    }
    uint32_t e = lo;
    while (e < w.n && skh[e] == kh) e++;
    if (e == lo) return false;  // indexHash has no entry: bh zero
    const bhg_handle last = rec[sorted[e - 1]];
    uint64_t lk; uint32_t ll;
    rec_user_key(base + last.offset, end, lk, ll);
    bool conflict = false;
    for (uint32_t q = lo; q + 1 < e && !conflict; q++) {
        uint64_t qk; uint32_t ql;
        rec_user_key(base + rec[sorted[q]].offset, end, qk, ql);
        conflict = !keq(lk, ll, qk, ql);
    }
    bhg_handle bh = {0, 0, 0};
    if (!conflict) {
        bh = last;
    } else {
        for (uint32_t q = e; q > lo; q--) {
            const bhg_handle r = rec[sorted[q - 1]];
            uint64_t qk; uint32_t ql;
            rec_user_key(base + r.offset, end, qk, ql);
            if (keq(kp, klen, qk, ql)) { bh = r; break; }
        }
    }
    if (bh.length == 0) return false;  // bh.Length <= 0: (nil, nil, nil)
    h = bh;
    return true;
}

// golang/snappy v0.0.4 Decode's error checks (decode.go decodedLen, decode_other.go decode) over
// the stream [p, p + n) without producing output: true iff Decode returns err == nil, with the
// decoded length in dlen.  Lane-serial byte loads: it runs only on open-writer hits.
__device__ bool snappy_stream_ok(uint64_t p, uint64_t n, uint64_t &dlen) {
    uint64_t x = 0, hdr = 0;
    uint32_t sh = 0;
    bool ok = false;
    for (uint64_t i = 0; i < n && i < 10; i++) {  // binary.Uvarint; > 0xffffffff -> ErrTooLarge
        const uint32_t b = ld8(p + i);
        if (b < 0x80) {
            if (i == 9 && b > 1) return false;
            x |= (uint64_t)b << sh;
            ok = x <= 0xffffffffull;
            hdr = i + 1;
            break;
        }
        x |= (uint64_t)(b & 0x7f) << sh;
        sh += 7;
    }
    if (!ok) return false;
    dlen = x;
    const uint64_t s0 = p + hdr, se = p + n;
    uint64_t s = s0, d = 0;
    while (s < se) {
        const uint32_t tag = ld8(s);
        uint64_t length, offset = 0;
        if ((tag & 3) == 0) {  // literal
            uint32_t v = tag >> 2, nb = v < 60 ? 0u : v - 59;
            if (s + 1 + nb > se) return false;
            if (nb) {
                v = 0;
                for (uint32_t q = 0; q < nb; q++) v |= (uint32_t)ld8(s + 1 + q) << (8 * q);
            }
            s += 1 + nb;
            length = (uint64_t)v + 1;
            if (length > dlen - d || length > se - s) return false;
            d += length;
            s += length;
            continue;
        }
        const uint32_t nb = (tag & 3) == 1 ? 1u : (tag & 3) == 2 ? 2u : 4u;
        if (s + 1 + nb > se) return false;
        if ((tag & 3) == 1) {
            length = 4 + ((tag >> 2) & 7);
            offset = ((tag & 0xe0u) << 3) | ld8(s + 1);
        } else {
            length = 1 + (tag >> 2);
            for (uint32_t q = 0; q < nb; q++) offset |= (uint64_t)ld8(s + 1 + q) << (8 * q);
        }
        s += 1 + nb;
        if (offset == 0 || d < offset || length > dlen - d) return false;
        d += length;
    }
    return d == dlen;
}

// Writer.Get's read of the record it found (writer.go:190-228): ReadAt inside the file,
// readRecord non-nil (block2.go:57-66), compressor.Decode without error and with a non-nil value
// (snappy.Decode of a 0-length stream returns a nil slice).  Any failure makes Bithash.Get fall
// through to GetFileNumMap -> Reader.Get (bithash.go:102-107).
__device__ bool writer_record_ok(uint64_t base, uint64_t src_len, const bhg_handle &h, int codec) {
    if (h.offset > src_len || (uint64_t)h.length > src_len - h.offset || h.length < 12) return false;
    const uint64_t p = base + h.offset, end = base + src_len;
    const uint32_t k = ldu32(p, end), v = ldu32(p + 4, end);
    if (k == 0 || v == 0 || (uint64_t)12 + k + v != (uint64_t)h.length) return false;
    if (codec != BHG_CODEC_SNAPPY) return true;  // noCompressor.Decode returns the non-empty value
    uint64_t dlen = 0;
    return snappy_stream_ok(p + 12 + k, v, dlen) && dlen != 0;
}

// Bithash.Get (bithash.go:101-119): the open writer of file_num first (Writer.Get, final only
// when it returns a value without error), then GetFileNumMap(fn) (:264-273; 0 ->
// ErrBhFileNumZero) and Reader.Get on that table
template <bool HAVE_HASH>
__global__ __launch_bounds__(256) void k_bithash_get(const uint8_t *__restrict__ src, uint64_t src_len,
                                                     const bhg_writer_index *__restrict__ writers, uint32_t nwriters,
                                                     const bhg_table *__restrict__ tables, uint32_t ntables,
                                                     const uint32_t *__restrict__ fn_map,
                                                     const uint32_t *__restrict__ fn_table, uint32_t fn_count,
                                                     const uint8_t *__restrict__ keys, const uint64_t *__restrict__ key_off,
                                                     const uint32_t *__restrict__ file_nums,
                                                     const uint32_t *__restrict__ khash, int codec, uint32_t n,
                                                     bhg_handle *__restrict__ out_h, uint32_t *__restrict__ out_st) {
    const uint64_t base = (uint64_t)src, end = base + src_len;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t fn = file_nums[i];
        const uint64_t k0 = key_off[i], k1 = key_off[i + 1];
        const uint64_t kp = (uint64_t)keys + k0;
        const uint32_t klen = (uint32_t)(k1 - k0);
        const uint32_t kh = HAVE_HASH ? khash[i] : query_hash(kp, klen);
        bhg_handle h = {0, 0, 0};
        uint32_t st = BHG_ST_NOT_FOUND;
        bool done = false;
        for (uint32_t w = 0; w < nwriters && !done; w++) {
            const bhg_writer_index W = writers[w];
            if (W.file_num == fn) {
                done = writer_lookup(base, end, W, kp, klen, kh, h) && writer_record_ok(base, src_len, h, codec);
                if (done) st = BHG_ST_OK;
                else h = bhg_handle{0, 0, 0};
                break;
            }
        }
        if (!done) {
            const uint32_t dst = fn < fn_count ? fn_map[fn] : 0u;
            if (dst == 0) {
                st = BHG_ST_FILE_NUM_ZERO;
            } else {
                const uint32_t ti = dst < fn_count ? fn_table[dst] : 0xffffffffu;
                if (ti < ntables) st = table_lookup(base, src_len, tables[ti], kp, klen, kh, h);
            }
        }
        out_h[i] = h;
        out_st[i] = st;
    }
}

// record i's khash -> sort key (stable radix sort by the low 32 bits)
__global__ __launch_bounds__(256) void k_widx_keys(const uint32_t *__restrict__ khash, uint32_t n, uint64_t *keys,
                                                   uint32_t *idx) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        keys[i] = khash[i];
        idx[i] = i;
    }
}
__global__ __launch_bounds__(256) void k_widx_lo(const uint64_t *__restrict__ keys, uint32_t n, uint32_t *out) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = (uint32_t)keys[i];
}

}  // namespace

hipError_t launch_get(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_table *tables, uint32_t ntables,
                      const uint8_t *keys, const uint64_t *key_off, const uint32_t *table_idx, const uint32_t *khash,
                      uint32_t n, bhg_handle *out_h, uint32_t *out_st) {
    uint64_t need = (n + 255) / 256;
    uint64_t cap = (uint64_t)L.num_cus * 16;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    if (khash)
        hipLaunchKernelGGL(k_get<true>, dim3(grid), dim3(256), 0, L.stream, src, src_len, tables, ntables, keys,
                           key_off, table_idx, khash, n, out_h, out_st);
    else
        hipLaunchKernelGGL(k_get<false>, dim3(grid), dim3(256), 0, L.stream, src, src_len, tables, ntables, keys,
                           key_off, table_idx, khash, n, out_h, out_st);
    return hipGetLastError();
}

hipError_t launch_bithash_get(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_writer_index *writers,
                              uint32_t nwriters, const bhg_table *tables, uint32_t ntables, const uint32_t *fn_map,
                              const uint32_t *fn_table, uint32_t fn_count, const uint8_t *keys, const uint64_t *key_off,
                              const uint32_t *file_nums, const uint32_t *khash, int codec, uint32_t n,
                              bhg_handle *out_h, uint32_t *out_st) {
    uint64_t need = (n + 255) / 256;
    uint64_t cap = (uint64_t)L.num_cus * 16;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    if (khash)
        hipLaunchKernelGGL(k_bithash_get<true>, dim3(grid), dim3(256), 0, L.stream, src, src_len, writers, nwriters,
                           tables, ntables, fn_map, fn_table, fn_count, keys, key_off, file_nums, khash, codec, n, out_h,
                           out_st);
    else
        hipLaunchKernelGGL(k_bithash_get<false>, dim3(grid), dim3(256), 0, L.stream, src, src_len, writers, nwriters,
                           tables, ntables, fn_map, fn_table, fn_count, keys, key_off, file_nums, khash, codec, n, out_h,
                           out_st);
    return hipGetLastError();
}

size_t writer_index_scratch_bytes(uint32_t n) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    return al(radix_sort_scratch_bytes(n)) + 2 * al((size_t)n * 8) + al((size_t)n * 4);
}

hipError_t launch_writer_index(const Launch &L, const uint32_t *khash, uint32_t n, uint32_t *sorted,
                               uint32_t *sorted_kh, void *scratch) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    uint8_t *s = reinterpret_cast<uint8_t *>(scratch);
    void *sort_buf = s;
    s += al(radix_sort_scratch_bytes(n));
    uint64_t *k = reinterpret_cast<uint64_t *>(s);
    s += al((size_t)n * 8);
    uint64_t *ks = reinterpret_cast<uint64_t *>(s);
    s += al((size_t)n * 8);
    uint32_t *idx = reinterpret_cast<uint32_t *>(s);
    const uint32_t g = lane_grid(L, n ? n : 1, 256);
    hipLaunchKernelGGL(k_widx_keys, dim3(g), dim3(256), 0, L.stream, khash, n, k, idx);
    hipError_t e = launch_radix_sort_pairs(L, k, ks, idx, sorted, n, 32, sort_buf);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_widx_lo, dim3(g), dim3(256), 0, L.stream, ks, n, sorted_kh);
    return hipGetLastError();
}

}  // namespace bhg
