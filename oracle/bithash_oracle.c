/*
 * bithash_oracle.c -- TEST INFRASTRUCTURE ONLY (see bithash_oracle.h).
 *
 * Plain-C restatement of the reference Go path, one function per reference
 * function, each citing the file:line it follows (paths relative to the
 * bitalosdb v2 source tree).  Used as the parity checker for the HIP path and
 * as bench.py's reported-only CPU baseline ("kind": "port").
 */
#include "bithash_oracle.h"

#include <pthread.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

/* ------------------------------------------------------------------ */
/* little-endian helpers (encoding/binary.LittleEndian)                */
/* ------------------------------------------------------------------ */
static inline uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
static inline uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | (uint64_t)le32(p + 4) << 32; }
static inline void put32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void put64(uint8_t *p, uint64_t v) { put32(p, (uint32_t)v); put32(p + 4, (uint32_t)(v >> 32)); }

/* ------------------------------------------------------------------ */
/* internal/crc/crc.go:19-33 -- CRC-32C (Castagnoli) + LevelDB mask     */
/* Go: var table = crc32.MakeTable(crc32.Castagnoli)  (reflected        */
/* polynomial 0x82F63B78); crc32.Update(c, tab, p) = ^update(^c, p).    */
/* ------------------------------------------------------------------ */
static uint32_t crc_tab[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_tab[i] = c;
    }
}

uint32_t bho_crc32c_update(uint32_t crc, const uint8_t *p, size_t n) {
    pthread_once(&crc_once, crc_init);
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; i++) c = crc_tab[(uint8_t)c ^ p[i]] ^ (c >> 8);
    return ~c;
}

/* Go's amd64 Castagnoli path uses the SSE4.2 crc32 instruction; this is the
 * same function computed the same way, used only to make the CPU baseline a
 * fair stand-in for the reference's speed. */
#if defined(__x86_64__)
__attribute__((target("sse4.2")))
static uint32_t crc_hw(uint32_t c, const uint8_t *p, size_t n) {
    while (n && ((uintptr_t)p & 7)) { c = _mm_crc32_u8(c, *p++); n--; }
    uint64_t c64 = c;
    while (n >= 8) { uint64_t w; memcpy(&w, p, 8); c64 = _mm_crc32_u64(c64, w); p += 8; n -= 8; }
    c = (uint32_t)c64;
    while (n--) c = _mm_crc32_u8(c, *p++);
    return c;
}
static int have_sse42(void) { return __builtin_cpu_supports("sse4.2"); }
#endif

uint32_t bho_crc32c_update_hw(uint32_t crc, const uint8_t *p, size_t n) {
#if defined(__x86_64__)
    if (have_sse42()) return ~crc_hw(~crc, p, n);
#endif
    return bho_crc32c_update(crc, p, n);
}

/* crc.go:31-33: uint32(c>>15|c<<17) + 0xa282ead8 */
uint32_t bho_crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
uint32_t bho_crc_masked(const uint8_t *p, size_t n) { return bho_crc_mask(bho_crc32c_update(0, p, n)); }
static uint32_t crc_masked_fast(const uint8_t *p, size_t n) { return bho_crc_mask(bho_crc32c_update_hw(0, p, n)); }

/* ------------------------------------------------------------------ */
/* internal/hash/fnv.go:19-23 -- hash/fnv.New32 = FNV-1 (mul, then xor) */
/* ------------------------------------------------------------------ */
uint32_t bho_fnv32(const uint8_t *p, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; i++) { h *= 16777619u; h ^= p[i]; }
    return h;
}

/* ------------------------------------------------------------------ */
/* golang/snappy v0.0.4 (go.mod:7): encode.go / encode_other.go         */
/* ------------------------------------------------------------------ */
enum { tagLiteral = 0, tagCopy1 = 1, tagCopy2 = 2, tagCopy4 = 3 };
#define SNAPPY_MAX_BLOCK 65536
#define SNAPPY_INPUT_MARGIN (16 - 1)
#define SNAPPY_MIN_NONLITERAL (1 + 1 + SNAPPY_INPUT_MARGIN)

/* encode.go MaxEncodedLen */
int64_t bho_snappy_max_encoded_len(int64_t srcLen) {
    uint64_t n = (uint64_t)srcLen;
    if (n > 0xffffffffull) return -1;
    n = 32 + n + n / 6;
    if (n > 0xffffffffull) return -1;
    return (int64_t)n;
}

static size_t put_uvarint(uint8_t *p, uint64_t x) {
    size_t i = 0;
    while (x >= 0x80) { p[i++] = (uint8_t)x | 0x80; x >>= 7; }
    p[i++] = (uint8_t)x;
    return i;
}

/* encode_other.go emitLiteral */
static size_t emit_literal(uint8_t *dst, const uint8_t *lit, size_t len) {
    size_t i; uint32_t n = (uint32_t)(len - 1);
    if (n < 60) { dst[0] = (uint8_t)(n << 2 | tagLiteral); i = 1; }
    else if (n < (1u << 8)) { dst[0] = 60 << 2 | tagLiteral; dst[1] = (uint8_t)n; i = 2; }
    else { dst[0] = 61 << 2 | tagLiteral; dst[1] = (uint8_t)n; dst[2] = (uint8_t)(n >> 8); i = 3; }
    memcpy(dst + i, lit, len);
    return i + len;
}

/* encode_other.go emitCopy */
static size_t emit_copy(uint8_t *dst, int offset, int length) {
    size_t i = 0;
    while (length >= 68) {
        dst[i + 0] = 63 << 2 | tagCopy2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3; length -= 64;
    }
    if (length > 64) {
        dst[i + 0] = 59 << 2 | tagCopy2; dst[i + 1] = (uint8_t)offset; dst[i + 2] = (uint8_t)(offset >> 8);
        i += 3; length -= 60;
    }
    if (length >= 12 || offset >= 2048) {
        dst[i + 0] = (uint8_t)((length - 1) << 2 | tagCopy2); dst[i + 1] = (uint8_t)offset;
        dst[i + 2] = (uint8_t)(offset >> 8);
        return i + 3;
    }
    dst[i + 0] = (uint8_t)((offset >> 8) << 5 | (length - 4) << 2 | tagCopy1);
    dst[i + 1] = (uint8_t)offset;
    return i + 2;
}

static inline uint32_t snappy_hash(uint32_t u, uint32_t shift) { return (u * 0x1e35a7bdu) >> shift; }

/* encode_other.go encodeBlock */
static size_t encode_block(uint8_t *dst, const uint8_t *src, int len) {
    enum { maxTableSize = 1 << 14, tableMask = maxTableSize - 1 };
    uint32_t shift = 32 - 8;
    for (int tableSize = 1 << 8; tableSize < maxTableSize && tableSize < len; tableSize *= 2) shift--;
    uint16_t table[maxTableSize];
    memset(table, 0, sizeof table);
    int sLimit = len - SNAPPY_INPUT_MARGIN;
    int nextEmit = 0;
    int s = 1;
    uint32_t nextHash = snappy_hash(le32(src + s), shift);
    size_t d = 0;
    for (;;) {
        int skip = 32;
        int nextS = s;
        int candidate = 0;
        for (;;) {
            s = nextS;
            int bytesBetweenHashLookups = skip >> 5;
            nextS = s + bytesBetweenHashLookups;
            skip += bytesBetweenHashLookups;
            if (nextS > sLimit) goto emit_remainder;
            candidate = table[nextHash & tableMask];
            table[nextHash & tableMask] = (uint16_t)s;
            nextHash = snappy_hash(le32(src + nextS), shift);
            if (le32(src + s) == le32(src + candidate)) break;
        }
        d += emit_literal(dst + d, src + nextEmit, (size_t)(s - nextEmit));
        for (;;) {
            int base = s;
            s += 4;
            for (int i = candidate + 4; s < len && src[i] == src[s]; i++, s++) {}
            d += emit_copy(dst + d, base - candidate, s - base);
            nextEmit = s;
            if (s >= sLimit) goto emit_remainder;
            uint64_t x = le64(src + s - 1);
            uint32_t prevHash = snappy_hash((uint32_t)(x >> 0), shift);
            table[prevHash & tableMask] = (uint16_t)(s - 1);
            uint32_t currHash = snappy_hash((uint32_t)(x >> 8), shift);
            candidate = table[currHash & tableMask];
            table[currHash & tableMask] = (uint16_t)s;
            if ((uint32_t)(x >> 8) != le32(src + candidate)) {
                nextHash = snappy_hash((uint32_t)(x >> 16), shift);
                s++;
                break;
            }
        }
    }
emit_remainder:
    if (nextEmit < len) d += emit_literal(dst + d, src + nextEmit, (size_t)(len - nextEmit));
    return d;
}

/* encode.go Encode */
size_t bho_snappy_encode(uint8_t *dst, const uint8_t *src, size_t n) {
    size_t d = put_uvarint(dst, n);
    while (n > 0) {
        size_t plen = n > SNAPPY_MAX_BLOCK ? SNAPPY_MAX_BLOCK : n;
        if (plen < SNAPPY_MIN_NONLITERAL) d += emit_literal(dst + d, src, plen);
        else d += encode_block(dst + d, src, (int)plen);
        src += plen; n -= plen;
    }
    return d;
}

/* decode.go decodedLen + encoding/binary.Uvarint */
int bho_snappy_decoded_len(const uint8_t *src, size_t n, uint64_t *dlen, size_t *hdr) {
    uint64_t x = 0; unsigned s = 0;
    for (size_t i = 0; i < n; i++) {
        uint8_t b = src[i];
        if (i == 10) return -1;                       /* overflow */
        if (b < 0x80) {
            if (i == 9 && b > 1) return -1;           /* overflow */
            x |= (uint64_t)b << s;
            if (x > 0xffffffffull) return -1;         /* ErrCorrupt */
            *dlen = x; *hdr = i + 1;
            return 0;
        }
        x |= (uint64_t)(b & 0x7f) << s;
        s += 7;
    }
    return -1;                                        /* n == 0 */
}

/* decode_other.go decode (0 ok, -1 ErrCorrupt) */
static int snappy_decode_body(uint8_t *dst, uint64_t dlen, const uint8_t *src, uint64_t slen) {
    uint64_t d = 0, s = 0, offset = 0, length = 0;
    while (s < slen) {
        switch (src[s] & 0x03) {
        case tagLiteral: {
            uint32_t x = src[s] >> 2;
            if (x < 60) { s++; }
            else if (x == 60) { s += 2; if (s > slen) return -1; x = src[s - 1]; }
            else if (x == 61) { s += 3; if (s > slen) return -1; x = src[s - 2] | (uint32_t)src[s - 1] << 8; }
            else if (x == 62) { s += 4; if (s > slen) return -1;
                x = src[s - 3] | (uint32_t)src[s - 2] << 8 | (uint32_t)src[s - 1] << 16; }
            else { s += 5; if (s > slen) return -1;
                x = src[s - 4] | (uint32_t)src[s - 3] << 8 | (uint32_t)src[s - 2] << 16 | (uint32_t)src[s - 1] << 24; }
            length = (uint64_t)x + 1;                 /* int is 64-bit: never <= 0 */
            if (length > dlen - d || length > slen - s) return -1;
            memcpy(dst + d, src + s, length);
            d += length; s += length;
            continue;
        }
        case tagCopy1:
            s += 2; if (s > slen) return -1;
            length = 4 + ((src[s - 2] >> 2) & 0x7);
            offset = ((uint32_t)(src[s - 2] & 0xe0) << 3) | src[s - 1];
            break;
        case tagCopy2:
            s += 3; if (s > slen) return -1;
            length = 1 + (src[s - 3] >> 2);
            offset = src[s - 2] | (uint32_t)src[s - 1] << 8;
            break;
        default: /* tagCopy4 */
            s += 5; if (s > slen) return -1;
            length = 1 + (src[s - 5] >> 2);
            offset = src[s - 4] | (uint32_t)src[s - 3] << 8 | (uint32_t)src[s - 2] << 16 | (uint64_t)src[s - 1] << 24;
            break;
        }
        if (offset == 0 || d < offset || length > dlen - d) return -1;
        for (uint64_t i = 0; i < length; i++) dst[d + i] = dst[d - offset + i];   /* forward copy */
        d += length;
    }
    return d == dlen ? 0 : -1;
}

int bho_snappy_decode(uint8_t *dst, uint64_t dlen, const uint8_t *src, size_t n) {
    uint64_t v; size_t hdr;
    if (bho_snappy_decoded_len(src, n, &v, &hdr) != 0 || v != dlen) return -1;
    return snappy_decode_body(dst, dlen, src + hdr, n - hdr);
}

/* ------------------------------------------------------------------ */
/* bithash/block2.go:73-105 block2Writer.set (+ base.InternalKey.Encode)*/
/* ------------------------------------------------------------------ */
size_t bho_record_set(uint8_t *dst, const uint8_t *ukey, size_t uklen, uint64_t trailer,
                      const uint8_t *val, size_t vlen, uint32_t file_num) {
    uint32_t keySize = (uint32_t)(uklen + 8);
    put32(dst + 0, keySize);
    put32(dst + 4, (uint32_t)vlen);
    put32(dst + 8, file_num);
    memcpy(dst + 12, ukey, uklen);
    put64(dst + 12 + uklen, trailer);
    memcpy(dst + 12 + keySize, val, vlen);
    return 12 + keySize + vlen;
}

/* ------------------------------------------------------------------ */
/* One block of Reader.readData (bithash/reader.go:233-272):            */
/*   bh.Length<=0 -> ErrBhIllegalBlockLength; ReadAt short -> error;     */
/*   readRecord (block2.go:57-66, readKV :38-55); compressor.Decode.     */
/* Plus the build's per-record masked CRC32C column.     */
/* ------------------------------------------------------------------ */
static void decode_one(const uint8_t *src, uint64_t src_len, const bho_handle *h, int codec,
                       const uint32_t *expected_crc, uint32_t i, bho_desc *d, uint8_t *out_vals,
                       const uint64_t *out_val_off, int fast_crc) {
    memset(d, 0, sizeof *d);
    if (h->length == 0) { d->status = BHO_ILLEGAL_LENGTH; return; }
    if (h->offset > src_len || (uint64_t)h->length > src_len - h->offset) { d->status = BHO_INCOMPLETE; return; }
    const uint8_t *rec = src + h->offset;
    uint32_t L = h->length;
    d->crc = fast_crc ? crc_masked_fast(rec, L) : bho_crc_masked(rec, L);
    /* readRecordHeader reads buf[0:12]; Go would panic for L < 12 -> RECORD_NIL here */
    if (L < 12) { d->status = BHO_RECORD_NIL; return; }
    uint32_t k = le32(rec), v = le32(rec + 4), fn = le32(rec + 8);
    /* recordLen := int(recordHeaderSize + ikeySize + valueSize); a uint32 wrap
     * would make Go read out of bounds -> treated as RECORD_NIL */
    if (k == 0 || v == 0 || (uint64_t)12 + k + v != (uint64_t)L) { d->status = BHO_RECORD_NIL; return; }
    d->file_num = fn;
    d->key_off = 12;
    if (k >= 8) { d->key_len = k - 8; d->trailer = le64(rec + 12 + k - 8); }
    else { d->key_len = 0; d->trailer = 255; }
    d->fnv1 = bho_fnv32(rec + 12, d->key_len);
    const uint8_t *val = rec + 12 + k;
    if (codec == 0) {                              /* noCompressor.Decode returns src (compress.go:57-59) */
        d->val_off = 12 + k; d->val_len = v;
    } else {                                       /* snappy.Decode(nil, val) (compress.go:83-85) */
        uint64_t dlen; size_t hdr;
        if (bho_snappy_decoded_len(val, v, &dlen, &hdr) != 0 || dlen * 3 > (uint64_t)(v - hdr) * 64) {
            d->status = BHO_SNAPPY_CORRUPT; return;
        }
        uint64_t cap = out_val_off[i + 1] - out_val_off[i];
        if (dlen > cap) { d->status = BHO_SNAPPY_TOO_LARGE; return; }
        if (snappy_decode_body(out_vals + out_val_off[i], dlen, val + hdr, v - hdr) != 0) {
            d->status = BHO_SNAPPY_CORRUPT; return;
        }
        d->val_off = 0; d->val_len = (uint32_t)dlen;
    }
    if (expected_crc && expected_crc[i] != d->crc) d->status = BHO_CRC_MISMATCH;
}

typedef struct {
    const uint8_t *src; uint64_t src_len; const bho_handle *h; uint32_t lo, hi; int codec;
    const uint32_t *expected_crc; bho_desc *out; uint8_t *out_vals; const uint64_t *out_val_off; int fast;
} dec_job;

static void *dec_worker(void *arg) {
    dec_job *j = (dec_job *)arg;
    for (uint32_t i = j->lo; i < j->hi; i++)
        decode_one(j->src, j->src_len, j->h + i, j->codec, j->expected_crc, i, j->out + i, j->out_vals,
                   j->out_val_off, j->fast);
    return NULL;
}

/* nthreads <= 0: single thread, reference-definition CRC (checker mode).
 * nthreads >= 1: that many threads, SSE4.2 CRC (baseline mode). */
void bho_decode_batch(const uint8_t *src, uint64_t src_len, const bho_handle *h, uint32_t n, int codec,
                      const uint32_t *expected_crc, bho_desc *out, uint8_t *out_vals,
                      const uint64_t *out_val_off, int nthreads) {
    int fast = nthreads >= 1;
    int nt = nthreads < 1 ? 1 : nthreads;
    if (nt > 256) nt = 256;
    pthread_t tid[256];
    dec_job jobs[256];
    for (int t = 0; t < nt; t++) {
        jobs[t] = (dec_job){src, src_len, h, (uint32_t)((uint64_t)n * t / nt), (uint32_t)((uint64_t)n * (t + 1) / nt),
                            codec, expected_crc, out, out_vals, out_val_off, fast};
    }
    if (nt == 1) { dec_worker(&jobs[0]); return; }
    for (int t = 0; t < nt; t++) pthread_create(&tid[t], NULL, dec_worker, &jobs[t]);
    for (int t = 0; t < nt; t++) pthread_join(tid[t], NULL);
}

/* Reader.readData as the reference runs it (reader.go:251): one ReadAt
 * (pread) of bh.Length bytes per block into a buffer, then readRecord /
 * Decode on that buffer.  A short read -> ErrBhReadAtIncomplete
 * (BHO_INCOMPLETE).  Baseline mode only (SSE4.2 CRC), codec NONE. */
typedef struct {
    int fd; const bho_handle *h; uint32_t lo, hi; const uint32_t *expected_crc; bho_desc *out;
} pread_job;

static void *pread_worker(void *arg) {
    pread_job *j = (pread_job *)arg;
    size_t cap = 1 << 16;
    uint8_t *buf = (uint8_t *)malloc(cap);
    for (uint32_t i = j->lo; i < j->hi && buf; i++) {
        const bho_handle *h = j->h + i;
        if (h->length > cap) {
            free(buf);
            cap = h->length;
            buf = (uint8_t *)malloc(cap);
            if (!buf) break;
        }
        ssize_t got = h->length ? pread(j->fd, buf, h->length, (off_t)h->offset) : 0;
        if (got < 0) got = 0;
        bho_handle local = {0, h->length, 0};
        decode_one(buf, (uint64_t)got, &local, 0, j->expected_crc, i, j->out + i, NULL, NULL, 1);
    }
    free(buf);
    return NULL;
}

void bho_decode_batch_pread(int fd, const bho_handle *h, uint32_t n, const uint32_t *expected_crc, bho_desc *out,
                            int nthreads) {
    int nt = nthreads < 1 ? 1 : nthreads;
    if (nt > 256) nt = 256;
    pthread_t tid[256];
    pread_job jobs[256];
    for (int t = 0; t < nt; t++)
        jobs[t] = (pread_job){fd, h, (uint32_t)((uint64_t)n * t / nt), (uint32_t)((uint64_t)n * (t + 1) / nt),
                              expected_crc, out};
    if (nt == 1) { pread_worker(&jobs[0]); return; }
    for (int t = 0; t < nt; t++) pthread_create(&tid[t], NULL, pread_worker, &jobs[t]);
    for (int t = 0; t < nt; t++) pthread_join(tid[t], NULL);
}

void bho_decode_sizes(const uint8_t *src, uint64_t src_len, const bho_handle *h, uint32_t n, uint64_t *out) {
    for (uint32_t i = 0; i < n; i++) {
        out[i] = 0;
        if (h[i].length < 12 || h[i].offset > src_len || (uint64_t)h[i].length > src_len - h[i].offset) continue;
        const uint8_t *rec = src + h[i].offset;
        uint32_t k = le32(rec), v = le32(rec + 4);
        if (k == 0 || v == 0 || (uint64_t)12 + k + v != (uint64_t)h[i].length) continue;
        uint64_t dlen; size_t hdr;
        if (bho_snappy_decoded_len(rec + 12 + k, v, &dlen, &hdr) != 0 || dlen * 3 > (uint64_t)(v - hdr) * 64) continue;
        out[i] = dlen;
    }
}

/* ------------------------------------------------------------------ */
/* BithashWriter.Add sequence: bithash/bithash_writer.go:25-67 over     */
/* Writer.Add/add (bithash/writer.go:230-283).                          */
/* ------------------------------------------------------------------ */
#define MAX_KEY_SIZE (33u << 10)
#define MAX_VALUE_SIZE (256u << 20)
#define DATA_MAX_SIZE (0xFFFFFFFFu - (256u << 20))

static int encode_seq(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                      const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                      const uint32_t *file_nums, int max_tables, uint32_t init_size, uint64_t table_max,
                      uint8_t *out, uint64_t *out_len, uint64_t *out_pos, uint32_t *out_bh_off,
                      uint32_t *out_bh_len, uint32_t *out_table, uint32_t *fnv, uint32_t *crc,
                      uint32_t *status, uint32_t *out_table_start, int fast);

int bho_encode_batch(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                     const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                     const uint32_t *file_nums, int max_tables, uint32_t init_size, uint64_t table_max,
                     uint8_t *out, uint64_t *out_len, uint64_t *out_pos, uint32_t *out_bh_off,
                     uint32_t *out_bh_len, uint32_t *out_table, uint32_t *fnv, uint32_t *crc,
                     uint32_t *status, uint32_t *out_table_start) {
    return encode_seq(keys, key_off, trailers, vals, val_off, n, codec, file_nums, max_tables, init_size,
                      table_max, out, out_len, out_pos, out_bh_off, out_bh_len, out_table, fnv, crc, status,
                      out_table_start, 0);
}

/* CPU baseline of the encode path on many cores (reported only): nthreads
 * independent BithashWriters (the reference serialises Adds per Writer,
 * writers run concurrently), thread t taking the contiguous pair range
 * [n t / T, n (t+1) / T) -- golang/snappy Encode + FNV-1 + record pack +
 * masked CRC-32C (SSE4.2) per pair, 128 MiB table splits.  Returns the total
 * bytes written, or 0 on allocation failure. */
typedef struct {
    const uint8_t *keys; const uint64_t *key_off; const uint64_t *trailers; const uint8_t *vals;
    const uint64_t *val_off; uint32_t lo, hi; int codec; uint64_t table_max; uint64_t written; int fail;
} enc_job;

static void *enc_worker(void *arg) {
    enc_job *j = (enc_job *)arg;
    uint32_t m = j->hi - j->lo;
    size_t cap = 1;
    for (uint32_t i = j->lo; i < j->hi; i++)
        cap += 20 + (size_t)(j->key_off[i + 1] - j->key_off[i]) +
               (size_t)bho_snappy_max_encoded_len((int64_t)(j->val_off[i + 1] - j->val_off[i])) + 16;
    uint8_t *out = (uint8_t *)malloc(cap);
    uint64_t *pos = (uint64_t *)malloc(((size_t)m + 1) * 8);
    uint32_t *u32 = (uint32_t *)malloc(((size_t)m + 1) * 4 * 6 + 4096 * 8);
    if (!out || !pos || !u32) { j->fail = 1; free(out); free(pos); free(u32); return NULL; }
    uint32_t *fns = u32 + ((size_t)m + 1) * 6, *tstart = fns + 4096;
    for (uint32_t t = 0; t < 4096; t++) fns[t] = t + 1;
    uint64_t len = 0;
    /* offsets are absolute: pass the range's own base pointers */
    const uint64_t *ko = j->key_off + j->lo, *vo = j->val_off + j->lo;
    uint64_t *kor = (uint64_t *)malloc(((size_t)m + 1) * 16);
    if (!kor) { j->fail = 1; free(out); free(pos); free(u32); return NULL; }
    uint64_t *vor = kor + m + 1;
    for (uint32_t i = 0; i <= m; i++) { kor[i] = ko[i] - ko[0]; vor[i] = vo[i] - vo[0]; }
    size_t q = (size_t)m + 1;
    int nt = encode_seq(j->keys + ko[0], kor, j->trailers + j->lo, j->vals + vo[0], vor, m, j->codec, fns, 4096, 0,
                        j->table_max, out, &len, pos, u32, u32 + q, u32 + 2 * q, u32 + 3 * q, u32 + 4 * q,
                        u32 + 5 * q, tstart, 1);
    j->fail = nt < 0;
    j->written = len;
    free(kor); free(out); free(pos); free(u32);
    return NULL;
}

uint64_t bho_encode_batch_mt(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                             const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                             uint64_t table_max, int nthreads) {
    int nt = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
    pthread_t tid[256];
    enc_job jobs[256];
    for (int t = 0; t < nt; t++)
        jobs[t] = (enc_job){keys, key_off, trailers, vals, val_off, (uint32_t)((uint64_t)n * t / nt),
                            (uint32_t)((uint64_t)n * (t + 1) / nt), codec, table_max, 0, 0};
    if (nt == 1) enc_worker(&jobs[0]);
    else {
        for (int t = 0; t < nt; t++) pthread_create(&tid[t], NULL, enc_worker, &jobs[t]);
        for (int t = 0; t < nt; t++) pthread_join(tid[t], NULL);
    }
    uint64_t total = 0;
    for (int t = 0; t < nt; t++) {
        if (jobs[t].fail) return 0;
        total += jobs[t].written;
    }
    return total;
}

static int encode_seq(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                      const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                      const uint32_t *file_nums, int max_tables, uint32_t init_size, uint64_t table_max,
                      uint8_t *out, uint64_t *out_len, uint64_t *out_pos, uint32_t *out_bh_off,
                      uint32_t *out_bh_len, uint32_t *out_table, uint32_t *fnv, uint32_t *crc,
                      uint32_t *status, uint32_t *out_table_start, int fast) {
    int t = 0;
    uint32_t size = init_size;          /* meta.Size == currentOffset for a data-only writer */
    uint64_t pos = 0;
    uint8_t *cbuf = NULL; size_t ccap = 0;
    if (max_tables < 1) return -1;
    out_table_start[0] = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *uk = keys + key_off[i];
        size_t uklen = (size_t)(key_off[i + 1] - key_off[i]);
        const uint8_t *v = vals + val_off[i];
        size_t vlen = (size_t)(val_off[i + 1] - val_off[i]);
        const uint8_t *c = v; size_t clen = vlen;
        if (codec == 1) {                                  /* writer.go:236-244 */
            size_t need = (size_t)bho_snappy_max_encoded_len((int64_t)vlen);
            if (need > ccap) { free(cbuf); ccap = need; cbuf = (uint8_t *)malloc(ccap); }
            clen = bho_snappy_encode(cbuf, v, vlen); c = cbuf;
        }
        fnv[i] = bho_fnv32(uk, uklen);                     /* writer.go:246 */
        out_pos[i] = UINT64_MAX; out_bh_off[i] = out_bh_len[i] = 0; out_table[i] = (uint32_t)t; crc[i] = 0;
        size_t keySize = uklen + 8;                        /* writer.go:258-265 */
        if (keySize > MAX_KEY_SIZE) { status[i] = BHO_KEY_TOO_LARGE; continue; }
        if (clen > MAX_VALUE_SIZE) { status[i] = BHO_VALUE_TOO_LARGE; continue; }
        uint32_t kvSize = (uint32_t)(keySize + clen + 12);
        if ((uint32_t)(size + kvSize) > DATA_MAX_SIZE) { status[i] = BHO_DATA_MAX_EXCEEDED; continue; }
        size_t L = bho_record_set(out + pos, uk, uklen, trailers[i], c, clen, file_nums[t]);
        status[i] = BHO_OK;
        out_pos[i] = pos;
        out_bh_off[i] = size; out_bh_len[i] = (uint32_t)L;  /* BlockHandle{currentOffset, length} */
        crc[i] = fast ? crc_masked_fast(out + pos, L) : bho_crc_masked(out + pos, L);
        pos += L;
        size += (uint32_t)L;
        if ((uint64_t)size >= table_max) {                  /* maybeSplitTable: isWriteFull after add */
            if (t + 1 >= max_tables) { free(cbuf); return -1; }
            t++;
            out_table_start[t] = i + 1;
            size = 0;
        }
    }
    free(cbuf);
    *out_len = pos;
    return t + 1;
}

/* ------------------------------------------------------------------ */
/* Sequential record scans over a table's bytes:                        */
/*  mode 0: TableIterator.findEntry (bithash/table.go:358-395)           */
/*  mode 1: Writer.rebuild          (bithash/writer.go:539-583)          */
/* ------------------------------------------------------------------ */
int64_t bho_scan_region(const uint8_t *data, uint64_t len, int mode, bho_handle *out, uint64_t max,
                        uint64_t *end_offset) {
    uint64_t off = 0; int64_t cnt = 0;
    for (;;) {
        if (len - off < 12 || off > len) break;            /* short header read */
        uint32_t k = le32(data + off), v = le32(data + off + 4);
        if (mode == 0) {
            if (k == 0 || v == 0) break;
            uint32_t kvLen = k + v;                         /* uint32 arithmetic */
            if (len - off - 12 < kvLen) break;              /* short kv read -> err */
            if ((uint64_t)cnt < max) { out[cnt].offset = off; out[cnt].length = 12 + kvLen; out[cnt].pad = 0; }
            cnt++;
            off += 12 + (uint64_t)kvLen;
        } else {
            if (k == 0) break;
            if (len - off - 12 < k) break;                  /* short key read */
            uint32_t recLen = 12 + k + v;                   /* uint32 arithmetic */
            if ((uint64_t)cnt < max) { out[cnt].offset = off; out[cnt].length = recLen; out[cnt].pad = 0; }
            cnt++;
            off += 12 + (uint64_t)(uint32_t)(k + v);
        }
    }
    if (end_offset) *end_offset = off;
    return cnt;
}
