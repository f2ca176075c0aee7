/*
 * bithash_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the zuoyebang/bitalosdb v2 bithash record codec path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this; the product library (bitalosdb_amd/) never links or calls it.
 *
 * Parity pinning: the Go reference cannot be built here (no Go toolchain,
 * GOEXPERIMENT=arenas, un-vendored golang/snappy v0.0.4).  This restatement
 * is pinned by the reference's own asserted known answers (see
 * tests/test_oracle_known_answers.py: K1 table split sizes / offsets,
 * K2 FNV-1 collision pairs + conflict counts, K3 updateHash semantics,
 * K4 ordered scan) plus standard-algorithm KATs (CRC-32C, FNV-1) and, for
 * snappy decode/encode validity, interop with pyarrow's Google C++ snappy.
 * golang/snappy *encode* byte-identity is "parity unpinned" (no golden
 * vector for it exists in the reference or in this container).
 */
#ifndef BITHASH_ORACLE_H
#define BITHASH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-block status codes (same numbering as include/bithashgpu.h). */
enum {
    BHO_OK = 0,
    BHO_RECORD_NIL = 1,       /* readRecord -> nil  (bithash/block2.go:57-66) */
    BHO_ILLEGAL_LENGTH = 2,   /* bh.Length <= 0     (bithash/reader.go:234-236) */
    BHO_INCOMPLETE = 3,       /* ReadAt n != length (bithash/reader.go:255-258) */
    BHO_SNAPPY_CORRUPT = 4,   /* snappy.ErrCorrupt */
    BHO_SNAPPY_TOO_LARGE = 5, /* decoded length exceeds caller capacity */
    BHO_CRC_MISMATCH = 6,     /* build extension: expected_crc[] given and differs */
    BHO_KEY_TOO_LARGE = 7,    /* ErrBhKeyTooLarge   (bithash/writer.go:260-262) */
    BHO_VALUE_TOO_LARGE = 8,  /* ErrBhValueTooLarge (bithash/writer.go:262-264) */
    BHO_DATA_MAX_EXCEEDED = 9 /* writer.go:266-269 */
};

typedef struct {
    uint64_t offset;
    uint32_t length;
    uint32_t pad;
} bho_handle;

typedef struct {
    uint32_t key_off, key_len; /* user key view, relative to record start */
    uint32_t val_off, val_len; /* none: value view rel. to record start; snappy: decoded len, val_off 0 */
    uint64_t trailer;          /* ikey trailer; 255 (InternalKeyKindInvalid) if ikeySize < 8 */
    uint32_t file_num;
    uint32_t fnv1;             /* hash.Fnv32(UserKey) */
    uint32_t crc;              /* crc.New(record[0:L]).Value() */
    uint32_t status;
} bho_desc;

/* ---- primitives ---- */
uint32_t bho_crc32c_update(uint32_t crc, const uint8_t *p, size_t n);  /* Go crc32.Update(crc, Castagnoli, p) */
uint32_t bho_crc32c_update_hw(uint32_t crc, const uint8_t *p, size_t n);/* SSE4.2 form, same result */
uint32_t bho_crc_mask(uint32_t crc);                                    /* crc.CRC.Value() */
uint32_t bho_crc_masked(const uint8_t *p, size_t n);                    /* crc.New(p).Value() */
uint32_t bho_fnv32(const uint8_t *p, size_t n);                         /* hash.Fnv32 (FNV-1) */

/* ---- snappy (golang/snappy v0.0.4 semantics) ---- */
int64_t bho_snappy_max_encoded_len(int64_t n);
size_t bho_snappy_encode(uint8_t *dst, const uint8_t *src, size_t n);
/* returns 0 ok, -1 corrupt; *dlen = decoded length, *hdr = varint bytes */
int bho_snappy_decoded_len(const uint8_t *src, size_t n, uint64_t *dlen, size_t *hdr);
/* returns 0 ok, -1 corrupt; dst must hold dlen bytes */
int bho_snappy_decode(uint8_t *dst, uint64_t dlen, const uint8_t *src, size_t n);

/* ---- record ---- */
size_t bho_record_set(uint8_t *dst, const uint8_t *ukey, size_t uklen, uint64_t trailer,
                      const uint8_t *val, size_t vlen, uint32_t file_num);

/* ---- batch decode: checker for the GPU path (and the CPU baseline) ----
 * codec 0 = NoCompressor, 1 = snappy.  For snappy, out_val_off has n+1
 * entries and block i's capacity is out_val_off[i+1]-out_val_off[i]. */
void bho_decode_batch(const uint8_t *src, uint64_t src_len, const bho_handle *h, uint32_t n,
                      int codec, const uint32_t *expected_crc, bho_desc *out,
                      uint8_t *out_vals, const uint64_t *out_val_off, int nthreads);
/* Reader.readData with one pread() per block into a buffer (reader.go:251),
 * codec 0, SSE4.2 CRC: the CPU baseline that pays the reference's per-block
 * ReadAt.  fd is an open descriptor of the table bytes. */
void bho_decode_batch_pread(int fd, const bho_handle *h, uint32_t n, const uint32_t *expected_crc, bho_desc *out,
                            int nthreads);
/* snappy decoded sizes (0 for blocks whose header / varint is invalid) */
void bho_decode_sizes(const uint8_t *src, uint64_t src_len, const bho_handle *h, uint32_t n,
                      uint64_t *out_sizes);

/* ---- batch encode (BithashWriter.Add sequence) ----
 * keys: concatenated user keys, key_off[n+1]; vals: concatenated raw
 * values, val_off[n+1]; trailers[n].  Tables: records are appended to
 * table t (file number file_nums[t]); the first table starts at
 * init_size bytes (its currentOffset == meta.Size); after every
 * successful add, meta.Size >= table_max starts the next table at 0.
 * Outputs: out (all records of all tables concatenated), out_pos[i]
 * (position of record i in out, or UINT64_MAX if its add failed),
 * out_bh_off/out_bh_len (BlockHandle inside its table), out_table[i],
 * fnv[i], crc[i], status[i]; out_table_start[t] = first record of
 * table t; returns number of tables used (>=1) or -1 if max_tables
 * is too small. *out_len = bytes written. */
/* reported-only CPU baseline: nthreads independent writers over contiguous pair ranges */
uint64_t bho_encode_batch_mt(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                             const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                             uint64_t table_max, int nthreads);
int bho_encode_batch(const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                     const uint8_t *vals, const uint64_t *val_off, uint32_t n, int codec,
                     const uint32_t *file_nums, int max_tables, uint32_t init_size,
                     uint64_t table_max, uint8_t *out, uint64_t *out_len, uint64_t *out_pos,
                     uint32_t *out_bh_off, uint32_t *out_bh_len, uint32_t *out_table,
                     uint32_t *fnv, uint32_t *crc, uint32_t *status, uint32_t *out_table_start);

/* ---- sequential data-region scan (TableIterator.findEntry / Writer.rebuild) ----
 * mode 0: TableIterator (stop when ikeySize==0 or valueSize==0, or short read)
 * mode 1: rebuild       (stop when ikeySize==0, or short header / key read)
 * returns number of records; writes handles (offset, length) up to max. */
int64_t bho_scan_region(const uint8_t *data, uint64_t len, int mode, bho_handle *out, uint64_t max,
                        uint64_t *end_offset);

#ifdef __cplusplus
}
#endif
#endif
