/*
 * bithashgpu.h -- C-ABI of the MI355X (gfx950) bithash block codec.
 *
 * This is the drop-in boundary a Go (cgo) caller binds.
 * Plain C types only: pointers, sizes, PODs.  No HIP/torch types appear in
 * any signature; streams are passed as opaque `void*` (a hipStream_t, or
 * NULL for the context's own stream).
 *
 * A "bithash block" is one data record of a .bht table file
 * (bithash/block2.go:26,31-36,73-105):
 *
 *     u32 ikeySize | u32 valueSize | u32 fileNum | ikey[ikeySize] | value[valueSize]
 *     ikey = userKey || u64 LE trailer (seq<<8 | kind)     (internal/base/internal.go:67-72,121-124)
 *
 * addressed by BlockHandle{Offset u32, Length u32} (bithash/block.go:26-39).
 * Blocks are independent: the batch entry points decode/encode N of them in
 * one launch sequence.  Unless a function says otherwise, every buffer
 * pointer is DEVICE memory (device-resident path); *_host variants take
 * host memory and include the H2D/D2H copies (end-to-end path).
 *
 * Ownership: the library never frees caller memory.  Device scratch is
 * allocated per call from the context's stream-ordered memory pool and freed
 * on the call's stream after its last kernel (hipMallocFromPoolAsync /
 * hipFreeAsync), so concurrent calls never share scratch.  Errors: functions return 0 (BHG_OK) or a negative
 * BHG_E* code; bhg_last_error() gives the text.  Nothing aborts or throws
 * across this boundary.  Per-block outcomes are reported in status columns
 * (BHG_ST_*), mapped 1:1 onto the reference's Go errors.
 *
 * Threading: a bhg_ctx may be used from several host threads on distinct
 * streams; calls on one stream are ordered.  The *_host entry points are
 * synchronous and serialise on the context (they own its staging buffers).
 * Multi-GPU: one ctx per device.
 */
#ifndef BITHASHGPU_H
#define BITHASHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BHG_ABI_VERSION 3  /* 3: bhg_bithash_get_batch gained its codec argument (round 5) */

/* ---- API return codes ---- */
#define BHG_OK 0
#define BHG_EINVAL (-1)     /* bad argument (null pointer, n too large, bad codec) */
#define BHG_EHIP (-2)       /* HIP runtime error */
#define BHG_ENOMEM (-3)     /* device allocation failed */
#define BHG_ENODEV (-4)     /* no such device / no GPU */
#define BHG_ECAPACITY (-5)  /* caller output buffer too small */

/* ---- codecs: internal/compress/compress.go:21-24 (CompressTypeNo / CompressTypeSnappy) ---- */
#define BHG_CODEC_NONE 0
#define BHG_CODEC_SNAPPY 1

/* ---- per-block status (decode) / per-record status (encode) ---- */
#define BHG_ST_OK 0
#define BHG_ST_RECORD_NIL 1        /* readRecord -> nil: ErrBhReadRecordNil (block2.go:57-66, reader.go:260-264, error.go) */
#define BHG_ST_ILLEGAL_LENGTH 2    /* bh.Length <= 0: ErrBhIllegalBlockLength (reader.go:234-236) */
#define BHG_ST_INCOMPLETE 3        /* handle past end of src: ReadAt short / io.EOF (reader.go:251-258) */
#define BHG_ST_SNAPPY_CORRUPT 4    /* snappy.ErrCorrupt (compress.go:83-85) */
#define BHG_ST_SNAPPY_TOO_LARGE 5  /* decoded length exceeds the output slot given to the block */
#define BHG_ST_CRC_MISMATCH 6      /* build extension: expected_crc given and != computed */
#define BHG_ST_KEY_TOO_LARGE 7     /* ErrBhKeyTooLarge  (writer.go:260-261) */
#define BHG_ST_VALUE_TOO_LARGE 8   /* ErrBhValueTooLarge (writer.go:262-263) */
#define BHG_ST_DATA_MAX_EXCEEDED 9 /* "bithash: panic add exceed data max size" (writer.go:266-269) */
#define BHG_ST_NOT_FOUND 10        /* HashIndex miss: ErrBhNotFound (reader.go:210-213) */
#define BHG_ST_NO_SPACE 11         /* encode: the record does not fit in out_cap (or max_tables ran out);
                                      nothing was written for it -- grow the buffer and re-run */
#define BHG_ST_SKIPPED 12          /* encode: live[i] == 0, the compaction filter dropped the record
                                      (bitree/bithash.go:225-228); not an error */
#define BHG_ST_FILE_NUM_ZERO 13    /* Bithash.Get: GetFileNumMap(fn) == 0 -> ErrBhFileNumZero
                                      (bithash.go:109-111, 264-273) */

/* BlockHandle (block.go:26-39) with the offset widened to 64 bits so one
 * batch may span many concatenated/mmap'd table files. 16 B. */
typedef struct bhg_handle {
    uint64_t offset;
    uint32_t length;
    uint32_t pad;
} bhg_handle;

/* One decoded block (40 B).  Mirrors readRecord's (*InternalKey, value,
 * FileNum) (block2.go:57-66) plus the build's CRC column:
 *   key_off/key_len : UserKey view, relative to the record start (12, ikeySize-8);
 *                     key_len = 0 when ikeySize < 8 (UserKey nil)
 *   val_off/val_len : codec NONE -> zero-copy value view relative to the record
 *                     start (noCompressor.Decode returns src, compress.go:57-59);
 *                     codec SNAPPY -> val_off = 0, val_len = decoded length, the
 *                     bytes at out_vals + out_val_off[i]
 *   trailer         : ikey trailer u64 (seq<<8|kind); 255 (InternalKeyKindInvalid)
 *                     when ikeySize < 8 (base.DecodeInternalKey)
 *   file_num        : header fileNum
 *   fnv1            : hash.Fnv32(UserKey) (internal/hash/fnv.go:19-23, FNV-1)
 *   crc             : crc.New(record[0:L]).Value() -- masked CRC-32C (internal/crc/crc.go:19-33)
 *                     computed whenever the handle lies inside src
 *   status          : BHG_ST_*
 * For RECORD_NIL / ILLEGAL_LENGTH / INCOMPLETE every field except crc and
 * status is 0.  For SNAPPY_* the key fields are filled, val_off/val_len 0, and the block's
 * slot in out_vals (out_val_off[i] .. [i+1]) holds unspecified bytes. */
typedef struct bhg_desc {
    uint32_t key_off, key_len;
    uint32_t val_off, val_len;
    uint64_t trailer;
    uint32_t file_num;
    uint32_t fnv1;
    uint32_t crc;
    uint32_t status;
} bhg_desc;

typedef struct bhg_ctx bhg_ctx;

/* ---- context / device ---- */
int bhg_abi_version(void);
int bhg_device_count(void);
/* device: HIP ordinal; flags: reserved (0).  Returns NULL on failure. */
bhg_ctx *bhg_create(int device, int flags);
void bhg_destroy(bhg_ctx *ctx);
const char *bhg_last_error(const bhg_ctx *ctx);
/* the context's own stream (a hipStream_t) */
void *bhg_stream(bhg_ctx *ctx);
int bhg_stream_sync(bhg_ctx *ctx, void *stream);

/* ---- memory helpers (so a cgo caller needs no HIP headers) ---- */
void *bhg_malloc_device(bhg_ctx *ctx, uint64_t bytes);
int bhg_free_device(bhg_ctx *ctx, void *p);
void *bhg_malloc_host(bhg_ctx *ctx, uint64_t bytes); /* pinned */
int bhg_free_host(bhg_ctx *ctx, void *p);
int bhg_memcpy_h2d(bhg_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
int bhg_memcpy_d2h(bhg_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
int bhg_memset_device(bhg_ctx *ctx, void *dst, int value, uint64_t bytes, void *stream);

/* ---- batch decode (device-resident) ----
 * Replaces, per block, Reader.readData's readRecord + compressor.Decode
 * (bithash/reader.go:233-272, bithash/writer.go:215-222 for open tables,
 * block2.go:57-66, compress.go:57-59 / 83-85), batched; adds FNV-1 of the
 * user key (hash.Fnv32, needed by Writer.rebuild writer.go:575 and compaction
 * bitree/bithash.go:224) and the masked CRC-32C of the record.
 *   src, src_len     : bytes the handles index into (e.g. concatenated .bht files)
 *   handles[n]       : block handles (offset relative to src)
 *   codec            : BHG_CODEC_NONE or BHG_CODEC_SNAPPY
 *   expected_crc     : nullable; if given, mismatching OK blocks -> BHG_ST_CRC_MISMATCH
 *   out_desc[n]      : descriptors
 *   SNAPPY only:
 *   out_val_off[n+1] : written by the library: exclusive scan of the decoded
 *                      lengths; out_val_off[n] = total bytes needed
 *   out_vals, out_vals_cap : decoded values; a block whose slot would end past
 *                      out_vals_cap gets BHG_ST_SNAPPY_TOO_LARGE.
 *                      out_vals NULL = sizing pass: only the header/CRC pass
 *                      and the scan run; descriptors then hold the header
 *                      pass's provisional val_off (compressed payload offset
 *                      in the record) and val_len (decoded length).
 * Asynchronous on `stream` (no host synchronisation inside).  All pointers
 * device memory. */
int bhg_decode_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                     uint32_t n, int codec, const uint32_t *expected_crc, bhg_desc *out_desc,
                     uint8_t *out_vals, uint64_t out_vals_cap, uint64_t *out_val_off, void *stream);

/* Same contract with HOST buffers (may be pageable, bhg_malloc_host or
 * bhg_host_register'ed): copies in, decodes, copies out; synchronous.  This
 * is the end-to-end path (mmap'd .bht -> H2D -> kernel -> D2H).  For codec
 * NONE with handles sorted by offset (table scans, compaction) the batch is
 * pipelined in <= 64 MiB chunks over 3 streams, so H2D, kernels and D2H
 * overlap (pin src and reuse a pinned out_desc for the link rate); with
 * unsorted handles a page-locked + mapped src (bhg_host_register,
 * bhg_malloc_host) is decoded in place over PCIe with no staging copy
 * (out_desc / handles / expected_crc used in place too when mapped);
 * otherwise src is copied whole first.  SNAPPY with handles sorted by offset
 * (every record within 64 MiB) and out_vals given: pipelined in <= 64 MiB src
 * chunks on two streams, chunk k + 1's H2D under chunk k's values, offsets and
 * descriptors coming back; a page-locked + mapped out_vals is written by a copy
 * kernel, a pageable one through page-locked staging and host copy threads
 * (pin src and out_vals for the link rate).  Otherwise SNAPPY stages src
 * whole in HBM.  SNAPPY: device value buffers are sized from the scanned totals
 * (not from out_vals_cap); out_vals NULL returns only out_val_off (the sizing
 * pass). */
int bhg_decode_batch_host(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                          uint32_t n, int codec, const uint32_t *expected_crc, bhg_desc *out_desc,
                          uint8_t *out_vals, uint64_t out_vals_cap, uint64_t *out_val_off);

/* Page-lock (pin) a caller host range, e.g. an mmap'd .bht file, and map it
 * into the device address space (hipHostRegister, mapped + portable): the
 * *_host paths then read it in place (NoCompressor) or copy it by DMA at the
 * link rate instead of through pageable staging.  Unregister before unmapping. */
int bhg_host_register(bhg_ctx *ctx, void *p, uint64_t bytes);
int bhg_host_unregister(bhg_ctx *ctx, void *p);

/* ---- primitives, batched (device) ----
 * crc.New(src[h.offset : h.offset+h.length]).Value() for each handle
 * (internal/crc/crc.go:23-33; the indexhash_checksum of writer.go:477 is one
 * such range).  Handles past src_len give 0. */
int bhg_crc32c_masked_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                            uint32_t n, uint32_t *out_crc, void *stream);
/* Same result as bhg_crc32c_masked_batch, each range spread over up to 64 workgroups: for
 * LONG ranges, e.g. verifying each table's indexhash_checksum
 * (bithash/writer.go:476-478 writes crc.New(indexhash_data).Value() as decimal;
 * bithash/reader.go:162-190 (readIndexHash) reads only indexhash_data, never the checksum -- SURVEY
 * 8(a) A6(ii) adds the check).  Handles past src_len give 0. */
int bhg_crc32c_masked_long(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                           uint32_t n, uint32_t *out_crc, void *stream);
/* hash.Fnv32 of each range (internal/hash/fnv.go:19-23) */
int bhg_fnv32_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                    uint32_t n, uint32_t *out_fnv, void *stream);

/* ---- batch encode (device-resident): BithashWriter.Add over N pairs ----
 * Replaces Writer.Add/add (bithash/writer.go:230-283) + block2Writer.set
 * (block2.go:73-105) + compressor.Encode (compress.go:67-69) + hash.Fnv32 +
 * maybeSplitTable (bithash_writer.go:47-67), batched:
 *   keys, key_off[n+1]      : concatenated user keys
 *   trailers[n]             : ikey trailers (seq<<8 | kind)
 *   vals, val_off[n+1]      : concatenated raw values
 *   vals_len                : val_off[n] (host-known total, sizes the snappy
 *                             scratch without a device read; values whose
 *                             encoding would overflow it get BHG_ST_NO_SPACE)
 *   codec                   : BHG_CODEC_NONE / BHG_CODEC_SNAPPY (golang/snappy v0.0.4 Encode)
 *   file_nums[max_tables]   : fileNum of table 0,1,2... (header fileNum of its records)
 *   init_size               : meta.Size/currentOffset of table 0 when the batch starts
 *   table_max               : TableMaxSize; after each successful add,
 *                             size >= table_max starts the next table at 0
 *   out, out_cap            : packed records of all tables, concatenated;
 *                             records ending past out_cap get BHG_ST_NO_SPACE
 * Outputs (device arrays, n entries unless noted) in bhg_encode_out.
 * Asynchronous on `stream` (no host synchronisation inside). */
typedef struct bhg_encode_out {
    uint64_t *pos;          /* byte position of record i in out (UINT64_MAX if its add failed) */
    uint32_t *bh_off;       /* BlockHandle.Offset inside its table */
    uint32_t *bh_len;       /* BlockHandle.Length */
    uint32_t *table;        /* table index (0-based) */
    uint32_t *fnv1;         /* hash.Fnv32(userKey) */
    uint32_t *crc;          /* masked CRC-32C of the packed record */
    uint32_t *status;       /* BHG_ST_OK / KEY_TOO_LARGE / VALUE_TOO_LARGE / DATA_MAX_EXCEEDED /
                               NO_SPACE / SKIPPED */
    uint32_t *table_start;  /* [max_tables] first record index of each table */
    uint64_t *summary;      /* [4]: bytes the batch occupies in out (out_cap >= this
                               writes every record), tables used (0 = max_tables too
                               small), failed adds (status not OK/SKIPPED), split failed */
    bhg_handle *rec;        /* nullable: {pos, bh_len} per record ({UINT64_MAX, 0} if not written):
                               the record list bhg_table_tail / bhg_decode_batch take */
    uint64_t *table_size;   /* nullable [max_tables]: currentOffset of each table after the
                               batch (its data-region size; bhg_table_tail's data_end) */
} bhg_encode_out;

int bhg_encode_batch(bhg_ctx *ctx, const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                     const uint8_t *vals, const uint64_t *val_off, uint64_t vals_len, uint32_t n, int codec,
                     const uint32_t *file_nums, uint32_t max_tables, uint32_t init_size, uint64_t table_max,
                     uint8_t *out, uint64_t out_cap, const bhg_encode_out *o, void *stream);

/* ---- compaction re-pack (device): BithashWriter.AddIkey over N records ----
 * Replaces the per-record loop of compactBithashFiles (bitree/bithash.go:217-239):
 * the liveness filter (findKey -> skip) and bw.AddIkey(ik, v, khash, fn)
 * (bithash_writer.go:43-45, writer.go:249-255): the value bytes are written
 * as given (already encoded: TableIterator hands out stored bytes), the
 * header fileNum is the record's SOURCE file, the khash is the caller's, and
 * all records go to ONE table (AddIkey never calls maybeSplitTable).
 *   keys/key_off/trailers/vals/val_off : as bhg_encode_batch (vals = stored value bytes)
 *   khash[n]        : nullable -> hash.Fnv32(userKey)
 *   rec_file_nums[n]: header fileNum of each record
 *   live[n]         : nullable u8 mask; 0 -> BHG_ST_SKIPPED, no bytes, no handle
 *   init_size       : the destination writer's currentOffset when the batch starts
 *   out, out_cap, o : as bhg_encode_batch; o->table_start needs 1 entry, table[] is 0.
 * Statuses: OK, SKIPPED, KEY_TOO_LARGE, VALUE_TOO_LARGE, DATA_MAX_EXCEEDED
 * (writer.go:266-269, per record against init_size + position), NO_SPACE.
 * The reference aborts the compaction at its first failed add; a caller
 * mirroring it stops at the first status not OK/SKIPPED. */
int bhg_encode_ikey_batch(bhg_ctx *ctx, const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                          const uint8_t *vals, const uint64_t *val_off, uint32_t n, const uint32_t *khash,
                          const uint32_t *rec_file_nums, const uint8_t *live, uint32_t init_size, uint8_t *out,
                          uint64_t out_cap, const bhg_encode_out *o, void *stream);

/* ---- compaction re-pack from stored records (device) ----
 * bhg_encode_ikey_batch with the AddIkey inputs read straight from the
 * source records: TableIterator hands compactBithashFiles each record's
 * ikey, stored value bytes and header fileNum (table.go:358-395), and
 * AddIkey writes them unchanged (writer.go:249-255), so the live records are
 * re-packed byte for byte into one destination table.
 *   src, src_len, handles[n] : source records (e.g. bhg_scan_tables mode 0
 *                              over the tables being compacted)
 *   live[n]   : nullable u8 mask (the findKey filter, bitree/bithash.go:225-228)
 *   khash[n]  : nullable -> hash.Fnv32(userKey)
 *   init_size, out, out_cap, o : as bhg_encode_ikey_batch
 * A handle that is not one whole record (out of range, ikeySize < 8,
 * 12 + ikeySize + valueSize != length) gets BHG_ST_RECORD_NIL. */
int bhg_repack_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                     const uint8_t *live, const uint32_t *khash, uint32_t init_size, uint8_t *out,
                     uint64_t out_cap, const bhg_encode_out *o, void *stream);

/* ---- table tail (device): Writer.writeTable for many tables at once ----
 * Replaces writeData's empty record header, writeConflict, writeIndexHash,
 * writeMeta and writeFooter (bithash/writer.go:312-338, 393-533), with
 * updateHash (writer.go:285-310) folded over the records in add order, the
 * HashIndex build/serialize (internal/bindex/hash_index.go:217-363), the
 * blockWriter format (block.go:595-729) and the footer (table.go:56-68).
 *   recs, rec[n]     : record bytes and each record's {position in recs, length}
 *                      (bhg_encode_out.rec, or bhg_rebuild_tables' handles)
 *   bh_off[n]        : BlockHandle.Offset of each record inside its table
 *   khash[n]         : the khash updateHash was given (hash.Fnv32(userKey) for Add)
 *   table[n]         : table index; records with table >= ntables are ignored
 *   status[n]        : nullable; records with status != BHG_ST_OK are ignored
 *   data_end[ntables]: each table's currentOffset before writeTable (its data size)
 *   tail, tail_cap   : output; table t's tail bytes are written at tail + tail_off[t]
 *   tail_off[ntables+1] : written: slot offsets (exclusive scan of per-table upper
 *                      bounds); tail_off[ntables] = bytes needed
 *   tail_len[ntables]: written: bytes of table t's tail (the file is its data region
 *                      followed by these bytes); 0 when its slot ends past tail_cap
 *   stats[4*ntables] : nullable; per table {index items, conflict keys, BHG_ST_OK or
 *                      BHG_ST_NO_SPACE, 0}
 * Records of one table must be given in add order (the order Add was called).
 * Asynchronous on `stream`. */
int bhg_table_tail(bhg_ctx *ctx, const uint8_t *recs, const bhg_handle *rec, const uint32_t *bh_off,
                   const uint32_t *khash, const uint32_t *table, const uint32_t *status, uint32_t n,
                   uint32_t ntables, const uint64_t *data_end, uint8_t *tail, uint64_t tail_cap,
                   uint64_t *tail_off, uint64_t *tail_len, uint32_t *stats, void *stream);

/* ---- rebuild (device): Writer.rebuild over footerless tables ----
 * Replaces writer.go:539-583 (and the reopen path that calls it): the mode-1
 * header chase of bhg_scan_tables, then per record bh = {offset inside the
 * table, 12 + ikeySize + valueSize}, khash = hash.Fnv32(UserKey) and the
 * table index -- exactly the inputs updateHash received, so bhg_table_tail
 * on them (with data_end = out_end) writes the tail Writer.writeTable would
 * write after the rebuild.
 *   src, table_off, ntables, out_handles, max_out, out_first, out_end : as
 *       bhg_scan_tables mode 1 (out_end[t] = the rebuilt currentOffset)
 *   out_khash, out_bh_off, out_table [max_out] : per record; entries past
 *       out_first[ntables] get table = UINT32_MAX */
int bhg_rebuild_tables(bhg_ctx *ctx, const uint8_t *src, const uint64_t *table_off, uint32_t ntables,
                       bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end,
                       uint32_t *out_khash, uint32_t *out_bh_off, uint32_t *out_table, void *stream);

/* ---- table data-region scan (device) ----
 * TableIterator.findEntry (bithash/table.go:358-395, mode 0) or Writer.rebuild
 * (bithash/writer.go:539-583, mode 1) over each table: the sequential header
 * chase that yields every record's handle in file order.
 *   src, table_off[ntables+1] : table files concatenated; table t = src[table_off[t] : table_off[t+1]]
 *   out_handles, max_out      : handles (offset relative to src), table t's
 *                               records start at out_first[t]
 *   out_first[ntables+1]      : written: exclusive scan of per-table counts
 *   out_end[ntables]          : written: offset (inside table) where the scan stopped */
int bhg_scan_tables(bhg_ctx *ctx, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                    bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end,
                    void *stream);

/* bhg_scan_tables plus, per table, which pass produced its handles (a diagnostic for tests and
 * tuning; the handles are the same): out_path[ntables] (device) = BHG_SCAN_PATH_*. */
#define BHG_SCAN_PATH_SEGMENTS 0  /* segment walks resolved by the stitch */
#define BHG_SCAN_PATH_REPLAY 1    /* serial count walk, write pass replayed from its step log */
#define BHG_SCAN_PATH_SERIAL 2    /* serial walk whose step log overflowed: walked again to write */
int bhg_scan_tables_paths(bhg_ctx *ctx, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                          bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end,
                          uint32_t *out_path, void *stream);
/* Device scratch (from the context's stream-ordered pool) one scan call over ntables takes: tables
 * are scanned 256 at a time through one scratch area, so this stops growing at 256 tables. */
uint64_t bhg_scan_scratch_bytes(uint32_t ntables);

/* ---- batched point lookup (device): Reader.Get minus the pread ----
 * One opened table (NewReader, bithash/reader.go:73-183, done by the host):
 *   base            : byte offset of the table file inside src
 *   index_off/len   : the HashIndex bytes (the indexhash_data value of the
 *                     indexhash block), offset inside src; len 0 = no keys
 *   conflict_off    : offset inside src of the conflict block
 *   conflict_bh_*   : conflictBH as read from the meta block (table-relative;
 *                     length 0 = no conflict block)                       40 B */
typedef struct bhg_table {
    uint64_t base;
    uint64_t index_off;
    uint64_t index_len;
    uint64_t conflict_off;
    uint32_t conflict_bh_off;
    uint32_t conflict_bh_len;
} bhg_table;

/* For each query i (UserKey keys[key_off[i] : key_off[i+1]] in table
 * tables[table_idx[i]]): khash = hash.Fnv32(key) unless khash[] is given,
 * HashIndex.Get64 (internal/bindex/hash_index.go:399-431), and for handles in
 * the conflict range the conflict block SeekGE (reader.go:218-228, 274-289;
 * block.go:274-350).  Writes out_handles[i] = {table base + bh.Offset,
 * bh.Length} (feed to bhg_decode_batch for readData) and out_status[i] =
 * BHG_ST_OK, BHG_ST_NOT_FOUND (ErrBhNotFound) or BHG_ST_ILLEGAL_LENGTH
 * (conflict miss -> ErrBhIllegalBlockLength).  Replaces Reader.Get /
 * Bithash.Get's index path (bithash.go:101-119).  All pointers device. */
int bhg_get_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_table *tables, uint32_t ntables,
                  const uint8_t *keys, const uint64_t *key_off, const uint32_t *table_idx, const uint32_t *khash,
                  uint32_t n, bhg_handle *out_handles, uint32_t *out_status, void *stream);

/* ---- Bithash.Get over open (mutable) tables, the fileNum map and opened tables (device) ----
 * An open table's index: Writer.indexHash + conflictKeys (writer.go:285-310) of a table still
 * being written, held as its records sorted by khash (stable: add order inside a khash).
 * Built by bhg_writer_index_build from the records' khash (bhg_encode_batch's fnv1 output, or
 * the AddIkey khash).  Writer.Get (writer.go:171-228) on it: a khash whose adds all carried one
 * UserKey answers the last add (ih.bh, whatever key is queried, as Go does); two or more
 * distinct keys (conflict) answer the last add of the queried key (conflictKeys) or nothing.
 * Assumption: one khash per UserKey (Writer.Add's hash.Fnv32, and every AddIkey caller in the
 * reference).  Go's conflictKeys is one map per writer, so a key added under two khash values
 * whose runs both conflict answers its last add in either run; here it answers its last add in
 * the queried run.
 *   rec       : device bhg_handle[n], the records in add order (offsets into src)
 *   sorted    : device uint32_t[n] record indices sorted by khash
 *   sorted_kh : device uint32_t[n] khash of sorted[j]
 *   file_num  : the writer's fileNum (the rwwWriters key, bithash.go:102)         32 B */
typedef struct bhg_writer_index {
    uint64_t rec;
    uint64_t sorted;
    uint64_t sorted_kh;
    uint32_t n;
    uint32_t file_num;
} bhg_writer_index;

/* sorted / sorted_kh of an open table from its records' khash[n] (device pointers). */
int bhg_writer_index_build(bhg_ctx *ctx, const uint32_t *khash, uint32_t n, uint32_t *sorted, uint32_t *sorted_kh,
                           void *stream);

/* Bithash.Get (bithash.go:101-119) for n queries (UserKey keys[key_off[i] : key_off[i+1]],
 * khash[i] or hash.Fnv32 of the key when khash is null, fileNum file_nums[i]):
 *   1. the open writer with that fileNum (writers[], nwriters): Writer.Get -> OK on a hit whose
 *      read succeeds (writer.go:190-228: the record inside src, readRecord non-nil, and with
 *      codec BHG_CODEC_SNAPPY a snappy stream that decodes without error to >= 1 byte); any
 *      other writer outcome falls through to 2, as Go's `err == nil && value != nil` test does;
 *   2. dst = fn_map[fn] (GetFileNumMap, :264-273; fn >= fn_count or 0 -> BHG_ST_FILE_NUM_ZERO);
 *   3. the opened table tables[fn_table[dst]] (bhtReaders; none -> BHG_ST_NOT_FOUND): Reader.Get's
 *      index path as bhg_get_batch (OK / NOT_FOUND / ILLEGAL_LENGTH).
 * out_handles[i] is rebased to src (feed to bhg_decode_batch for readData / Writer.Get's read).
 * fn_map and fn_table are indexed by fileNum, fn_count entries each.  All pointers device. */
int bhg_bithash_get_batch(bhg_ctx *ctx, const uint8_t *src, uint64_t src_len, const bhg_writer_index *writers,
                          uint32_t nwriters, const bhg_table *tables, uint32_t ntables, const uint32_t *fn_map,
                          const uint32_t *fn_table, uint32_t fn_count, const uint8_t *keys, const uint64_t *key_off,
                          const uint32_t *file_nums, const uint32_t *khash, int codec, uint32_t n,
                          bhg_handle *out_handles, uint32_t *out_status, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* BITHASHGPU_H */
