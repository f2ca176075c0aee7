// bhg_internal.h -- host-side glue shared by the kernel translation units
// and the C-ABI implementation (bhg_api.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bithashgpu.h"

namespace bhg {

struct Launch {
    hipStream_t stream;
    int num_cus;           // 256 on MI355X
    const uint32_t *ztab;  // device copy of build_tile_ztab() (owned by the context)
    const uint32_t *stab;  // device copy of build_stream_tab(kStreamWin, kStreamNch) (owned by the context)
    const uint32_t *xtab;  // device copy of build_xtab() (owned by the context)
};

// persistent grid for lane-per-item kernels: enough workgroups to fill the
// chip, never more than the work needs
inline uint32_t lane_grid(const Launch &L, uint64_t n, uint32_t block) {
    uint64_t need = (n + block - 1) / block;
    uint64_t cap = (uint64_t)L.num_cus * 4;
    uint64_t g = need < cap ? need : cap;
    return g == 0 ? 1u : (uint32_t)g;
}

// Workgroups of `block` threads of `kernel` that are resident on one CU at once: the
// runtime's occupancy figure, capped by 160 KiB of LDS in 2-KiB allocation granules
// (MI355X, measured: the runtime figure alone over-counted k_snappy_enc -- 12 where 11
// fit, the 12th wave of each CU then ran after the others, +38 % time -- and a 12.5-KiB
// variant that 1-KiB granules would put at 12 per CU ran 1.54x slower, as 11 would).
// `fallback` if the queries fail.
inline uint32_t resident_per_cu(const void *kernel, int block, uint32_t fallback) {
    int b = 0;
    hipFuncAttributes fa;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, block, 0) != hipSuccess || b <= 0 ||
        hipFuncGetAttributes(&fa, kernel) != hipSuccess)
        return fallback;
    const size_t lds = (fa.sharedSizeBytes + 2047) & ~(size_t)2047;
    if (lds) {
        const int by_lds = (int)((160u * 1024u) / lds);
        if (by_lds < b) b = by_lds;
    }
    return b > 0 ? (uint32_t)b : 1u;
}

// bhg_decode.hip: descriptors for codec NONE (complete) or the snappy header
// pass (sizes[i] = decoded length; the values follow with launch_snappy)
// lists: null, or (snappy) the decode lists of snappy_list_bytes(n) -- the header pass sorts the
// blocks to decode into them by size for launch_snappy (which must get the same pointer)
// long_scratch (snappy): null, or long_crc_scratch_bytes(n, src_len) -- then the records longer than
// kLongRec are CRC'd by the long-record pass after the header pass (a batch of long records: long_batch)
hipError_t launch_decode(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         int codec, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes,
                         uint32_t *lists = nullptr, void *long_scratch = nullptr);
// bhg_decode_tile.hip: the NoCompressor decode kernel.  long_scratch: null, or long_crc_scratch_bytes(n,
// src_len) bytes -- then records longer than kLongRec are CRC'd by the long-record pass (a batch of long
// records: see long_batch)
hipError_t launch_decode_tile(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              const uint32_t *expected_crc, bhg_desc *out, void *long_scratch = nullptr);
// bhg_longcrc.hip: masked CRC-32C of the records longer than kLongRec, the whole chip at once (8-KiB
// pieces, one wave each), completing descriptors the LONG tile kernel left (crc 0, status unchecked),
// or (the encoder) the CRCs of the long records k_enc_pack left to k_enc_lcopy
// (4 KiB: the tile kernel's 8 lanes per record load a record's windows past the first 9 one pass at
// a time, synchronously; at 16 KiB the records of 4-16 KiB kept the bigval NoCompressor step's tile
// kernel at 0.19 ms of 0.62)
constexpr uint32_t kLongRec = 4096;
// the dispatch's rule: the long-record passes run for batches whose mean record (decode) or value
// (encode, repack) is past this (the tile kernel's and k_enc_pack's own paths stay for the rest: they
// handle any length, a long record at one wave's or 8 lanes' pace)
constexpr uint64_t kLongMean = 8192;
inline bool long_batch(uint64_t src_len, uint32_t n) { return n != 0 && src_len > (uint64_t)n * kLongMean; }
size_t long_crc_scratch_bytes(uint32_t n, uint64_t src_len);
// the same for a piece list of cap entries (a record whose pieces pass it is walked by one wave instead)
size_t long_crc_scratch_bytes_cap(uint32_t n, uint64_t cap);
// crc_out (the encoder): non-null -> crc_out[i] = the masked CRC of each long record i, descriptors untouched;
// list_cap: 0 (room for every piece of src_len) or the list capacity the scratch was sized for
hipError_t launch_long_crc(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           const uint32_t *expected_crc, bhg_desc *out, void *scratch, uint32_t *crc_out = nullptr,
                           uint64_t list_cap = 0);
// bhg_decode_stream.hip: mode 0 NoCompressor, mode 1 snappy header pass;
// the shift tables it reads (Launch::stab) are built on the host once per context
size_t stream_tab_words();
void build_stream_tab_default(uint32_t *out);
hipError_t launch_decode_stream(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                                int mode, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes,
                                uint32_t *lists, void *long_scratch = nullptr);
// bhg_snappy_dec.hip: golang/snappy value decode (lane per block)
// list: the decode lists the header pass filled (launch_decode with the same pointer, of
// snappy_list_bytes(n)): the blocks for the 1-KiB LDS slots, those for the 4-KiB slots in
// kSnapBuckets buckets of decoded size, and the ones left for the global-memory pass; null ->
// every block through the global-memory kernel.  Layout (u32 words): [0, 64) the small
// sub-lists' sizes, [64, 64 + 64 kSnapBuckets) the large ones' (largest bucket first), then the
// global-memory list's size; from kSnapListHdr the sub-lists themselves, snappy_sub_cap(n)
// entries apart (small, then large in the same order), then the global-memory list (n).  A
// header-pass tile t (64 handles) appends to sub-list t mod 64 of its class, so no sub-list takes
// more than snappy_sub_cap(n) and the appends of ~16k tiles spread over 64 counters per class.
// big: snappy_big_bytes(n, out_cap) bytes of scratch for the blocks past the LDS tiers (chunk-parallel)
hipError_t launch_snappy(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                         bhg_desc *out, uint8_t *out_vals, uint64_t out_cap, const uint64_t *val_off,
                         uint32_t *list, void *big);
size_t snappy_big_bytes(uint32_t n, uint64_t out_cap);
// size buckets of the 4-KiB tier, so a wave's blocks walk alike (it runs as long as its longest):
// mixdec 4.89 -> 4.28 ms with 4; 8 and 12 buckets 4.31-4.32 / 4.36-4.39 (profiles/r5/snappy_buckets)
constexpr uint32_t kSnapBuckets = 4;
constexpr uint32_t kSnapBucketBytes = 3072 / kSnapBuckets;  // decoded bytes per bucket above 1 KiB
constexpr uint32_t kSnapSubs = 64 * (1 + kSnapBuckets);
constexpr uint32_t kSnapRtCount = kSnapSubs;  // word of the global-memory list's size
constexpr uint32_t kSnapListHdr = (kSnapSubs + 1 + 255) / 256 * 256;  // the sizes, rounded to 1 KiB
constexpr uint32_t kSnapBigCtr = 384;  // 4 words of the header for launch_snappy's big-block path (zeroed with it)
constexpr uint32_t kSnapSmallMax = 1024;   // decoded bytes a tier-1 slot takes ...
constexpr uint32_t kSnapSmallSlot = 1088;  // ... and its slot (the stream + 24 must fit too)
inline size_t snappy_sub_cap(uint32_t n) { return 64 * (((size_t)n + 64 * 64 - 1) / (64 * 64)); }
inline size_t snappy_list_bytes(uint32_t n) { return 4 * (kSnapListHdr + (size_t)kSnapSubs * snappy_sub_cap(n) + (size_t)n); }
hipError_t launch_crc_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out);
// one workgroup per range (long ranges: the per-table indexhash checksum)
size_t crc_long_scratch_bytes(uint32_t n);
// scratch: crc_long_scratch_bytes(n) bytes
hipError_t launch_crc_long(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                           uint32_t *out, void *scratch);
hipError_t launch_fnv_ranges(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                             uint32_t *out);

// bhg_get.hip
hipError_t launch_get(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_table *tables, uint32_t ntables,
                      const uint8_t *keys, const uint64_t *key_off, const uint32_t *table_idx, const uint32_t *khash,
                      uint32_t n, bhg_handle *out_h, uint32_t *out_st);

// bhg_get.hip: Bithash.Get over open writers + the fileNum map + opened tables
hipError_t launch_bithash_get(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_writer_index *writers,
                              uint32_t nwriters, const bhg_table *tables, uint32_t ntables, const uint32_t *fn_map,
                              const uint32_t *fn_table, uint32_t fn_count, const uint8_t *keys, const uint64_t *key_off,
                              const uint32_t *file_nums, const uint32_t *khash, int codec, uint32_t n,
                              bhg_handle *out_h, uint32_t *out_st);
size_t writer_index_scratch_bytes(uint32_t n);
hipError_t launch_writer_index(const Launch &L, const uint32_t *khash, uint32_t n, uint32_t *sorted,
                               uint32_t *sorted_kh, void *scratch);

// bhg_encode.hip
struct EncodeLaunch {
    const uint8_t *keys;
    const uint64_t *key_off;
    const uint64_t *trailers;
    const uint8_t *vbase;      // value' bytes (raw values or snappy scratch)
    const uint64_t *vpos;      // value' offsets into vbase
    const uint64_t *vlen;      // value' lengths
    const uint8_t *vend;       // end of the buffer vbase points into (nullable: unknown)
    uint32_t n;
    const uint32_t *file_nums;      // per table
    const uint32_t *rec_file_nums;  // per record (AddIkey), nullable
    const uint8_t *live;            // per record liveness (compaction), nullable
    const uint32_t *khash;          // per record given khash (AddIkey), nullable -> FNV-1 of the key
    const uint32_t *key_len;        // nullable: per-record key length (keys not contiguous)
    const uint32_t *pre_status;     // nullable: records with a non-OK status here are not added
    int single_table;               // AddIkey: one table, no split; dataMaxSize checked per record
    uint32_t max_tables;
    uint32_t init_size;
    uint64_t table_max;
    uint8_t *out;
    uint64_t out_cap;
    uint64_t *lens;            // scratch n+1
    void *scan_scratch;
    // nullable: enc_long_scratch_bytes(n, vend - vbase) bytes -> records longer than kLongRec are copied
    // and CRC'd by whole-chip passes instead of one wave of k_enc_pack each (a batch of long values)
    void *long_scratch;
    bhg_encode_out o;
};
// vbound: the bytes of the buffer the values' (value') bytes lie in (EncodeLaunch vend - vbase)
size_t enc_long_scratch_bytes(uint32_t n, uint64_t vbound);
hipError_t launch_encode(const Launch &L, const EncodeLaunch &E);
hipError_t launch_enc_rawvals(const Launch &L, const uint64_t *val_off, uint32_t n, uint64_t *vlen);
// bhg_repack_batch: AddIkey inputs parsed from stored records
hipError_t launch_repack_prep(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                              uint64_t *key_off, uint32_t *key_len, uint64_t *trailers, uint64_t *vpos,
                              uint64_t *vlen, uint32_t *fns, uint32_t *pre);

// bhg_snappy_enc.hip
hipError_t launch_snappy_maxlen(const Launch &L, const uint64_t *val_off, uint32_t n, uint64_t *out);
size_t snappy_enc_list_bytes(uint32_t n);  // the value-class lists launch_snappy_enc needs
// the block path's scratch (values > 4 KiB: their 64-KiB blocks, each a work item)
size_t snappy_block_scratch_bytes(uint32_t n, uint64_t vals_len);
hipError_t launch_snappy_enc(const Launch &L, const uint8_t *vals, const uint64_t *val_off, uint32_t n, uint64_t vals_len,
                             uint8_t *scratch, uint64_t scap, const uint64_t *soff, uint64_t *clen, uint32_t *lists,
                             void *block_scratch);

// bhg_tail.hip: Writer.writeTable's tail for many tables (include/bithashgpu.h bhg_table_tail)
struct TailLaunch {
    const uint8_t *recs;
    const bhg_handle *rec;
    const uint32_t *bh_off, *khash, *table, *status;
    uint32_t n, ntables;
    const uint64_t *data_end;
    uint8_t *tail;
    uint64_t tail_cap;
    uint64_t *tail_off, *tail_len;
    uint32_t *stats;
};
size_t tail_scratch_bytes(uint32_t n, uint32_t ntables);
hipError_t launch_table_tail(const Launch &L, const TailLaunch &T, void *scratch);
// bhg_tscan.hip: per-record rebuild outputs after a mode-1 scan (khash, table-relative offset, table)
hipError_t launch_rebuild_recs(const Launch &L, const uint8_t *src, const uint64_t *table_off, uint32_t ntables,
                               const bhg_handle *h, uint64_t max_out, const uint64_t *first, uint32_t *khash,
                               uint32_t *bh_off, uint32_t *table);

// bhg_scan.hip: exclusive prefix sum of n u64 in place into out[0..n], out[n] = total.
// scratch must hold scan_scratch_bytes(n).
size_t scan_scratch_bytes(uint64_t n);
// bhg_sort.hip: stable LSD radix sort of (u64 key, u32 value) pairs over key bits [0, end_bit);
// the sorted pairs land in keys_out / vals_out, keys / vals are overwritten
size_t radix_sort_scratch_bytes(uint32_t n);
hipError_t launch_radix_sort_pairs(const Launch &L, uint64_t *keys, uint64_t *keys_out, uint32_t *vals,
                                   uint32_t *vals_out, uint32_t n, uint32_t end_bit, void *scratch);
hipError_t launch_exclusive_scan_u64(const Launch &L, const uint64_t *in, uint64_t *out, uint64_t n, void *scratch);
// p[i * stride] += add (mod 2^64), i in [0, n)
hipError_t launch_add_u64(const Launch &L, uint64_t *p, uint64_t n, uint64_t add, uint32_t stride);
// dst (mapped host memory) <- src, n bytes; src == dst mod 16
hipError_t launch_copy_out(const Launch &L, const uint8_t *src, uint8_t *dst, uint64_t n);

// bhg_tscan.hip: table data-region scan (uniform prefixes -> count -> scan -> write); first[ntables+1],
// scan_scratch holds scan_scratch_bytes(ntables), uni_scratch tscan_uni_bytes(ntables).
size_t tscan_uni_bytes(uint32_t ntables);
// bhg_snappy_enc.hip: *bad = 0 iff the highest lane's byte stays when lanes of one ds_write_b8
// store to the same byte (the encoder's duplicate-bucket check relies on it)
hipError_t launch_lds_order_probe(hipStream_t stream, uint32_t *bad);
hipError_t launch_tscan(const Launch &L, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                        bhg_handle *out, uint64_t max_out, uint64_t *first, uint64_t *out_end, void *scan_scratch,
                        void *uni_scratch, uint32_t *out_path = nullptr);

}  // namespace bhg
