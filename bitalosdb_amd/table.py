"""Host side of the .bht table format around the GPU codec.

Product code (no oracle import).  Two halves, both small control logic the
reference runs once per table:

* open (NewReader, bithash/reader.go:73-183): footer (table.go:90-127) ->
  meta block -> data / conflict / indexhash handles -> the HashIndex bytes
  (indexhash_data value) located inside the file.  The result is a
  ``TABLE_DT`` record for ``bhg_get_batch``.
* close (Writer.writeTable, bithash/writer.go:312-338, 393-533): given the
  records a batch encode packed into one table (handles, FNV-1 hashes and
  user keys in add order), build the tail -- 12-byte terminator, conflict
  block, indexhash block {indexhash_data: HashIndex, indexhash_checksum:
  masked CRC-32C in decimal}, meta block, 21-byte footer.  updateHash
  (writer.go:285-310) is applied as a grouped pass over the key hashes; the
  HashIndex (internal/bindex/hash_index.go:267-363) is written with numpy
  (one sort of the unique hashes).  The masked CRC-32C is taken from the
  caller (the GPU primitive bhg_crc32c_masked_batch in codec.py).
"""
import struct

import numpy as np

from ._lib import HANDLE_DT, TABLE_DT

RECORD_HEADER_SIZE = 12
BLOCK_RESTART_INTERVAL = 16          # block.go:607
FOOTER_LEN = 21                      # table.go:29-51: [checksum type][metaBH 8][version 4][magic 8]
MAGIC = b"\xf7\xcf\xf4\x85\xb7\x41\xe2\x88"
FORMAT_VERSION2 = 2
CHECKSUM_CRC32C = 1
HASH_INDEX_SHARDS = 1 << 16          # bindex.HashIndexShardsNum
SUCCINCT_HEADER_SIZE = 8
SUCCINCT_VERSION = 1
ITEM_OFFSET = SUCCINCT_HEADER_SIZE + 4 * HASH_INDEX_SHARDS
TRAILER_SET_SEQ1 = (1 << 8) | 1      # MakeInternalKey(key, 1, InternalKeyKindSet)

META_DATA_BH = b"data_blockhandle"
META_CONFLICT_BH = b"conflict_blockhandle"
META_INDEXHASH_BH = b"indexhash_blockhandle"
INDEXHASH_DATA = b"indexhash_data"
INDEXHASH_CHECKSUM = b"indexhash_checksum"


class TableError(Exception):
    pass


# ------------------------------------------------------------------ prefix blocks (block.go)

def _uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _varint32(buf, p):
    """readEntry's varint32 (block.go:115-172): at most 5 bytes."""
    x = 0
    for i in range(5):
        b = buf[p + i]
        if b < 128 or i == 4:
            return (x | (b << (7 * i))) & 0xFFFFFFFF, p + i + 1
        x |= (b & 0x7F) << (7 * i)
    return x, p + 5


def block_build(entries):
    """blockWriter.add/finish (block.go:595-729): entries = [(ikey bytes, value bytes)] in order."""
    buf = bytearray()
    restarts = []
    prev = b""
    for n, (k, v) in enumerate(entries):
        shared = 0
        if n % BLOCK_RESTART_INTERVAL == 0:
            restarts.append(len(buf))
        else:
            m = min(len(k), len(prev))
            while shared < m and k[shared] == prev[shared]:
                shared += 1
        buf += _uvarint(shared) + _uvarint(len(k) - shared) + _uvarint(len(v)) + k[shared:] + v
        prev = k
    if not entries:
        restarts = [0]
    return bytes(buf) + b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))


def block_iter(buf, off, length):
    """blockIter First/Next (block.go:112-182, 452-505): yields (ikey, value_off, value_len), offsets in buf."""
    if length < 4:
        raise TableError("bithash invalid table block size")
    nres = struct.unpack_from("<I", buf, off + length - 4)[0]
    if nres == 0:
        raise TableError("bithash invalid table block has no restart points")
    end = off + length - 4 * (1 + nres)
    p, full = off, b""
    while p < end:
        shared, p = _varint32(buf, p)
        unshared, p = _varint32(buf, p)
        vlen, p = _varint32(buf, p)
        full = full[:shared] + bytes(buf[p:p + unshared])
        p += unshared
        yield full, p, vlen
        p += vlen


def _ikey(ukey):
    return bytes(ukey) + struct.pack("<Q", TRAILER_SET_SEQ1)


def _bh(off, length):
    return struct.pack("<II", off, length)


# ------------------------------------------------------------------ open (NewReader)

def open_table(buf, base=0):
    """NewReader's footer/meta/indexhash reads over one table file image.

    buf: the bytes of the file (bytes/bytearray/np.uint8); base: its offset
    inside the src the GPU sees.  Returns (TABLE_DT record, info dict)."""
    b = memoryview(np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf).cast("B")
    size = len(b)
    if size < FOOTER_LEN:
        raise TableError("ErrBhInvalidTableSize")
    f = bytes(b[size - FOOTER_LEN:])
    if struct.unpack_from("<I", f, 9)[0] != FORMAT_VERSION2:
        raise TableError("bithash unsupported format version")
    moff, mlen = struct.unpack_from("<II", f, 1)
    if (moff + mlen) & 0xFFFFFFFF > size:            # uint32 sum, as decodeTableFooter
        raise TableError("ErrBhInvalidTableMeta")
    meta = {}
    for ik, vo, vl in block_iter(b, moff, mlen):
        if vl != 8:
            raise TableError("bithash: bad meta block handle")
        meta[bytes(ik[:-8])] = struct.unpack_from("<II", b, vo)
    if len(meta) != 3:
        raise TableError("bithash: read meta blockHandleSum mismatch")
    ioff, ilen = meta[META_INDEXHASH_BH]
    index_off, index_len, checksum = 0, 0, None
    for ik, vo, vl in block_iter(b, ioff, ilen):
        uk = bytes(ik[:-8])
        if uk == INDEXHASH_DATA:
            index_off, index_len = vo, vl
        elif uk == INDEXHASH_CHECKSUM:
            checksum = int(bytes(b[vo:vo + vl]).decode())
    coff, clen = meta[META_CONFLICT_BH]
    rec = np.zeros((), dtype=TABLE_DT)
    rec["base"] = base
    rec["index_off"] = base + index_off
    rec["index_len"] = index_len
    rec["conflict_off"] = base + coff
    rec["conflict_bh_off"] = coff
    rec["conflict_bh_len"] = clen
    info = dict(data_bh=meta[META_DATA_BH], conflict_bh=(coff, clen), index_bh=(ioff, ilen),
                index_data=(index_off, index_len), index_checksum=checksum, meta_bh=(moff, mlen))
    return rec, info


def verify_index_checksums(codec, src_t, infos, bases):
    """The CRC-verify build contract for tables: for each
    opened table, masked CRC-32C of its indexhash_data on the GPU against the
    decimal indexhash_checksum that Writer.writeIndexHash stored
    (bithash/writer.go:476-478).  The reference reader never checks it
    (reader.go:162-183 reads only indexhash_data).

    codec: BithashCodec; src_t: device bytes holding the tables; infos: the
    info dicts of open_table; bases: each table's offset in src_t.
    Returns (ok bool[n], computed uint32[n]); a table without the checksum
    entry compares as not ok."""
    from .codec import handles_tensor
    n = len(infos)
    h = np.zeros(n, dtype=HANDLE_DT)
    for t, (info, b) in enumerate(zip(infos, bases)):
        off, ln = info["index_data"]
        h[t] = (b + off, ln, 0)
    if n == 0:
        return np.zeros(0, dtype=bool), np.zeros(0, dtype=np.uint32)
    got = codec.crc_long(src_t, handles_tensor(h, codec.device), n).cpu().numpy().view(np.uint32)
    want = np.array([-1 if i["index_checksum"] is None else i["index_checksum"] for i in infos], dtype=np.int64)
    return got.astype(np.int64) == want, got


# ------------------------------------------------------------------ close (Writer.writeTable)

def update_hash_groups(khash, keys):
    """updateHash (writer.go:285-310) over the adds of one table, in order.

    khash: uint32 [n]; keys: list of user keys (bytes).  Returns
      order    : the distinct khashes in first-add order (Go indexArray)
      last     : index of the last add per distinct khash (its BlockHandle wins)
      conflict : bool per distinct khash (>= 2 distinct user keys)
      ckeys    : {user key: index of its last add} for keys of conflicting hashes
    """
    khash = np.asarray(khash, dtype=np.uint32)
    n = len(khash)
    uniq, first, inv = np.unique(khash, return_index=True, return_inverse=True)
    last = np.full(len(uniq), -1, dtype=np.int64)
    np.maximum.at(last, inv, np.arange(n))            # the last add of each hash
    cnt = np.bincount(inv, minlength=len(uniq))
    conflict = np.zeros(len(uniq), dtype=bool)
    ckeys = {}
    rep = np.nonzero(cnt[inv] > 1)[0]                 # adds whose hash repeats: overwrite or collision
    if rep.size:
        rep = rep[np.argsort(inv[rep], kind="stable")]  # grouped by hash, add order kept inside a group
        bounds = np.flatnonzero(np.diff(inv[rep])) + 1
        for grp in np.split(rep, bounds):
            ks = {}
            for i in grp:
                ks[bytes(keys[i])] = int(i)
            if len(ks) > 1:
                conflict[inv[grp[0]]] = True
                ckeys.update(ks)
    order = np.argsort(first, kind="stable")
    return uniq, order, last, conflict, ckeys


def hash_index_bytes(khash_sorted, values):
    """HashIndex serialization (hash_index.go:267-363), 64-bit items, big-endian:
    header {u16 version, u16 0, u32 shards} | u32 cumulative count per shard |
    items {u16 lo16, u64 value} grouped by hi16, sorted by lo16 (unique)."""
    kh = np.asarray(khash_sorted, dtype=np.uint32)
    hi = (kh >> 16).astype(np.int64)
    counts = np.bincount(hi, minlength=HASH_INDEX_SHARDS)
    cum = np.cumsum(counts).astype(">u4")
    items = np.zeros(len(kh), dtype=[("lo", ">u2"), ("v", ">u8")])
    items["lo"] = (kh & 0xFFFF).astype(np.uint16)
    items["v"] = np.asarray(values, dtype=np.uint64)
    hdr = struct.pack(">HHI", SUCCINCT_VERSION, 0, HASH_INDEX_SHARDS)
    return hdr + cum.tobytes() + items.tobytes()


def table_tail(data_end, bh_off, bh_len, khash, keys, crc_masked):
    """Writer.writeTable's tail for one table whose records occupy [0, data_end).

    bh_off/bh_len/khash: per add, in add order; keys: the user keys (bytes);
    crc_masked: callable(bytes) -> masked CRC-32C (crc.New(b).Value()).
    Returns the bytes that follow the data region (terminator .. footer)."""
    bh_off = np.asarray(bh_off, dtype=np.uint64)
    bh_len = np.asarray(bh_len, dtype=np.uint64)
    out = bytearray(12)                                # writeData: 12-byte terminator (writer.go:393-407)
    cur = data_end + 12
    uniq, order, last, conflict, ckeys = update_hash_groups(khash, keys) if len(khash) else (
        np.zeros(0, np.uint32), np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, bool), {})
    # writeConflict (writer.go:409-433): sorted keys, value = 8-B handle
    if not ckeys:
        conflict_bh = (cur, 0)
    else:
        blk = block_build([(_ikey(k), _bh(int(bh_off[i]), int(bh_len[i]))) for k, i in sorted(ckeys.items())])
        conflict_bh = (cur, len(blk))
        out += blk
        cur += len(blk)
    # writeIndexHash (writer.go:435-490)
    entries = []
    data = b""
    if len(uniq):
        li = last
        vals = bh_off[li] | (bh_len[li] << np.uint64(32))
        cval = np.uint64(conflict_bh[0]) | (np.uint64(conflict_bh[1]) << np.uint64(32))
        vals = np.where(conflict, cval, vals)
        data = hash_index_bytes(uniq, vals)            # np.unique output is sorted by khash
        entries.append((_ikey(INDEXHASH_DATA), data))
    entries.append((_ikey(INDEXHASH_CHECKSUM), str(crc_masked(data)).encode()))
    blk = block_build(entries)
    index_bh = (cur, len(blk))
    out += blk
    cur += len(blk)
    # writeMeta (writer.go:492-520): data, conflict, indexhash handles
    blk = block_build([(_ikey(META_DATA_BH), _bh(0, data_end + 12)),
                       (_ikey(META_CONFLICT_BH), _bh(*conflict_bh)),
                       (_ikey(META_INDEXHASH_BH), _bh(*index_bh))])
    meta_bh = (cur, len(blk))
    out += blk
    cur += len(blk)
    # writeFooter (table.go:56-68)
    out += bytes([CHECKSUM_CRC32C]) + _bh(*meta_bh) + struct.pack("<I", FORMAT_VERSION2) + MAGIC
    return bytes(out)
