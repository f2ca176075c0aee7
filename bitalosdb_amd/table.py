"""Host side of the .bht table format around the GPU codec: table open.

Product code (no oracle import).  NewReader (bithash/reader.go:73-183) is
control logic run once per table: footer (table.go:90-127) -> meta block ->
data / conflict / indexhash handles -> the HashIndex bytes (indexhash_data
value) located inside the file.  The result is a ``TABLE_DT`` record for
``bhg_get_batch``; ``verify_index_checksums`` adds the indexhash checksum
check on the GPU.  Closing a table (Writer.writeTable's tail) runs on the
GPU: bhg_table_tail (bitalosdb_amd/csrc/bhg_tail.hip, codec.table_tail).
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

META_DATA_BH = b"data_blockhandle"
META_CONFLICT_BH = b"conflict_blockhandle"
META_INDEXHASH_BH = b"indexhash_blockhandle"
INDEXHASH_DATA = b"indexhash_data"
INDEXHASH_CHECKSUM = b"indexhash_checksum"


class TableError(Exception):
    pass


# ------------------------------------------------------------------ prefix blocks (block.go)

def _varint32(buf, p):
    """readEntry's varint32 (block.go:115-172): at most 5 bytes."""
    x = 0
    for i in range(5):
        b = buf[p + i]
        if b < 128 or i == 4:
            return (x | (b << (7 * i))) & 0xFFFFFFFF, p + i + 1
        x |= (b & 0x7F) << (7 * i)
    return x, p + 5


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
