"""Python restatement of the bithash table format (writer + reader + scans).

TEST INFRASTRUCTURE ONLY (small cases: the fixtures and the reference's
known-answer tests).  Byte arithmetic is delegated to the C restatement in
oracle.py (CRC-32C, FNV-1, snappy); this module restates the table-level
control logic:

  * blockWriter / blockIter          bithash/block.go:26-39, 112-182, 274-350, 595-729
  * HashIndex (64-bit items)         internal/bindex/hash_index.go:83-100, 217-233, 267-363, 399-503
  * footer                           bithash/table.go:29-127
  * Writer.add / updateHash / tail   bithash/writer.go:230-338, 393-537
  * Writer.rebuild                   bithash/writer.go:539-583
  * BithashWriter split / Finish     bithash/bithash_writer.go:25-87
  * Reader.Get / readData / conflict bithash/reader.go:117-289
  * TableIterator                    bithash/table.go:296-395
"""
import struct

from . import oracle as O

RECORD_HEADER_SIZE = 12
BLOCK_RESTART_INTERVAL = 16
BLOCK_HANDLE_LEN = 8
FOOTER_LEN = 1 + BLOCK_HANDLE_LEN + 4 + 8
MAGIC = b"\xf7\xcf\xf4\x85\xb7\x41\xe2\x88"
FORMAT_VERSION2 = 2
CHECKSUM_CRC32C = 1
MAX_KEY_SIZE = 33 << 10
MAX_VALUE_SIZE = 256 << 20
DATA_MAX_SIZE = 0xFFFFFFFF - (256 << 20)
KIND_SET = 1
KIND_INVALID = 255

META_INDEXHASH_BH = b"indexhash_blockhandle"
META_CONFLICT_BH = b"conflict_blockhandle"
META_DATA_BH = b"data_blockhandle"
INDEXHASH_DATA = b"indexhash_data"
INDEXHASH_CHECKSUM = b"indexhash_checksum"

HASH_INDEX_SHARDS = 64 << 10
SUCCINCT_HEADER_SIZE = 8
SUCCINCT_VERSION = 1


class BithashError(Exception):
    pass


def make_ikey(ukey, seq, kind=KIND_SET):
    return bytes(ukey) + struct.pack("<Q", (seq << 8) | kind)


def encode_bh(off, length):
    return struct.pack("<II", off, length)


def decode_bh(b):
    return struct.unpack_from("<II", b, 0)


def _uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _read_uvarint32(buf, p):
    # readEntry's unrolled varint32 decode (block.go:115-172): up to 5 bytes.
    shift, x = 0, 0
    for i in range(5):
        b = buf[p + i]
        if b < 128 or i == 4:
            x |= b << shift
            return x & 0xFFFFFFFF, p + i + 1
        x |= (b & 0x7F) << shift
        shift += 7


class BlockWriter:
    """blockWriter (block.go:595-729)."""

    def __init__(self, restart_interval=BLOCK_RESTART_INTERVAL):
        self.restart_interval = restart_interval
        self.n_entries = 0
        self.next_restart = 0
        self.buf = bytearray()
        self.restarts = []
        self.prev_key = b""

    def add(self, ikey, value):
        cur = bytes(ikey)
        shared = 0
        if self.n_entries == self.next_restart:
            self.next_restart = self.n_entries + self.restart_interval
            self.restarts.append(len(self.buf))
        else:
            n = min(len(cur), len(self.prev_key))
            while shared < n and cur[shared] == self.prev_key[shared]:
                shared += 1
        self.buf += _uvarint(shared) + _uvarint(len(cur) - shared) + _uvarint(len(value))
        self.buf += cur[shared:] + bytes(value)
        self.prev_key = cur
        self.n_entries += 1

    def finish(self):
        restarts = self.restarts if self.n_entries else [0]
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))
        self.__init__(self.restart_interval)
        return out


def block_entries(block):
    """All (ikey, value) entries of a block, in order (blockIter First/Next)."""
    block = bytes(block)
    num_restarts = struct.unpack_from("<I", block, len(block) - 4)[0]
    if num_restarts == 0:
        raise BithashError("bithash invalid table block has no restart points")
    end = len(block) - 4 * (1 + num_restarts)
    out, p, full = [], 0, b""
    while p < end:
        shared, p = _read_uvarint32(block, p)
        unshared, p = _read_uvarint32(block, p)
        vlen, p = _read_uvarint32(block, p)
        full = full[:shared] + block[p:p + unshared]
        p += unshared
        out.append((full, block[p:p + vlen]))
        p += vlen
    return out


def split_ikey(ikey):
    """base.DecodeInternalKey (internal/base/internal.go:92-106)."""
    n = len(ikey) - 8
    if n >= 0:
        return ikey[:n], struct.unpack_from("<Q", ikey, n)[0]
    return None, KIND_INVALID


def block_seek_ge(block, ukey):
    """blockIter.SeekGE on user key (entries are sorted by InternalCompare)."""
    for ik, v in block_entries(block):
        uk, _ = split_ikey(ik)
        if uk is not None and uk >= ukey:
            return uk, v
    return None, None


class HashIndex:
    """bindex.HashIndex, 64-bit items, big-endian serialization."""

    def __init__(self):
        self.shards = [[] for _ in range(HASH_INDEX_SHARDS)]
        self.length = 0

    def add(self, khash, value):
        self.shards[khash >> 16].append((khash & 0xFFFF, value))
        self.length += 1

    def serialize(self):
        # unique64Internal: sort by lo16, drop repeated lo16 (keeps first after sort)
        items_total = 0
        shard_words = []
        item_bytes = bytearray()
        for s in self.shards:
            s.sort(key=lambda it: it[0])
            uniq, prev = [], -1
            for lo, v in s:
                if lo == prev:
                    continue
                uniq.append((lo, v))
                prev = lo
            items_total += len(uniq)
            shard_words.append(struct.pack(">I", items_total))
            for lo, v in uniq:
                item_bytes += struct.pack(">HQ", lo, v)
        hdr = struct.pack(">HHI", SUCCINCT_VERSION, 0, HASH_INDEX_SHARDS)
        return hdr + b"".join(shard_words) + bytes(item_bytes)


def hash_index_get64(data, khash):
    """HashIndex.Get64 (hash_index.go:399-431) + findItem (:487-503)."""
    item_off = SUCCINCT_HEADER_SIZE + HASH_INDEX_SHARDS * 4
    if data is None or len(data) <= item_off:
        return None
    hid, lid = khash >> 16, khash & 0xFFFF
    origin = 0
    if hid > 0:
        origin = struct.unpack_from(">I", data, SUCCINCT_HEADER_SIZE + (hid - 1) * 4)[0]
    dest = struct.unpack_from(">I", data, SUCCINCT_HEADER_SIZE + hid * 4)[0]
    if dest <= origin:
        return None
    n = dest - origin
    cur = item_off + origin * 10
    i, j = 0, n
    while i < j:
        h = (i + j) >> 1
        if struct.unpack_from(">H", data, cur + 10 * h)[0] < lid:
            i = h + 1
        else:
            j = h
    if i < n and struct.unpack_from(">H", data, cur + 10 * i)[0] == lid:
        return struct.unpack_from(">Q", data, cur + 10 * i + 2)[0]
    return None


class Writer:
    """bithash Writer (writer.go:69-583) over an in-memory file (bytearray)."""

    def __init__(self, file_num, table_max_size, compressor=0, file=None):
        self.file_num = file_num
        self.data_block_size = table_max_size
        self.compressor = compressor
        self.file = bytearray() if file is None else file
        self.current_offset = 0
        self.size = 0
        self.key_num = 0
        self.conflict_key_num = 0
        self.index_hash = {}       # khash -> [bh(off,len), userKey, conflict]
        self.index_order = []      # insertion order (Go indexArray)
        self.conflict_keys = {}
        self.err = None
        self.closed = False

    # writer.go:230-247
    def add(self, ikey_ukey, trailer, value):
        if self.err:
            raise self.err
        compressed = O.snappy_encode(value) if self.compressor == 1 else bytes(value)
        return self._add(ikey_ukey, trailer, compressed, O.fnv32(ikey_ukey), self.file_num)

    # writer.go:249-255
    def add_ikey(self, ukey, trailer, value, khash, file_num):
        if self.err:
            raise self.err
        return self._add(ukey, trailer, bytes(value), khash, file_num)

    # writer.go:257-283
    def _add(self, ukey, trailer, value, khash, file_num):
        key_size = len(ukey) + 8
        if key_size > MAX_KEY_SIZE:
            raise BithashError("ErrBhKeyTooLarge")
        if len(value) > MAX_VALUE_SIZE:
            raise BithashError("ErrBhValueTooLarge")
        kv = key_size + len(value) + RECORD_HEADER_SIZE
        if ((self.size + kv) & 0xFFFFFFFF) > DATA_MAX_SIZE:
            raise BithashError("bithash: panic add exceed data max size")
        rec = O.record_set(ukey, trailer, value, file_num)
        self.file[self.current_offset:self.current_offset + len(rec)] = rec
        bh = (self.current_offset, len(rec))
        self.current_offset += len(rec)
        self.size += len(rec)
        self.key_num += 1
        self.update_hash(bytes(ukey), khash, bh)
        return bh

    # writer.go:285-310
    def update_hash(self, key, khash, bh):
        ih = self.index_hash.get(khash)
        if ih is None:
            self.index_hash[khash] = [bh, key, False]
            self.index_order.append(khash)
        elif ih[2]:
            self.conflict_keys[key] = bh
        elif ih[1] == key:
            ih[0] = bh
        else:
            ih[2] = True
            self.conflict_keys[key] = bh
            self.conflict_keys[ih[1]] = ih[0]

    def is_write_full(self):
        return self.size >= self.data_block_size

    # writer.go:312-338 (+ :393-533)
    def write_table(self, force):
        if self.err:
            raise self.err
        if not (force or self.is_write_full()):
            return
        out = self.file
        # writeData: 12 zero bytes, dataBH = {0, currentOffset}
        out[self.current_offset:self.current_offset + 12] = bytes(12)
        self.current_offset += 12
        data_bh = (0, self.current_offset)
        # writeConflict
        self.conflict_key_num = len(self.conflict_keys)
        if self.conflict_key_num == 0:
            conflict_bh = (self.current_offset, 0)
        else:
            bw = BlockWriter()
            for k in sorted(self.conflict_keys):
                bw.add(make_ikey(k, 1), encode_bh(*self.conflict_keys[k]))
            b = bw.finish()
            out[self.current_offset:self.current_offset + len(b)] = b
            conflict_bh = (self.current_offset, len(b))
            self.current_offset += len(b)
        # writeIndexHash
        ibw = BlockWriter()
        data = b""
        if self.index_hash:
            hi = HashIndex()
            for khash in self.index_order:
                bh, _, conflict = self.index_hash[khash]
                hbh = conflict_bh if conflict else bh
                hi.add(khash, struct.unpack("<Q", encode_bh(*hbh))[0])
            data = hi.serialize()
            ibw.add(make_ikey(INDEXHASH_DATA, 1), data)
        checksum = O.crc_masked(data)
        ibw.add(make_ikey(INDEXHASH_CHECKSUM, 1), str(checksum).encode())
        b = ibw.finish()
        out[self.current_offset:self.current_offset + len(b)] = b
        index_bh = (self.current_offset, len(b))
        self.current_offset += len(b)
        # writeMeta
        mbw = BlockWriter()
        mbw.add(make_ikey(META_DATA_BH, 1), encode_bh(*data_bh))
        mbw.add(make_ikey(META_CONFLICT_BH, 1), encode_bh(*conflict_bh))
        mbw.add(make_ikey(META_INDEXHASH_BH, 1), encode_bh(*index_bh))
        b = mbw.finish()
        out[self.current_offset:self.current_offset + len(b)] = b
        meta_bh = (self.current_offset, len(b))
        self.current_offset += len(b)
        # writeFooter (table.go:56-68)
        footer = bytes([CHECKSUM_CRC32C]) + encode_bh(*meta_bh) + struct.pack("<I", FORMAT_VERSION2) + MAGIC
        out[self.current_offset:self.current_offset + len(footer)] = footer
        self.err = BithashError("ErrBhWriterClosed")

    # writer.go:539-583
    def rebuild(self):
        handles, _ = O.scan_region(bytes(self.file), mode=1)
        for off, length, _ in handles:
            off, length = int(off), int(length)
            k = struct.unpack_from("<I", self.file, off)[0]
            ikey = bytes(self.file[off + 12:off + 12 + k])
            uk, _ = split_ikey(ikey)
            self.current_offset = (self.current_offset + length) & 0xFFFFFFFF
            self.size = (self.size + length) & 0xFFFFFFFF
            self.key_num += 1
            self.update_hash(uk if uk is not None else b"", O.fnv32(uk or b""), (off, length))


class Store:
    """A minimal Bithash store: numbered in-memory table files, flush sessions
    (BithashWriter, bithash_writer.go) and point reads (Bithash.Get)."""

    def __init__(self, table_max_size, compressor=0):
        self.table_max_size = table_max_size
        self.compressor = compressor
        self.files = {}          # fileNum -> bytearray
        self.closed_meta = {}    # fileNum -> (keyNum, conflictKeyNum)
        self.next_file_num = 1
        self.mutable = []        # writers not yet full

    def _new_writer(self):
        fn = self.next_file_num
        self.next_file_num += 1
        w = Writer(fn, self.table_max_size, self.compressor)
        self.files[fn] = w.file
        return w

    def flush_start(self):
        w = self.mutable.pop() if self.mutable else self._new_writer()
        return FlushSession(self, w)

    def close_table(self, w, force):
        w.write_table(force)
        self.closed_meta[w.file_num] = (w.key_num, w.conflict_key_num)

    def get(self, ukey, file_num):
        for w in self.mutable:
            if w.file_num == file_num:
                return _writer_get(w, ukey)
        return table_get(bytes(self.files[file_num]), ukey, self.compressor)


class FlushSession:
    """BithashWriter (bithash_writer.go:19-95)."""

    def __init__(self, store, w, compact=False):
        self.store, self.wr, self.compact = store, w, compact

    def add(self, ukey, seq, value, kind=KIND_SET):
        self.wr.add(ukey, (seq << 8) | kind, value)
        fn = self.wr.file_num
        if self.wr.is_write_full():                 # maybeSplitTable (:47-67)
            old = self.wr
            self.wr = self.store._new_writer()
            self.store.close_table(old, False)
        return fn

    def finish(self):                               # :69-87
        if self.compact:
            self.store.close_table(self.wr, True)
        elif not self.wr.is_write_full():
            self.store.mutable.append(self.wr)


def _writer_get(w, ukey):
    """Writer.Get (writer.go:171-228)."""
    ih = w.index_hash.get(O.fnv32(ukey))
    if ih is None:
        return None
    bh = w.conflict_keys.get(bytes(ukey), (0, 0)) if ih[2] else ih[0]
    if bh[1] <= 0:
        return None
    return _read_data(bytes(w.file), bh, w.compressor)


def writer_get_handle(w, ukey, khash=None):
    """Writer.Get's index (writer.go:171-228): the handle it reads, or None (bh.Length <= 0)."""
    ih = w.index_hash.get(O.fnv32(ukey) if khash is None else khash)
    if ih is None:
        return None
    bh = w.conflict_keys.get(bytes(ukey), (0, 0)) if ih[2] else ih[0]
    return bh if bh[1] > 0 else None


def bithash_get_handle(writers, files, fn_map, ukey, fn, khash=None):
    """Bithash.Get (bithash.go:101-119) without the read: writers = {fileNum: open Writer}
    (rwwWriters), files = {fileNum: closed table bytes} (bhtReaders), fn_map = GetFileNumMap's map.
    Returns (status, fileNum, (off, len)) with status "OK", "NOT_FOUND", "ILLEGAL_LENGTH" or
    "FILE_NUM_ZERO".  A writer hit is final only when Writer.Get returns err == nil and a
    non-nil value (bithash.go:102-107): its read (writer.go:190-228) can fail on the record
    (ErrBhReadRecordNil, ErrBhReadAtIncomplete) or the snappy stream, and snappy.Decode of a
    0-length stream returns a nil slice; each of those falls through to GetFileNumMap."""
    w = writers.get(fn)
    if w is not None:
        bh = writer_get_handle(w, ukey, khash)
        if bh is not None:
            try:
                val = _read_data(bytes(w.file), bh, w.compressor)
            except (BithashError, O.SnappyCorrupt):
                val = None
            if val is not None and (w.compressor != 1 or len(val) > 0):
                return "OK", fn, bh
    dst = fn_map.get(fn, 0)
    if dst == 0:
        return "FILE_NUM_ZERO", 0, (0, 0)
    if dst not in files:
        return "NOT_FOUND", dst, (0, 0)
    st, off, ln = get_handle(files[dst], ukey) if khash is None else _get_handle_kh(files[dst], ukey, khash)
    return st, dst, (off, ln)


def _get_handle_kh(f, ukey, khash):
    t = open_table(f)
    v = hash_index_get64(t["index_data"], khash)
    if v is None:
        return "NOT_FOUND", 0, 0
    off, length = v & 0xFFFFFFFF, v >> 32
    coff, clen = t["conflict_bh"]
    if clen != 0 and off >= coff and length <= clen:
        uk, cv = block_seek_ge(t["conflict_buf"], bytes(ukey))
        off, length = decode_bh(cv) if cv is not None and uk == bytes(ukey) else (0, 0)
        if (off, length) == (0, 0):
            return "ILLEGAL_LENGTH", 0, 0
    return "OK", off, length


def read_footer(f):
    """readTableFooter + decodeTableFooter (table.go:90-127)."""
    if len(f) < FOOTER_LEN:
        raise BithashError("ErrBhInvalidTableSize")
    buf = f[len(f) - FOOTER_LEN:]
    if struct.unpack_from("<I", buf, 9)[0] != FORMAT_VERSION2:
        raise BithashError("bithash unsupported format version")
    off, length = decode_bh(buf[1:])
    if off + length > len(f):
        raise BithashError("ErrBhInvalidTableMeta")
    return off, length


def open_table(f):
    """NewReader: footer -> readMeta -> readIndexHash (reader.go:73-183)."""
    moff, mlen = read_footer(f)
    handles = {}
    for ik, v in block_entries(f[moff:moff + mlen]):
        uk, _ = split_ikey(ik)
        handles[uk] = decode_bh(v)
    if len(handles) != 3:
        raise BithashError("bithash: read meta blockHandleSum mismatch")
    ioff, ilen = handles[META_INDEXHASH_BH]
    idx_data = None
    checksum = None
    for ik, v in block_entries(f[ioff:ioff + ilen]):
        uk, _ = split_ikey(ik)
        if uk == INDEXHASH_DATA:
            idx_data = v
        elif uk == INDEXHASH_CHECKSUM:
            checksum = v
    coff, clen = handles[META_CONFLICT_BH]
    return dict(data_bh=handles[META_DATA_BH], conflict_bh=(coff, clen), index_bh=(ioff, ilen),
                index_data=idx_data, index_checksum=checksum,
                conflict_buf=f[coff:coff + clen] if clen > 0 else None)


def table_get(f, ukey, compressor=0, khash=None):
    """Reader.Get (reader.go:209-231); khash is the caller's (Bithash.Get passes FNV-1 of the
    key, the default here; AddIkey callers may have written another)."""
    t = open_table(f)
    v = hash_index_get64(t["index_data"], O.fnv32(ukey) if khash is None else khash)
    if v is None:
        raise BithashError("ErrBhNotFound")
    off, length = v & 0xFFFFFFFF, v >> 32
    coff, clen = t["conflict_bh"]
    if clen != 0 and off >= coff and length <= clen:
        _, cv = block_seek_ge(t["conflict_buf"], bytes(ukey))
        bh = decode_bh(cv) if cv is not None and _ == bytes(ukey) else (0, 0)
        if bh == (0, 0):
            raise BithashError("ErrBhIllegalBlockLength")
        off, length = bh
    return _read_data(f, (off, length), compressor)


def get_handle(f, ukey):
    """Reader.Get's index path (reader.go:209-231) without readData:
    returns (status, bh_off, bh_len) with status "OK", "NOT_FOUND" or "ILLEGAL_LENGTH"."""
    t = open_table(f)
    v = hash_index_get64(t["index_data"], O.fnv32(ukey))
    if v is None:
        return "NOT_FOUND", 0, 0
    off, length = v & 0xFFFFFFFF, v >> 32
    coff, clen = t["conflict_bh"]
    if clen != 0 and off >= coff and length <= clen:
        uk, cv = block_seek_ge(t["conflict_buf"], bytes(ukey))
        off, length = decode_bh(cv) if cv is not None and uk == bytes(ukey) else (0, 0)
        if (off, length) == (0, 0):
            return "ILLEGAL_LENGTH", 0, 0
    return "OK", off, length


def _read_data(f, bh, compressor):
    """Reader.readData (reader.go:233-272) for one handle."""
    off, length = bh
    if length <= 0:
        raise BithashError("ErrBhIllegalBlockLength")
    buf = bytes(f[off:off + length])
    if len(buf) != length:
        raise BithashError("ErrBhReadAtIncomplete")
    k, v = struct.unpack_from("<II", buf, 0)
    if k == 0 or v == 0 or len(buf) != 12 + k + v:
        raise BithashError("ErrBhReadRecordNil")
    val = buf[12 + k:12 + k + v]
    return O.snappy_decode(val) if compressor == 1 else val


def table_iter(f):
    """TableIterator over a table file: yields (userKey, trailer, raw value, fileNum)."""
    handles, _ = O.scan_region(bytes(f), mode=0)
    for off, length, _ in handles:
        off = int(off)
        k, v, fn = struct.unpack_from("<III", f, off)
        ikey = bytes(f[off + 12:off + 12 + k])
        uk, tr = split_ikey(ikey)
        yield uk, tr, bytes(f[off + 12 + k:off + 12 + k + v]), fn
