"""Host-side mirror of the reference's bithash record-codec surface, backed by
the gfx950 kernels through the C-ABI (include/bithashgpu.h).

Reference surface this mirrors (zuoyebang/bitalosdb v2):
  * compress.Compressor: NoCompressor / SnappyCompressor     internal/compress/compress.go:26-89
  * block2Reader.readRecord -> (*InternalKey, value, FileNum)  bithash/block2.go:57-66
  * Reader.readData errors                                     bithash/reader.go:233-272, error.go
  * Writer.Add / BithashWriter.Add + maybeSplitTable           bithash/writer.go:230-283, bithash_writer.go:25-67
  * hash.Fnv32, crc.New(b).Value()                             internal/hash/fnv.go:19-23, internal/crc/crc.go
  * TableIterator / Writer.rebuild scans                       bithash/table.go:358-395, writer.go:539-583

torch is used only as device-memory plumbing (tensors hold the buffers; their
data_ptr()s cross the C-ABI).  Every computation happens in the HIP library.
"""
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as B
from ._lib import CODEC_NONE, CODEC_SNAPPY, DESC_DT, HANDLE_DT  # noqa: F401

# compress.CompressTypeNo / CompressTypeSnappy (compress.go:21-24)
NoCompressor = CODEC_NONE
SnappyCompressor = CODEC_SNAPPY

# Go sentinel errors each per-block status maps onto (bithash/error.go, golang/snappy)
STATUS_ERRORS = {
    B.ST_RECORD_NIL: "bithash: read record nil",                 # ErrBhReadRecordNil
    B.ST_ILLEGAL_LENGTH: "bithash: illegal block handle length", # ErrBhIllegalBlockLength
    B.ST_INCOMPLETE: "bithash: readAt incomplete",               # ErrBhReadAtIncomplete / io.EOF
    B.ST_SNAPPY_CORRUPT: "snappy: corrupt input",                # snappy.ErrCorrupt
    B.ST_SNAPPY_TOO_LARGE: "snappy: decoded block is too large",
    B.ST_CRC_MISMATCH: "bithash: record crc mismatch",
    B.ST_KEY_TOO_LARGE: "bithash: key too large",                # ErrBhKeyTooLarge
    B.ST_VALUE_TOO_LARGE: "bithash: value too large",            # ErrBhValueTooLarge
    B.ST_DATA_MAX_EXCEEDED: "bithash: panic add exceed data max size",
    B.ST_NOT_FOUND: "bithash: not found",                        # ErrBhNotFound
    B.ST_NO_SPACE: "bithash: encode output buffer too small",
    B.ST_FILE_NUM_ZERO: "bithash: fileNum zero",                 # ErrBhFileNumZero
}


class BithashCodecError(Exception):
    def __init__(self, status):
        super().__init__(STATUS_ERRORS.get(int(status), "status %d" % int(status)))
        self.status = int(status)


def _ptr(t):
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr() if t.numel() else None
    if isinstance(t, np.ndarray):
        return t.ctypes.data if t.size else None
    return int(t)


def as_device_bytes(x, device):
    """numpy/bytes -> uint8 CUDA tensor (plumbing)."""
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.uint8) if x.device != device else x.view(torch.uint8)
    a = np.frombuffer(bytes(x), dtype=np.uint8) if isinstance(x, (bytes, bytearray)) else np.ascontiguousarray(x).view(np.uint8).reshape(-1)
    return torch.from_numpy(a.copy()).to(device)


def handles_tensor(handles, device):
    a = np.ascontiguousarray(handles, dtype=HANDLE_DT)
    return torch.from_numpy(a.view(np.uint8).copy()).to(device)


def desc_numpy(desc_t):
    return desc_t.cpu().numpy().view(DESC_DT).reshape(-1)


@dataclass
class DecodedBatch:
    desc: torch.Tensor          # uint8 [n*40] device: bhg_desc[n]
    vals: torch.Tensor          # uint8 device (snappy) or None
    val_off: torch.Tensor       # uint8 view of u64[n+1] (snappy) or None

    def desc_np(self):
        return desc_numpy(self.desc)

    def val_off_np(self):
        return None if self.val_off is None else self.val_off.cpu().numpy().view(np.uint64)


class BithashCodec:
    """One bhg_ctx on one GPU (the cgo shim's Go-side object, in Python)."""

    def __init__(self, device=0):
        if not torch.cuda.is_available():
            raise B.BhgError("no GPU visible: the bithash codec has no CPU path")
        self.device = torch.device("cuda", device)
        self.L = B.lib()
        self.ctx = self.L.bhg_create(device, 0)
        if not self.ctx:
            raise B.BhgError("bhg_create(%d) failed" % device)
        # torch work for this codec (allocations, copies, events) runs on the
        # context's own HIP stream, so every launch is ordered with it
        self.stream = torch.cuda.ExternalStream(self.L.bhg_stream(self.ctx), device=self.device)

    def close(self):
        if self.ctx:
            self.L.bhg_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return self.stream.cuda_stream

    def sync(self):
        self.stream.synchronize()

    # ---- decode ----
    def decode_batch(self, src, src_len, handles, n, compressor=NoCompressor, expected_crc=None,
                     out_desc=None, out_vals=None, out_val_off=None, stream=None):
        """Device-resident batch decode (bhg_decode_batch).  src/handles/... are
        CUDA tensors (or raw device pointers as ints)."""
        dev = self.device
        if out_desc is None:
            out_desc = torch.empty(n * DESC_DT.itemsize, dtype=torch.uint8, device=dev)
        cap = 0
        if compressor == SnappyCompressor:
            if out_val_off is None:
                out_val_off = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
            if out_vals is not None:
                cap = out_vals.numel() if isinstance(out_vals, torch.Tensor) else int(out_vals[1])
                out_vals = out_vals if isinstance(out_vals, torch.Tensor) else out_vals[0]
        rc = self.L.bhg_decode_batch(self.ctx, _ptr(src), src_len, _ptr(handles), n, compressor,
                                     _ptr(expected_crc), _ptr(out_desc), _ptr(out_vals), cap, _ptr(out_val_off),
                                     stream if stream is not None else self._stream())
        B.check(self.ctx, rc, "bhg_decode_batch")
        return DecodedBatch(out_desc, out_vals, out_val_off)

    def decode(self, src, handles, compressor=NoCompressor, expected_crc=None):
        """Convenience: host arrays in, device decode, results as numpy.
        Snappy runs two passes: sizes -> allocate -> decode (the library fills val_off)."""
        with torch.cuda.stream(self.stream):
            return self._decode(src, handles, compressor, expected_crc)

    def _decode(self, src, handles, compressor, expected_crc):
        dev = self.device
        src_t = as_device_bytes(src, dev)
        h_t = handles_tensor(handles, dev)
        n = len(handles)
        exp_t = None
        if expected_crc is not None:
            exp_t = torch.from_numpy(np.ascontiguousarray(expected_crc, dtype=np.uint32).view(np.int32).copy()).to(dev)
        if compressor == SnappyCompressor:
            probe = self.decode_batch(src_t, src_t.numel(), h_t, n, compressor, exp_t)
            self.sync()
            total = int(probe.val_off_np()[-1]) if n else 0
            vals = torch.zeros(max(total, 1), dtype=torch.uint8, device=dev)
            res = self.decode_batch(src_t, src_t.numel(), h_t, n, compressor, exp_t, out_vals=vals)
            self.sync()
            return res.desc_np(), vals.cpu().numpy()[:total], res.val_off_np()
        res = self.decode_batch(src_t, src_t.numel(), h_t, n, compressor, exp_t)
        self.sync()
        return res.desc_np(), None, None

    def decode_host(self, src, handles, compressor=NoCompressor, expected_crc=None, out_vals_cap=None,
                    out_desc=None, out_vals=None):
        """End-to-end path: host buffers in and out (bhg_decode_batch_host).
        Snappy with out_vals_cap None runs the sizing pass first (out_vals NULL)
        and allocates exactly out_val_off[n] bytes.  out_desc: an optional
        caller-owned DESC_DT array of n entries (e.g. host_register'ed once and
        reused: the NoCompressor path then writes it in place).  out_vals: an
        optional caller-owned contiguous uint8 array for the snappy values (its
        size is the capacity when out_vals_cap is None; no sizing pass then)."""
        src = np.ascontiguousarray(np.frombuffer(src, np.uint8) if isinstance(src, (bytes, bytearray)) else src,
                                   dtype=np.uint8)
        h = np.ascontiguousarray(handles, dtype=HANDLE_DT)
        n = len(h)
        if out_desc is not None:
            if out_desc.dtype != DESC_DT or len(out_desc) < n or not out_desc.flags["C_CONTIGUOUS"]:
                raise ValueError("out_desc must be a contiguous DESC_DT array of >= n entries")
            desc = out_desc[:n]
        else:
            desc = np.empty(n, dtype=DESC_DT)
        exp = None if expected_crc is None else np.ascontiguousarray(expected_crc, dtype=np.uint32)
        off = np.zeros(n + 1, dtype=np.uint64) if compressor == SnappyCompressor else None
        cap = 0
        vals = None
        if compressor == SnappyCompressor:
            if out_vals is not None:
                if out_vals.dtype != np.uint8 or out_vals.ndim != 1 or not out_vals.flags["C_CONTIGUOUS"]:
                    raise ValueError("out_vals must be a contiguous 1-D uint8 array")
                out_vals_cap = out_vals.size if out_vals_cap is None else min(out_vals_cap, out_vals.size)
            if out_vals_cap is None:
                rc = self.L.bhg_decode_batch_host(self.ctx, _ptr(src), src.size, _ptr(h), n, compressor, _ptr(exp),
                                                  _ptr(desc), None, 0, _ptr(off))
                B.check(self.ctx, rc, "bhg_decode_batch_host(sizing)")
                out_vals_cap = int(off[-1])
            cap = out_vals_cap
            vals = out_vals if out_vals is not None else np.zeros(max(cap, 1), dtype=np.uint8)
        rc = self.L.bhg_decode_batch_host(self.ctx, _ptr(src), src.size, _ptr(h), n, compressor, _ptr(exp),
                                          _ptr(desc), _ptr(vals), cap, _ptr(off))
        B.check(self.ctx, rc, "bhg_decode_batch_host")
        return desc, (None if vals is None else vals[:min(cap, int(off[-1]))]), off

    def get_batch(self, src_t, tables, keys, table_idx, khash=None):
        """Batched Reader.Get index path (bhg_get_batch): returns device tensors
        (handles [n] as int64 pairs in HANDLE_DT layout, status [n] int32).

        src_t: device uint8 tensor holding the table files; tables: TABLE_DT
        array (bitalosdb_amd.table.open_table records); keys: list of user
        keys or (bytes, key_off[n+1]); table_idx: per query."""
        if isinstance(keys, tuple):
            kb, ko = keys
        else:
            ko = np.zeros(len(keys) + 1, dtype=np.uint64)
            ko[1:] = np.cumsum([len(k) for k in keys])
            kb = b"".join(bytes(k) for k in keys)
        n = len(ko) - 1
        dev = self.device
        with torch.cuda.stream(self.stream):
            tab_t = torch.from_numpy(np.ascontiguousarray(tables, dtype=B.TABLE_DT).view(np.uint8).copy()).to(dev)
            kb_t = torch.from_numpy(np.frombuffer(kb, np.uint8).copy() if len(kb) else np.zeros(1, np.uint8)).to(dev)
            ko_t = torch.from_numpy(np.ascontiguousarray(ko, dtype=np.uint64).view(np.int64)).to(dev)
            ti_t = torch.from_numpy(np.ascontiguousarray(table_idx, dtype=np.uint32).view(np.int32)).to(dev)
            kh_t = None if khash is None else torch.from_numpy(
                np.ascontiguousarray(khash, dtype=np.uint32).view(np.int32)).to(dev)
            out_h = torch.empty(max(n, 1) * 2, dtype=torch.int64, device=dev)
            out_s = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        self.get_batch_dev(src_t, tab_t, len(tables), kb_t, ko_t, ti_t, kh_t, n, out_h, out_s)
        return out_h[:2 * n], out_s[:n]

    def get_batch_dev(self, src_t, tab_t, ntables, kb_t, ko_t, ti_t, kh_t, n, out_h, out_s):
        """bhg_get_batch on device-resident inputs (no copies)."""
        rc = self.L.bhg_get_batch(self.ctx, _ptr(src_t), src_t.numel(), _ptr(tab_t), ntables, _ptr(kb_t),
                                  _ptr(ko_t), _ptr(ti_t), _ptr(kh_t), n, _ptr(out_h), _ptr(out_s), self._stream())
        B.check(self.ctx, rc, "bhg_get_batch")

    def writer_index(self, khash_t, n):
        """bhg_writer_index_build: an open table's Writer.indexHash / conflictKeys as its records
        sorted by khash (device int32 tensors sorted, sorted_kh)."""
        with torch.cuda.stream(self.stream):
            srt = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
            skh = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        rc = self.L.bhg_writer_index_build(self.ctx, _ptr(khash_t), n, _ptr(srt), _ptr(skh), self._stream())
        B.check(self.ctx, rc, "bhg_writer_index_build")
        return srt, skh

    def bithash_get(self, src_t, writers, tables, fn_map, fn_table, keys, file_nums, khash=None, compressor=0):
        """Bithash.Get over a batch (bhg_bithash_get_batch): the open writer of each query's
        fileNum first (Writer.Get; final only when its read would return a value: the record
        checks and, for compressor 1, the snappy stream), then GetFileNumMap and Reader.Get on
        the mapped table.

        writers: WRITER_INDEX_DT array (device pointers: record handles, writer_index outputs);
        tables: TABLE_DT; fn_map / fn_table: per fileNum (dst fileNum or 0 / table index or
        0xffffffff); keys: list of user keys.  Returns device tensors (handles as int64 pairs in
        HANDLE_DT layout, status int32)."""
        ko = np.zeros(len(keys) + 1, dtype=np.uint64)
        ko[1:] = np.cumsum([len(k) for k in keys])
        kb = b"".join(bytes(k) for k in keys)
        n = len(keys)
        dev = self.device

        def t32(a):
            a = np.ascontiguousarray(a, dtype=np.uint32)
            return torch.from_numpy(a.view(np.int32).copy() if a.size else np.zeros(1, np.int32)).to(dev)

        def tbytes(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            return torch.from_numpy(a.view(np.uint8).copy() if a.size else np.zeros(8, np.uint8)).to(dev)
        with torch.cuda.stream(self.stream):
            w_t = tbytes(writers, B.WRITER_INDEX_DT)
            tab_t = tbytes(tables, B.TABLE_DT)
            fm_t, ft_t, fn_t = t32(fn_map), t32(fn_table), t32(file_nums)
            kb_t = torch.from_numpy(np.frombuffer(kb, np.uint8).copy() if len(kb) else np.zeros(1, np.uint8)).to(dev)
            ko_t = torch.from_numpy(ko.view(np.int64)).to(dev)
            kh_t = None if khash is None else t32(khash)
            out_h = torch.empty(max(n, 1) * 2, dtype=torch.int64, device=dev)
            out_s = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        rc = self.L.bhg_bithash_get_batch(self.ctx, _ptr(src_t), src_t.numel(), _ptr(w_t), len(writers), _ptr(tab_t),
                                          len(tables), _ptr(fm_t), _ptr(ft_t), len(fn_map), _ptr(kb_t), _ptr(ko_t),
                                          _ptr(fn_t), _ptr(kh_t), int(compressor), n, _ptr(out_h), _ptr(out_s),
                                          self._stream())
        B.check(self.ctx, rc, "bhg_bithash_get_batch")
        return out_h[:2 * n], out_s[:n]

    def crc_masked_bytes(self, b):
        """crc.New(b).Value() of one host byte string, on the GPU (bhg_crc32c_masked_batch)."""
        with torch.cuda.stream(self.stream):
            t = torch.from_numpy(np.frombuffer(bytes(b), np.uint8).copy() if len(b) else np.zeros(1, np.uint8))
            t = t.to(self.device)
            h = np.zeros(1, dtype=HANDLE_DT)
            h["length"] = len(b)
            ht = handles_tensor(h, self.device)
            out = self.crc_batch(t, ht, 1)
            self.sync()
        return int(out.cpu().numpy().view(np.uint32)[0])

    def multi_get(self, src_t, tables, keys, table_idx, compressor=NoCompressor):
        """Bithash.Get over a batch: index lookup, then readData of the found
        handles (bhg_decode_batch).  Returns (status per query, desc, vals, val_off)
        as numpy; status BHG_ST_* with NOT_FOUND / ILLEGAL_LENGTH from the index
        path and the decode status otherwise."""
        with torch.cuda.stream(self.stream):
            h_t, s_t = self.get_batch(src_t, tables, keys, table_idx)
            n = s_t.numel()
            vals = None
            if compressor == SnappyCompressor:
                probe = self.decode_batch(src_t, src_t.numel(), h_t, n, compressor)
                self.sync()
                total = int(probe.val_off_np()[-1]) if n else 0
                vals = torch.zeros(max(total, 1), dtype=torch.uint8, device=self.device)
            res = self.decode_batch(src_t, src_t.numel(), h_t, n, compressor=compressor, out_vals=vals)
            self.sync()
        st = s_t.cpu().numpy().view(np.uint32).copy()
        desc = res.desc_np()
        ok = st == B.ST_OK
        st[ok] = desc["status"][ok]
        if compressor == SnappyCompressor:
            off = res.val_off_np()
            return st, desc, vals.cpu().numpy()[:int(off[-1])], off
        return st, desc, None, None

    def host_register(self, arr):
        """Pin a host numpy buffer (bhg_host_register) for DMA-rate *_host copies."""
        B.check(self.ctx, self.L.bhg_host_register(self.ctx, _ptr(arr), arr.nbytes), "bhg_host_register")

    def host_unregister(self, arr):
        B.check(self.ctx, self.L.bhg_host_unregister(self.ctx, _ptr(arr)), "bhg_host_unregister")

    # ---- primitives ----
    def crc_batch(self, src_t, handles_t, n):
        with torch.cuda.stream(self.stream):
            out = torch.empty(n, dtype=torch.int32, device=self.device)
        rc = self.L.bhg_crc32c_masked_batch(self.ctx, _ptr(src_t), src_t.numel(), _ptr(handles_t), n, _ptr(out),
                                            self._stream())
        B.check(self.ctx, rc, "bhg_crc32c_masked_batch")
        return out

    def crc_long(self, src_t, handles_t, n):
        """bhg_crc32c_masked_long: crc.New(range).Value() per range, one workgroup
        per range (long ranges, e.g. each table's indexhash_data)."""
        with torch.cuda.stream(self.stream):
            out = torch.empty(n, dtype=torch.int32, device=self.device)
        rc = self.L.bhg_crc32c_masked_long(self.ctx, _ptr(src_t), src_t.numel(), _ptr(handles_t), n, _ptr(out),
                                           self._stream())
        B.check(self.ctx, rc, "bhg_crc32c_masked_long")
        return out

    def fnv_batch(self, src_t, handles_t, n):
        with torch.cuda.stream(self.stream):
            out = torch.empty(n, dtype=torch.int32, device=self.device)
        rc = self.L.bhg_fnv32_batch(self.ctx, _ptr(src_t), src_t.numel(), _ptr(handles_t), n, _ptr(out),
                                    self._stream())
        B.check(self.ctx, rc, "bhg_fnv32_batch")
        return out

    def table_tail(self, recs_t, rec_t, bh_off_t, khash_t, table_t, status_t, n, ntables, data_end_t, tail_cap=None):
        """bhg_table_tail: Writer.writeTable's tail for `ntables` tables on the GPU.
        All inputs are device tensors (rec_t: bhg_handle[n] as int64 pairs).
        tail_cap None sizes the buffer exactly (one sizing call first).
        Returns (tail uint8 tensor, tail_off int64 [ntables+1], tail_len int64
        [ntables], stats int32 [4*ntables])."""
        dev = self.device
        with torch.cuda.stream(self.stream):
            off = torch.zeros(ntables + 1, dtype=torch.int64, device=dev)
            ln = torch.zeros(max(ntables, 1), dtype=torch.int64, device=dev)
            stats = torch.zeros(max(ntables, 1) * 4, dtype=torch.int32, device=dev)
        args = lambda tail, cap: (self.ctx, _ptr(recs_t), _ptr(rec_t), _ptr(bh_off_t), _ptr(khash_t), _ptr(table_t),
                                  _ptr(status_t), n, ntables, _ptr(data_end_t), _ptr(tail), cap, _ptr(off), _ptr(ln),
                                  _ptr(stats), self._stream())
        if tail_cap is None:
            B.check(self.ctx, self.L.bhg_table_tail(*args(None, 0)), "bhg_table_tail(sizing)")
            self.sync()
            tail_cap = int(off[ntables].item())
        with torch.cuda.stream(self.stream):
            tail = torch.zeros(max(tail_cap, 1), dtype=torch.uint8, device=dev)
        B.check(self.ctx, self.L.bhg_table_tail(*args(tail, tail_cap)), "bhg_table_tail")
        return tail, off, ln[:ntables], stats[:4 * ntables]

    def rebuild_tables(self, src_t, table_off):
        """bhg_rebuild_tables (Writer.rebuild, writer.go:539-583) over footerless
        tables src_t[table_off[t]:table_off[t+1]].  Returns device tensors
        (handles int64 pairs [count], first [ntables+1], end [ntables],
        khash/bh_off/table int32 [count])."""
        ntab = len(table_off) - 1
        dev = self.device
        with torch.cuda.stream(self.stream):
            toff = table_off if torch.is_tensor(table_off) else _u64_tensor(table_off, dev)
            first = torch.zeros(ntab + 1, dtype=torch.int64, device=dev)
            end = torch.zeros(max(ntab, 1), dtype=torch.int64, device=dev)
        rc = self.L.bhg_scan_tables(self.ctx, _ptr(src_t), _ptr(toff), ntab, 1, None, 0, _ptr(first), _ptr(end),
                                    self._stream())
        B.check(self.ctx, rc, "bhg_scan_tables(count)")
        self.sync()
        cnt = int(first[ntab].item())
        with torch.cuda.stream(self.stream):
            h = torch.empty((max(cnt, 1), 2), dtype=torch.int64, device=dev)
            kh, bo, tb = (torch.empty(max(cnt, 1), dtype=torch.int32, device=dev) for _ in range(3))
        rc = self.L.bhg_rebuild_tables(self.ctx, _ptr(src_t), _ptr(toff), ntab, _ptr(h), cnt, _ptr(first), _ptr(end),
                                       _ptr(kh), _ptr(bo), _ptr(tb), self._stream())
        B.check(self.ctx, rc, "bhg_rebuild_tables")
        return h[:cnt], first, end[:ntab], kh[:cnt], bo[:cnt], tb[:cnt]

    def scan_tables(self, src_t, table_off, mode=0, max_out=None, paths=False):
        """TableIterator (mode 0, table.go:358-395) / Writer.rebuild (mode 1,
        writer.go:539-583) header chase over each table src_t[table_off[t]:table_off[t+1]].

        Returns device tensors (handles [count] HANDLE_DT-shaped int64 pairs,
        first [ntables+1] int64, end [ntables] int64).  max_out=None counts first
        (one extra scan) and sizes the handle buffer exactly.  paths=True adds a
        fourth tensor: per table, the pass that wrote its handles (B.SCAN_PATH_*)."""
        ntab = len(table_off) - 1
        with torch.cuda.stream(self.stream):
            toff = table_off if torch.is_tensor(table_off) else _u64_tensor(table_off, self.device)
            first = torch.zeros(ntab + 1, dtype=torch.int64, device=self.device)
            end = torch.zeros(max(ntab, 1), dtype=torch.int64, device=self.device)
            path = torch.full((max(ntab, 1),), -1, dtype=torch.int32, device=self.device)
        if max_out is None:
            rc = self.L.bhg_scan_tables(self.ctx, _ptr(src_t), _ptr(toff), ntab, mode, None, 0, _ptr(first),
                                        _ptr(end), self._stream())
            B.check(self.ctx, rc, "bhg_scan_tables")
            self.sync()
            max_out = int(first[ntab].item())
        with torch.cuda.stream(self.stream):
            out = torch.empty((max(max_out, 1), 2), dtype=torch.int64, device=self.device)
        if paths:
            rc = self.L.bhg_scan_tables_paths(self.ctx, _ptr(src_t), _ptr(toff), ntab, mode, _ptr(out), max_out,
                                              _ptr(first), _ptr(end), _ptr(path), self._stream())
            B.check(self.ctx, rc, "bhg_scan_tables_paths")
            return out[:max_out], first, end[:ntab], path[:ntab]
        rc = self.L.bhg_scan_tables(self.ctx, _ptr(src_t), _ptr(toff), ntab, mode, _ptr(out), max_out, _ptr(first),
                                    _ptr(end), self._stream())
        B.check(self.ctx, rc, "bhg_scan_tables")
        return out[:max_out], first, end[:ntab]


def read_record_status(desc_row):
    """block2Reader.readRecord (block2.go:57-66) outcome for one descriptor:
    raises the Go sentinel the reader would return, else (key_off, key_len, val_off, val_len)."""
    if int(desc_row["status"]) != B.ST_OK:
        raise BithashCodecError(desc_row["status"])
    return (int(desc_row["key_off"]), int(desc_row["key_len"]), int(desc_row["val_off"]), int(desc_row["val_len"]))


def _u64_tensor(a, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64).copy()).to(device)


def _u32_tensor(a, device):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32).copy()).to(device)


class EncodeBuffers:
    """Device outputs of bhg_encode_batch (bhg_encode_out)."""

    def __init__(self, n, max_tables, device):
        z = lambda k, dt: torch.zeros(k, dtype=dt, device=device)
        self.pos = z(n, torch.int64)
        self.bh_off = z(n, torch.int32)
        self.bh_len = z(n, torch.int32)
        self.table = z(n, torch.int32)
        self.fnv1 = z(n, torch.int32)
        self.crc = z(n, torch.int32)
        self.status = z(n, torch.int32)
        self.table_start = z(max_tables, torch.int32)
        self.summary = z(4, torch.int64)
        self.rec = z(max(n, 1) * 2, torch.int64)           # bhg_handle[n]
        self.table_size = z(max_tables, torch.int64)

    def struct(self):
        return B.EncodeOut(*[_ptr(getattr(self, f)) for f, _ in B.EncodeOut._fields_])


def _encode_codec(self, keys_t, key_off_t, trailers_t, vals_t, val_off_t, n, codec, file_nums_t, max_tables,
                  init_size, table_max, out_t, bufs, stream=None, vals_len=None):
    """Device-resident bhg_encode_batch (all tensors on the codec's device).
    vals_len = val_off[n] (defaults to vals_t.numel(), an upper bound)."""
    o = bufs.struct()
    if vals_len is None:
        vals_len = vals_t.numel()
    rc = self.L.bhg_encode_batch(self.ctx, _ptr(keys_t), _ptr(key_off_t), _ptr(trailers_t), _ptr(vals_t),
                                 _ptr(val_off_t), vals_len, n, codec, _ptr(file_nums_t), max_tables, init_size,
                                 table_max, _ptr(out_t), out_t.numel(), ctypes.byref(o),
                                 stream if stream is not None else self._stream())
    B.check(self.ctx, rc, "bhg_encode_batch")
    return bufs


def _encode_ikey_codec(self, keys_t, key_off_t, trailers_t, vals_t, val_off_t, n, khash_t, rec_file_nums_t, live_t,
                       init_size, out_t, bufs, stream=None):
    """Device-resident bhg_encode_ikey_batch: BithashWriter.AddIkey over a batch
    (compaction re-pack, bitree/bithash.go:217-239)."""
    o = bufs.struct()
    rc = self.L.bhg_encode_ikey_batch(self.ctx, _ptr(keys_t), _ptr(key_off_t), _ptr(trailers_t), _ptr(vals_t),
                                      _ptr(val_off_t), n, _ptr(khash_t), _ptr(rec_file_nums_t), _ptr(live_t),
                                      init_size, _ptr(out_t), out_t.numel(), ctypes.byref(o),
                                      stream if stream is not None else self._stream())
    B.check(self.ctx, rc, "bhg_encode_ikey_batch")
    return bufs


def _encode_result(bufs, out, nt):
    summ = bufs.summary.cpu().numpy().view(np.uint64)
    total = int(summ[0])
    u32 = lambda t: t.cpu().numpy().view(np.uint32)
    return dict(out=out[:min(total, out.numel())].cpu().numpy(), pos=bufs.pos.cpu().numpy().view(np.uint64),
                bh_off=u32(bufs.bh_off), bh_len=u32(bufs.bh_len), table=u32(bufs.table), fnv=u32(bufs.fnv1),
                crc=u32(bufs.crc), status=u32(bufs.status), table_start=u32(bufs.table_start)[:nt], ntables=nt,
                summary=summ.copy(), bufs=bufs, out_t=out)


def _encode(self, keys, trailers, values, compressor=NoCompressor, file_nums=(1,), init_size=0,
            table_max=128 << 20, out_cap=None):
    """BithashWriter.Add over a host batch (lists of bytes); results as numpy (oracle-shaped dict)."""
    dev = self.device
    with torch.cuda.stream(self.stream):
        n = len(keys)
        key_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([len(k) for k in keys], out=key_off[1:])
        val_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([len(v) for v in values], out=val_off[1:])
        kb = as_device_bytes(b"".join(keys) or b"\0", dev)
        vb = as_device_bytes(b"".join(values) or b"\0", dev)
        if out_cap is None:
            out_cap = int(sum(20 + len(k) + len(v) + len(v) // 6 + 32 for k, v in zip(keys, values))) + 16
        out = torch.zeros(max(out_cap, 1), dtype=torch.uint8, device=dev)
        bufs = EncodeBuffers(n, len(file_nums), dev)
        self.encode_batch(kb, _u64_tensor(key_off, dev), _u64_tensor(trailers, dev), vb, _u64_tensor(val_off, dev),
                          n, compressor, _u32_tensor(file_nums, dev), len(file_nums), init_size, table_max, out, bufs,
                          vals_len=int(val_off[-1]))
        self.sync()
        nt = int(bufs.summary.cpu().numpy().view(np.uint64)[1])
        if nt == 0:
            raise ValueError("not enough file numbers for the table splits")
        return _encode_result(bufs, out, nt)


def _encode_ikey(self, keys, trailers, values, rec_file_nums, live=None, khash=None, init_size=0, out_cap=None):
    """BithashWriter.AddIkey over a host batch: values are written as given
    (stored bytes), header fileNum per record, records with live[i] == 0
    skipped (BHG_ST_SKIPPED).  Results as numpy (oracle-shaped dict)."""
    dev = self.device
    with torch.cuda.stream(self.stream):
        n = len(keys)
        key_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([len(k) for k in keys], out=key_off[1:])
        val_off = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([len(v) for v in values], out=val_off[1:])
        kb = as_device_bytes(b"".join(keys) or b"\0", dev)
        vb = as_device_bytes(b"".join(values) or b"\0", dev)
        if out_cap is None:
            out_cap = int(sum(20 + len(k) + len(v) for k, v in zip(keys, values))) + 16
        out = torch.zeros(max(out_cap, 1), dtype=torch.uint8, device=dev)
        bufs = EncodeBuffers(n, 1, dev)
        live_t = None if live is None else torch.from_numpy(np.ascontiguousarray(live, dtype=np.uint8)).to(dev)
        kh_t = None if khash is None else _u32_tensor(khash, dev)
        self.encode_ikey_batch(kb, _u64_tensor(key_off, dev), _u64_tensor(trailers, dev), vb,
                               _u64_tensor(val_off, dev), n, kh_t, _u32_tensor(rec_file_nums, dev), live_t, init_size,
                               out, bufs)
        self.sync()
        return _encode_result(bufs, out, 1)


BithashCodec.encode_batch = _encode_codec
BithashCodec.encode_ikey_batch = _encode_ikey_codec
BithashCodec.encode = _encode
BithashCodec.encode_ikey = _encode_ikey


def _encode_tables(self, keys, trailers, values, compressor=NoCompressor, file_nums=(1,), table_max=128 << 20):
    """A whole flush on the GPU: BithashWriter.Add over the batch (table
    splits included), then every table closed with Writer.writeTable
    (bhg_table_tail).  Returns {fileNum: table file bytes} plus the encode
    result; the mirror of FlushStart/Add.../FlushFinish on a compacting flush
    (bithash_writer.go:25-87) where every table is finished."""
    res = self.encode(keys, trailers, values, compressor=compressor, file_nums=file_nums, table_max=table_max)
    dev = self.device
    nt = res["ntables"]
    bufs = res["bufs"]
    with torch.cuda.stream(self.stream):
        out_t = res["out_t"]
        tail, off, ln, stats = self.table_tail(out_t, bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table, bufs.status,
                                               len(keys), nt, bufs.table_size)
        self.sync()
    tail = tail.cpu().numpy()
    off = off.cpu().numpy()
    ln = ln.cpu().numpy()
    sizes = bufs.table_size.cpu().numpy()[:nt]
    out = res["out"]
    files = {}
    ts = list(res["table_start"]) + [len(keys)]
    pos = res["pos"]
    for t in range(nt):
        ok = [i for i in range(ts[t], ts[t + 1]) if res["status"][i] == 0]
        start = int(pos[ok[0]]) - int(res["bh_off"][ok[0]]) if ok else 0
        data = out[start:start + int(sizes[t])].tobytes() if ok else b""
        files[int(file_nums[t])] = data + tail[int(off[t]):int(off[t]) + int(ln[t])].tobytes()
    return files, res, stats.cpu().numpy().view(np.uint32).reshape(-1, 4)


BithashCodec.encode_tables = _encode_tables


def _repack_batch(self, src_t, handles_t, n, live_t=None, khash_t=None, init_size=0, out_t=None, bufs=None):
    """bhg_repack_batch: the live records of a TableIterator pass re-packed
    byte for byte into one destination table (compaction's AddIkey loop)."""
    dev = self.device
    with torch.cuda.stream(self.stream):
        if out_t is None:
            out_t = torch.zeros(max(src_t.numel(), 1), dtype=torch.uint8, device=dev)
        if bufs is None:
            bufs = EncodeBuffers(n, 1, dev)
    o = bufs.struct()
    rc = self.L.bhg_repack_batch(self.ctx, _ptr(src_t), src_t.numel(), _ptr(handles_t), n, _ptr(live_t),
                                 _ptr(khash_t), init_size, _ptr(out_t), out_t.numel(), ctypes.byref(o), self._stream())
    B.check(self.ctx, rc, "bhg_repack_batch")
    return out_t, bufs


def _compact(self, src_t, table_off, live=None, init_size=0):
    """compactBithashFiles (bitree/bithash.go:158-270) for the bithash side, all
    on the GPU: TableIterator scan of every source table (bhg_scan_tables mode
    0), the liveness filter + AddIkey re-pack (bhg_repack_batch), and the
    destination's Writer.writeTable (bhg_table_tail).  live: per scanned record
    (scan order), host or device u8; None keeps everything.
    Returns (table file bytes, per-record statuses, handles numpy)."""
    dev = self.device
    h_t, first, _ = self.scan_tables(src_t, table_off, mode=0)
    self.sync()
    n = int(h_t.shape[0]) if int(first[-1].item()) else 0
    with torch.cuda.stream(self.stream):
        live_t = None
        if live is not None:
            live_t = live if torch.is_tensor(live) else torch.from_numpy(np.ascontiguousarray(live, np.uint8)).to(dev)
    out_t, bufs = self.repack_batch(src_t, h_t, n, live_t, None, init_size)
    tail, off, ln, stats = self.table_tail(out_t, bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table, bufs.status, n, 1,
                                           bufs.table_size)
    self.sync()
    size = int(bufs.table_size[0].item())
    data = out_t[:size - init_size].cpu().numpy().tobytes()
    t = tail.cpu().numpy()
    return data + t[int(off[0]):int(off[0]) + int(ln[0])].tobytes(), bufs.status.cpu().numpy().view(np.uint32)[:n], \
        h_t.cpu().numpy().view(HANDLE_DT).reshape(-1)[:n]


BithashCodec.repack_batch = _repack_batch
BithashCodec.compact = _compact
