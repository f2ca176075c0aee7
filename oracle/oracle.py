"""ctypes wrapper over the C restatement (oracle/bithash_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

HANDLE_DT = np.dtype([("offset", "<u8"), ("length", "<u4"), ("pad", "<u4")])
DESC_DT = np.dtype([("key_off", "<u4"), ("key_len", "<u4"), ("val_off", "<u4"), ("val_len", "<u4"),
                    ("trailer", "<u8"), ("file_num", "<u4"), ("fnv1", "<u4"), ("crc", "<u4"),
                    ("status", "<u4")])
assert HANDLE_DT.itemsize == 16 and DESC_DT.itemsize == 40

OK, RECORD_NIL, ILLEGAL_LENGTH, INCOMPLETE, SNAPPY_CORRUPT, SNAPPY_TOO_LARGE, CRC_MISMATCH = range(7)
KEY_TOO_LARGE, VALUE_TOO_LARGE, DATA_MAX_EXCEEDED = 7, 8, 9
NOT_FOUND, NO_SPACE, SKIPPED = 10, 11, 12  # include/bithashgpu.h (encode-side statuses of the C-ABI)

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, U32, U64, SZ, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
        L.bho_crc32c_update.restype = U32
        L.bho_crc32c_update.argtypes = [U32, P, SZ]
        L.bho_crc32c_update_hw.restype = U32
        L.bho_crc32c_update_hw.argtypes = [U32, P, SZ]
        L.bho_crc_mask.restype = U32
        L.bho_crc_mask.argtypes = [U32]
        L.bho_crc_masked.restype = U32
        L.bho_crc_masked.argtypes = [P, SZ]
        L.bho_fnv32.restype = U32
        L.bho_fnv32.argtypes = [P, SZ]
        L.bho_snappy_max_encoded_len.restype = ctypes.c_int64
        L.bho_snappy_max_encoded_len.argtypes = [ctypes.c_int64]
        L.bho_snappy_encode.restype = SZ
        L.bho_snappy_encode.argtypes = [P, P, SZ]
        L.bho_snappy_decoded_len.restype = I
        L.bho_snappy_decoded_len.argtypes = [P, SZ, ctypes.POINTER(U64), ctypes.POINTER(SZ)]
        L.bho_snappy_decode.restype = I
        L.bho_snappy_decode.argtypes = [P, U64, P, SZ]
        L.bho_record_set.restype = SZ
        L.bho_record_set.argtypes = [P, P, SZ, U64, P, SZ, U32]
        L.bho_decode_batch.restype = None
        L.bho_decode_batch.argtypes = [P, U64, P, U32, I, P, P, P, P, I]
        L.bho_decode_batch_pread.restype = None
        L.bho_decode_batch_pread.argtypes = [I, P, U32, P, P, I]
        L.bho_decode_sizes.restype = None
        L.bho_decode_sizes.argtypes = [P, U64, P, U32, P]
        L.bho_encode_batch.restype = I
        L.bho_encode_batch.argtypes = [P, P, P, P, P, U32, I, P, I, U32, U64, P, P, P, P, P, P, P, P, P, P]
        L.bho_encode_batch_mt.restype = U64
        L.bho_encode_batch_mt.argtypes = [P, P, P, P, P, U32, I, U64, I]
        L.bho_scan_region.restype = ctypes.c_int64
        L.bho_scan_region.argtypes = [P, U64, I, P, U64, ctypes.POINTER(U64)]
        _lib = L
    return _lib


def _buf(b):
    """bytes/bytearray/np.ndarray -> (keepalive, pointer, length)."""
    if isinstance(b, np.ndarray):
        a = np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    else:
        a = np.frombuffer(bytes(b), dtype=np.uint8)
    return a, (a.ctypes.data if a.size else None), a.size


def _ptr(a):
    return None if a is None else a.ctypes.data


def crc32c(data, crc=0, hw=False):
    a, p, n = _buf(data)
    return (lib().bho_crc32c_update_hw if hw else lib().bho_crc32c_update)(crc, p, n)


def crc_mask(c):
    return lib().bho_crc_mask(c)


def crc_masked(data):
    a, p, n = _buf(data)
    return lib().bho_crc_masked(p, n)


def fnv32(data):
    a, p, n = _buf(data)
    return lib().bho_fnv32(p, n)


def snappy_max_encoded_len(n):
    return lib().bho_snappy_max_encoded_len(n)


def snappy_encode(data):
    a, p, n = _buf(data)
    out = np.empty(max(1, snappy_max_encoded_len(n)), dtype=np.uint8)
    m = lib().bho_snappy_encode(out.ctypes.data, p, n)
    return out[:m].tobytes()


class SnappyCorrupt(Exception):
    """snappy: corrupt input (golang/snappy ErrCorrupt)."""


def snappy_decoded_len(data):
    a, p, n = _buf(data)
    v, h = ctypes.c_uint64(), ctypes.c_size_t()
    if lib().bho_snappy_decoded_len(p, n, ctypes.byref(v), ctypes.byref(h)) != 0:
        raise SnappyCorrupt("snappy: corrupt input")
    return v.value, h.value


def snappy_decode(data):
    dlen, _ = snappy_decoded_len(data)
    a, p, n = _buf(data)
    out = np.empty(max(1, dlen), dtype=np.uint8)
    if lib().bho_snappy_decode(out.ctypes.data, dlen, p, n) != 0:
        raise SnappyCorrupt("snappy: corrupt input")
    return out[:dlen].tobytes()


def record_set(ukey, trailer, value, file_num):
    out = np.empty(12 + len(ukey) + 8 + len(value), dtype=np.uint8)
    ka, kp, kn = _buf(ukey)
    va, vp, vn = _buf(value)
    m = lib().bho_record_set(out.ctypes.data, kp, kn, trailer, vp, vn, file_num)
    return out[:m].tobytes()


def _u8(src):
    if isinstance(src, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(src), dtype=np.uint8)
    return np.ascontiguousarray(src).view(np.uint8).reshape(-1)


def decode_sizes(src, handles):
    src = _u8(src)
    handles = np.ascontiguousarray(handles, dtype=HANDLE_DT)
    out = np.zeros(len(handles), dtype=np.uint64)
    lib().bho_decode_sizes(_ptr(src), src.size, _ptr(handles), len(handles), _ptr(out))
    return out


def decode_batch(src, handles, codec=0, expected_crc=None, nthreads=0, out_val_off=None):
    """Batch Reader.readData semantics.  Returns (desc, out_vals, out_val_off).

    nthreads=0: single thread, reference-definition CRC (checker mode);
    nthreads>=1: threaded, SSE4.2 CRC (baseline mode)."""
    src = _u8(src)
    handles = np.ascontiguousarray(handles, dtype=HANDLE_DT)
    n = len(handles)
    desc = np.zeros(n, dtype=DESC_DT)
    vals = None
    if codec == 1:
        if out_val_off is None:
            sizes = decode_sizes(src, handles)
            out_val_off = np.zeros(n + 1, dtype=np.uint64)
            np.cumsum(sizes, out=out_val_off[1:])
        out_val_off = np.ascontiguousarray(out_val_off, dtype=np.uint64)
        vals = np.zeros(max(1, int(out_val_off[-1])), dtype=np.uint8)
    exp = None if expected_crc is None else np.ascontiguousarray(expected_crc, dtype=np.uint32)
    lib().bho_decode_batch(_ptr(src), src.size, _ptr(handles), n, codec, _ptr(exp), _ptr(desc),
                           _ptr(vals), _ptr(out_val_off), nthreads)
    return desc, vals, out_val_off


def decode_batch_pread(fd, handles, expected_crc=None, nthreads=1):
    """Reader.readData with one pread per block (reader.go:251), codec NONE,
    baseline mode.  fd: an open file descriptor of the table bytes."""
    handles = np.ascontiguousarray(handles, dtype=HANDLE_DT)
    desc = np.zeros(len(handles), dtype=DESC_DT)
    exp = None if expected_crc is None else np.ascontiguousarray(expected_crc, dtype=np.uint32)
    lib().bho_decode_batch_pread(fd, _ptr(handles), len(handles), _ptr(exp), _ptr(desc), nthreads)
    return desc


def encode_batch(keys, trailers, values, codec=0, file_nums=(1,), init_size=0, table_max=128 << 20):
    """BithashWriter.Add over a batch. keys/values: lists of bytes."""
    n = len(keys)
    key_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(k) for k in keys], out=key_off[1:])
    val_off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum([len(v) for v in values], out=val_off[1:])
    kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
    vb = np.frombuffer(b"".join(values) or b"\0", dtype=np.uint8)
    tr = np.ascontiguousarray(trailers, dtype=np.uint64)
    fns = np.ascontiguousarray(file_nums, dtype=np.uint32)
    cap = int(sum(12 + len(k) + 8 + max(len(v), snappy_max_encoded_len(len(v)) if codec else 0)
                  for k, v in zip(keys, values))) + 1
    out = np.zeros(cap, dtype=np.uint8)
    out_len = ctypes.c_uint64()
    pos = np.zeros(n, dtype=np.uint64)
    bh_off = np.zeros(n, dtype=np.uint32)
    bh_len = np.zeros(n, dtype=np.uint32)
    tab = np.zeros(n, dtype=np.uint32)
    fnv = np.zeros(n, dtype=np.uint32)
    crc = np.zeros(n, dtype=np.uint32)
    st = np.zeros(n, dtype=np.uint32)
    tstart = np.zeros(len(fns), dtype=np.uint32)
    nt = lib().bho_encode_batch(_ptr(kb), _ptr(key_off), _ptr(tr), _ptr(vb), _ptr(val_off), n, codec,
                                _ptr(fns), len(fns), init_size, table_max, _ptr(out), ctypes.byref(out_len),
                                _ptr(pos), _ptr(bh_off), _ptr(bh_len), _ptr(tab), _ptr(fnv), _ptr(crc),
                                _ptr(st), _ptr(tstart))
    if nt < 0:
        raise ValueError("not enough file numbers for the table splits")
    return dict(out=out[:out_len.value], pos=pos, bh_off=bh_off, bh_len=bh_len, table=tab, fnv=fnv,
                crc=crc, status=st, table_start=tstart[:nt], ntables=nt)


def encode_batch_mt(keys, key_off, trailers, vals, val_off, n, codec=1, table_max=128 << 20, nthreads=1):
    """CPU baseline of the encode path (bho_encode_batch_mt): flat numpy keys /
    values with u64 offsets[n+1]; nthreads independent writers over contiguous
    pair ranges.  Returns the bytes written."""
    kb, vb = _u8(keys), _u8(vals)
    ko = np.ascontiguousarray(key_off, dtype=np.uint64)
    vo = np.ascontiguousarray(val_off, dtype=np.uint64)
    tr = np.ascontiguousarray(trailers, dtype=np.uint64)
    w = lib().bho_encode_batch_mt(_ptr(kb), _ptr(ko), _ptr(tr), _ptr(vb), _ptr(vo), n, codec, table_max, nthreads)
    if w == 0 and n:
        raise MemoryError("bho_encode_batch_mt")
    return w


def scan_region(data, mode=0, max_records=None):
    a, p, n = _buf(data)
    if max_records is None:
        max_records = n // 12 + 1
    out = np.zeros(max_records, dtype=HANDLE_DT)
    end = ctypes.c_uint64()
    cnt = lib().bho_scan_region(p, n, mode, _ptr(out), max_records, ctypes.byref(end))
    return out[:min(cnt, max_records)], end.value
