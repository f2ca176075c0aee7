"""ctypes binding of libbithashgpu.so (include/bithashgpu.h).

The product path is the HIP library: if the shared object is missing or no
GPU is visible, every call raises -- there is no CPU fallback.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BHG_LIB_PATH") or os.path.join(_HERE, "lib", "libbithashgpu.so")  # override: lab builds
CSRC = os.path.join(_HERE, "csrc")

HANDLE_DT = np.dtype([("offset", "<u8"), ("length", "<u4"), ("pad", "<u4")])
DESC_DT = np.dtype([("key_off", "<u4"), ("key_len", "<u4"), ("val_off", "<u4"), ("val_len", "<u4"),
                    ("trailer", "<u8"), ("file_num", "<u4"), ("fnv1", "<u4"), ("crc", "<u4"),
                    ("status", "<u4")])
assert HANDLE_DT.itemsize == 16 and DESC_DT.itemsize == 40

# include/bithashgpu.h
BHG_OK, BHG_EINVAL, BHG_EHIP, BHG_ENOMEM, BHG_ENODEV, BHG_ECAPACITY = 0, -1, -2, -3, -4, -5
CODEC_NONE, CODEC_SNAPPY = 0, 1
ST_OK, ST_RECORD_NIL, ST_ILLEGAL_LENGTH, ST_INCOMPLETE, ST_SNAPPY_CORRUPT, ST_SNAPPY_TOO_LARGE, \
    ST_CRC_MISMATCH, ST_KEY_TOO_LARGE, ST_VALUE_TOO_LARGE, ST_DATA_MAX_EXCEEDED, ST_NOT_FOUND, \
    ST_NO_SPACE, ST_SKIPPED, ST_FILE_NUM_ZERO = range(14)
SCAN_PATH_SEGMENTS, SCAN_PATH_REPLAY, SCAN_PATH_SERIAL = range(3)
ABI_VERSION = 3
TABLE_DT = np.dtype([("base", "<u8"), ("index_off", "<u8"), ("index_len", "<u8"), ("conflict_off", "<u8"),
                     ("conflict_bh_off", "<u4"), ("conflict_bh_len", "<u4")])
WRITER_INDEX_DT = np.dtype([("rec", "<u8"), ("sorted", "<u8"), ("sorted_kh", "<u8"), ("n", "<u4"),
                            ("file_num", "<u4")])
assert TABLE_DT.itemsize == 40 and WRITER_INDEX_DT.itemsize == 32

EXPORTS = [
    "bhg_abi_version", "bhg_device_count", "bhg_create", "bhg_destroy", "bhg_last_error", "bhg_stream",
    "bhg_stream_sync", "bhg_malloc_device", "bhg_free_device", "bhg_malloc_host", "bhg_free_host",
    "bhg_memcpy_h2d", "bhg_memcpy_d2h", "bhg_memset_device", "bhg_decode_batch", "bhg_decode_batch_host",
    "bhg_crc32c_masked_batch", "bhg_crc32c_masked_long", "bhg_fnv32_batch", "bhg_encode_batch",
    "bhg_encode_ikey_batch", "bhg_scan_tables", "bhg_table_tail", "bhg_rebuild_tables",
    "bhg_repack_batch",
    "bhg_host_register", "bhg_host_unregister", "bhg_get_batch", "bhg_writer_index_build",
    "bhg_bithash_get_batch", "bhg_scan_tables_paths", "bhg_scan_scratch_bytes",
]


class BhgError(RuntimeError):
    pass


class EncodeOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("pos", "bh_off", "bh_len", "table", "fnv1", "crc", "status", "table_start", "summary", "rec",
                 "table_size")]


_lib = None


def build(force=False):
    """Compile the HIP sources for gfx950 into lib/libbithashgpu.so (hipcc cross-compiles; no GPU needed)."""
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(["make", "-s", "-j8", "-C", CSRC])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BhgError("libbithashgpu.so not built: run bitalosdb_amd._lib.build() / __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        if L.bhg_abi_version() != ABI_VERSION:
            raise BhgError("libbithashgpu.so ABI %d, bindings expect %d: rebuild" % (L.bhg_abi_version(), ABI_VERSION))
        P, U32, U64, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        sig = {
            "bhg_abi_version": (I, []),
            "bhg_device_count": (I, []),
            "bhg_create": (P, [I, I]),
            "bhg_destroy": (None, [P]),
            "bhg_last_error": (ctypes.c_char_p, [P]),
            "bhg_stream": (P, [P]),
            "bhg_stream_sync": (I, [P, P]),
            "bhg_malloc_device": (P, [P, U64]),
            "bhg_free_device": (I, [P, P]),
            "bhg_malloc_host": (P, [P, U64]),
            "bhg_free_host": (I, [P, P]),
            "bhg_memcpy_h2d": (I, [P, P, P, U64, P]),
            "bhg_memcpy_d2h": (I, [P, P, P, U64, P]),
            "bhg_memset_device": (I, [P, P, I, U64, P]),
            "bhg_decode_batch": (I, [P, P, U64, P, U32, I, P, P, P, U64, P, P]),
            "bhg_decode_batch_host": (I, [P, P, U64, P, U32, I, P, P, P, U64, P]),
            "bhg_crc32c_masked_batch": (I, [P, P, U64, P, U32, P, P]),
            "bhg_crc32c_masked_long": (I, [P, P, U64, P, U32, P, P]),
            "bhg_fnv32_batch": (I, [P, P, U64, P, U32, P, P]),
            "bhg_encode_batch": (I, [P, P, P, P, P, P, U64, U32, I, P, U32, U32, U64, P, U64,
                                     ctypes.POINTER(EncodeOut), P]),
            "bhg_encode_ikey_batch": (I, [P, P, P, P, P, P, U32, P, P, P, U32, P, U64,
                                          ctypes.POINTER(EncodeOut), P]),
            "bhg_scan_tables": (I, [P, P, P, U32, I, P, U64, P, P, P]),
            "bhg_scan_tables_paths": (I, [P, P, P, U32, I, P, U64, P, P, P, P]),
            "bhg_scan_scratch_bytes": (U64, [U32]),
            "bhg_table_tail": (I, [P, P, P, P, P, P, P, U32, U32, P, P, U64, P, P, P, P]),
            "bhg_rebuild_tables": (I, [P, P, P, U32, P, U64, P, P, P, P, P, P]),
            "bhg_repack_batch": (I, [P, P, U64, P, U32, P, P, U32, P, U64, ctypes.POINTER(EncodeOut), P]),
            "bhg_host_register": (I, [P, P, U64]),
            "bhg_host_unregister": (I, [P, P]),
            "bhg_get_batch": (I, [P, P, U64, P, U32, P, P, P, P, U32, P, P, P]),
            "bhg_writer_index_build": (I, [P, P, U32, P, P, P]),
            "bhg_bithash_get_batch": (I, [P, P, U64, P, U32, P, U32, P, P, U32, P, P, P, P, I, U32, P, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(ctx, rc, what):
    if rc != BHG_OK:
        msg = lib().bhg_last_error(ctx)
        raise BhgError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))
