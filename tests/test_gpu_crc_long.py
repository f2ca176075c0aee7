"""GPU parity for bhg_crc32c_masked_long (one workgroup per range) and the
per-table indexhash_checksum verify built on it (SURVEY 8(a) A6(ii);
the checksum is written at bithash/writer.go:476-478)."""
import os
import random

import numpy as np
import pytest
import torch

from bitalosdb_amd import table as BT
from oracle import oracle as O
from oracle import table as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd import _lib
    from bitalosdb_amd.codec import BithashCodec
    _lib.lib()
    c = BithashCodec(0)
    yield c
    c.close()


def test_long_ranges_match_restatement(codec):
    """Span-boundary lengths (256-B spans aligned to the range end, 64 x 256 of them before the
    span doubles at 4 MiB, 8 MiB, 16 MiB ...; four chains per full span, one for a partial
    first span; round 4's 1-KiB spans kept in the list), odd alignments, empty and out-of-range
    handles, a range ending at the last byte of the source."""
    from bitalosdb_amd.codec import as_device_bytes, handles_tensor
    rng = np.random.default_rng(21)
    size = 20 << 20
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    dsrc = as_device_bytes(data, codec.device)
    K = 4096
    M16 = 16 << 20
    M4 = 4 << 20
    lens = [0, 1, 3, 4, 5, 63, 64, 255, 256, 257, 511, 512, 513, 767, 1023, 1024, 1025, 4095, K, K + 1,
            2 * K - 1, 2 * K, 2 * K + 1, 1_510_000, M4 - 1, M4, M4 + 1, M4 + 255, M4 + 257, 2 * M4 - 1,
            2 * M4 + 1, 2048 * K - 1, 2048 * K, 2048 * K + 1, M16 - 1, M16, M16 + 1, M16 + 1023, M16 + 1025,
            17 << 20]
    hs = []
    for ln in lens:
        for off in (0, 1, 2, 3, 1001):
            if off + ln <= size:
                hs.append((off, ln, 0))
    hs += [(size, 0, 0), (size - 10, 11, 0), (size + 1, 0, 0), (0, size, 0), (1, size - 1, 0),
           (size - 4099, 4099, 0), (size - M4 - 3, M4 + 3, 0)]
    h = np.array(hs, dtype=O.HANDLE_DT)
    got = codec.crc_long(dsrc, handles_tensor(h, codec.device), len(h)).cpu().numpy().view(np.uint32)
    short = codec.crc_batch(dsrc, handles_tensor(h, codec.device), len(h)).cpu().numpy().view(np.uint32)
    for i, (o, ln, _) in enumerate(hs):
        exp = O.crc_masked(data[o:o + ln]) if o + ln <= size else 0
        assert got[i] == exp, (o, ln)
        assert short[i] == exp, (o, ln)   # the lane-per-range primitive agrees
    assert got[hs.index((0, 0, 0))] == 0xA282EAD8                # crc.New("") masked


def test_verify_index_checksums(codec):
    """Every table the restated writer produced (K2 golden table + random
    tables incl. an empty one) verifies; a flipped indexhash byte does not."""
    from bitalosdb_amd.codec import as_device_bytes
    blobs = [open(os.path.join(GOLD, "k2.bht"), "rb").read()]
    rng = random.Random(3)
    for n in (0, 1, 500, 5000):
        w = T.Writer(10 + n, 1 << 30)
        for i in range(n):
            w.add(bytes(rng.randrange(97, 123) for _ in range(32)), (i + 1) << 8 | 1, b"v" * rng.randrange(1, 64))
        w.write_table(True)
        blobs.append(bytes(w.file))
    infos, bases, base = [], [], 0
    for b in blobs:
        infos.append(BT.open_table(b, base=base)[1])
        bases.append(base)
        base += len(b)
    src = bytearray(b"".join(blobs))
    ok, got = BT.verify_index_checksums(codec, as_device_bytes(bytes(src), codec.device), infos, bases)
    assert ok.all()
    for b, info, g in zip(blobs, infos, got):
        off, ln = info["index_data"]
        assert g == O.crc_masked(b[off:off + ln])
    # corrupt one byte of the last table's HashIndex items
    off, ln = infos[-1]["index_data"]
    src[bases[-1] + off + ln - 1] ^= 0x5A
    ok, _ = BT.verify_index_checksums(codec, as_device_bytes(bytes(src), codec.device), infos, bases)
    assert list(ok) == [True] * (len(blobs) - 1) + [False]
