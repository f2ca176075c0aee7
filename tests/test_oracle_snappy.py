"""Snappy restatement (golang/snappy v0.0.4, go.mod:7) -- interop and edge cases.

golang/snappy is an un-vendored third-party dependency.  The
decode side is pinned by interop with an independent implementation
(pyarrow's Google C++ snappy) in both directions; the encode side is checked
for validity + round trip; golang byte-identity of encoded streams is
"parity unpinned" (no golden vector exists in the reference).
"""
import random

import numpy as np
import pyarrow as pa
import pytest

from oracle import oracle as O


def compressible(rng, n):
    dictionary = bytes(rng.randrange(256) for _ in range(4096))
    out = bytearray()
    while len(out) < n:
        if rng.random() < 0.2:
            out += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 16)))
        else:
            ln = rng.randrange(4, 64)
            st = rng.randrange(0, 4096 - ln)
            out += dictionary[st:st + ln]
    return bytes(out[:n])


SIZES = [0, 1, 2, 15, 16, 17, 18, 31, 59, 60, 61, 62, 64, 255, 256, 257, 1000, 1024, 4096, 65535, 65536,
         65537, 140000]


@pytest.mark.parametrize("n", SIZES)
def test_encode_roundtrip_and_pyarrow_decodes_ours(n):
    rng = random.Random(n)
    for data in (compressible(rng, n), bytes(rng.randrange(256) for _ in range(min(n, 5000))), b"a" * n):
        enc = O.snappy_encode(data)
        assert len(enc) <= O.snappy_max_encoded_len(len(data))
        assert O.snappy_decode(enc) == data
        got = pa.decompress(enc, decompressed_size=len(data), codec="snappy", asbytes=True)
        assert got == data


@pytest.mark.parametrize("n", SIZES)
def test_we_decode_pyarrow(n):
    rng = random.Random(1000 + n)
    data = compressible(rng, n)
    enc = pa.compress(data, codec="snappy", asbytes=True)
    assert O.snappy_decode(enc) == data


def test_encode_known_shapes():
    # < 17 bytes: a single literal (minNonLiteralBlockSize = 1 + 1 + inputMargin)
    assert O.snappy_encode(b"") == b"\x00"
    assert O.snappy_encode(b"abc") == b"\x03\x08abc"
    # 16 x 'a': still a literal
    assert O.snappy_encode(b"a" * 16) == b"\x10" + bytes([15 << 2]) + b"a" * 16
    # 17 x 'a': literal 'a' then copy offset 1 (emitCopy -> tagCopy1 len 16 is >= 12 -> tagCopy2)
    enc = O.snappy_encode(b"a" * 17)
    assert O.snappy_decode(enc) == b"a" * 17
    assert enc[:3] == b"\x11\x00a"


def _stream(dlen, body):
    x, out = dlen, bytearray()
    while x >= 0x80:
        out.append(x & 0x7F | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out) + body


def test_decode_edge_streams():
    # literal forms 60/61/62/63 (1..4 extra length bytes)
    lit = bytes(range(200))
    assert O.snappy_decode(_stream(200, bytes([60 << 2, 199]) + lit)) == lit
    assert O.snappy_decode(_stream(200, bytes([61 << 2, 199, 0]) + lit)) == lit
    assert O.snappy_decode(_stream(200, bytes([62 << 2, 199, 0, 0]) + lit)) == lit
    assert O.snappy_decode(_stream(200, bytes([63 << 2, 199, 0, 0, 0]) + lit)) == lit
    # copy1 (len 4..11, offset < 2048), overlapping (offset 1 run-length)
    body = bytes([0 << 2, ord("x")]) + bytes([(11 - 4) << 2 | 1, 1])
    assert O.snappy_decode(_stream(12, body)) == b"x" * 12
    # copy2 len 64 offset 2 (periodic overlap)
    body = bytes([1 << 2]) + b"ab" + bytes([63 << 2 | 2, 2, 0])
    assert O.snappy_decode(_stream(66, body)) == b"ab" * 33
    # copy4
    body = bytes([3 << 2]) + b"wxyz" + bytes([3 << 2 | 3, 4, 0, 0, 0])
    assert O.snappy_decode(_stream(8, body)) == b"wxyz" * 2
    # corrupt: offset 0, offset > written, short output, long output, truncated tag
    bad = [
        _stream(5, bytes([0 << 2, 1]) + bytes([0 << 2 | 1, 0])),
        _stream(9, bytes([0 << 2, 1]) + bytes([(8 - 4) << 2 | 1, 2])),
        _stream(3, bytes([0 << 2, 1])),
        _stream(1, bytes([1 << 2, 1, 2])),
        _stream(5, bytes([0 << 2, 1, 2])),
        _stream(8, bytes([60 << 2])),
        b"",
        b"\xff" * 11,
        b"\x80\x80\x80\x80\x80\x80\x80\x80\x80\x02",
        b"\xff\xff\xff\xff\x1f",         # > 0xffffffff
    ]
    for b in bad:
        with pytest.raises(O.SnappyCorrupt):
            O.snappy_decode(b)
    # non-canonical (6-byte) varint of a small length is accepted (binary.Uvarint)
    assert O.snappy_decode(b"\x83\x80\x80\x80\x80\x00" + bytes([2 << 2]) + b"abc") == b"abc"


def test_block_boundary_64k():
    rng = random.Random(9)
    data = compressible(rng, 3 * 65536 + 5)
    enc = O.snappy_encode(data)
    # every 64 KiB chunk is encoded independently: no copy reaches back across it
    assert O.snappy_decode(enc) == data
    assert pa.decompress(enc, decompressed_size=len(data), codec="snappy", asbytes=True) == data
