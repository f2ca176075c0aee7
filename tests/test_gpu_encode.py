"""GPU parity for the batched BithashWriter.Add path (bhg_encode_batch) against
the CPU restatement of writer.go:230-283 + bithash_writer.go:25-67."""
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd.codec import BithashCodec
    c = BithashCodec(0)
    yield c
    c.close()


def rb(rng, n):
    return bytes(rng.randrange(256) for _ in range(n))


def check(got, exp):
    assert got["ntables"] == exp["ntables"]
    assert np.array_equal(got["table_start"], exp["table_start"])
    for f in ("status", "fnv", "bh_off", "bh_len", "table", "crc", "pos"):
        g, e = got[f], exp[f]
        ok = e["status"] == 0 if False else None
        bad = np.nonzero(g != e)[0]
        assert bad.size == 0, (f, bad[:8], g[bad[:8]], e[bad[:8]])
    assert got["out"].tobytes() == exp["out"].tobytes()


@pytest.mark.parametrize("seed,table_max,init", [(1, 128 << 20, 0), (2, 1 << 16, 0), (3, 1 << 16, 40000),
                                                 (4, 5000, 4999), (5, 3000, 0)])
def test_encode_none_matches_restatement(codec, seed, table_max, init):
    rng = random.Random(seed)
    n = 3000
    keys = [rb(rng, rng.choice([0, 1, 7, 31, 32, 33, 64])) for _ in range(n)]
    vals = [rb(rng, rng.choice([0, 1, 3, 64, 100, 1024, 4096])) for _ in range(n)]
    trailers = [((i + 1) << 8) | 1 for i in range(n)]
    fns = list(range(10, 10 + 2000))
    got = codec.encode(keys, trailers, vals, file_nums=fns, init_size=init, table_max=table_max)
    exp = O.encode_batch(keys, trailers, vals, file_nums=fns, init_size=init, table_max=table_max)
    check(got, exp)


def test_encode_k1_split_sizes(codec):
    """K1: 1200 x 2 KiB values, TableMaxSize 1 MiB -> tables of 1,049,651 / 1,049,767 B, third at 405,072."""
    rng = random.Random(7)
    keys = [b"bithash_testkey_%d" % i for i in range(1200)]
    vals = [rb(rng, 2048) for _ in range(1200)]
    tr = [((i + 1) << 8) | 1 for i in range(1200)]
    got = codec.encode(keys, tr, vals, file_nums=[1, 2, 3, 4], table_max=1 << 20)
    exp = O.encode_batch(keys, tr, vals, file_nums=[1, 2, 3, 4], table_max=1 << 20)
    check(got, exp)
    assert got["ntables"] == 3
    ts = list(got["table_start"]) + [1200]
    sizes = [int(got["bh_off"][ts[t + 1] - 1] + got["bh_len"][ts[t + 1] - 1]) for t in range(3)]
    assert sizes == [1049651, 1049767, 405072]


def test_encode_too_large(codec):
    rng = random.Random(8)
    keys = [b"a" * 10, b"b" * ((33 << 10) - 7), b"c" * 5, b"d" * ((33 << 10) - 8)]
    vals = [b"x" * 10, b"y", b"z" * 3, b"w"]
    tr = [1 << 8 | 1] * 4
    got = codec.encode(keys, tr, vals, file_nums=[5, 6])
    exp = O.encode_batch(keys, tr, vals, file_nums=[5, 6])
    check(got, exp)
    assert list(got["status"]) == [0, O.KEY_TOO_LARGE, 0, 0]


def test_encode_then_decode_roundtrip(codec):
    rng = random.Random(9)
    n = 2000
    keys = [rb(rng, 32) for _ in range(n)]
    vals = [rb(rng, rng.randrange(64, 4097)) for _ in range(n)]
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, file_nums=[1, 2, 3], table_max=4 << 20)
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = got["pos"]
    h["length"] = got["bh_len"]
    desc, _, _ = codec.decode(got["out"], h)
    assert (desc["status"] == 0).all()
    assert np.array_equal(desc["crc"], got["crc"])
    assert np.array_equal(desc["fnv1"], got["fnv"])
    out = got["out"]
    for i in (0, 1, 999, n - 1):
        o = int(h["offset"][i]) + int(desc["val_off"][i])
        assert out[o:o + int(desc["val_len"][i])].tobytes() == vals[i]


def compressible(rng, n):
    d = rb(rng, 700)
    out = bytearray()
    while len(out) < n:
        if rng.random() < 0.2:
            out += rb(rng, rng.randrange(1, 16))
        else:
            ln = rng.randrange(4, 64)
            st = rng.randrange(0, 700 - ln)
            out += d[st:st + ln]
    return bytes(out[:n])


@pytest.mark.parametrize("seed", [11, 12])
def test_encode_snappy_byte_exact(codec, seed):
    """golang/snappy v0.0.4 Encode on the GPU == the restated encoder, byte for byte
    (incl. values > 4 KiB -> serial block path, and > 64 KiB -> block split)."""
    rng = random.Random(seed)
    n = 1500
    sizes = [rng.choice([0, 1, 16, 17, 18, 40, 64, 100, 1024, 2048, 4095, 4096, 4097, 9000]) for _ in range(n)]
    sizes[7] = 70000
    sizes[8] = 131072 + 5
    keys = [rb(rng, 32) for _ in range(n)]
    vals = []
    for i, sz in enumerate(sizes):
        kind = i % 4
        if kind == 0:
            vals.append(compressible(rng, sz))
        elif kind == 1:
            vals.append(rb(rng, sz))
        elif kind == 2:
            vals.append((b"abcd" * (sz // 4 + 1))[:sz])
        else:
            vals.append(bytes(sz))
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, compressor=1, file_nums=list(range(1, 50)), table_max=1 << 20)
    exp = O.encode_batch(keys, tr, vals, codec=1, file_nums=list(range(1, 50)), table_max=1 << 20)
    check(got, exp)
    # and the records decode back (GPU snappy decode) to the raw values
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = got["pos"]
    h["length"] = got["bh_len"]
    desc, dv, doff = codec.decode(got["out"], h, compressor=1)
    assert (desc["status"] == 0).all()
    for i in range(0, n, 37):
        assert dv[int(doff[i]):int(doff[i + 1])].tobytes() == vals[i]
