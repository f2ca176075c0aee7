"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU half: the restatement reproduces every committed fixture byte for byte,
the K1/K2 fixtures carry the reference's asserted known answers
(bithash_test.go:643-766), and every snappy stream agrees with an independent
implementation (pyarrow's C++ snappy).  GPU half (marked gpu): the HIP path
reproduces the fixtures through the C-ABI without calling the oracle.
"""
import hashlib
import json
import os
import random
import sys

import numpy as np
import pytest

from oracle import oracle as O
from oracle import table as T

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
import make_golden as MG  # noqa: E402

FIELDS = ["key_off", "key_len", "val_off", "val_len", "trailer", "file_num", "fnv1", "crc", "status"]


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def read(name):
    return open(os.path.join(GOLD, name), "rb").read()


def snappy_cases():
    z = load("snappy_edges.npz")
    cut = lambda k, i: z[k][int(z[k + "_off"][i]):int(z[k + "_off"][i + 1])].tobytes()
    return [(cut("raw", i), cut("go", i), cut("pyarrow", i)) for i in range(len(z["raw_off"]) - 1)]


# ---------------------------------------------------------------- CPU ----

def test_k1_manifest_known_answers():
    m = json.load(open(os.path.join(GOLD, "k1_manifest.json")))
    assert m["closed_data_sizes"] == [1049651, 1049767]      # bithash_test.go:725-755
    assert m["mutable_current_offset"] == 405072
    assert MG.k1_manifest() == m


def test_k2_table_fixture():
    b = read("k2.bht")
    assert b == MG.k2_table()
    t = T.open_table(b)
    assert t["index_checksum"] == str(O.crc_masked(t["index_data"])).encode()
    assert len(T.block_entries(t["conflict_buf"])) == 12
    h, end = O.scan_region(b, mode=0)
    g = np.load(os.path.join(GOLD, "k2_scan.npy"), allow_pickle=False)
    assert len(g) == 112 and (h == g).all()


@pytest.mark.parametrize("name,codec", [("rec_none", 0), ("rec_snappy", 1)])
def test_record_fixtures(name, codec):
    src = read(name + ".bin")
    z = load(name + ".npz")
    s2, h2 = MG.records(random.Random(100 + codec), codec)
    assert s2 == src and (h2 == z["handles"]).all()
    desc, vals, voff = O.decode_batch(src, z["handles"], codec=codec)
    for f in FIELDS:
        assert (desc[f] == z["desc"][f]).all(), f
    assert (z["desc"]["status"][:266] == 0).all() and (z["desc"]["status"][266:] != 0).all()
    if codec:
        assert (voff == z["val_off"]).all()
        assert vals[:int(voff[-1])].tobytes() == z["vals"].tobytes()


def test_snappy_edges_vs_pyarrow():
    import pyarrow as pa
    c = pa.Codec("snappy")
    cases = snappy_cases()
    assert len(cases) > 60
    for raw, go, pae in cases:
        assert O.snappy_encode(raw) == go                      # golang/snappy v0.0.4 bytes
        assert c.decompress(go, decompressed_size=len(raw)).to_pybytes() == raw
        assert O.snappy_decode(pae) == raw


def test_encode_fixture():
    z = load("encode.npz")
    keys = [z["keys"][int(z["key_off"][i]):int(z["key_off"][i + 1])].tobytes() for i in range(64)]
    vals = [z["vals"][int(z["val_off"][i]):int(z["val_off"][i + 1])].tobytes() for i in range(64)]
    for codec in (0, 1):
        e = O.encode_batch(keys, z["trailers"], vals, codec=codec, file_nums=[11, 12, 13, 14], table_max=64 << 10)
        assert e["ntables"] == int(z["c%d_ntables" % codec][0]) > 1
        for k in ("out", "pos", "bh_off", "bh_len", "table", "fnv", "crc", "status", "table_start"):
            assert (np.asarray(e[k]) == z["c%d_%s" % (codec, k)]).all(), (codec, k)


# ---------------------------------------------------------------- GPU ----

@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd import _lib
    from bitalosdb_amd.codec import BithashCodec
    _lib.lib()
    c = BithashCodec(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name,cod", [("rec_none", 0), ("rec_snappy", 1)])
def test_gpu_record_fixtures(codec, name, cod):
    src = read(name + ".bin")
    z = load(name + ".npz")
    got, vals, voff = codec.decode(src, z["handles"], compressor=cod)
    for f in FIELDS:
        assert (got[f] == z["desc"][f]).all(), f
    if cod:
        assert (np.asarray(voff) == z["val_off"]).all()
        assert np.asarray(vals)[:int(z["val_off"][-1])].tobytes() == z["vals"].tobytes()


@pytest.mark.gpu
def test_gpu_scan_k2(codec):
    import torch
    b = read("k2.bht")
    src = torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).to(codec.device)
    h, first, end = codec.scan_tables(src, np.array([0, len(b)], dtype=np.uint64), mode=0)
    codec.sync()
    h = h.cpu().numpy().view(np.uint8).reshape(-1).view(O.HANDLE_DT)
    g = np.load(os.path.join(GOLD, "k2_scan.npy"), allow_pickle=False)
    assert (h["offset"] == g["offset"]).all() and (h["length"] == g["length"]).all()


@pytest.mark.gpu
def test_gpu_encode_fixture(codec):
    z = load("encode.npz")
    keys = [z["keys"][int(z["key_off"][i]):int(z["key_off"][i + 1])].tobytes() for i in range(64)]
    vals = [z["vals"][int(z["val_off"][i]):int(z["val_off"][i + 1])].tobytes() for i in range(64)]
    for cod in (0, 1):
        e = codec.encode(keys, z["trailers"], vals, compressor=cod, file_nums=[11, 12, 13, 14], table_max=64 << 10)
        assert e["ntables"] == int(z["c%d_ntables" % cod][0])
        for k in ("out", "pos", "bh_off", "bh_len", "table", "fnv", "crc", "status", "table_start"):
            assert (np.asarray(e[k]) == z["c%d_%s" % (cod, k)]).all(), (cod, k)


@pytest.mark.gpu
def test_gpu_snappy_edges(codec):
    """GPU snappy encoder emits the golang/snappy bytes; GPU decoder reads the
    C++-snappy (pyarrow) streams -- both carried as record values."""
    cases = snappy_cases()
    keys = [b"k%03d" % i for i in range(len(cases))]
    trs = np.arange(1, len(cases) + 1, dtype=np.uint64) << np.uint64(8)
    e = codec.encode(keys, trs, [c[0] for c in cases], compressor=1, file_nums=[1])
    exp = b"".join(O.record_set(k, int(t), c[1], 1) for k, t, c in zip(keys, trs, cases))
    assert e["out"].tobytes() == exp
    src = b"".join(O.record_set(k, int(t), c[2], 1) for k, t, c in zip(keys, trs, cases))
    lens = [12 + len(k) + 8 + len(c[2]) for k, c in zip(keys, cases)]
    hs = np.zeros(len(cases), dtype=O.HANDLE_DT)
    hs["offset"] = np.concatenate([[0], np.cumsum(lens)[:-1]])
    hs["length"] = lens
    got, vals, voff = codec.decode(src, hs, compressor=1)
    assert (got["status"] == 0).all()
    vals = np.asarray(vals)
    voff = np.asarray(voff)
    for i, c in enumerate(cases):
        assert vals[int(voff[i]):int(voff[i + 1])].tobytes() == c[0], i
