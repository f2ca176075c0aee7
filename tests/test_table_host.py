"""Host table open (bitalosdb_amd/table.py, NewReader's footer/meta/indexhash
parse) vs the restatement (oracle/table.py) on tables the restated writer
built.  CPU only.  (The tail bytes themselves are built on the GPU and
checked in tests/test_gpu_tail.py.)"""
import os
import random
import struct

import pytest

from bitalosdb_amd import table as BT
from oracle import table as T


def _build(keys, values, table_max=1 << 30):
    w = T.Writer(7, table_max)
    for i, (k, v) in enumerate(zip(keys, values)):
        w.add(k, ((i + 1) << 8) | 1, v)
    w.write_table(True)
    return bytes(w.file)


def _k2_keys():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "kat", os.path.join(os.path.dirname(__file__), "test_oracle_known_answers.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return list(m.K2_KEYS)


def _check_open(f, base=0):
    rec, info = BT.open_table(f, base=base)
    t = T.open_table(f)
    io, il = info["index_data"]
    if t["index_data"] is None:
        assert il == 0
    else:
        assert f[io:io + il] == t["index_data"]
    assert info["conflict_bh"] == t["conflict_bh"] and info["index_checksum"] == int(t["index_checksum"])
    assert info["data_bh"] == t["data_bh"] and info["index_bh"] == t["index_bh"]
    assert int(rec["index_off"]) == base + io and int(rec["conflict_bh_len"]) == t["conflict_bh"][1]
    return rec, info


@pytest.mark.parametrize("seed,n,dup", [(1, 50, 0.0), (2, 3000, 0.2), (3, 1, 0.0)])
def test_open_matches_writer(seed, n, dup):
    rng = random.Random(seed)
    keys = []
    for i in range(n):
        if keys and rng.random() < dup:
            keys.append(rng.choice(keys))
        else:
            keys.append(bytes(rng.randrange(97, 123) for _ in range(rng.choice([1, 8, 32]))))
    vals = [bytes(rng.randrange(256) for _ in range(rng.choice([1, 100, 1024]))) for _ in range(n)]
    _check_open(_build(keys, vals), base=seed * 1000)


def test_open_with_fnv_collisions():
    """The K2 collision pairs (bithash_test.go:650-663) give a conflict block."""
    keys = _k2_keys()
    vals = [b"v%d" % i * 10 for i in range(len(keys))]
    rec, info = _check_open(_build(keys + keys[:3], vals + vals[:3]))
    assert info["conflict_bh"][1] > 0


def test_open_empty_table():
    rec, info = _check_open(_build([], []))
    assert info["index_checksum"] == 2726488792   # crc of "" masked
    assert info["index_data"] == (0, 0)


def test_open_matches_oracle_k2():
    b = open(os.path.join(os.path.dirname(__file__), "golden", "k2.bht"), "rb").read()
    _check_open(b, base=100)


def test_block_iter_matches_restatement():
    entries = [(T.make_ikey(b"key%03d" % i, 1), struct.pack("<II", i, i * 2)) for i in range(40)]
    bw = T.BlockWriter()
    for k, v in entries:
        bw.add(k, v)
    blk = bw.finish()
    got = [(k, blk[vo:vo + vl]) for k, vo, vl in BT.block_iter(blk, 0, len(blk))]
    assert got == T.block_entries(blk)


def test_bad_footer_rejected():
    with pytest.raises(BT.TableError):
        BT.open_table(b"\0" * 10)
    f = bytearray(_build([b"a"], [b"b"]))
    f[-12] ^= 0xFF                                  # format version
    with pytest.raises(BT.TableError):
        BT.open_table(bytes(f))
