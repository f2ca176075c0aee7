"""Host table logic (bitalosdb_amd/table.py) vs the restatement (oracle/table.py):
the tail bytes of Writer.writeTable and NewReader's footer/meta/index parse.
CPU only: the masked CRC-32C comes from the C restatement here."""
import random
import struct

import numpy as np
import pytest

from bitalosdb_amd import table as BT
from oracle import oracle as O
from oracle import table as T


def _build(keys, values, table_max=1 << 30):
    w = T.Writer(7, table_max)
    adds = []
    for i, (k, v) in enumerate(zip(keys, values)):
        bh = w.add(k, ((i + 1) << 8) | 1, v)
        adds.append((bh[0], bh[1], O.fnv32(k), bytes(k)))
    data_end = w.current_offset
    w.write_table(True)
    return bytes(w.file), data_end, adds


def _tail(data_end, adds):
    return BT.table_tail(data_end, [a[0] for a in adds], [a[1] for a in adds], [a[2] for a in adds],
                         [a[3] for a in adds], O.crc_masked)


def _k2_keys():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "kat", os.path.join(os.path.dirname(__file__), "test_oracle_known_answers.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return list(m.K2_KEYS)


@pytest.mark.parametrize("seed,n,dup", [(1, 50, 0.0), (2, 3000, 0.2), (3, 1, 0.0)])
def test_tail_matches_writer(seed, n, dup):
    rng = random.Random(seed)
    keys = []
    for i in range(n):
        if keys and rng.random() < dup:
            keys.append(rng.choice(keys))            # overwrite: same key, later handle wins
        else:
            keys.append(bytes(rng.randrange(97, 123) for _ in range(rng.choice([1, 8, 32]))))
    vals = [bytes(rng.randrange(256) for _ in range(rng.choice([1, 100, 1024]))) for _ in range(n)]
    f, data_end, adds = _build(keys, vals)
    assert f[data_end:] == _tail(data_end, adds)


def test_tail_with_fnv_collisions():
    """The K2 collision pairs (bithash_test.go:650-663) go through the conflict block."""
    keys = _k2_keys()
    vals = [b"v%d" % i * 10 for i in range(len(keys))]
    f, data_end, adds = _build(keys + keys[:3], vals + vals[:3])
    assert f[data_end:] == _tail(data_end, adds)
    rec, info = BT.open_table(f)
    assert info["conflict_bh"][1] > 0


def test_empty_table_tail():
    f, data_end, adds = _build([], [])
    assert f[data_end:] == _tail(data_end, adds)
    assert BT.open_table(f)[1]["index_checksum"] == 2726488792   # crc of "" masked


def test_open_matches_oracle_k2():
    import os
    b = open(os.path.join(os.path.dirname(__file__), "golden", "k2.bht"), "rb").read()
    rec, info = BT.open_table(b, base=100)
    t = T.open_table(b)
    io, il = info["index_data"]
    assert b[io:io + il] == t["index_data"]
    assert info["conflict_bh"] == t["conflict_bh"] and info["index_checksum"] == int(t["index_checksum"])
    assert int(rec["index_off"]) == 100 + io and int(rec["conflict_bh_len"]) == t["conflict_bh"][1]


def test_block_build_matches_writer():
    entries = [(T.make_ikey(b"key%03d" % i, 1), struct.pack("<II", i, i * 2)) for i in range(40)]
    bw = T.BlockWriter()
    for k, v in entries:
        bw.add(k, v)
    assert BT.block_build(entries) == bw.finish()
    blk = BT.block_build(entries)
    got = [(k, blk[vo:vo + vl]) for k, vo, vl in BT.block_iter(blk, 0, len(blk))]
    assert got == T.block_entries(blk)
