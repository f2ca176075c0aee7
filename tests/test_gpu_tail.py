"""GPU parity for the table tail (bhg_table_tail: Writer.writeTable's
writeData/Conflict/IndexHash/Meta/Footer) and Writer.rebuild
(bhg_rebuild_tables), byte for byte against the restated writer
(oracle/table.py: Writer.update_hash / write_table / rebuild).

Cases: K1 (1200 x 2 KiB, three 1 MiB tables, bithash_test.go:725-764), the
K2 FNV-1 collision keys (conflict block, bithash_test.go:643-723) mixed with
overwrites, hand-made multi-key collision groups with repeated adds, an
empty table, a 128 MiB C4-shaped table, and the K1 rebuild (405,072)."""
import importlib.util
import os
import random

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import table as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd.codec import BithashCodec
    c = BithashCodec(0)
    yield c
    c.close()


def _k2_keys():
    spec = importlib.util.spec_from_file_location("kat", os.path.join(os.path.dirname(__file__),
                                                                      "test_oracle_known_answers.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return list(m.K2_KEYS)


def rb(rng, n):
    return bytes(rng.randrange(256) for _ in range(n))


def oracle_files(keys, trs, vals, table_max, compressor=0):
    """Store + compacting flush: every table finished by write_table."""
    st = T.Store(table_max, compressor=compressor)
    s = st.flush_start()
    for k, tr, v in zip(keys, trs, vals):
        s.wr.add(k, tr, v)
        if s.wr.is_write_full():
            old = s.wr
            s.wr = st._new_writer()
            st.close_table(old, False)
    s.compact = True
    s.finish()
    return {fn: bytes(f) for fn, f in st.files.items()}, st


def assert_files_equal(got, exp):
    assert sorted(got) == sorted(exp)
    for fn in exp:
        g, e = got[fn], exp[fn]
        if g != e:
            bad = next(i for i in range(min(len(g), len(e))) if g[i] != e[i]) if min(len(g), len(e)) else 0
            raise AssertionError("table %d: len %d vs %d, first diff at %d" % (fn, len(g), len(e), bad))


def test_tail_k1_tables(codec):
    rng = random.Random(7)
    keys = [b"bithash_testkey_%d" % i for i in range(1200)]
    vals = [rb(rng, 2048) for _ in range(1200)]
    trs = [((i + 1) << 8) | 1 for i in range(1200)]
    exp, st = oracle_files(keys, trs, vals, 1 << 20)
    got, res, stats = codec.encode_tables(keys, trs, vals, file_nums=[1, 2, 3, 4], table_max=1 << 20)
    assert res["ntables"] == 3
    assert_files_equal(got, exp)
    assert list(stats[:, 2]) == [0, 0, 0]
    assert [int(x) for x in stats[:, 1]] == [st.closed_meta[fn][1] for fn in (1, 2, 3)]
    # the GPU-built files open and serve every key (restated Reader.Get)
    for i in range(0, 1200, 97):
        fn = next(f for f in (1, 2, 3) if i < sum(int(stats[t, 0]) for t in range(f)))
        assert T.table_get(got[fn], keys[i]) == vals[i]


@pytest.mark.parametrize("compressor", [0, 1])
def test_tail_conflicts_and_overwrites(codec, compressor):
    """K2 collision pairs + 3-way collisions + repeated keys (overwrite: last add
    wins; a colliding key re-added after the conflict: conflictKeys updated)."""
    rng = random.Random(11 + compressor)
    k2 = _k2_keys()
    base = [rb(rng, rng.choice([4, 16, 32])) for _ in range(3000)]
    seq = []
    for i in range(4000):
        r = rng.random()
        if r < 0.05:
            seq.append(rng.choice(k2))
        elif r < 0.2 and seq:
            seq.append(rng.choice(seq))        # overwrite of an earlier key
        else:
            seq.append(base[i % len(base)])
    seq += k2 + k2[::-1]
    trs = [((i + 1) << 8) | 1 for i in range(len(seq))]
    vals = [rb(rng, rng.choice([1, 30, 500, 3000])) for _ in seq]
    exp, st = oracle_files(seq, trs, vals, 1 << 20, compressor)
    fns = list(range(1, 40))
    got, res, stats = codec.encode_tables(seq, trs, vals, compressor=compressor, file_nums=fns, table_max=1 << 20)
    assert_files_equal(got, exp)
    assert int(stats[:, 1].sum()) > 0                       # conflict blocks were built
    assert [int(x) for x in stats[:, 1]] == [st.closed_meta[fn][1] for fn in sorted(exp)]


def test_tail_empty_and_tiny_tables(codec):
    """ntables beyond the used ones: an empty writer's tail (no indexhash_data
    entry, checksum of nothing); a table holding one record."""
    from bitalosdb_amd.codec import _u64_tensor
    w0 = T.Writer(1, 1 << 20)
    w0.add(b"only", 1 << 8 | 1, b"value")
    w0.write_table(True)
    w1 = T.Writer(2, 1 << 20)
    w1.write_table(True)
    res = codec.encode([b"only"], [1 << 8 | 1], [b"value"], file_nums=[1, 2], table_max=1 << 20)
    bufs = res["bufs"]
    with torch.cuda.stream(codec.stream):
        de = _u64_tensor([int(res["bh_len"][0]), 0], codec.device)
        tail, off, ln, stats = codec.table_tail(res["out_t"], bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table,
                                                bufs.status, 1, 2, de)
        codec.sync()
    tail, off, ln = tail.cpu().numpy(), off.cpu().numpy(), ln.cpu().numpy()
    f0 = res["out"].tobytes() + tail[off[0]:off[0] + ln[0]].tobytes()
    f1 = tail[off[1]:off[1] + ln[1]].tobytes()
    assert f0 == bytes(w0.file)
    assert f1 == bytes(w1.file)


def test_tail_small_cap_reports_no_space(codec):
    rng = random.Random(3)
    keys = [rb(rng, 12) for _ in range(500)]
    vals = [rb(rng, 100) for _ in range(500)]
    trs = [((i + 1) << 8) | 1 for i in range(500)]
    res = codec.encode(keys, trs, vals, file_nums=list(range(1, 20)), table_max=20000)
    nt = res["ntables"]
    bufs = res["bufs"]
    _, off_full, ln_full, _ = codec.table_tail(res["out_t"], bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table,
                                               bufs.status, 500, nt, bufs.table_size)
    codec.sync()
    offs = off_full.cpu().numpy()
    cap = int(offs[1])                                       # room for table 0's slot only
    tail, off, ln, stats = codec.table_tail(res["out_t"], bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table,
                                            bufs.status, 500, nt, bufs.table_size, tail_cap=cap)
    codec.sync()
    ln, stats = ln.cpu().numpy(), stats.cpu().numpy().view(np.uint32).reshape(-1, 4)
    assert ln[0] == ln_full.cpu().numpy()[0] and (ln[1:] == 0).all()
    assert stats[0, 2] == 0 and (stats[1:, 2] == O.NO_SPACE).all()


def test_tail_c4_shaped_128mib(codec):
    """C4 shape: U[64, 4096] values, TableMaxSize 128 MiB (2 full tables + tail)."""
    rng = np.random.default_rng(5)
    n = 140_000
    sizes = rng.integers(64, 4097, n)
    blob = rng.integers(0, 256, int(sizes.sum()) + 64, dtype=np.uint8).tobytes()
    offs = np.concatenate([[0], np.cumsum(sizes)])
    vals = [blob[offs[i]:offs[i + 1]] for i in range(n)]
    keys = [b"c4key_%010d" % i for i in range(n)]
    trs = [((i + 1) << 8) | 1 for i in range(n)]
    got, res, stats = codec.encode_tables(keys, trs, vals, file_nums=[1, 2, 3, 4], table_max=128 << 20)
    assert res["ntables"] == 3
    exp, _ = oracle_files(keys, trs, vals, 128 << 20)
    assert_files_equal(got, exp)


def test_rebuild_k1_table(codec):
    """K1 rebuild: the third table's data region + b"panic" (bithash_test.go:725-756):
    the GPU rebuild yields currentOffset 405,072 and the handles/khash updateHash
    saw; its tail equals the restated rebuild + writeTable, and the rebuilt table
    equals the original third table."""
    from bitalosdb_amd.codec import as_device_bytes
    rng = random.Random(7)
    keys = [b"bithash_testkey_%d" % i for i in range(1200)]
    vals = [rb(rng, 2048) for _ in range(1200)]
    trs = [((i + 1) << 8) | 1 for i in range(1200)]
    exp, st = oracle_files(keys, trs, vals, 1 << 20)
    data3 = bytes(st.files[3][:405072])
    w = T.Writer(3, 1 << 20)
    w.file = bytearray(data3 + b"panic")
    w.rebuild()
    assert w.current_offset == 405072
    w.write_table(True)
    want_tail = bytes(w.file[405072:])
    src = data3 + b"panic"
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src_t = as_device_bytes(src, dev)
        h, first, end, kh, bo, tb = codec.rebuild_tables(src_t, [0, len(src)])
        codec.sync()
        assert int(end[0].item()) == 405072
        cnt = int(first[1].item())
        tail, off, ln, stats = codec.table_tail(src_t, h, bo, kh, tb, None, cnt, 1, end)
        codec.sync()
    t = tail.cpu().numpy()
    got_tail = t[int(off[0]):int(off[0]) + int(ln[0])].tobytes()
    assert got_tail == want_tail
    assert data3 + got_tail == exp[3]
    # the rebuilt khash / handles are the scan + FNV-1 of every key
    hh = h.cpu().numpy().view(O.HANDLE_DT).reshape(-1)
    khn = kh.cpu().numpy().view(np.uint32)
    for i in (0, 1, cnt - 1):
        o = int(hh["offset"][i])
        k = int.from_bytes(src[o:o + 4], "little")
        assert khn[i] == O.fnv32(src[o + 12:o + 12 + k - 8])


def test_rebuild_multi_table_roundtrip(codec):
    """Several footerless tables (snappy values, overwrites, K2 collisions) in
    one rebuild call; tails of all of them equal the restated rebuild+writeTable."""
    from bitalosdb_amd.codec import as_device_bytes
    rng = random.Random(19)
    k2 = _k2_keys()
    datas, wants = [], []
    for t in range(4):
        w = T.Writer(t + 1, 1 << 30, compressor=1)
        written = []
        for i in range(300 + 200 * t):
            if rng.random() < 0.05:
                k = rng.choice(k2)
            elif written and rng.random() < 0.1:
                k = rng.choice(written)
            else:
                k = rb(rng, rng.choice([0, 5, 24]))
            w.add(k, ((i + 1) << 8) | 1, rb(rng, rng.choice([1, 100, 1500])))
            written.append(k)
        data = bytes(w.file[:w.current_offset])
        w2 = T.Writer(t + 1, 1 << 30, compressor=1)
        w2.file = bytearray(data)
        w2.rebuild()
        w2.write_table(True)
        datas.append(data)
        wants.append(bytes(w2.file[len(data):]))
    src = b"".join(datas)
    toff = np.cumsum([0] + [len(d) for d in datas]).tolist()
    with torch.cuda.stream(codec.stream):
        src_t = as_device_bytes(src, codec.device)
        h, first, end, kh, bo, tb = codec.rebuild_tables(src_t, toff)
        codec.sync()
        cnt = int(first[4].item())
        tail, off, ln, stats = codec.table_tail(src_t, h, bo, kh, tb, None, cnt, 4, end)
        codec.sync()
    t = tail.cpu().numpy()
    off, ln = off.cpu().numpy(), ln.cpu().numpy()
    for i in range(4):
        assert t[off[i]:off[i] + ln[i]].tobytes() == wants[i], i


def _ikey_table(codec, keys, trs, vals, khash, fn=9):
    """AddIkey over the batch with caller-given khash (bhg_encode_ikey_batch), then
    writeTable (bhg_table_tail): one whole table file."""
    n = len(keys)
    res = codec.encode_ikey(keys, trs, vals, [fn] * n, khash=khash)
    assert (res["status"] == 0).all()
    assert np.array_equal(res["fnv"], np.asarray(khash, np.uint32))
    bufs = res["bufs"]
    with torch.cuda.stream(codec.stream):
        tail, off, ln, stats = codec.table_tail(res["out_t"], bufs.rec, bufs.bh_off, bufs.fnv1, bufs.table,
                                               bufs.status, n, 1, bufs.table_size)
        codec.sync()
    size = int(bufs.table_size[0].item())
    t = tail.cpu().numpy()
    stats = stats.cpu().numpy().view(np.uint32).reshape(-1, 4)     # per table: flat [4 * ntables]
    return res["out"][:size].tobytes() + t[int(off[0]):int(off[0]) + int(ln[0])].tobytes(), stats


def _oracle_ikey_table(keys, trs, vals, khash, fn=9):
    w = T.Writer(fn, 1 << 40)
    for k, tr, v, kh in zip(keys, trs, vals, khash):
        w.add_ikey(k, tr, v, kh, fn)
    w.write_table(True)
    return bytes(w.file), w


def test_tail_conflict_block_past_one_restart(codec):
    """A conflict block of 41 keys (restart points at entries 0, 16, 32) whose keys
    share long prefixes, so every entry between restarts is prefix-compressed:
    all 41 under one khash, some re-added after the group turned conflicting."""
    rng = random.Random(41)
    keys = [b"shared/prefix/of/conflict/keys/%03d" % (i * 7 % 41) for i in range(41)]
    keys += [keys[i] for i in (3, 17, 40, 0)]                     # re-adds: conflictKeys updated
    keys += [b"other_%d" % i for i in range(30)]                  # ordinary index items
    khash = [0xABCD1234] * 45 + [O.fnv32(k) for k in keys[45:]]
    trs = [((i + 1) << 8) | 1 for i in range(len(keys))]
    vals = [rb(rng, rng.choice([5, 100, 700])) for _ in keys]
    got, stats = _ikey_table(codec, keys, trs, vals, khash)
    exp, w = _oracle_ikey_table(keys, trs, vals, khash)
    assert len(w.conflict_keys) == 41 and int(stats[0, 1]) == 41
    assert got == exp
    for k in (keys[0], keys[20], keys[44]):
        last = max(i for i in range(len(keys)) if keys[i] == k)
        assert T.table_get(got, k, khash=khash[last]) == vals[last]


def test_tail_one_key_under_two_khash(codec):
    """AddIkey lets the caller pick khash: one user key added under two khash
    values, each group conflicting with other keys.  conflictKeys is one map per
    table, so the key is written once, with the handle of whichever group
    assigned it last -- including the case where that assignment is the first
    key's re-assignment at the add that makes its group conflict."""
    rng = random.Random(42)
    A, B = 0x11110000, 0x22220000
    cases = [
        # (key, khash): "dup" first in group A (assigned again when A conflicts), later in group B
        [(b"dup", A), (b"x1", B), (b"dup", B), (b"a2", A)],
        # dup last assigned in A by a plain re-add after both groups conflict
        [(b"dup", B), (b"y1", B), (b"dup", A), (b"y2", A), (b"dup", A)],
        # dup never re-added: B's conflict-making add assigns it after A's
        [(b"dup", A), (b"z1", A), (b"dup", B), (b"z2", B)],
    ]
    for spec in cases:
        spec = spec + [(b"fill_%d" % i, O.fnv32(b"fill_%d" % i)) for i in range(20)]
        keys = [k for k, _ in spec]
        khash = [h for _, h in spec]
        trs = [((i + 1) << 8) | 1 for i in range(len(spec))]
        vals = [rb(rng, rng.choice([3, 60])) for _ in spec]
        got, stats = _ikey_table(codec, keys, trs, vals, khash)
        exp, w = _oracle_ikey_table(keys, trs, vals, khash)
        assert int(stats[0, 1]) == len(w.conflict_keys)
        assert got == exp, spec[:5]


def test_tail_conflict_keys_prefix_edge_cases(codec):
    """k_conf_rank / k_tail_dedupe compare keys by their big-endian 8-byte prefix first and
    fall back to the bytes only on equal prefixes: keys that are prefixes of each other, keys
    with zero bytes where the prefix pads with zeros, keys shorter than 8 B, the empty key, and
    keys equal in the first 8 bytes -- one conflict group, plus a second group holding some of
    the same keys (dedupe across two khash values)."""
    rng = random.Random(43)
    edge = [b"", b"\x00", b"\x00\x00", b"a", b"a\x00", b"a\x00\x00", b"a\x00b", b"ab", b"abcdefgh",
            b"abcdefgh\x00", b"abcdefgh\x00\x00", b"abcdefghi", b"abcdefgh\xff", b"abcdefg", b"\xff" * 9]
    A, B = 0x5A5A0001, 0x5A5A0002
    spec = [(k, A) for k in edge]
    spec += [(b"a\x00", B), (b"abcdefgh", B), (b"zz", B), (b"a\x00", A), (b"", B)]
    spec += [(b"fill_%d" % i, O.fnv32(b"fill_%d" % i)) for i in range(20)]
    rng.shuffle(spec)
    keys = [k for k, _ in spec]
    khash = [h for _, h in spec]
    trs = [((i + 1) << 8) | 1 for i in range(len(spec))]
    vals = [rb(rng, rng.choice([1, 9, 70])) for _ in spec]
    got, stats = _ikey_table(codec, keys, trs, vals, khash)
    exp, w = _oracle_ikey_table(keys, trs, vals, khash)
    assert int(stats[0, 1]) == len(w.conflict_keys)
    assert got == exp
