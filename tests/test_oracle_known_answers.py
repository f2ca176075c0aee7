"""Pins the CPU restatement (oracle/) to the reference's own asserted tests.

K1  bithash/bithash_test.go:725-766  TestBithashOpenTableErrRebuild
K2  bithash/bithash_test.go:643-723  TestBithashKeyHashConflict
K3  bithash/writer_test.go:150-195   TestWriterUpdateIndex
K4  bithash/bithash_test.go:247-291  TestBithashCompactIter (scaled: 2,000 records)
plus standard-algorithm KATs for CRC-32C (internal/crc/crc.go) and FNV-1
(internal/hash/fnv.go), which the reference does not test itself.
"""
import random
import struct

import pytest

from oracle import oracle as O
from oracle import table as T


def rand_bytes(rng, n):
    # utils.FuncRandBytes alphabet (internal/utils/func.go:22-30), seeded here
    alpha = b"1qaz2wsx3edc4rfv5tgb6yhn7ujm8ik9ol0pabcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    return bytes(rng.choice(alpha) for _ in range(n))


def test_crc32c_kat():
    assert O.crc32c(b"123456789") == 0xE3069283
    assert O.crc32c(b"123456789", hw=True) == 0xE3069283
    assert O.crc_masked(b"123456789") == 0xC78AB0E5 == 3347755237
    # empty indexhash payload -> "2726488792" (writer.go:477-478)
    assert O.crc_masked(b"") == 0xA282EAD8 == 2726488792
    # incremental Update == one-shot (crc.go:27-29)
    assert O.crc32c(b"6789", O.crc32c(b"12345")) == 0xE3069283
    rng = random.Random(1)
    for n in (0, 1, 3, 7, 8, 9, 63, 64, 1076, 4099):
        b = rand_bytes(rng, n)
        assert O.crc32c(b) == O.crc32c(b, hw=True)


def test_fnv1_kat():
    assert O.fnv32(b"") == 0x811C9DC5
    assert O.fnv32(b"a") == 0x050C5D7E        # FNV-1, not FNV-1a (0xE40C292C)
    assert O.fnv32(b"foobar") == 0x31F0B262


K2_KEYS = [b"l41khazkyppk4sBj7BhdQxpfMGF2bKH9", b"zZah6yQoo4ElihZfMVwragoejhuHaocb",
           b"yBZrxusPKQdo1rKauI6rtOfs5tjbySx6", b"l0asXWDhSamz5qncres4xJSsaUK2Jhtz",
           b"wmoVNuhDBJOblKUS8wiSXNNmTjvcxrc7", b"H7fyvszFYYZqM0NnmfmjRjPoslT1V4nu",
           b"NplhsekvJnBm7gJHge5qsgJcqb68GCJu", b"1gncjKqtxufeiqwGfdpVrJubtEabsOyl",
           b"AqLMVOYwsi67FbCqHr2aivuoyKZH1eiW", b"zSpkzpkG9xbvR4IgqNcfF24pdg351Any",
           b"tk0F3dTRD8BGqaPAekliaDiZvRojoTk1", b"dzurIotnFYUPynzW6V9DzyfdzTzs2chx"]


def test_k2_fnv1_collision_pairs():
    hs = [O.fnv32(k) for k in K2_KEYS]
    assert len(set(hs)) == 6
    for i in range(0, 12, 2):
        assert hs[i] == hs[i + 1]
    assert sorted(set(hs)) == sorted([0x622DF638, 0x4A6A5057, 0xD523CEF4, 0xC832452C, 0xBE5B12A2, 0xB46DD5A0])


def _fnv1a(b):
    h = 0x811C9DC5
    for c in b:
        h = ((h ^ c) * 16777619) & 0xFFFFFFFF
    return h


def test_k2_not_fnv1a():
    assert len({_fnv1a(k) for k in K2_KEYS}) == 12


def test_k2_key_hash_conflict_store():
    rng = random.Random(2)
    st = T.Store(64 << 20)
    seq = 1
    kv = [(b"bithash_testkey_%d" % i, rand_bytes(rng, 2048)) for i in range(100)]
    ckv = [(k, rand_bytes(rng, 2048)) for k in K2_KEYS]
    fns, cfns = [0] * 100, [0] * 12
    s = st.flush_start()
    for i, (k, v) in enumerate(kv):
        fns[i] = s.add(k, seq, v)
        seq += 1
        if i == 50:
            for j, (ck, cv) in enumerate(ckv):
                cfns[j] = s.add(ck, seq, cv)
                seq += 1
    s.finish()

    def read():
        for (k, v), fn in zip(kv + ckv, fns + cfns):
            assert st.get(k, fn) == v

    read()
    s = st.flush_start()
    s.compact = True
    s.finish()
    assert not st.mutable
    read()
    assert st.closed_meta[1] == (112, 12)
    t = T.open_table(bytes(st.files[1]))
    # indexhash_checksum is the decimal masked CRC32C of indexhash_data (writer.go:477-478)
    assert t["index_checksum"] == str(O.crc_masked(t["index_data"])).encode()
    # 106 distinct hashes -> 106 HashIndex items; 12 conflict keys in the conflict block
    assert len(t["index_data"]) == 8 + 65536 * 4 + 10 * 106
    assert len(T.block_entries(t["conflict_buf"])) == 12


def test_k1_table_split_and_rebuild():
    rng = random.Random(3)
    st = T.Store(1 << 20)
    kv = [(b"bithash_testkey_%d" % i, rand_bytes(rng, 2048)) for i in range(1200)]
    s = st.flush_start()
    fns = []
    for i, (k, v) in enumerate(kv):
        fns.append(s.add(k, i + 1, v))
    s.finish()
    # two closed tables (split after the add that crosses 1 MiB) + a mutable third
    assert sorted(st.closed_meta) == [1, 2]
    w = st.mutable[-1]
    assert w.file_num == 3
    assert w.current_offset == 405072
    sizes = []
    for fn in (1, 2):
        t = T.open_table(bytes(st.files[fn]))
        sizes.append(t["data_bh"][1] - 12)
    assert sizes == [1049651, 1049767]
    # append 5 garbage bytes to the mutable table; reopen -> rebuild
    w.file += b"panic"
    assert len(w.file) == 405077
    w2 = T.Writer(3, 1 << 20, file=bytearray(w.file))
    w2.rebuild()
    assert w2.current_offset == 405072
    for (k, v), fn in zip(kv, fns):
        if fn == 3:
            assert T._writer_get(w2, k) == v
        else:
            assert st.get(k, fn) == v


def test_k3_update_hash_semantics():
    w = T.Writer(1, 1 << 20)
    w.update_hash(b"key1", 100, (1, 1))
    w.update_hash(b"key2", 200, (2, 2))
    assert w.index_hash[100][1] == b"key1" and w.index_hash[200][1] == b"key2"
    assert w.index_hash[100][0] == (1, 1) and w.index_hash[200][0] == (2, 2)
    assert len(w.index_hash) == 2 and not w.conflict_keys
    w.update_hash(b"key1", 100, (3, 3))
    assert w.index_hash[100][0] == (3, 3) and w.index_hash[100][2] is False
    w.update_hash(b"key11", 100, (4, 4))
    assert w.index_hash[100][2] is True
    assert w.conflict_keys == {b"key1": (3, 3), b"key11": (4, 4)}
    w.update_hash(b"key111", 100, (5, 5))
    w.update_hash(b"key1", 100, (6, 6))
    assert w.conflict_keys == {b"key1": (6, 6), b"key11": (4, 4), b"key111": (5, 5)}


def test_k4_ordered_table_scan():
    rng = random.Random(4)
    st = T.Store(512 << 20)
    kv = [(b"bithash_testkey_%d" % i, rand_bytes(rng, 2048)) for i in range(2000)]
    s = st.flush_start()
    for i, (k, v) in enumerate(kv):
        s.add(k, i + 1, v)
    s.compact = True
    s.finish()
    got = list(T.table_iter(bytes(st.files[1])))
    assert len(got) == len(kv)
    for i, ((k, v), (uk, tr, val, fn)) in enumerate(zip(kv, got)):
        assert uk == k and tr >> 8 == i + 1 and val == v and fn == 1


def test_block_writer_restart_roundtrip():
    bw = T.BlockWriter()
    entries = [(T.make_ikey(b"key%04d" % i, i + 1), struct.pack("<Q", i * 7)) for i in range(40)]
    for k, v in entries:
        bw.add(k, v)
    b = bw.finish()
    nres = struct.unpack_from("<I", b, len(b) - 4)[0]
    assert nres == 3                    # entries 0, 16, 32
    assert T.block_entries(b) == entries
    empty = T.BlockWriter().finish()
    assert empty == struct.pack("<II", 0, 1)


def test_scan_stop_rules():
    recs = b"".join(O.record_set(b"k%d" % i, (i + 1) << 8 | 1, b"v" * (i + 1), 9) for i in range(5))
    # TableIterator: stops at the 12-zero terminator
    h, end = O.scan_region(recs + bytes(12) + b"tail")
    assert len(h) == 5 and end == len(recs)
    # rebuild stops only on ikeySize == 0: a zero valueSize record is still counted
    odd = O.record_set(b"z", 1, b"", 9)
    h0, _ = O.scan_region(recs + odd + bytes(12), mode=0)
    h1, _ = O.scan_region(recs + odd + bytes(12), mode=1)
    assert len(h0) == 5 and len(h1) == 6
    # short header (the K1 "panic" garbage) ends both scans
    h, end = O.scan_region(recs + b"panic", mode=1)
    assert len(h) == 5 and end == len(recs)
