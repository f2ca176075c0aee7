"""GPU parity: batched Reader.Get (bhg_get_batch: FNV-1 -> HashIndex.Get64 ->
conflict-block SeekGE) and Bithash.Get over a batch (get + readData) vs the
restatement (oracle/table.py get_handle / table_get).

Tables: the K2 known-answer table (6 FNV-1 collision pairs -> conflict block,
bithash_test.go:643-723), writer-built tables with overwrites, snappy values,
an empty table, and hash-colliding keys that were never written (they hit the
conflict range and miss in SeekGE -> ErrBhIllegalBlockLength)."""
import os
import random

import numpy as np
import pytest
import torch

from bitalosdb_amd import table as BT
from bitalosdb_amd._lib import ST_ILLEGAL_LENGTH, ST_NOT_FOUND, ST_OK
from oracle import oracle as O
from oracle import table as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
ST = {"OK": ST_OK, "NOT_FOUND": ST_NOT_FOUND, "ILLEGAL_LENGTH": ST_ILLEGAL_LENGTH}


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd import _lib
    from bitalosdb_amd.codec import BithashCodec
    _lib.lib()
    c = BithashCodec(0)
    yield c
    c.close()


def _writer_table(rng, n, fn, compressor=0, dup=0.1, keys=None):
    w = T.Writer(fn, 1 << 30, compressor=compressor)
    written = []
    for i in range(n):
        if keys is not None:
            k = keys[i]
        elif written and rng.random() < dup:
            k = rng.choice(written)
        else:
            k = bytes(rng.randrange(97, 123) for _ in range(rng.choice([3, 16, 32])))
        v = bytes(rng.randrange(65, 91) for _ in range(rng.choice([1, 50, 700])))
        w.add(k, ((i + 1) << 8) | 1, v)
        written.append(k)
    w.write_table(True)
    return bytes(w.file), written


def _k2_keys():
    import importlib.util
    spec = importlib.util.spec_from_file_location("kat", os.path.join(os.path.dirname(__file__),
                                                                      "test_oracle_known_answers.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return list(m.K2_KEYS)


def _concat(files):
    src = bytearray()
    recs = []
    for f in files:
        base = len(src) + 5                # odd padding between tables: bases need no alignment
        src += bytes(5) + f
        rec, _ = BT.open_table(f, base=base)
        recs.append(rec)
    return bytes(src), np.array(recs, dtype=recs[0].dtype)


def _check(codec, files, queries):
    src, tabs = _concat(files)
    src_t = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).to(codec.device)
    keys = [q[1] for q in queries]
    tidx = np.array([q[0] for q in queries], dtype=np.uint32)
    h_t, s_t = codec.get_batch(src_t, tabs, keys, tidx)
    codec.sync()
    h = h_t.cpu().numpy().view(np.uint8).view(O.HANDLE_DT)
    st = s_t.cpu().numpy().view(np.uint32)
    for i, (t, k) in enumerate(queries):
        es, eo, el = T.get_handle(files[t], k)
        assert st[i] == ST[es], (i, k, es, st[i])
        if es == "OK":
            assert int(h["offset"][i]) == int(tabs["base"][t]) + eo and int(h["length"][i]) == el, (i, k)
    return src_t, tabs, keys, tidx


def test_get_k2_conflict_table(codec):
    b = open(os.path.join(GOLD, "k2.bht"), "rb").read()
    keys2 = _k2_keys()
    t = T.open_table(b)
    all_keys = [uk for uk, _, _, _ in T.table_iter(b)]
    rng = random.Random(5)
    missing = [bytes(rng.randrange(97, 123) for _ in range(20)) for _ in range(200)]
    qs = [(0, k) for k in all_keys + keys2 + missing]
    _check(codec, [b], qs)
    assert t["conflict_bh"][1] > 0


def test_get_conflict_range_miss(codec):
    """A key whose FNV-1 equals a conflicting hash but was never written:
    HashIndex hit on conflictBH, SeekGE miss -> ILLEGAL_LENGTH."""
    keys2 = _k2_keys()
    f, _ = _writer_table(random.Random(1), 3, 9, keys=[keys2[0], keys2[1], b"solo"])
    # keys2[0], keys2[1] collide; build a third collider of the same pair by reusing the hash via a table of
    # only keys2[0] and looking up keys2[1] in a table where keys2[0] collides with another written key
    qs = [(0, keys2[0]), (0, keys2[1]), (0, b"solo"), (0, b"absent")]
    _check(codec, [f], qs)
    f2, _ = _writer_table(random.Random(2), 3, 9, keys=[keys2[0], keys2[1], keys2[2]])
    # keys2[3] pairs with keys2[2]: its hash is in the index as a plain (non-conflict) entry -> OK with keys2[2]'s
    # handle (Reader.Get does not compare keys outside the conflict block, reader.go:209-231)
    _check(codec, [f2], [(0, k) for k in keys2[:6]])


@pytest.mark.parametrize("compressor", [0, 1])
def test_multi_table_multiget(codec, compressor):
    rng = random.Random(10 + compressor)
    files, written = [], []
    for t in range(3):
        f, w = _writer_table(rng, 400, 20 + t, compressor=compressor)
        files.append(f)
        written.append(w)
    empty, _ = _writer_table(rng, 0, 30)
    files.append(empty)
    qs = []
    for _ in range(3000):
        t = rng.randrange(4)
        if t < 3 and rng.random() < 0.8:
            qs.append((t, rng.choice(written[t])))
        else:
            qs.append((t, bytes(rng.randrange(97, 123) for _ in range(rng.choice([3, 16, 32])))))
    src_t, tabs, keys, tidx = _check(codec, files, qs)
    st, desc, vals, voff = codec.multi_get(src_t, tabs, keys, tidx, compressor=compressor)
    for i, (t, k) in enumerate(qs):
        try:
            exp = T.table_get(files[t], k, compressor)
        except T.BithashError as e:
            assert st[i] != ST_OK, (i, str(e))
            continue
        assert st[i] == ST_OK
        if compressor:
            got = vals[int(voff[i]):int(voff[i + 1])].tobytes()
        else:
            off = int(tabs["base"][t])
            hoff = int(T.get_handle(files[t], k)[1])
            got = bytes(files[t][hoff + int(desc["val_off"][i]):hoff + int(desc["val_off"][i]) + int(desc["val_len"][i])])
            assert off >= 0
        assert got == exp, i


def test_given_khash_matches(codec):
    rng = random.Random(3)
    f, w = _writer_table(rng, 300, 4)
    src, tabs = _concat([f])
    src_t = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).to(codec.device)
    keys = w[:200]
    kh = np.array([O.fnv32(k) for k in keys], dtype=np.uint32)
    h1, s1 = codec.get_batch(src_t, tabs, keys, np.zeros(200, np.uint32))
    h2, s2 = codec.get_batch(src_t, tabs, keys, np.zeros(200, np.uint32), khash=kh)
    codec.sync()
    assert torch.equal(h1, h2) and torch.equal(s1, s2)
    assert (s1.cpu().numpy() == ST_OK).all()


def test_bithash_get_open_writer_and_filenum_map(codec):
    """Bithash.Get (bithash.go:101-119) over a batch (bhg_bithash_get_batch): queries on a
    still-open table go through Writer.Get's in-memory index (writer.go:171-228, rebuilt on
    the device by bhg_writer_index_build) -- overwritten keys answer the last add, the K2
    collision pairs added to the open table take the conflictKeys path, a never-written key
    sharing a non-conflict khash answers the stored key's handle as Go does; writer misses fall
    through GetFileNumMap to the closed tables (a compacted fileNum remapped to its
    destination, an unmapped fileNum -> ErrBhFileNumZero).  Checked against the restated
    Bithash.Get (oracle/table.py bithash_get_handle)."""
    from bitalosdb_amd._lib import ST_FILE_NUM_ZERO, WRITER_INDEX_DT
    from bitalosdb_amd.codec import handles_tensor
    rng = random.Random(77)
    keys2 = _k2_keys()
    k2 = open(os.path.join(GOLD, "k2.bht"), "rb").read()
    f5, w5 = _writer_table(rng, 300, 5)
    f6, w6 = _writer_table(rng, 300, 6)
    files = {3: k2, 5: f5, 6: f6}
    order = [3, 5, 6]
    src, tabs = _concat([files[fn] for fn in order])
    # the open table (fileNum 8): plain keys with overwrites, two K2 collision pairs (conflict), and
    # one key of a third pair alone (a non-conflict khash shared with a never-written key)
    w = T.Writer(8, 1 << 30)
    plain = [bytes(rng.randrange(97, 123) for _ in range(rng.choice([5, 16, 32]))) for _ in range(150)]
    adds = plain + plain[:40] + keys2[:4] + [keys2[0], keys2[3]] + [keys2[4]]
    rng.shuffle(adds)
    for i, k in enumerate(adds):
        w.add(k, ((i + 1) << 8) | 1, bytes(rng.randrange(65, 91) for _ in range(rng.choice([3, 60, 400]))))
    wbase = len(src) + 3
    src = src + bytes(3) + bytes(w.file)
    recs = []
    off = 0
    for k in adds:                                   # the writer's records in add order
        ln = 12 + len(k) + 8 + struct_len(w.file, off)
        recs.append((wbase + off, ln, 0))
        off += ln
    rec_h = np.array(recs, dtype=O.HANDLE_DT)
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src_t = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).to(dev)
        rec_t = handles_tensor(rec_h, dev)
        kh_t = torch.from_numpy(np.array([O.fnv32(k) for k in adds], dtype=np.uint32).view(np.int32)).to(dev)
        srt, skh = codec.writer_index(kh_t, len(adds))
    writers = np.zeros(1, dtype=WRITER_INDEX_DT)
    writers[0] = (rec_t.data_ptr(), srt.data_ptr(), skh.data_ptr(), len(adds), 8)
    fn_map_d = {3: 3, 4: 6, 5: 5, 6: 6, 8: 8}          # 4 was compacted into 6; 7 is unmapped
    fn_count = 10
    fn_map = np.zeros(fn_count, np.uint32)
    for s_, d_ in fn_map_d.items():
        fn_map[s_] = d_
    fn_table = np.full(fn_count, 0xFFFFFFFF, np.uint32)
    for ti, fn in enumerate(order):
        fn_table[fn] = ti
    missing = [bytes(rng.randrange(97, 123) for _ in range(12)) for _ in range(60)]
    qs = [(8, k) for k in plain + keys2 + missing]
    qs += [(5, k) for k in w5[:100]] + [(4, k) for k in w6[:100]] + [(6, k) for k in missing[:20]]
    qs += [(3, k) for k in keys2] + [(7, k) for k in plain[:10]] + [(12, k) for k in plain[:5]]
    rng.shuffle(qs)
    h_t, s_t = codec.bithash_get(src_t, writers, tabs, fn_map, fn_table, [q[1] for q in qs], [q[0] for q in qs])
    codec.sync()
    h = h_t.cpu().numpy().view(np.uint8).view(O.HANDLE_DT)
    st = s_t.cpu().numpy().view(np.uint32)
    code = dict(ST, FILE_NUM_ZERO=ST_FILE_NUM_ZERO)
    base_of = {fn: int(tabs["base"][ti]) for ti, fn in enumerate(order)}
    base_of[8] = wbase
    seen = set()
    for i, (fn, k) in enumerate(qs):
        es, efn, (eo, el) = T.bithash_get_handle({8: w}, files, fn_map_d, k, fn)
        assert st[i] == code[es], (i, fn, k, es, st[i])
        if es == "OK":
            assert int(h["offset"][i]) == base_of[efn] + eo and int(h["length"][i]) == el, (i, fn, k)
            seen.add((fn == 8, efn == 8))
    assert (True, True) in seen and (False, False) in seen          # writer hits and table hits
    assert {code["FILE_NUM_ZERO"], code["NOT_FOUND"]} <= set(st.tolist())
    # the conflict path ran: the two K2 pairs added to the open table answer their own records
    for k in keys2[:4]:
        es, efn, bh = T.bithash_get_handle({8: w}, files, fn_map_d, k, 8)
        assert es == "OK" and efn == 8 and w.index_hash[O.fnv32(k)][2]


def struct_len(buf, off):
    import struct
    return struct.unpack_from("<I", buf, off + 4)[0]


@pytest.mark.parametrize("compressor", [0, 1])
def test_bithash_get_writer_read_failure_falls_through(codec, compressor):
    """Bithash.Get keeps an open writer's answer only when Writer.Get returns a value without
    error (bithash.go:102-107).  Open-writer records that read as nil -- an empty value
    (NoCompressor: readRecord nil, ErrBhReadRecordNil; snappy: a 0-length stream decodes to a nil
    slice), a corrupted valueSize, a corrupted snappy stream -- fall through GetFileNumMap to the
    closed table (hit or ErrBhNotFound); a later good add of the same key is final again.
    Checked against the restated Bithash.Get (oracle/table.py bithash_get_handle)."""
    import struct
    from bitalosdb_amd._lib import ST_FILE_NUM_ZERO, WRITER_INDEX_DT
    from bitalosdb_amd.codec import handles_tensor
    rng = random.Random(1000 + compressor)
    f5, w5 = _writer_table(rng, 300, 5)
    files = {5: f5}
    src, tabs = _concat([f5])
    uniq5 = list(dict.fromkeys(w5))
    rng.shuffle(uniq5)
    good, empty, corrupt, healed = uniq5[:30], uniq5[30:60], uniq5[60:80], uniq5[80:100]
    fresh_empty = [b"fe%03d" % i for i in range(10)]
    fresh_good = [b"fg%03d" % i for i in range(10)]
    w = T.Writer(9, 1 << 30, compressor=compressor)

    def val():
        return bytes(rng.randrange(65, 91) for _ in range(rng.randrange(10, 100)))
    adds = [(k, val()) for k in good + corrupt + fresh_good] + [(k, b"") for k in empty + fresh_empty + healed]
    rng.shuffle(adds)
    adds += [(k, val()) for k in healed]              # the last add of a healed key is good
    recs, corrupt_at = [], {}
    for i, (k, v) in enumerate(adds):
        off = w.current_offset
        w.add(k, ((i + 1) << 8) | 1, v)
        recs.append((off, w.current_offset - off))
        if k in corrupt:
            corrupt_at[k] = off
    for k, off in corrupt_at.items():                 # after the adds: the index keeps the handles
        kl, vl = struct.unpack_from("<II", w.file, off)
        if compressor == 0:
            struct.pack_into("<I", w.file, off + 4, vl + 1)            # 12 + k + v != len(buf)
        else:
            assert w.file[off + 12 + kl] < 127
            w.file[off + 12 + kl] += 1                                 # decodedLen one past the body
    wbase = len(src) + 3
    src = src + bytes(3) + bytes(w.file)
    rec_h = np.array([(wbase + o, ln, 0) for o, ln in recs], dtype=O.HANDLE_DT)
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src_t = torch.from_numpy(np.frombuffer(src, np.uint8).copy()).to(dev)
        rec_t = handles_tensor(rec_h, dev)
        kh_t = torch.from_numpy(np.array([O.fnv32(k) for k, _ in adds], dtype=np.uint32).view(np.int32)).to(dev)
        srt, skh = codec.writer_index(kh_t, len(adds))
    writers = np.zeros(1, dtype=WRITER_INDEX_DT)
    writers[0] = (rec_t.data_ptr(), srt.data_ptr(), skh.data_ptr(), len(adds), 9)
    fn_map_d = {5: 5, 9: 5}
    fn_count = 12
    fn_map = np.zeros(fn_count, np.uint32)
    for s_, d_ in fn_map_d.items():
        fn_map[s_] = d_
    fn_table = np.full(fn_count, 0xFFFFFFFF, np.uint32)
    fn_table[5] = 0
    missing = [b"zz%03d" % i for i in range(10)]
    qs = [(9, k) for k in good + empty + corrupt + healed + fresh_empty + fresh_good + missing]
    qs += [(5, k) for k in good[:10]] + [(10, k) for k in empty[:5]]
    h_t, s_t = codec.bithash_get(src_t, writers, tabs, fn_map, fn_table, [q[1] for q in qs], [q[0] for q in qs],
                                 compressor=compressor)
    codec.sync()
    h = h_t.cpu().numpy().view(np.uint8).view(O.HANDLE_DT)
    st = s_t.cpu().numpy().view(np.uint32)
    code = dict(ST, FILE_NUM_ZERO=ST_FILE_NUM_ZERO)
    base_of = {5: int(tabs["base"][0]), 9: wbase}
    fell = hit = 0
    for i, (fn, k) in enumerate(qs):
        es, efn, (eo, el) = T.bithash_get_handle({9: w}, files, fn_map_d, k, fn)
        assert st[i] == code[es], (i, fn, k, es, st[i])
        if es == "OK":
            assert int(h["offset"][i]) == base_of[efn] + eo and int(h["length"][i]) == el, (i, fn, k)
            if fn == 9:
                fell += efn == 5
                hit += efn == 9
    # every failure class fell through to table 5, every good writer record answered itself
    assert fell == len(empty) + len(corrupt) and hit == len(good) + len(healed) + len(fresh_good)
