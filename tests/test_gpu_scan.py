"""GPU parity for the table data-region scan (bhg_scan_tables).

The HIP header chase vs the CPU restatement bho_scan_region (oracle), which
follows TableIterator.findEntry (bithash/table.go:358-395, mode 0) and
Writer.rebuild (bithash/writer.go:539-583, mode 1).  Bit-exact on every
handle, on the per-table counts (out_first) and on the stop offsets (out_end).
Cases: uniform C2-shaped tables (speculative path), mixed lengths with uniform
runs (window chase and the switch between the two), complete .bht files from
the restated writer (K1/K4), the stop rules (12-zero terminator, valueSize 0,
ikeySize 0, short header, short key/value, value running past the end),
uint32 wrap of keySize+valueSize, empty/tiny tables, and max_out truncation.
"""
import random
import struct

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import table as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd import _lib
    from bitalosdb_amd.codec import BithashCodec
    _lib.lib()
    c = BithashCodec(0)
    yield c
    c.close()


def expected(tables, mode):
    hs, first, ends, base = [], [0], [], 0
    for b in tables:
        h, end = O.scan_region(b, mode=mode)
        h = h.copy()
        h["offset"] += base
        hs.append(h)
        first.append(first[-1] + len(h))
        ends.append(end)
        base += len(b)
    h = np.concatenate(hs) if hs else np.zeros(0, dtype=O.HANDLE_DT)
    return h, np.array(first, dtype=np.uint64), np.array(ends, dtype=np.uint64)


def run_scan(codec, tables, mode, max_out=None):
    src = b"".join(tables)
    off = np.zeros(len(tables) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in tables])
    src_t = torch.from_numpy(np.frombuffer(src + b"\0", dtype=np.uint8).copy()).to(codec.device)
    h, first, end = codec.scan_tables(src_t, off, mode=mode, max_out=max_out)
    codec.sync()
    h = h.cpu().numpy().view(np.uint8).reshape(-1).view(O.HANDLE_DT)[:len(h)] if len(h) else np.zeros(0, O.HANDLE_DT)
    return h, first.cpu().numpy().view(np.uint64), end.cpu().numpy().view(np.uint64)


def check(codec, tables, mode):
    eh, ef, ee = expected(tables, mode)
    gh, gf, ge = run_scan(codec, tables, mode)
    assert (gf == ef).all(), (gf[:8], ef[:8])
    assert (ge == ee).all(), (np.nonzero(ge != ee)[0][:8], ge[:8], ee[:8])
    assert len(gh) == len(eh)
    for f in ("offset", "length"):
        bad = np.nonzero(gh[f] != eh[f])[0]
        assert bad.size == 0, "%s differs at %s: got %s exp %s" % (f, bad[:8], gh[f][bad[:8]], eh[f][bad[:8]])
    return len(eh)


def rec(k, v, fn=7, seq=1):
    return O.record_set(k, seq << 8 | 1, v, fn)


def rand_bytes(rng, n):
    return rng.randbytes(n)


def uniform_table(rng, n, klen, vlen, term=True):
    k = rand_bytes(rng, klen)
    v = rand_bytes(rng, vlen)
    body = b"".join(rec(k, v, seq=i + 1) for i in range(n))
    return body + (bytes(12) if term else b"")


@pytest.mark.parametrize("mode", [0, 1])
def test_uniform_tables(codec, mode):
    rng = random.Random(1)
    tables = [uniform_table(rng, n, 32, 1024) for n in (1, 63, 64, 65, 1023, 1024, 1025, 5000)]
    tables.append(uniform_table(rng, 3000, 7, 13))            # ikeySize < 8, short records
    tables.append(uniform_table(rng, 2048, 32, 1024, term=False))  # data runs to the end of the table
    assert check(codec, tables, mode) > 10000


@pytest.mark.parametrize("mode", [0, 1])
def test_uniform_prefix_edges(codec, mode):
    """The grid-wide uniform-prefix pass (records i * G0 of the first record's length G0) hands
    the walk over at the first record that differs: prefixes broken by one odd record and then
    resumed at the same length (the resumed run is the walk's), a first record of another length,
    a prefix of one record, a prefix ending in every stop rule, and a prefix long enough to span
    many of the pass's 16,384-record strides."""
    rng = random.Random(12)
    k, v = rand_bytes(rng, 32), rand_bytes(rng, 1000)
    run = lambda n: b"".join(rec(k, v, seq=i + 1) for i in range(n))
    odd = rec(b"odd-one", rand_bytes(rng, 77))
    tables = [
        run(1000) + odd + run(500) + bytes(12),
        odd + run(1000) + bytes(12),
        run(1) + odd + run(3) + bytes(12),
        run(2),
        run(300) + rec(b"z", b"") + run(5) + bytes(12),               # valueSize 0 after the prefix
        run(300) + struct.pack("<III", 0, 9, 1) + b"x" * 40,          # ikeySize 0
        run(300) + struct.pack("<III", 4, 1 << 20, 1) + b"abcd",      # value past the end
        run(300) + b"panic",                                          # short header
        run(40000) + bytes(12),
        run(6)[:-100],                                                # the last record's value cut short
        struct.pack("<III", 4, 1 << 20, 1) + b"abcd",                 # record 0 runs past the end
    ]
    assert check(codec, tables, mode) > 42000


@pytest.mark.parametrize("mode", [0, 1])
def test_segment_walks_and_their_misses(codec, mode):
    """Tables past 1 MiB are walked as up to 64 segments from guessed entry points and stitched
    (k_tscan_seg / k_tscan_stitch / k_tscan_segw).  Random values: the guesses hold.  Values
    that hold 10 record-shaped sub-records and then noise: a segment that starts early in such a
    value guesses a sub-record chain that survives the guess test but never meets the true chain,
    so the stitch misses and the table takes the serial walk.  Both must match the restatement,
    as must a chain that jumps over whole segments (one 3-MiB value)."""
    rng = random.Random(21)
    recs = [rec(rand_bytes(rng, rng.randrange(8, 40)), rand_bytes(rng, rng.randrange(100, 4000)), seq=i + 1)
            for i in range(3000)]
    plain = b"".join(recs)
    sub = lambda: b"".join(struct.pack("<III", 2, 3, 1) + b"ab" + b"xyz" for _ in range(10))
    nested = b"".join(rec(rand_bytes(rng, 16), sub() + rand_bytes(rng, 7), seq=i + 1) for i in range(60000))
    jump = b"".join(recs[:100]) + rec(b"huge", rand_bytes(rng, 3 << 20)) + b"".join(recs[100:300])
    large = b"".join(rec(rand_bytes(rng, 24), rand_bytes(rng, rng.randrange(5000, 12000)), seq=i + 1)
                     for i in range(1500))  # a guess may leave the window after 3 records
    tables = [plain + bytes(12), nested + bytes(12), jump + bytes(12), plain * 3, large + bytes(12)]
    assert check(codec, tables, mode) > 60000


def test_step_log_overflow_falls_back_to_the_serial_walk(codec):
    """The write pass replays the count walk's logged steps (k_tscan_logw); a table whose walk
    takes more than TS_LOG_CAP = 4,096 steps is walked again to write (k_tscan<true>).  To get
    there the segment walks must miss: the records hold values with sub-record chains (as in
    test_segment_walks_and_their_misses), so guesses land on false chains and the stitch sends
    the table to the serial walk, whose ~4,400 windows of 128 KiB (a ~560-MB table after a
    uniform prefix) overflow the log.  Beside it a smaller table of the same records takes the replay
    and one with random values the segment walks.  out_path shows which pass wrote each table."""
    from bitalosdb_amd import _lib as B
    rng = random.Random(13)
    sub = lambda: b"".join(struct.pack("<III", 2, 3, 1) + b"ab" + b"xyz" for _ in range(10))
    chunk = b"".join(rec(rand_bytes(rng, 16), sub() + rand_bytes(rng, rng.randrange(1, 300)), seq=i + 1)
                     for i in range(2000))
    k, v = rand_bytes(rng, 32), rand_bytes(rng, 1000)
    prefix = b"".join(rec(k, v, seq=i + 1) for i in range(3000))
    reps = (540 << 20) // len(chunk) + 1
    big = prefix + chunk * reps + bytes(12)
    small = chunk * 8 + bytes(12)  # ~5 MB: 5 segments, a missed guess among them -> the replay
    recs = [rec(rand_bytes(rng, rng.randrange(8, 40)), rand_bytes(rng, rng.randrange(100, 4000)), seq=i + 1)
            for i in range(300)]
    plain = b"".join(recs * 20) + bytes(12)  # random values: the guesses hold
    tables = [big, small, plain]
    eh, ef, ee = expected(tables, 0)
    src = b"".join(tables)
    off = np.zeros(len(tables) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(b) for b in tables])
    src_t = torch.from_numpy(np.frombuffer(src + b"\0", dtype=np.uint8).copy()).to(codec.device)
    gh, gf, ge, gp = codec.scan_tables(src_t, off, mode=0, max_out=int(ef[-1]), paths=True)
    codec.sync()
    gh = gh.cpu().numpy().view(np.uint8).reshape(-1).view(O.HANDLE_DT)
    assert (gf.cpu().numpy().view(np.uint64) == ef).all()
    assert (ge.cpu().numpy().view(np.uint64) == ee).all()
    assert (gh["offset"] == eh["offset"]).all() and (gh["length"] == eh["length"]).all()
    assert gp.cpu().tolist() == [B.SCAN_PATH_SERIAL, B.SCAN_PATH_REPLAY, B.SCAN_PATH_SEGMENTS]


@pytest.mark.parametrize("mode", [0, 1])
def test_many_small_tables(codec, mode):
    """More tables than one scratch pass holds (256): the per-table counts of later passes are
    rebased on the earlier ones' totals (k_tscan_carry).  600 small tables of mixed shapes."""
    rng = random.Random(31)
    tables = []
    for t in range(600):
        kind = t % 4
        if kind == 0:
            tables.append(uniform_table(rng, rng.randrange(0, 40), 16, 100))
        elif kind == 1:
            tables.append(b"".join(rec(rand_bytes(rng, rng.randrange(1, 30)), rand_bytes(rng, rng.randrange(1, 300)))
                                   for _ in range(rng.randrange(0, 30))) + bytes(12))
        elif kind == 2:
            tables.append(b"")
        else:
            tables.append(uniform_table(rng, 5, 8, 40, term=False) + b"panic")
    assert check(codec, tables, mode) > 3000


@pytest.mark.parametrize("mode", [0, 1])
def test_mixed_lengths_and_runs(codec, mode):
    rng = random.Random(2)
    tables = []
    for t in range(12):
        parts = []
        for _ in range(rng.randrange(1, 40)):
            klen, vlen = rng.randrange(1, 80), rng.randrange(1, 3000)
            run = rng.choice([1, 1, 2, 5, 40, 300, 1500])
            if run == 1:
                parts.append(rec(rand_bytes(rng, klen), rand_bytes(rng, vlen), seq=len(parts) + 1))
            else:
                parts.append(uniform_table(rng, run, klen, vlen, term=False))
        tail = rng.choice([bytes(12), bytes(12) + b"tail", b"", b"panic", bytes(5)])
        tables.append(b"".join(parts) + tail)
    assert check(codec, tables, mode) > 1000


@pytest.mark.parametrize("mode", [0, 1])
def test_stop_rules(codec, mode):
    rng = random.Random(3)
    base = b"".join(rec(b"k%d" % i, b"v" * (i + 1)) for i in range(5))
    long_hdr = struct.pack("<III", 4, 1 << 20, 1) + b"abcd"      # value runs past the end
    tables = [
        b"",                                                    # empty table
        bytes(5), bytes(11), bytes(12), b"x" * 11,
        base + bytes(12) + b"tail",                             # terminator
        base + rec(b"z", b"") + base + bytes(12),               # valueSize 0: stops mode 0 only
        base + struct.pack("<III", 0, 9, 1) + b"x" * 40,        # ikeySize 0
        base + b"panic",                                        # short header
        base + struct.pack("<III", 50, 1, 1) + b"short",        # short key
        base + struct.pack("<III", 4, 100, 1) + b"keyXval",     # short value (mode 0 stop, mode 1 handle)
        base + long_hdr,
        base + struct.pack("<III", 1, 0xFFFFFFFF, 1) + b"Q" + rec(b"after", b"wrap") * 3 + bytes(12),  # u32 wrap
        struct.pack("<III", 0xFFFFFFF0, 0x20, 1) + b"k" * 64,   # u32 wrap on the first record
    ]
    tables += [uniform_table(rng, 2000, 24, 600, term=False) + long_hdr]
    check(codec, tables, mode)


@pytest.mark.parametrize("mode", [0, 1])
def test_writer_tables(codec, mode):
    """Complete .bht files (data, conflict, hash index, meta, footer) from the
    restated writer: K1 (three tables after splits) and a K4-style table."""
    rng = random.Random(9)
    st = T.Store(1 << 20)
    s = st.flush_start()
    for i in range(1200):
        s.add(b"bithash_testkey_%d" % i, i + 1, rand_bytes(rng, rng.randrange(1, 4096)))
    s.compact = True
    s.finish()
    tables = [bytes(st.files[fn]) for fn in sorted(st.files)]
    assert check(codec, tables, mode) == 1200


def test_random_garbage_rebuild(codec):
    """Rebuild over garbage after valid records: random headers with small keys."""
    rng = random.Random(5)
    tables = []
    for t in range(20):
        body = b"".join(rec(rand_bytes(rng, rng.randrange(1, 20)), rand_bytes(rng, rng.randrange(0, 50)))
                        for _ in range(rng.randrange(0, 200)))
        junk = b"".join(struct.pack("<II", rng.randrange(1, 16), rng.randrange(0, 64)) + rand_bytes(rng, rng.randrange(0, 40))
                        for _ in range(rng.randrange(0, 50)))
        tables.append(body + junk)
    for mode in (0, 1):
        check(codec, tables, mode)


def test_max_out_truncation(codec):
    rng = random.Random(6)
    tables = [uniform_table(rng, 3000, 16, 100), uniform_table(rng, 10, 16, 100)]
    eh, ef, ee = expected(tables, 0)
    gh, gf, ge = run_scan(codec, tables, 0, max_out=2000)
    assert (gf == ef).all() and (ge == ee).all()
    assert (gh["offset"] == eh["offset"][:2000]).all()


def test_c2_size_scan(codec):
    """configs[1]-sized region (1M records of 1076 B in 128 MiB tables):
    handles equal the generator's, counts per table, stops at the terminators."""
    from bitalosdb_amd import synth
    n = 1 << 20
    src, h, meta = synth.uniform_tables(n, device=codec.device)
    tb = meta["table_bytes"]
    off = np.array([min(t * tb, meta["src_bytes"]) for t in range(meta["tables"])] + [meta["src_bytes"]], dtype=np.uint64)
    gh, gf, ge = codec.scan_tables(src, off, mode=0)
    codec.sync()
    gh = gh.cpu().numpy().view(np.uint8).reshape(-1).view(O.HANDLE_DT)
    assert len(gh) == n
    assert (gh["offset"] == h["offset"]).all() and (gh["length"] == h["length"]).all()
    ge = ge.cpu().numpy().view(np.uint64)
    assert (ge == np.diff(off) - 12).all()
