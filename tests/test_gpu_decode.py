"""GPU parity: the HIP decode path (through the C-ABI) vs the CPU restatement.

Bit-exact on every descriptor field and every decoded byte.  Cases follow
what the reference tests / reads exercise: uniform 32 B/1 KiB records
(C2 shape), mixed sizes, arbitrary byte alignment, the readRecord nil rules
(block2.go:57-66), zero/over-long handles (reader.go:234-258), ikeySize < 8
(base.DecodeInternalKey), snappy values incl. corrupt streams, the K1/K2
known-answer tables, and the full-size C2 batch.
"""
import random

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import table as T

pytestmark = pytest.mark.gpu

FIELDS = ["key_off", "key_len", "val_off", "val_len", "trailer", "file_num", "fnv1", "crc", "status"]


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd.codec import BithashCodec
    c = BithashCodec(0)
    yield c
    c.close()


def assert_desc_equal(got, exp):
    assert len(got) == len(exp)
    for f in FIELDS:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, "field %s differs at %s: got %s exp %s" % (
            f, bad[:8], got[f][bad[:8]], exp[f][bad[:8]])


def make_records(rng, specs, gap_max=0, codec=0):
    """specs: list of (ukey, value, file_num). Returns (src bytes, handles)."""
    buf = bytearray()
    hs = []
    for i, (k, v, fn) in enumerate(specs):
        buf += bytes(rng.randrange(256) for _ in range(rng.randrange(gap_max + 1))) if gap_max else b""
        val = O.snappy_encode(v) if codec == 1 else v
        rec = O.record_set(k, (i + 1) << 8 | 1, val, fn)
        hs.append((len(buf), len(rec), 0))
        buf += rec
    return bytes(buf), np.array(hs, dtype=O.HANDLE_DT)


def rand_bytes(rng, n):
    return bytes(rng.randrange(256) for _ in range(n))


def test_uniform_c2_shape(codec):
    rng = random.Random(11)
    specs = [(rand_bytes(rng, 32), rand_bytes(rng, 1024), 1 + i // 1000) for i in range(3000)]
    src, h = make_records(rng, specs)
    got, _, _ = codec.decode(src, h)
    exp, _, _ = O.decode_batch(src, h)
    assert_desc_equal(got, exp)
    assert (got["status"] == 0).all() and (got["val_len"] == 1024).all()


@pytest.mark.parametrize("gap", [0, 3, 17])
def test_mixed_sizes_and_alignment(codec, gap):
    rng = random.Random(gap)
    specs = []
    for i in range(1500):
        kl = rng.choice([0, 1, 5, 7, 8, 16, 31, 32, 33, 35, 36, 37, 39, 40, 41, 48, 100])
        vl = rng.choice([1, 2, 3, 4, 5, 63, 64, 65, 300, 1024, 1025, 4096, 9000])
        specs.append((rand_bytes(rng, kl), rand_bytes(rng, vl), rng.randrange(1 << 32)))
    src, h = make_records(rng, specs, gap_max=gap)
    got, _, _ = codec.decode(src, h)
    exp, _, _ = O.decode_batch(src, h)
    assert_desc_equal(got, exp)


def test_status_edge_cases(codec):
    rng = random.Random(5)
    src, h = make_records(rng, [(b"k" * 32, b"v" * 1024, 7), (b"abc", b"x" * 10, 8), (b"", b"y", 9)])
    src = bytearray(src)
    extra = []
    # raw ikeySize < 8 record (UserKey nil, trailer = InternalKeyKindInvalid)
    small = bytearray(np.array([3, 2, 5], dtype="<u4").tobytes()) + b"abc" + b"zz"
    extra.append((len(src), len(small)))
    src += small
    # zero valueSize / zero ikeySize / length mismatch / too short
    for k, v, pay in ((8, 0, b"\0" * 8), (0, 4, b"wxyz"), (8, 4, b"\0" * 8 + b"abc")):
        rec = bytearray(np.array([k, v, 1], dtype="<u4").tobytes()) + pay
        extra.append((len(src), len(rec)))
        src += rec
    extra.append((0, 5))                      # L < 12
    extra.append((0, 0))                      # ILLEGAL_LENGTH
    extra.append(("END-3", 10))               # past the end -> INCOMPLETE
    extra.append(("END+100", 1))              # offset past the end
    # uint32-wrapping header: 12 + k + v wraps to L
    wrap = bytearray(np.array([0xFFFFFFF0, 0x20, 1], dtype="<u4").tobytes()) + b"\0" * 16
    extra.append((len(src), 28))
    src += wrap
    # a record that ends exactly at the (unaligned) end of src
    tail = O.record_set(b"tailkey", 99 << 8 | 1, b"q" * 13, 3)
    src += b"\x01"
    extra.append((len(src), len(tail)))
    src += tail
    end = len(src)
    fix = {"END-3": end - 3, "END+100": end + 100}
    hs = np.concatenate([h, np.array([(fix.get(o, o), l, 0) for o, l in extra], dtype=O.HANDLE_DT)])
    got, _, _ = codec.decode(bytes(src), hs)
    exp, _, _ = O.decode_batch(bytes(src), hs)
    assert_desc_equal(got, exp)
    st = list(exp["status"])
    assert st[:3] == [0, 0, 0]
    assert st[3] == 0 and exp["trailer"][3] == 255 and exp["key_len"][3] == 0
    assert st[4:7] == [O.RECORD_NIL] * 3
    assert st[7:11] == [O.RECORD_NIL, O.ILLEGAL_LENGTH, O.INCOMPLETE, O.INCOMPLETE]
    assert st[11] == O.RECORD_NIL and st[12] == 0


def test_expected_crc(codec):
    rng = random.Random(6)
    specs = [(rand_bytes(rng, 32), rand_bytes(rng, 200), 1) for _ in range(500)]
    src, h = make_records(rng, specs, gap_max=5)
    exp0, _, _ = O.decode_batch(src, h)
    want = exp0["crc"].copy()
    want[::7] ^= 1
    got, _, _ = codec.decode(src, h, expected_crc=want)
    exp, _, _ = O.decode_batch(src, h, expected_crc=want)
    assert_desc_equal(got, exp)
    assert (got["status"][::7] == O.CRC_MISMATCH).all()


def np_bytes(g, n):
    return g.integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("seed", [1, 2])
def test_long_record_batches(codec, seed):
    """A NoCompressor batch whose mean record is past 8 KiB takes the long-record pass
    (bhg_longcrc.hip): records over 4 KiB are CRC'd as 8-KiB pieces by the whole chip and the
    tile kernel leaves their CRC / status to it.  Mixed with short records, odd offsets, the
    readRecord / readData statuses, lengths at the 4-KiB, 16-KiB, 128-B, 8-KiB and 64-KiB edges, 1-3 MiB
    records, and expected CRCs with some flipped."""
    rng = random.Random(seed)
    g = np.random.default_rng(seed)
    vlens = [g.integers(16400, 400000) for _ in range(150)] + [g.integers(1, 16000) for _ in range(30)]
    vlens += [(1 << 20) + int(g.integers(0, 2 << 20)) for _ in range(4)]
    vlens += [16384 - 60, 16384 - 59, 65536 - 60, 65536 - 59, 131072 - 52, 128 * 1000 - 52, 65536 * 3 + 1]
    vlens += [4096 - 60, 4096 - 59, 4096 - 58, 8192 - 60, 8192 - 59, 8192 + 68, 12288 - 60]
    rng.shuffle(vlens)
    specs = [(rand_bytes(rng, rng.randrange(0, 48)), np_bytes(g, int(v)), rng.randrange(1 << 32)) for v in vlens]
    src, h = make_records(rng, specs, gap_max=3)
    h = h.copy()
    h["length"][5] -= 1                 # RECORD_NIL (its CRC is still computed)
    h["length"][6] = 0                  # ILLEGAL_LENGTH
    h["offset"][7] = len(src) - 100     # INCOMPLETE
    assert len(src) > 8192 * len(h)
    exp0, _, _ = O.decode_batch(src, h)
    want = exp0["crc"].copy()
    want[::5] ^= 1
    got, _, _ = codec.decode(src, h, expected_crc=want)
    exp, _, _ = O.decode_batch(src, h, expected_crc=want)
    assert_desc_equal(got, exp)
    assert (got["status"] == O.CRC_MISMATCH).sum() > 20


def test_long_record_pass_overflow_list(codec):
    """Handles that overlap (the same 3-MiB record many times) give more pieces than the piece
    list holds (src_len / 8 KiB + n + 1): those records take the overflow walk, one wave per
    record; the results must not depend on which path a record took."""
    rng = random.Random(3)
    g = np.random.default_rng(3)
    src, h1 = make_records(rng, [(b"big-key", np_bytes(g, 3 << 20), 7), (b"small", b"v" * 100, 8)])
    h = np.concatenate([np.repeat(h1[:1], 150), h1[1:], np.repeat(h1[:1], 50)])
    h["length"][10] -= 7  # one of them RECORD_NIL
    got, _, _ = codec.decode(src, h)
    exp, _, _ = O.decode_batch(src, h)
    assert_desc_equal(got, exp)


def compressible(rng, n):
    d = rand_bytes(rng, 512)
    out = bytearray()
    while len(out) < n:
        if rng.random() < 0.2:
            out += rand_bytes(rng, rng.randrange(1, 16))
        else:
            ln = rng.randrange(4, 64)
            st = rng.randrange(0, 512 - ln)
            out += d[st:st + ln]
    return bytes(out[:n])


def test_snappy_values(codec):
    rng = random.Random(7)
    specs = []
    for i in range(1200):
        vl = rng.choice([1, 5, 16, 17, 100, 1024, 1024, 1024, 3000, 5000, 70000 if i % 300 == 0 else 2000])
        v = compressible(rng, vl) if i % 3 else b"ab" * (vl // 2) + b"c" * (vl % 2)
        specs.append((rand_bytes(rng, 32), v, 2))
    src, h = make_records(rng, specs, gap_max=2, codec=1)
    got, gvals, goff = codec.decode(src, h, compressor=1)
    exp, evals, eoff = O.decode_batch(src, h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    assert gvals.tobytes() == evals[:int(eoff[-1])].tobytes()
    for i in (0, 1, 2, 300, 1199):
        assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == specs[i][1]


def test_snappy_corrupt_streams(codec):
    rng = random.Random(8)
    good = O.snappy_encode(compressible(rng, 1024))
    bad_streams = [
        good[:-1],                                   # truncated
        b"\x05" + bytes([0 << 2]) + b"a" + bytes([0x01, 0x00]),   # copy1 with offset 0
        b"\x05" + bytes([0 << 2, 1]),                # short output
        b"\xff\xff\xff\xff\x1f" + b"\0" * 8,         # decodedLen > 0xffffffff
        b"\xff\xff\x03" + bytes([0 << 2, 1]),        # absurd decodedLen (> 64/3 x payload)
        b"\x08" + bytes([60 << 2]),                  # truncated literal length
        b"\x00",                                     # empty value -> ok (dLen 0)
        b"\x03" + bytes([2 << 2]) + b"abc",          # ok
    ]
    specs_src = bytearray()
    hs = []
    for i, s in enumerate(bad_streams):
        rec = O.record_set(b"key%d" % i, 1 << 8 | 1, s, 4)
        hs.append((len(specs_src), len(rec), 0))
        specs_src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(specs_src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(specs_src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    assert list(exp["status"][:6]) == [O.SNAPPY_CORRUPT] * 6
    assert list(exp["status"][6:]) == [0, 0]


def _uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append(x & 0x7f | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def test_snappy_inplace_spill_and_oversize(codec):
    """The LDS decoder decodes in place (stream at the slot end, output from the
    start).  A valid stream whose output runs far ahead of its stream -- 700 B of
    RLE copies first, then 324 one-byte copies (3 stream bytes each) -- would
    overwrite its own unread tags: the walk must hand it to the global-memory
    pass.  Mixed with ordinary blocks, oversize blocks (> 1 KiB out) and
    incompressible ones, so the fallback list holds a few blocks among many."""
    rng = random.Random(21)
    body = bytes([0 << 2]) + b"x"                      # literal "x"
    body += (bytes([(64 - 1) << 2 | 2]) + (1).to_bytes(2, "little")) * 10   # 10 x copy-2, n 64, offset 1
    body += bytes([(59 - 1) << 2 | 2]) + (1).to_bytes(2, "little")          # copy n 59 -> 700 B so far
    body += (bytes([0 << 2 | 2]) + (7).to_bytes(2, "little")) * 324        # 324 x copy-2, n 1, offset 7
    spill = _uvarint(1024) + body
    assert len(spill) <= 1024
    want = O.snappy_decode(spill)
    assert want is not None and len(want) == 1024
    streams = []
    for i in range(3000):
        k = i % 6
        if k == 0:
            streams.append(spill)
        elif k == 1:
            streams.append(O.snappy_encode(rand_bytes(rng, 1024)))         # incompressible: clen > 1 KiB
        elif k == 2:
            streams.append(O.snappy_encode(compressible(rng, 3000)))       # oversize output
        else:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([16, 500, 1024]))))
    src = bytearray()
    hs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"spill%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert (exp["status"] == 0).all()
    assert np.array_equal(goff, eoff)
    assert gvals.tobytes() == evals[:int(eoff[-1])].tobytes()
    assert gvals[int(goff[0]):int(goff[1])].tobytes() == want


def _lit(data):
    n = len(data)
    if n <= 60:
        return bytes([(n - 1) << 2]) + data
    if n <= 256:
        return bytes([60 << 2, n - 1]) + data
    return bytes([61 << 2]) + (n - 1).to_bytes(2, "little") + data


def _lit_any(data):
    """emitLiteral for any length (1-4 length bytes)."""
    n = len(data) - 1
    if n < 60:
        return bytes([n << 2]) + data
    nb = (n.bit_length() + 7) // 8
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + data


def _copy2(off, ln):
    return bytes([(ln - 1) << 2 | 2]) + off.to_bytes(2, "little")


@pytest.mark.parametrize("seed", [1, 2])
def test_snappy_big_blocks_chunked(codec, seed):
    """Blocks past the LDS tiers decode chunk-parallel: a wave parses the tags and cuts the block at
    every 64 KiB of output (k_sb_parse), a lane walks each chunk (k_sb_walk); irregular blocks fall
    to the serial pass.  Golang-encoded values of 5 KiB - 3 MiB (compressible, random, zeros),
    hand-built streams whose copies reach back across a 64-KiB output boundary (valid snappy the
    chunked walk cannot decode: serial pass), a literal longer than 64 KiB with a 3-byte length, and
    corrupted big streams -- statuses, offsets and values equal the restated decoder's."""
    rng = random.Random(seed)
    g = np.random.default_rng(seed)
    vals = []
    for i in range(60):
        sz = rng.choice([5000, 70000, 65536, 65537, 131072 + 9, 300000, (1 << 20) + 7, 3 << 20])
        k = i % 3
        vals.append(compressible(rng, sz) if k == 0 else g.integers(0, 256, sz, dtype=np.uint8).tobytes()
                    if k == 1 else bytes(sz))
    streams = [O.snappy_encode(v) for v in vals]
    big = g.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    cross = _lit_any(big) + _copy2(30000, 64) * 100 + _copy2(1, 60)  # copies from 30 KB back at d >= 64 KiB
    streams.append(_uvarint(70000 + 6400 + 60) + cross)
    lit3 = _lit_any(big + big[:1000])                              # one literal of 71,000 B (3-byte length)
    streams.append(_uvarint(71000) + lit3 + _copy2(71000 % 65536, 40))
    streams[-1] = _uvarint(71040) + lit3 + _copy2(5000, 40)
    bad = bytearray(O.snappy_encode(compressible(rng, 500000)))
    bad[len(bad) // 2] ^= 0xff                                     # corrupted big stream
    streams.append(bytes(bad))
    trunc = O.snappy_encode(compressible(rng, 200000))
    streams.append(trunc[:-7])                                     # truncated: ends early
    small = [O.snappy_encode(compressible(rng, rng.choice([16, 500, 1024, 3000]))) for _ in range(200)]
    allst = streams + small
    rng.shuffle(allst)
    src = bytearray()
    hs = []
    for i, st in enumerate(allst):
        rec = O.record_set(b"big%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    ok = np.nonzero(exp["status"] == 0)[0]
    assert len(ok) >= len(allst) - 3
    for i in ok:
        assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == evals[int(eoff[i]):int(eoff[i + 1])].tobytes(), i


def _lit_runs(rng, data, lo, hi):
    """data as literals of rng lengths in [lo, hi]."""
    out, j = [], 0
    while j < len(data):
        k = min(len(data) - j, rng.randint(lo, hi))
        out.append(_lit_any(data[j:j + k]))
        j += k
    return b"".join(out)


@pytest.mark.parametrize("seed", [3, 4])
def test_snappy_segment_parse(codec, seed):
    """Streams longer than 32 KiB are parsed in 16-KiB segments (k_sb_seg: 64 speculative chains
    per segment, k_sb_stitch: the block's chain through them, k_sb_emit: the 64-KiB chunk slots).
    Cases: golang-encoded compressible values of 100 KiB - 2 MiB; literals of 65-300 B (a literal
    over a segment start: the stitch walks that segment itself); streams of 1-byte literals (stream
    twice the output: more segments than the scratch holds, so some blocks take the one-wave parse);
    a 200-KiB literal (one element over three 64-KiB output boundaries: empty chunks); a copy
    offset past the output in a late segment, a literal length past the stream, a trailing extra
    byte (irregular: serial pass); stream lengths at the 32-KiB edge."""
    rng = random.Random(seed)
    g = np.random.default_rng(seed)
    streams = []
    for sz in [100000, 300000, (1 << 20) + 3, 2 << 20]:
        streams.append(O.snappy_encode(compressible(rng, sz)))
    for _ in range(6):
        d = np_bytes(g, rng.choice([70000, 150000, 400000]))
        st = _lit_runs(rng, d, 65, 300)
        streams.append(_uvarint(len(d)) + st)
    for _ in range(40):  # 1-byte literals: 2 stream bytes per output byte
        d = np_bytes(g, rng.choice([66000, 120000, 250000]))
        streams.append(_uvarint(len(d)) + b"".join(bytes([0]) + d[j:j + 1] for j in range(len(d))))
    d = np_bytes(g, 200000)
    streams.append(_uvarint(200000 + 64) + _lit_any(d) + _copy2(1000, 64))
    for edge in [32767, 32768, 32769, 32770]:  # stream lengths (after the uvarint) around kSbSegMin
        body = _lit_any(np_bytes(g, 1000))
        y = 2 * (edge - len(body)) % 3  # 3 x + 2 y = the rest
        x = (edge - len(body) - 2 * y) // 3
        body += _copy2(1000, 64) * x + bytes([(11 - 4) << 2 | 1, 100]) * y  # copy-2s, then copy-1s of 11 B
        assert len(body) == edge
        streams.append(_uvarint(1000 + 64 * x + 11 * y) + body)
    base = O.snappy_encode(compressible(rng, 600000))
    lastcp = len(base) - 200
    while base[lastcp] & 3 != 2:
        lastcp += 1
    b1 = bytearray(base)
    b1[lastcp + 1:lastcp + 3] = (0xffff).to_bytes(2, "little")  # copy offset past the output written
    streams.append(bytes(b1))
    d = np_bytes(g, 80000)
    streams.append(_uvarint(80000) + _lit_any(d)[:-10])               # literal past the stream
    streams.append(O.snappy_encode(compressible(rng, 90000)) + b"\x00")  # extra byte after dlen
    small = [O.snappy_encode(compressible(rng, rng.choice([16, 900, 3000]))) for _ in range(100)]
    allst = streams + small
    rng.shuffle(allst)
    src = bytearray()
    hs = []
    for i, st in enumerate(allst):
        rec = O.record_set(b"seg%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    # a batch of long records (mean past 8 KiB): the header pass leaves the records over 4 KiB to
    # the long-record CRC pass; expected CRCs with every 7th flipped check its status
    assert len(src) > 8192 * len(h)
    e0, _, _ = O.decode_batch(bytes(src), h, codec=1)
    ecrc = e0["crc"].astype(np.uint32).copy()
    ecrc[::7] ^= 1
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1, expected_crc=ecrc)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1, expected_crc=ecrc)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    assert (exp["status"] == O.CRC_MISMATCH).sum() >= len(h) // 7 - 6
    ok = np.nonzero((exp["status"] == O.OK) | (exp["status"] == O.CRC_MISMATCH))[0]
    assert len(ok) >= len(allst) - 6
    for i in ok:
        assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == evals[int(eoff[i]):int(eoff[i + 1])].tobytes(), i


@pytest.mark.parametrize("seed", [7, 8])
def test_snappy_big_streams_fuzzed(codec, seed):
    """Long golang/snappy streams (the segment parse, the chunk walk) with 1-3 bytes flipped at
    random places, each flip a stream of its own; random bytes behind a valid uvarint of a large
    decoded length; truncations at random points.  Every descriptor and every decoded value must
    equal the restated decoder's -- a corrupt stream is reported, never decoded into other bytes."""
    rng = random.Random(seed)
    g = np.random.default_rng(seed)
    bases = [O.snappy_encode(compressible(rng, n)) for n in (70000, 200000, 700000)]
    bases.append(O.snappy_encode(np_bytes(g, 150000)))
    streams = []
    for b in bases:
        streams.append(b)
        for _ in range(12):
            x = bytearray(b)
            for _ in range(rng.randint(1, 3)):
                x[rng.randrange(4, len(x))] ^= rng.randrange(1, 256)
            streams.append(bytes(x))
        for _ in range(3):
            streams.append(b[:rng.randrange(len(b) // 2, len(b))])
    for n in (40000, 100000, 300000):
        streams.append(_uvarint(2 * n) + np_bytes(g, n))
    small = [O.snappy_encode(compressible(rng, rng.choice([50, 900, 3000]))) for _ in range(60)]
    allst = streams + small
    rng.shuffle(allst)
    src = bytearray()
    hs = []
    for i, st in enumerate(allst):
        rec = O.record_set(b"fz%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    ok = np.nonzero(exp["status"] == 0)[0]
    assert len(ok) >= len(small) + len(bases)
    assert (exp["status"] == O.SNAPPY_CORRUPT).sum() >= 20
    for i in ok:
        assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == evals[int(eoff[i]):int(eoff[i + 1])].tobytes(), i


def test_snappy_long_streams_in_lds(codec):
    """Streams longer than the 64 chunks a lane-per-chunk staging covers (1,025 .. 1,064 B
    for a <= 1 KiB value: values snappy cannot shrink) are decoded in their LDS slot, the
    bytes past 1 KiB loaded separately; longer ones still go to the global-memory pass.
    k one-byte literals then one literal of the rest: stream = 1,028 + k bytes for 1,024 out.
    The last record (the end of src) is one of the longest LDS-path streams."""
    rng = random.Random(33)
    streams = []
    for i in range(1200):
        k = rng.choice([0, 3, 10, 22, 28, 36, 40, 42, 60])
        out = rand_bytes(rng, 1024)
        st = _uvarint(1024) + b"".join(_lit(out[j:j + 1]) for j in range(k)) + _lit(out[k:])
        assert O.snappy_decode(st) == out
        streams.append(st)
        if i % 5 == 0:
            streams.append(O.snappy_encode(rand_bytes(rng, rng.choice([1000, 1010, 1024]))))
    streams.append(_uvarint(1024) + b"".join(_lit(bytes([j])) for j in range(36)) + _lit(rand_bytes(rng, 988)))
    src = bytearray()
    hs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"long%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert (exp["status"] == 0).all()
    assert np.array_equal(goff, eoff)
    assert gvals.tobytes() == evals[:int(eoff[-1])].tobytes()


def test_snappy_tier2_slots(codec):
    """Values decoding to 1-4 KiB go to the second LDS tier (4,160-B slots, 4 stream
    chunks per lane): ordinary 1,025..4,096-B blocks, tier-1 spill hand-overs, streams past
    4 KiB (incompressible 4,000..4,096-B values: the tail loaded at the dump), a tier-2
    in-place spill (2,800 B of RLE copies, then 1,296 one-byte copies) and corrupt
    1-4 KiB streams, mixed with > 4 KiB blocks for the global-memory pass.  The last
    record (the end of src) is a tier-2 stream past 4 KiB."""
    rng = random.Random(44)
    body = bytes([0 << 2]) + b"x"
    body += (bytes([(64 - 1) << 2 | 2]) + (1).to_bytes(2, "little")) * 43   # 2,753 B
    body += bytes([(47 - 1) << 2 | 2]) + (1).to_bytes(2, "little")          # 2,800 B
    body += (bytes([0 << 2 | 2]) + (7).to_bytes(2, "little")) * 1296       # 4,096 B
    spill2 = _uvarint(4096) + body
    assert O.snappy_decode(spill2) is not None and len(spill2) + 24 <= 4160
    streams = []
    for i in range(2400):
        k = i % 10
        if k == 0:
            streams.append(spill2)
        elif k == 1:
            streams.append(O.snappy_encode(rand_bytes(rng, rng.choice([4000, 4070, 4096]))))
        elif k == 2:
            good = O.snappy_encode(compressible(rng, rng.choice([1500, 4096])))
            streams.append(good[:-rng.randrange(1, 6)] if i % 20 == 2 else good[:5] + b"\x01\xff" + good[7:])
        elif k == 3:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([4097, 6000]))))
        elif k == 4:
            streams.append(O.snappy_encode(rand_bytes(rng, 1024)))
        else:
            streams.append(O.snappy_encode(compressible(rng, rng.randrange(1025, 4097))))
    streams.append(O.snappy_encode(rand_bytes(rng, 4096)))
    src = bytearray()
    hs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"t2-%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    # a corrupt block's slot holds no value (the reference returns snappy.ErrCorrupt): ok blocks only
    bad = [(i, int(eoff[i + 1] - eoff[i]), len(streams[i])) for i in range(len(streams))
           if exp["status"][i] == 0 and gvals[int(goff[i]):int(goff[i + 1])].tobytes() != evals[int(eoff[i]):int(eoff[i + 1])].tobytes()]
    assert not bad, "blocks differ (index, dlen, clen): %s of %d" % (bad[:12], len(bad))
    st = exp["status"]
    assert (st[0::10] == 0).all() and (st[1::10] == 0).all() and (st[5::10] == 0).all()
    assert (st[2::10] == O.SNAPPY_CORRUPT).sum() > 100


def test_snappy_small_majority_with_large_minority(codec):
    """Tier 1 walks the batch in its own order when >= 7/8 of the blocks are <= 1 KiB (and the
    header pass's list otherwise): a batch of 1-KiB blocks with a minority of 1-4 KiB and
    > 4 KiB blocks, spills and incompressible 1 KiB values, corrupt and oversize streams among
    them -- the minority must be decoded by tier 2 / the global pass exactly once."""
    rng = random.Random(55)
    streams = []
    for i in range(2400):
        k = i % 40
        if k == 0:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([1500, 3000, 4096]))))
        elif k == 1:
            streams.append(O.snappy_encode(compressible(rng, 9000)))
        elif k == 2:
            streams.append(O.snappy_encode(rand_bytes(rng, 1024)))        # stream > 1,064 B: the 4-KiB tier
        elif k == 3:
            good = O.snappy_encode(compressible(rng, 1024))
            streams.append(good[:-2])                                    # corrupt
        else:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([16, 500, 1000, 1024]))))
    src = bytearray()
    hs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"nat-%d" % i, 1 << 8 | 1, st, 4)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    ok = [i for i in range(len(streams)) if exp["status"][i] == 0]
    assert len(ok) >= 2300
    for i in ok:
        assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == evals[int(eoff[i]):int(eoff[i + 1])].tobytes(), i


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 130, 4097])
def test_snappy_lists_shuffled_duplicates_small_batches(codec, n):
    """The header pass files each block into a decode list by its wave's tile (sub-list =
    tile mod 64), and the roles read the lists back by a per-wave binary search over the
    sub-list sizes: batch sizes around the wave and sub-list boundaries (1 .. 4,097 handles,
    4,097 = one handle past 64 tiles), handles in shuffled order with duplicates (one record
    decoded into two output slots), every size class present."""
    rng = random.Random(1000 + n)
    streams = []
    for i in range(min(n, 400)):
        k = i % 6
        if k == 0:
            streams.append(O.snappy_encode(compressible(rng, rng.randrange(1025, 4097))))
        elif k == 1:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([4097, 7000]))))
        elif k == 2:
            streams.append(O.snappy_encode(rand_bytes(rng, rng.choice([900, 1024, 2000]))))
        elif k == 3:
            streams.append(O.snappy_encode(compressible(rng, rng.randrange(0, 1025)))[:-1] if i % 12 == 3
                           else O.snappy_encode(compressible(rng, rng.randrange(0, 1025))))
        else:
            streams.append(O.snappy_encode(compressible(rng, rng.randrange(1, 1025))))
    src = bytearray()
    recs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"sl-%d" % i, 1 << 8 | 1, st, 5)
        recs.append((len(src), len(rec), 0))
        src += rec
    pick = [rng.randrange(len(recs)) for _ in range(n)]
    if n >= 2:
        pick[-1] = pick[0]                     # a duplicate handle at the far end of the batch
    h = np.array([recs[j] for j in pick], dtype=O.HANDLE_DT)
    got, gvals, goff = codec.decode(bytes(src), h, compressor=1)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(goff, eoff)
    for i in range(n):
        if exp["status"][i] == 0:
            assert gvals[int(goff[i]):int(goff[i + 1])].tobytes() == evals[int(eoff[i]):int(eoff[i + 1])].tobytes(), i


def _view_with_bit31(nbytes, dev):
    """A uint8 device view of nbytes whose address has bit 31 of its low word set
    over its whole length (low word in [0x80000100, 0xFFFFFFFF])."""
    assert nbytes < (1 << 30)
    big = torch.empty((1 << 31) + 2 * nbytes + (1 << 20), dtype=torch.uint8, device=dev)
    lo = big.data_ptr() & 0xFFFFFFFF
    if 0x80000100 <= lo <= 0xFFFFFFFF - nbytes - 4096:
        off = 0
    elif lo < 0x80000100:
        off = 0x80000100 - lo
    else:
        off = (1 << 32) - lo + 0x80000100
    v = big[off:off + nbytes]
    a = v.data_ptr()
    assert (a & 0xFFFFFFFF) >= 0x80000000 and ((a + nbytes - 1) & 0xFFFFFFFF) >= 0x80000000
    return big, v


def test_snappy_addresses_with_bit31_set(codec):
    """Round 2's intermittent fault, pinned: src and out_vals placed where the low
    32 bits of every device address have bit 31 set, so a sign-extending
    composition of a readlane'd address would fault or write elsewhere.  The
    batch mixes slot-resident blocks (k_snappy_lds), in-place spill hand-overs
    and oversize / incompressible blocks (k_snappy_rt)."""
    from bitalosdb_amd.codec import handles_tensor
    rng = random.Random(31)
    body = bytes([0 << 2]) + b"x"
    body += (bytes([(64 - 1) << 2 | 2]) + (1).to_bytes(2, "little")) * 10
    body += bytes([(59 - 1) << 2 | 2]) + (1).to_bytes(2, "little")
    body += (bytes([0 << 2 | 2]) + (7).to_bytes(2, "little")) * 324
    spill = _uvarint(1024) + body
    streams = []
    for i in range(4000):
        k = i % 5
        if k == 0:
            streams.append(spill)
        elif k == 1:
            streams.append(O.snappy_encode(rand_bytes(rng, 1024)))
        elif k == 2:
            streams.append(O.snappy_encode(compressible(rng, 2500)))
        else:
            streams.append(O.snappy_encode(compressible(rng, rng.choice([16, 700, 1024]))))
    src = bytearray()
    hs = []
    for i, st in enumerate(streams):
        rec = O.record_set(b"bit31-%d" % i, (i + 1) << 8 | 1, st, 5)
        hs.append((len(src), len(rec), 0))
        src += rec
    h = np.array(hs, dtype=O.HANDLE_DT)
    exp, evals, eoff = O.decode_batch(bytes(src), h, codec=1)
    assert (exp["status"] == 0).all()
    total = int(eoff[-1])
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        big_s, src_t = _view_with_bit31(len(src), dev)
        src_t.copy_(torch.frombuffer(bytearray(src), dtype=torch.uint8).to(dev))
        big_v, vals_t = _view_with_bit31(total + 64, dev)
        ht = handles_tensor(h, dev)
        res = codec.decode_batch(src_t, len(src), ht, len(h), 1, out_vals=vals_t)
        codec.sync()
        got = res.desc_np()
        gv = vals_t[:total].cpu().numpy()
    assert_desc_equal(got, exp)
    assert np.array_equal(res.val_off_np(), eoff)
    assert gv.tobytes() == evals[:total].tobytes()
    del big_s, big_v


def test_known_answer_tables(codec):
    """K1 + K2 tables written by the restated writer, scanned, decoded on GPU."""
    rng = random.Random(9)
    st = T.Store(1 << 20)
    s = st.flush_start()
    for i in range(1200):
        s.add(b"bithash_testkey_%d" % i, i + 1, rand_bytes(rng, 2048))
    s.compact = True
    s.finish()
    blobs = [bytes(st.files[fn]) for fn in sorted(st.files)]
    src = b"".join(blobs)
    hs, base = [], 0
    for b in blobs:
        h, _ = O.scan_region(b, mode=0)
        h = h.copy()
        h["offset"] += base
        hs.append(h)
        base += len(b)
    h = np.concatenate(hs)
    assert len(h) == 1200
    got, _, _ = codec.decode(src, h)
    exp, _, _ = O.decode_batch(src, h)
    assert_desc_equal(got, exp)
    assert list(np.unique(got["file_num"])) == [1, 2, 3]
    assert (got["trailer"] >> 8 == np.arange(1, 1201)).all()


def test_crc_fnv_primitives(codec):
    rng = random.Random(10)
    data = rand_bytes(rng, 100000)
    hs = [(0, 0, 0), (0, 9, 0), (1, 1, 0), (3, 4096, 0), (99999, 1, 0), (5, 99995, 0), (100000, 0, 0)]
    hs += [(rng.randrange(0, 90000), rng.randrange(0, 10000), 0) for _ in range(500)]
    h = np.array(hs, dtype=O.HANDLE_DT)
    from bitalosdb_amd.codec import as_device_bytes, handles_tensor
    dsrc = as_device_bytes(data, codec.device)
    dh = handles_tensor(h, codec.device)
    crc = codec.crc_batch(dsrc, dh, len(h)).cpu().numpy().view(np.uint32)
    fnv = codec.fnv_batch(dsrc, dh, len(h)).cpu().numpy().view(np.uint32)
    for i, (o, l, _) in enumerate(hs):
        assert crc[i] == O.crc_masked(data[o:o + l])
        assert fnv[i] == O.fnv32(data[o:o + l])


def test_host_path_matches_device(codec):
    rng = random.Random(12)
    specs = [(rand_bytes(rng, 32), compressible(rng, 1024), 1) for _ in range(700)]
    src, h = make_records(rng, specs, gap_max=1, codec=1)
    d1, v1, o1 = codec.decode(src, h, compressor=1)
    d2, v2, o2 = codec.decode_host(src, h, compressor=1)
    assert_desc_equal(d2, d1)
    assert np.array_equal(o1, o2) and v1.tobytes() == v2.tobytes()
    src0, h0 = make_records(rng, specs[:300], gap_max=3)
    a, _, _ = codec.decode(src0, h0)
    b, _, _ = codec.decode_host(src0, h0)
    assert_desc_equal(b, a)


def test_full_size_c2_parity(codec):
    """BASELINE configs[1] at full size: 1M 32 B/1 KiB blocks in 128 MiB tables.
    Exact parity on all 1M descriptors (oracle in threaded SSE4.2 mode, whose
    CRC equals the table-driven definition: tests/test_oracle_known_answers)."""
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    n = 1_000_000
    with torch.cuda.stream(codec.stream):
        _full_size(codec, synth, handles_tensor, n)


def _full_size(codec, synth, handles_tensor, n):
    src_t, h, meta = synth.uniform_tables(n, device=codec.device)
    assert meta["tables"] == 9 and meta["records_per_table"] == 124738
    dh = handles_tensor(h, codec.device)
    res = codec.decode_batch(src_t, src_t.numel(), dh, n)
    codec.sync()
    got = res.desc_np()
    src = src_t.cpu().numpy()
    exp, _, _ = O.decode_batch(src, h, nthreads=8)
    assert_desc_equal(got, exp)
    assert (got["status"] == 0).all()
    assert (got["trailer"] >> 8 == np.arange(1, n + 1)).all()


def test_tile_window_edges(codec):
    """Record lengths around the 144-B / 128-B window grid of the tile kernels:
    heads of 1..4 bytes, exactly 8 / 9 / 17 windows, records of 1..3 bytes
    (raw handles, RECORD_NIL but CRC still reported), arbitrary alignment."""
    rng = random.Random(77)
    specs = []
    for L in list(range(13, 40)) + [140, 143, 144, 145, 146, 147, 148, 149, 287, 288, 289, 290, 291,
                                    1076, 1151, 1152, 1153, 1154, 1155, 1156, 1157, 1280, 1281, 1296,
                                    1297, 1300, 2448, 2449, 2453, 4100, 9000]:
        for kl in (0, 7, 32):
            vl = L - 12 - 8 - kl
            if vl >= 1:
                specs.append((rand_bytes(rng, kl), rand_bytes(rng, vl), rng.randrange(1, 9)))
    rng.shuffle(specs)
    src, h = make_records(rng, specs, gap_max=3)
    extra = [(rng.randrange(0, len(src) - 8), rng.randrange(1, 4), 0) for _ in range(40)]
    extra += [(rng.randrange(0, len(src) - 300), rng.randrange(4, 300), 0) for _ in range(200)]
    extra += [(0, 1, 0), (0, 3, 0), (len(src) - 1, 1, 0), (len(src) - 3, 3, 0), (len(src) - 4, 4, 0)]
    hs = np.concatenate([h, np.array(extra, dtype=O.HANDLE_DT)])
    order = np.array(list(range(len(hs))))
    rng.shuffle(order)
    hs = hs[order]
    got, _, _ = codec.decode(src, hs)
    exp, _, _ = O.decode_batch(src, hs)
    assert_desc_equal(got, exp)


@pytest.mark.parametrize("seed", [0, 1])
def test_snappy_value_shapes(codec, seed):
    """Snappy values of every element shape the decoder distinguishes: short
    and long literals, copies with offset < length (LZ77 overlap, periods
    1..3), incompressible values, a 70 KiB value (several 64 KiB blocks)."""
    rng = random.Random(300 + seed)
    specs = []
    for i in range(1500):
        vl = rng.choice([1, 3, 15, 16, 17, 31, 64, 100, 1024, 1024, 3000, 5000, 70000 if i % 500 == 0 else 2000])
        kind = i % 4
        v = compressible(rng, vl) if kind == 0 else (b"abc" * vl)[:vl] if kind == 1 else \
            (b"a" * vl) if kind == 2 else rand_bytes(rng, vl)
        specs.append((rand_bytes(rng, 32), v, 2))
    src, h = make_records(rng, specs, gap_max=5, codec=1)
    got, gv, go = codec.decode(src, h, compressor=1)
    exp, ev, eo = O.decode_batch(src, h, codec=1)
    assert_desc_equal(got, exp)
    assert np.array_equal(go, eo) and gv.tobytes() == ev[:int(eo[-1])].tobytes()


def test_snappy_sizing_pass_and_small_cap(codec):
    """out_vals NULL = sizing pass (scan only, provisional descriptors); an
    out_vals_cap below the total gives SNAPPY_TOO_LARGE exactly to the blocks
    whose slot ends past it, the others decode normally."""
    from bitalosdb_amd.codec import as_device_bytes, handles_tensor
    rng = random.Random(41)
    specs = [(rand_bytes(rng, 16), compressible(rng, rng.choice([10, 500, 1024, 4000])), 3) for _ in range(400)]
    src, h = make_records(rng, specs, codec=1)
    exp, ev, eo = O.decode_batch(src, h, codec=1)
    with torch.cuda.stream(codec.stream):
        st = as_device_bytes(src, codec.device)
        ht = handles_tensor(h, codec.device)
        probe = codec.decode_batch(st, st.numel(), ht, len(h), 1)
        codec.sync()
        assert np.array_equal(probe.val_off_np(), eo)
        pd = probe.desc_np()
        assert (pd["status"] == 0).all()
        assert np.array_equal(pd["val_len"], exp["val_len"])       # provisional: decoded length
        cap = int(eo[250]) + 7                                      # blocks 250.. end past cap
        vals = torch.zeros(cap, dtype=torch.uint8, device=codec.device)
        res = codec.decode_batch(st, st.numel(), ht, len(h), 1, out_vals=vals)
        codec.sync()
    d = res.desc_np()
    ends = eo[1:]
    assert (d["status"][ends > cap] == O.SNAPPY_TOO_LARGE).all()
    ok = ends <= cap
    assert (d["status"][ok] == 0).all()
    for f in FIELDS:
        assert np.array_equal(d[f][ok], exp[f][ok]), f
    assert vals.cpu().numpy()[:int(eo[250])].tobytes() == ev[:int(eo[250])].tobytes()
    # host path: exact sizing and a small cap
    d2, v2, o2 = codec.decode_host(src, h, compressor=1)
    assert_desc_equal(d2, exp)
    assert v2.tobytes() == ev[:int(eo[-1])].tobytes()
    d3, v3, _ = codec.decode_host(src, h, compressor=1, out_vals_cap=cap)
    assert (d3["status"][ends > cap] == O.SNAPPY_TOO_LARGE).all() and (d3["status"][ok] == 0).all()
    assert v3[:int(eo[250])].tobytes() == ev[:int(eo[250])].tobytes()


def test_two_threads_two_streams(codec):
    """One context, two host threads, each on its own HIP stream, running
    snappy decode (per-call scan scratch) and encode (per-call scratch)
    concurrently many times: every result equals the restatement."""
    import threading
    from bitalosdb_amd.codec import as_device_bytes, handles_tensor, _u64_tensor, _u32_tensor, EncodeBuffers
    rng = random.Random(55)
    specs = [(rand_bytes(rng, 24), compressible(rng, rng.choice([100, 1024, 3000])), 2) for _ in range(2000)]
    src, h = make_records(rng, specs, codec=1)
    exp, ev, eo = O.decode_batch(src, h, codec=1)
    keys = [rand_bytes(rng, 20) for _ in range(1500)]
    vals = [compressible(rng, rng.choice([64, 700, 2048])) for _ in range(1500)]
    trs = [(i + 1) << 8 | 1 for i in range(1500)]
    eexp = O.encode_batch(keys, trs, vals, codec=1, file_nums=[1, 2, 3, 4], table_max=1 << 20)
    errors = []
    dev = codec.device
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    with torch.cuda.stream(streams[0]):
        st = as_device_bytes(src, dev)
        ht = handles_tensor(h, dev)
    with torch.cuda.stream(streams[1]):
        ko = np.zeros(len(keys) + 1, np.uint64); np.cumsum([len(k) for k in keys], out=ko[1:])
        vo = np.zeros(len(vals) + 1, np.uint64); np.cumsum([len(v) for v in vals], out=vo[1:])
        kb = as_device_bytes(b"".join(keys), dev); vb = as_device_bytes(b"".join(vals), dev)
        kot, vot, trt = _u64_tensor(ko, dev), _u64_tensor(vo, dev), _u64_tensor(trs, dev)
        fns = _u32_tensor([1, 2, 3, 4], dev)
    torch.cuda.synchronize()

    def dec_worker():
        try:
            s = streams[0]
            with torch.cuda.stream(s):
                for _ in range(8):
                    vals_t = torch.zeros(int(eo[-1]), dtype=torch.uint8, device=dev)
                    off_t = torch.empty((len(h) + 1) * 8, dtype=torch.uint8, device=dev)
                    res = codec.decode_batch(st, st.numel(), ht, len(h), 1, out_vals=vals_t, out_val_off=off_t,
                                             stream=s.cuda_stream)
                    s.synchronize()
                    assert np.array_equal(res.val_off_np(), eo)
                    assert vals_t.cpu().numpy().tobytes() == ev[:int(eo[-1])].tobytes()
                    assert np.array_equal(res.desc_np()["crc"], exp["crc"])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def enc_worker():
        try:
            s = streams[1]
            with torch.cuda.stream(s):
                for _ in range(8):
                    out = torch.zeros(int(vo[-1]) * 2 + 64 * len(keys), dtype=torch.uint8, device=dev)
                    bufs = EncodeBuffers(len(keys), 4, dev)
                    codec.encode_batch(kb, kot, trt, vb, vot, len(keys), 1, fns, 4, 0, 1 << 20, out, bufs,
                                       stream=s.cuda_stream, vals_len=int(vo[-1]))
                    s.synchronize()
                    total = int(bufs.summary.cpu().numpy()[0])
                    assert out[:total].cpu().numpy().tobytes() == eexp["out"].tobytes()
                    assert np.array_equal(bufs.crc.cpu().numpy().view(np.uint32), eexp["crc"])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    ts = [threading.Thread(target=dec_worker), threading.Thread(target=enc_worker)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("chunk,big", [(4096, False), (1 << 20, False), (4096, True)])
def test_host_pipelined_sorted(chunk, big, monkeypatch):
    """bhg_decode_batch_host, NoCompressor, handles sorted by offset: the
    chunked 3-stream pipeline (tiny chunks force many chunks, records larger
    than a chunk force the whole-batch fallback) equals the restatement,
    including zero-length / out-of-range handles and expected_crc."""
    from bitalosdb_amd.codec import BithashCodec
    monkeypatch.setenv("BHG_HOST_CHUNK_BYTES", str(chunk))
    c = BithashCodec(0)
    rng = random.Random(chunk)
    sizes = [1, 64, 1024, 3000] + ([9000] if big else [])
    specs = [(rand_bytes(rng, rng.choice([0, 7, 32, 40])), rand_bytes(rng, rng.choice(sizes)), 9)
             for _ in range(3000)]
    src, h = make_records(rng, specs, gap_max=5)
    h = h.copy()
    h["length"][100] = 0                       # ErrBhIllegalBlockLength
    h["length"][2999] += 7                     # runs past src: INCOMPLETE
    exp, _, _ = O.decode_batch(src, h)
    expected = exp["crc"].copy()
    expected[5::97] ^= 1
    got, _, _ = c.decode_host(np.frombuffer(src, np.uint8).copy(), h, expected_crc=expected)
    exp2, _, _ = O.decode_batch(src, h, expected_crc=expected)
    assert_desc_equal(got, exp2)
    assert (got["status"] == 6).sum() > 0
    c.close()


def test_host_pipelined_registered(codec):
    """Pinned (bhg_host_register) host source: the zero-copy path (the kernel
    reads the mapped source in place)."""
    rng = random.Random(77)
    specs = [(rand_bytes(rng, 32), rand_bytes(rng, 1024), 3) for _ in range(4000)]
    src, h = make_records(rng, specs)
    buf = np.frombuffer(src, np.uint8).copy()
    codec.host_register(buf)
    try:
        got, _, _ = codec.decode_host(buf, h)
    finally:
        codec.host_unregister(buf)
    exp, _, _ = O.decode_batch(src, h)
    assert_desc_equal(got, exp)


@pytest.mark.parametrize("pin_desc", [False, True])
def test_host_mapped_unsorted(codec, pin_desc):
    """Zero-copy host path: page-locked + mapped source, handles in random order
    (no pipeline needed), edge statuses, expected_crc, and a reused descriptor
    buffer that is itself mapped (written in place) or pageable (D2H)."""
    from bitalosdb_amd.codec import DESC_DT
    rng = random.Random(91)
    specs = [(rand_bytes(rng, rng.choice([0, 7, 32, 40])), rand_bytes(rng, rng.choice([1, 64, 1024, 3000])), 4)
             for _ in range(3000)]
    src, h = make_records(rng, specs, gap_max=3)
    h = h.copy()
    h["length"][10] = 0                        # ErrBhIllegalBlockLength
    h["offset"][20] = len(src) - 5             # runs past src: INCOMPLETE
    perm = np.random.default_rng(5).permutation(len(h))
    h = h[perm]
    exp0, _, _ = O.decode_batch(src, h)
    expected = exp0["crc"].copy()
    expected[3::89] ^= 1
    buf = np.frombuffer(src, np.uint8).copy()
    out = np.empty(len(h), dtype=DESC_DT)
    codec.host_register(buf)
    if pin_desc:
        codec.host_register(out)
    try:
        got, _, _ = codec.decode_host(buf, h, expected_crc=expected, out_desc=out)
    finally:
        if pin_desc:
            codec.host_unregister(out)
        codec.host_unregister(buf)
    exp, _, _ = O.decode_batch(src, h, expected_crc=expected)
    assert_desc_equal(got, exp)
    assert (got["status"] == O.CRC_MISMATCH).sum() > 0


@pytest.mark.parametrize("pin", [False, True])
def test_host_pipelined_then_unsorted(pin, monkeypatch):
    """bhg_decode_batch_host with handles in offset order up to an index and out of
    order after it: the pipeline decodes the ordered prefix (several chunks), the rest
    goes to the mapped (pinned src) or whole-batch (pageable) path; every descriptor
    equals the restatement's."""
    from bitalosdb_amd.codec import BithashCodec
    monkeypatch.setenv("BHG_HOST_CHUNK_BYTES", str(1 << 16))
    c = BithashCodec(0)
    rng = random.Random(123)
    specs = [(rand_bytes(rng, 32), rand_bytes(rng, rng.choice([64, 1024, 2000])), 5) for _ in range(3000)]
    src, h = make_records(rng, specs, gap_max=3)
    h = h.copy()
    cut = 1700
    tail = h[cut:].copy()
    h[cut:] = tail[np.random.default_rng(8).permutation(len(tail))]
    h["length"][50] = 0                        # ErrBhIllegalBlockLength inside the ordered prefix
    exp0, _, _ = O.decode_batch(src, h)
    expected = exp0["crc"].copy()
    expected[7::61] ^= 1
    buf = np.frombuffer(src, np.uint8).copy()
    if pin:
        c.host_register(buf)
    try:
        got, _, _ = c.decode_host(buf, h, expected_crc=expected)
    finally:
        if pin:
            c.host_unregister(buf)
    exp, _, _ = O.decode_batch(src, h, expected_crc=expected)
    assert_desc_equal(got, exp)
    assert (got["status"] == O.CRC_MISMATCH).sum() > 0
    c.close()


@pytest.mark.parametrize("seed", [101, 202])
def test_fuzz_corrupt_records(codec, seed):
    """Randomised corruption of valid records, both codecs, every descriptor field and
    decoded byte against the restatement: flipped bytes in the 12-B header (key / value
    sizes, fileNum), in the key, trailer and value or snappy stream; handles cut short,
    stretched past the record or past src, zero-length; expected CRCs wrong for some."""
    rng = random.Random(seed)
    n = 4000
    for cdc in (0, 1):
        specs = []
        for i in range(n):
            kl = rng.choice([0, 1, 7, 8, 20, 32, 40])
            vl = rng.choice([1, 5, 60, 200, 1024, 1500])
            v = bytes((b"snappy-" * 300)[:vl]) if rng.random() < 0.5 else rand_bytes(rng, vl)
            specs.append((rand_bytes(rng, kl), v, 1 + i % 5))
        src, h = make_records(rng, specs, gap_max=3, codec=cdc)
        buf = bytearray(src)
        h = h.copy()
        crc = np.array([O.crc_masked(bytes(buf[int(o):int(o) + int(ln)])) for o, ln in zip(h["offset"], h["length"])],
                       dtype=np.uint32)
        for i in range(n):
            o, ln = int(h["offset"][i]), int(h["length"][i])
            r = rng.random()
            if r < 0.10:      # a header byte (key size, value size or fileNum)
                buf[o + rng.randrange(12)] ^= 1 << rng.randrange(8)
            elif r < 0.25:    # a byte of the key, trailer or value / snappy stream
                if ln > 12:
                    buf[o + 12 + rng.randrange(ln - 12)] ^= 1 << rng.randrange(8)
            elif r < 0.30:    # handle cut short
                h["length"][i] = rng.randrange(ln)
            elif r < 0.33:    # handle stretched into the next record
                h["length"][i] = ln + rng.randrange(1, 64)
            elif r < 0.35:    # handle past src
                h["offset"][i] = len(buf) - rng.randrange(1, 32)
            elif r < 0.40:    # a wrong expected CRC
                crc[i] ^= 1 << rng.randrange(32)
        got, gv, go = codec.decode(bytes(buf), h, compressor=cdc, expected_crc=crc)
        exp, ev, eo = O.decode_batch(bytes(buf), h, codec=cdc, expected_crc=crc)
        assert_desc_equal(got, exp)
        if cdc == 1:
            # decoded values of the blocks Decode returns (OK, or OK but CRC-mismatched); a
            # corrupt block's slot holds no value (the reference returns snappy.ErrCorrupt)
            assert np.array_equal(go, eo)
            for i in np.nonzero((exp["status"] == 0) | (exp["status"] == 6))[0]:
                a, b = int(eo[i]), int(eo[i + 1])
                assert gv[a:b].tobytes() == ev[a:b].tobytes(), (i, int(exp["status"][i]))
        st = np.bincount(exp["status"], minlength=16)
        assert st[0] > n // 2 and (st[1:] > 0).sum() >= 3, st   # most OK, several failure kinds hit


@pytest.mark.parametrize("chunk,cap_at,big,pin", [(4096, None, False, False), (1 << 16, None, False, False),
                                                  (1 << 16, 1900, False, False), (1 << 16, 2600, False, False),
                                                  (4096, None, True, False), (1 << 16, None, False, True),
                                                  (4096, 2600, False, True)])
def test_host_snappy_pipelined(chunk, cap_at, big, pin, monkeypatch):
    """bhg_decode_batch_host, SnappyCompressor, handles sorted by offset: the
    two-stage chunked pipeline (offsets rebased per chunk, chunk k + 1's H2D under
    chunk k's D2H) equals the restatement: descriptors, value offsets and
    values, with empty values, a zero-length handle, a handle running past src,
    flipped expected CRCs, a caller cap that ends inside a later chunk (the
    same SNAPPY_TOO_LARGE verdicts as the device path, empty values past it
    included), and records larger than a chunk (the whole-batch fallback).
    pin: source, values and descriptors page-locked (bhg_host_register), so the
    values go back by the copy kernel into the mapped buffer, at every offset
    mod 16 the chunk bases fall on."""
    from bitalosdb_amd.codec import BithashCodec
    monkeypatch.setenv("BHG_HOST_CHUNK_BYTES", str(chunk))
    c = BithashCodec(0)
    rng = random.Random(chunk + (cap_at or 0) + big)
    sizes = [0, 1, 64, 1024, 3000] + ([20000] if big else [])
    specs = [(rand_bytes(rng, rng.choice([0, 7, 32])), compressible(rng, rng.choice(sizes)), 3) for _ in range(3000)]
    src, h = make_records(rng, specs, gap_max=3, codec=1)
    h = h.copy()
    h["length"][100] = 0                       # ErrBhIllegalBlockLength
    h["length"][2999] += 9                     # runs past src: INCOMPLETE
    exp0, _, _ = O.decode_batch(src, h, codec=1)
    expected = exp0["crc"].copy()
    expected[5::97] ^= 1
    exp, ev, eo = O.decode_batch(src, h, codec=1, expected_crc=expected)
    buf = np.frombuffer(src, np.uint8).copy()
    cap = None if cap_at is None else int(eo[cap_at]) + 5
    kw = {}
    pinned = []
    if pin:
        from bitalosdb_amd.codec import DESC_DT
        kw = {"out_vals": np.full(int(eo[-1]) + 100 if cap is None else cap, 0xEE, dtype=np.uint8),
              "out_desc": np.empty(len(h), dtype=DESC_DT)}
        pinned = [buf, kw["out_vals"], kw["out_desc"]]
        for a in pinned:
            c.host_register(a)
    try:
        got, gv, go = c.decode_host(buf, h, compressor=1, expected_crc=expected, out_vals_cap=cap, **kw)
    finally:
        for a in pinned[::-1]:
            c.host_unregister(a)
    if pin and cap is None:
        assert (kw["out_vals"][int(eo[-1]):] == 0xEE).all()          # nothing written past the values
    if cap_at is None:
        assert_desc_equal(got, exp)
        assert np.array_equal(go, eo) and gv.tobytes() == ev[:int(eo[-1])].tobytes()
        assert (got["status"] == O.CRC_MISMATCH).sum() > 0
    else:
        assert np.array_equal(go, eo)
        ends = eo[1:]
        live = (exp["status"] == 0) | (exp["status"] == O.CRC_MISMATCH)
        assert (got["status"][live & (ends > cap)] == O.SNAPPY_TOO_LARGE).all()
        assert ((ends > cap) & live & (exp["val_len"] == 0)).sum() > 0     # empty values past the cap
        ok = ~(live & (ends > cap))
        for f in FIELDS:
            assert np.array_equal(got[f][ok], exp[f][ok]), f
        assert gv[:int(eo[cap_at])].tobytes() == ev[:int(eo[cap_at])].tobytes()
    c.close()


@pytest.mark.parametrize("pin", [False, True])
def test_host_snappy_unsorted(codec, pin):
    """bhg_decode_batch_host, SnappyCompressor, handles in random order (the
    whole-batch path): descriptors, value offsets (in handle order) and values
    equal the restatement; with out_vals page-locked the values go back by the
    copy kernel into the mapped buffer, and nothing past them is written."""
    from bitalosdb_amd.codec import DESC_DT
    rng = random.Random(404)
    specs = [(rand_bytes(rng, rng.choice([0, 7, 32])), compressible(rng, rng.choice([0, 1, 64, 1024, 3000])), 2)
             for _ in range(2500)]
    src, h = make_records(rng, specs, gap_max=3, codec=1)
    h = h[np.random.default_rng(17).permutation(len(h))].copy()
    h["length"][7] = 0                         # ErrBhIllegalBlockLength
    exp0, _, _ = O.decode_batch(src, h, codec=1)
    expected = exp0["crc"].copy()
    expected[3::89] ^= 1
    exp, ev, eo = O.decode_batch(src, h, codec=1, expected_crc=expected)
    buf = np.frombuffer(src, np.uint8).copy()
    vals = np.full(int(eo[-1]) + 100, 0xEE, dtype=np.uint8)
    desc = np.empty(len(h), dtype=DESC_DT)
    pinned = [buf, vals, desc] if pin else []
    for a in pinned:
        codec.host_register(a)
    try:
        got, gv, go = codec.decode_host(buf, h, compressor=1, expected_crc=expected, out_desc=desc, out_vals=vals)
    finally:
        for a in pinned[::-1]:
            codec.host_unregister(a)
    assert_desc_equal(got, exp)
    assert np.array_equal(go, eo) and gv.tobytes() == ev[:int(eo[-1])].tobytes()
    assert (vals[int(eo[-1]):] == 0xEE).all()
    assert (got["status"] == O.CRC_MISMATCH).sum() > 0
