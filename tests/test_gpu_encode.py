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


@pytest.mark.parametrize("compressor", [0, 1])
def test_encode_long_keys_big_values(codec, compressor):
    """User keys of 37..64 B (past the pack kernel's 36-B register prefix) with
    values of several KiB: the lane writes the prefix, the wave copies the value
    (phase B) -- byte-exact with the restated writer at every alignment."""
    rng = random.Random(40 + compressor)
    n = 400
    keys = [rb(rng, rng.choice([37, 40, 41, 48, 63, 64])) for _ in range(n)]
    vals = [compressible(rng, rng.choice([1, 5, 3000, 4096, 9001, 20000])) if i % 2 else
            rb(rng, rng.choice([2, 700, 5000, 16384])) for i in range(n)]
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, compressor=compressor, file_nums=list(range(1, 20)), table_max=1 << 20)
    exp = O.encode_batch(keys, tr, vals, codec=compressor, file_nums=list(range(1, 20)), table_max=1 << 20)
    check(got, exp)


@pytest.mark.parametrize("compressor", [0, 1])
def test_encode_long_batch(codec, compressor):
    """A batch of long values (mean past 8 KiB): records longer than 4 KiB are left by k_enc_pack
    to k_enc_lcopy (16-KiB output segments, one wave each) and their CRCs to the long-record pass over
    the packed output.  Records of 4-5 KiB (one segment), values of several segments, user keys past
    36 B, a long key with a 1-byte value (the whole value in the prefix dwords), a key too large and
    short records in between; table splits at 1 MiB -- byte-exact with the restated writer, then
    decoded back."""
    rng = random.Random(70 + compressor)
    g = np.random.default_rng(70 + compressor)
    n = 120
    keys, vals = [], []
    for i in range(n):
        kind = i % 6
        klen = rng.choice([0, 1, 16, 32, 37, 64, 200])
        if kind == 0:
            v = rng.choice([4050, 4096, 4200, 5000, 16384 - 60, 16384 + 17])
        elif kind == 1:
            v = rng.choice([40000, 65536, 70001, 200000])
        elif kind == 2:
            v = rng.choice([1, 7, 300, 3000])
        elif kind == 3:
            v = rng.choice([100000, 333333])
        elif kind == 4:
            v = 1
            klen = 5000  # L > 4 KiB from the key alone
        else:
            v = rng.choice([8192, 12000, 50000])
        keys.append(rb(rng, klen))
        vals.append(compressible(rng, v) if i % 2 else g.integers(0, 256, v, dtype=np.uint8).tobytes())
    keys[11] = b"k" * ((33 << 10) - 7)  # KEY_TOO_LARGE
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, compressor=compressor, file_nums=list(range(1, 40)), table_max=1 << 20)
    exp = O.encode_batch(keys, tr, vals, codec=compressor, file_nums=list(range(1, 40)), table_max=1 << 20)
    assert sum(len(v) for v in vals) > 8192 * n  # a long batch (bhg_encode_batch's rule)
    check(got, exp)
    assert got["status"][11] == O.KEY_TOO_LARGE
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = got["pos"]
    h["length"] = got["bh_len"]
    ok = np.nonzero(got["status"] == 0)[0]
    desc, dv, doff = codec.decode(got["out"], h[ok], compressor=compressor)
    assert (desc["status"] == 0).all()
    assert (desc["crc"] == got["crc"][ok]).all()
    for j, i in enumerate(ok):
        if compressor:
            assert dv[int(doff[j]):int(doff[j + 1])].tobytes() == vals[i]


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


@pytest.mark.parametrize("seed", [21, 22])
def test_encode_snappy_block_path(codec, seed):
    """Values past 4 KiB: every 64-KiB block is a work item of its own (k_snappy_enc_blocks),
    then each value's uvarint header and block outputs are joined (k_snappy_bcopy).  Sizes at
    the block edges (a last block of 16 bytes is emitLiteral'd, of 17 encodeBlock'd), 1-2 MiB
    values, incompressible / compressible / periodic / zero data, small values interleaved --
    byte-exact with the restated encoder, and decoded back on the GPU."""
    rng = random.Random(seed)
    g = np.random.default_rng(seed)
    sizes = [4097, 65535, 65536, 65537, 65536 + 16, 65536 + 17, 131072, 131072 + 3, 196608 - 1,
             (1 << 20) + 5, (2 << 20) - 77, 100, 3000, 0, 17]
    sizes += [rng.randrange(4097, 300000) for _ in range(40)]
    rng.shuffle(sizes)
    n = len(sizes)
    keys = [rb(rng, 32) for _ in range(n)]
    vals = []
    for i, sz in enumerate(sizes):
        kind = i % 4
        if kind == 0:
            vals.append(compressible(rng, sz))
        elif kind == 1:
            vals.append(g.integers(0, 256, sz, dtype=np.uint8).tobytes())
        elif kind == 2:
            vals.append((b"0123456789abcdefXYZ" * (sz // 19 + 1))[:sz])
        else:
            vals.append(bytes(sz))
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, compressor=1, file_nums=list(range(1, 50)), table_max=4 << 20)
    exp = O.encode_batch(keys, tr, vals, codec=1, file_nums=list(range(1, 50)), table_max=4 << 20)
    check(got, exp)
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = got["pos"]
    h["length"] = got["bh_len"]
    desc, dv, doff = codec.decode(got["out"], h, compressor=1)
    assert (desc["status"] == 0).all()
    for i in range(n):
        assert dv[int(doff[i]):int(doff[i + 1])].tobytes() == vals[i]


@pytest.mark.parametrize("sizes", [[0], [3000], [100, 3000], [2048, 2049], [4096] * 7, [1500] * 65,
                                   [5000, 17, 2048, 4097, 0, 64]])
def test_encode_snappy_tiny_batches(codec, sizes):
    """The encoder's class lists and work queue at batch sizes far below the grid:
    one value, empty small or large list, the 2 KiB / 4 KiB class edges, a class
    list longer than one wave's first take (the queue hands out the rest) --
    byte-exact with the restatement."""
    rng = random.Random(len(sizes) * 7 + sizes[0])
    n = len(sizes)
    keys = [rb(rng, 24) for _ in range(n)]
    vals = [compressible(rng, sz) if i % 2 == 0 else rb(rng, sz) for i, sz in enumerate(sizes)]
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    got = codec.encode(keys, tr, vals, compressor=1, file_nums=[5, 6], table_max=1 << 20)
    exp = O.encode_batch(keys, tr, vals, codec=1, file_nums=[5, 6], table_max=1 << 20)
    check(got, exp)


def test_encode_out_cap_too_small(codec):
    """Records that end past out_cap are not written: status NO_SPACE, pos
    UINT64_MAX, counted in summary[2]; summary[0] still reports the bytes the
    whole batch needs; everything before the cut equals the restatement."""
    rng = random.Random(21)
    n = 1000
    keys = [rb(rng, 16) for _ in range(n)]
    vals = [rb(rng, rng.choice([10, 300, 1000])) for _ in range(n)]
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    exp = O.encode_batch(keys, tr, vals, file_nums=[1, 2], table_max=64 << 20)
    cap = int(exp["pos"][600]) + 5
    got = codec.encode(keys, tr, vals, file_nums=[1, 2], table_max=64 << 20, out_cap=cap)
    fits = exp["pos"] + exp["bh_len"] <= cap
    assert fits[:600].all() and not fits[600:].any()
    assert (got["status"][fits] == 0).all() and (got["status"][~fits] == O.NO_SPACE).all()
    assert (got["pos"][~fits] == np.iinfo(np.uint64).max).all()
    assert int(got["summary"][2]) == int((~fits).sum())
    assert int(got["summary"][0]) == len(exp["out"])
    for f in ("fnv", "bh_off", "bh_len", "crc", "pos"):
        assert np.array_equal(got[f][fits], exp[f][fits]), f
    assert got["out"][:int(exp["pos"][600])].tobytes() == exp["out"][:int(exp["pos"][600])].tobytes()


def test_encode_snappy_vals_len_too_small(codec):
    """A vals_len below val_off[n] cannot overflow the snappy scratch: the
    values past the bound get NO_SPACE, the rest encode exactly."""
    import torch
    from bitalosdb_amd.codec import EncodeBuffers, as_device_bytes, _u32_tensor, _u64_tensor
    rng = random.Random(22)
    n = 300
    keys = [rb(rng, 8) for _ in range(n)]
    vals = [compressible(rng, 1000) for _ in range(n)]
    tr = [((i + 1) << 8) | 1 for i in range(n)]
    exp = O.encode_batch(keys, tr, vals, codec=1, file_nums=[3], table_max=64 << 20)
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        ko = np.zeros(n + 1, np.uint64); np.cumsum([len(k) for k in keys], out=ko[1:])
        vo = np.zeros(n + 1, np.uint64); np.cumsum([len(v) for v in vals], out=vo[1:])
        out = torch.zeros(len(exp["out"]) + 64, dtype=torch.uint8, device=dev)
        bufs = EncodeBuffers(n, 1, dev)
        codec.encode_batch(as_device_bytes(b"".join(keys), dev), _u64_tensor(ko, dev), _u64_tensor(tr, dev),
                           as_device_bytes(b"".join(vals), dev), _u64_tensor(vo, dev), n, 1, _u32_tensor([3], dev),
                           1, 0, 64 << 20, out, bufs, vals_len=int(vo[-1]) // 2)
        codec.sync()
    st = bufs.status.cpu().numpy().view(np.uint32)
    assert (st[:100] == 0).all() and (st[-50:] == O.NO_SPACE).all()
    ok = st == 0
    first_bad = int(np.argmin(ok))
    assert ok[:first_bad].all() and not ok[first_bad:].any()
    crc = bufs.crc.cpu().numpy().view(np.uint32)
    assert np.array_equal(crc[:first_bad], exp["crc"][:first_bad])


@pytest.mark.parametrize("codec_kind", [0, 1])
def test_encode_ikey_compaction_repack(codec, codec_kind):
    """Compaction re-pack (bitree/bithash.go:217-239): source tables scanned
    and decoded on the GPU (stored value bytes, source fileNum), a liveness
    mask, then bhg_encode_ikey_batch == the restated Writer.AddIkey sequence
    (one destination table, source fileNums in the headers, given khash)."""
    from oracle import table as T
    from bitalosdb_amd.codec import as_device_bytes, _u64_tensor
    rng = random.Random(30 + codec_kind)
    st = T.Store(1 << 20, compressor=codec_kind)
    s = st.flush_start()
    for i in range(1500):
        s.add(b"compact_key_%05d" % i, i + 1, compressible(rng, rng.choice([100, 900, 2000])))
    s.compact = True
    s.finish()
    blobs = [bytes(st.files[fn]) for fn in sorted(st.files)]
    src = b"".join(blobs)
    toff = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    h_t, first, _ = codec.scan_tables(as_device_bytes(src, codec.device), _u64_tensor(toff, codec.device), mode=0)
    codec.sync()
    h = h_t.cpu().numpy().view(O.HANDLE_DT).reshape(-1)
    assert len(h) == 1500
    desc, _, _ = codec.decode(src, h)          # stored bytes: NoCompressor view even for snappy tables
    assert (desc["status"] == 0).all()
    sb = np.frombuffer(src, np.uint8)
    keys, vals, trs, fns = [], [], [], []
    for i in range(len(h)):
        o = int(h["offset"][i])
        keys.append(sb[o + 12:o + 12 + int(desc["key_len"][i])].tobytes())
        vals.append(sb[o + int(desc["val_off"][i]):o + int(desc["val_off"][i]) + int(desc["val_len"][i])].tobytes())
        trs.append(int(desc["trailer"][i]))
        fns.append(int(desc["file_num"][i]))
    live = np.array([rng.random() < 0.7 for _ in keys], dtype=np.uint8)
    init = 4096
    got = codec.encode_ikey(keys, trs, vals, fns, live=live, khash=desc["fnv1"], init_size=init)
    w = T.Writer(99, 1 << 40, compressor=codec_kind)
    w.current_offset = w.size = init
    w.file += bytes(init)
    exp_bh = []
    for i in range(len(keys)):
        if live[i]:
            exp_bh.append(w.add_ikey(keys[i], trs[i], vals[i], int(desc["fnv1"][i]), fns[i]))
    assert (got["status"][live == 0] == O.SKIPPED).all() and (got["status"][live == 1] == 0).all()
    assert int(got["summary"][2]) == 0
    gbh = list(zip(got["bh_off"][live == 1].tolist(), got["bh_len"][live == 1].tolist()))
    assert gbh == exp_bh
    assert got["out"].tobytes() == bytes(w.file[init:w.current_offset])
    assert (got["table"] == 0).all() and np.array_equal(got["fnv"], desc["fnv1"])
    # the re-packed records decode with their source fileNums and CRCs
    hh = np.zeros(int(live.sum()), dtype=O.HANDLE_DT)
    hh["offset"] = got["pos"][live == 1]
    hh["length"] = got["bh_len"][live == 1]
    d2, _, _ = codec.decode(got["out"], hh)
    assert (d2["status"] == 0).all()
    assert np.array_equal(d2["file_num"], np.array(fns, np.uint32)[live == 1])
    assert np.array_equal(d2["crc"], got["crc"][live == 1])
