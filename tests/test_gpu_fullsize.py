"""Full-size GPU parity for BASELINE configs[2] and configs[3] (the C2 batch
is in test_gpu_decode.py::test_full_size_c2_parity):

* C3: 1M snappy blocks (32 B key / 1 KiB value, the SURVEY §8d dictionary
  generator and the 16-B-chunk generator, GPU-encoded into 128 MiB tables): every descriptor and every
  decoded byte against the restatement, and every value against its input;
* C4: 1M pairs with values U[64, 4096] B (both generators) through bhg_encode_batch (snappy,
  TableMaxSize 128 MiB): records, positions, handles, tables, FNV-1, CRCs and
  statuses against the restated BithashWriter.Add sequence -- every split
  boundary, u64 positions past 1 GiB and the scan over 489+ chunks included."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd.codec import BithashCodec
    c = BithashCodec(0)
    yield c
    c.close()


def _encode(codec, n, val_lens, seed, compressor, gen="dict"):
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import EncodeBuffers
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        keys, key_off, tr, vals, val_off = synth.kv_pairs_gpu(n, val_lens, device=dev, seed=seed, gen=gen)
        out = torch.empty(int(n * 64 + vals.numel() * 7 // 6 + 64), dtype=torch.uint8, device=dev)
        maxt = 256
        fns = torch.arange(1, maxt + 1, dtype=torch.int32, device=dev)
        bufs = EncodeBuffers(n, maxt, dev)
        codec.encode_batch(keys, key_off, tr, vals, val_off, n, compressor, fns, maxt, 0, 128 << 20, out, bufs,
                           vals_len=int(vals.numel()))
        codec.sync()
    return (keys, key_off, tr, vals, val_off), out, bufs


@pytest.mark.parametrize("gen", ["dict", "chunk16"])
def test_full_size_c3_parity(codec, gen):
    from bitalosdb_amd.codec import handles_tensor
    n = 1_000_000
    val_lens = torch.full((n,), 1024, dtype=torch.int64)
    (keys, _, _, vals, _), out, bufs = _encode(codec, n, val_lens, 0xC3, 1, gen)
    total = int(bufs.summary[0].item())
    assert int(bufs.summary[2].item()) == 0 and total > 1 << 29
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = bufs.pos.cpu().numpy().view(np.uint64)
    h["length"] = bufs.bh_len.cpu().numpy().view(np.uint32)
    exp_crc = bufs.crc.cpu().numpy().view(np.uint32)
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src = out[:total]
        ht = handles_tensor(h, dev)
        ec = bufs.crc
        probe = codec.decode_batch(src, total, ht, n, 1, expected_crc=ec)
        codec.sync()
        tot = int(probe.val_off_np()[-1])
        assert tot == n * 1024
        dv = torch.empty(tot, dtype=torch.uint8, device=dev)
        res = codec.decode_batch(src, total, ht, n, 1, expected_crc=ec, out_vals=dv)
        codec.sync()
    got = res.desc_np()
    assert (got["status"] == 0).all()
    host = src.cpu().numpy()
    exp, ev, eo = O.decode_batch(host, h, codec=1, expected_crc=exp_crc, nthreads=16)
    for f in exp.dtype.names:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, (f, bad[:8])
    gv = dv.cpu().numpy()
    assert np.array_equal(res.val_off_np(), eo)
    assert gv.tobytes() == ev[:tot].tobytes()
    assert gv.tobytes() == vals.cpu().numpy().tobytes()          # round trip to the encoder's input


@pytest.mark.parametrize("gen", ["dict", "chunk16"])
def test_full_size_c4_parity(codec, gen):
    n = 1_000_000
    g = torch.Generator().manual_seed(0xC4)
    val_lens = torch.randint(64, 4097, (n,), generator=g, dtype=torch.int64)
    (keys, key_off, tr, vals, val_off), out, bufs = _encode(codec, n, val_lens, 0xC4, 1, gen)
    nt = int(bufs.summary[1].item())
    assert nt >= 8
    kb = keys.cpu().numpy().tobytes()
    vb = vals.cpu().numpy().tobytes()
    vo = val_off.cpu().numpy()
    ks = [kb[32 * i:32 * i + 32] for i in range(n)]
    vs = [vb[vo[i]:vo[i + 1]] for i in range(n)]
    exp = O.encode_batch(ks, tr.cpu().numpy(), vs, codec=1, file_nums=list(range(1, 257)), table_max=128 << 20)
    assert exp["ntables"] == nt
    u32 = lambda t: t.cpu().numpy().view(np.uint32)
    got = dict(pos=bufs.pos.cpu().numpy().view(np.uint64), bh_off=u32(bufs.bh_off), bh_len=u32(bufs.bh_len),
               table=u32(bufs.table), fnv=u32(bufs.fnv1), crc=u32(bufs.crc), status=u32(bufs.status))
    for f, v in got.items():
        bad = np.nonzero(v != exp[f])[0]
        assert bad.size == 0, (f, bad[:8])
    assert np.array_equal(u32(bufs.table_start)[:nt], exp["table_start"])
    total = int(bufs.summary[0].item())
    assert total == len(exp["out"]) and total > 1 << 29
    assert out[:total].cpu().numpy().tobytes() == exp["out"].tobytes()


@pytest.mark.parametrize("compressor", [0, 1])
def test_full_size_mixed_decode_parity(codec, compressor):
    """The C4-shaped tables decoded (bench.py --config mixdec): 1M pairs with values U[64, 4096] B
    of the dict generator, GPU-encoded with either codec into 128 MiB tables, then the whole batch
    decoded with the writer's CRCs.  Every descriptor and every decoded byte against the C
    restatement, and every value against the encoder's input -- for snappy that runs both LDS
    tiers (76 % of the blocks decode to more than 1 KiB) and leaves k_snappy_rt nothing."""
    from bitalosdb_amd.codec import handles_tensor
    n = 1_000_000
    g = torch.Generator().manual_seed(0xD4)
    val_lens = torch.randint(64, 4097, (n,), generator=g, dtype=torch.int64)
    (keys, _, _, vals, val_off), out, bufs = _encode(codec, n, val_lens, 0xD4, compressor)
    total = int(bufs.summary[0].item())
    assert int(bufs.summary[2].item()) == 0 and total > 1 << 29
    h = np.zeros(n, dtype=O.HANDLE_DT)
    h["offset"] = bufs.pos.cpu().numpy().view(np.uint64)
    h["length"] = bufs.bh_len.cpu().numpy().view(np.uint32)
    exp_crc = bufs.crc.cpu().numpy().view(np.uint32)
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src = out[:total]
        ht = handles_tensor(h, dev)
        ec = bufs.crc
        if compressor == 1:
            probe = codec.decode_batch(src, total, ht, n, 1, expected_crc=ec)
            codec.sync()
            tot = int(probe.val_off_np()[-1])
            assert tot == int(val_off[-1].item())
            dv = torch.empty(tot, dtype=torch.uint8, device=dev)
            res = codec.decode_batch(src, total, ht, n, 1, expected_crc=ec, out_vals=dv)
        else:
            res = codec.decode_batch(src, total, ht, n, 0, expected_crc=ec)
        codec.sync()
    got = res.desc_np()
    assert (got["status"] == 0).all()
    host = src.cpu().numpy()
    exp, ev, eo = O.decode_batch(host, h, codec=compressor, expected_crc=exp_crc, nthreads=16)
    for f in exp.dtype.names:
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, (f, bad[:8])
    vin = vals.cpu().numpy()
    if compressor == 1:
        gv = dv.cpu().numpy()
        assert np.array_equal(res.val_off_np(), eo)
        assert gv.tobytes() == ev[:tot].tobytes()
        assert gv.tobytes() == vin.tobytes()                       # round trip to the encoder's input
    else:
        # NoCompressor values are views into src: gather them and compare with the input
        vo = got["val_off"].astype(np.int64) + h["offset"].astype(np.int64)
        vl = got["val_len"].astype(np.int64)
        assert np.array_equal(vl, np.diff(val_off.cpu().numpy()))
        assert np.concatenate([host[a:a + b] for a, b in zip(vo.tolist(), vl.tolist())]).tobytes() == vin.tobytes()
