"""BASELINE configs[4] (C5) on one GPU, at full size: the fixed corpus of 184
bithash tables x 124,738 records (32 B key / 1 KiB value; 24.7 GB
NoCompressor, 13.3 GB SnappyCompressor) -- the corpus bench.py shards by
table over N GPUs -- decoded in ONE bhg_decode_batch per codec.  Reference:
the full-table decode Reader.readData does per record
(/root/reference/bithash/reader.go:233-272), tables opened independently
(table.go:129-179, 296-315).

What full size adds over the 1M-block tests: 23M handles in one launch,
u64 record offsets far past 4 GiB into src, and (snappy) 23.5 GB of decoded
values with out_val_off past 4 GiB.  Checks:
  * every status OK (the expected CRCs are the writer's);
  * the one-launch digest equals the sum of the per-table digests, each table
    decoded by its own launch;
  * every table bit-exact against the restatement (descriptors, and the
    decoded bytes for snappy), one table at a time on the host;
  * snappy: every decoded value equals the generator's input value.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

T, R = 184, 124_738


@pytest.fixture(scope="module")
def codec():
    from bitalosdb_amd.codec import BithashCodec
    c = BithashCodec(0)
    yield c
    c.close()
    torch.cuda.empty_cache()


def _digest(d):
    from bitalosdb_amd import shard
    return shard.block_digest(d["crc"], d["fnv1"], d["trailer"], d["status"])


def _add(a, b):
    return (((a & 0xFFFFFFFF) + (b & 0xFFFFFFFF)) & 0xFFFFFFFF) | ((((a >> 32) + (b >> 32)) & 0xFFFFFFFF) << 32)


def _check_table_vs_restatement(src_t, h, exp_crc_t, d, t, snappy, vals_t=None, voff=None):
    rows = np.arange(t * R, (t + 1) * R)
    hs = h[rows].copy()
    lo = int(hs["offset"].min())
    hi = int((hs["offset"] + hs["length"]).max())
    hs["offset"] -= np.uint64(lo)
    host = src_t[lo:hi].cpu().numpy()
    ecrc = exp_crc_t[t * R:(t + 1) * R].cpu().numpy().view(np.uint32)
    e, ev, eo = O.decode_batch(host, hs, codec=1 if snappy else 0, expected_crc=ecrc, nthreads=16)
    dd = d[rows]
    for f in O.DESC_DT.names:
        if snappy and f == "val_off":
            continue
        bad = np.nonzero(e[f] != dd[f])[0]
        assert bad.size == 0, (t, f, bad[:8])
    if snappy:
        v0, v1 = int(voff[t * R]), int(voff[(t + 1) * R])
        assert np.array_equal(voff[t * R:(t + 1) * R + 1] - voff[t * R], eo)
        assert vals_t[v0:v1].cpu().numpy().tobytes() == ev[:int(eo[-1])].tobytes()


def test_c5_none_one_launch(codec):
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src_t, h, meta = synth.table_set(list(range(T)), R, device=dev, seed=synth.SEED, first_file_num=1)
        n = len(h)
        assert n == T * R and src_t.numel() > 24_000_000_000
        h_t = handles_tensor(h, dev)
        exp_crc = codec.crc_batch(src_t, h_t, n)
        res = codec.decode_batch(src_t, src_t.numel(), h_t, n, expected_crc=exp_crc)
        codec.sync()
        d = res.desc_np()
        assert (d["status"] == 0).all()
        assert (d["file_num"] == np.repeat(np.arange(1, T + 1, dtype=np.uint32), R)).all()
        assert (d["trailer"] >> np.uint64(8) == np.arange(1, n + 1, dtype=np.uint64)).all()
        whole = _digest(d)
        # per-table launches over each table's own byte range
        tb = meta["table_bytes"]
        summed = 0
        for t in range(T):
            ht = h[t * R:(t + 1) * R].copy()
            ht["offset"] -= np.uint64(t * tb)
            r = codec.decode_batch(src_t[t * tb:(t + 1) * tb], tb, handles_tensor(ht, dev), R,
                                   expected_crc=exp_crc[t * R:(t + 1) * R])
            summed = _add(summed, _digest(r.desc_np()))
        assert summed == whole
        for t in range(T):
            _check_table_vs_restatement(src_t, h, exp_crc, d, t, snappy=False)
        del src_t, h_t, exp_crc, res
    torch.cuda.empty_cache()


def test_c5_snappy_one_launch(codec):
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    dev = codec.device
    with torch.cuda.stream(codec.stream):
        src_t, h, exp_crc, raw = synth.table_set_snappy(codec, list(range(T)), R, device=dev, seed=synth.SEED)
        n = len(h)
        assert n == T * R and raw == n * 1024 and src_t.numel() > 12_000_000_000
        h_t = handles_tensor(h, dev)
        vals_t = torch.empty(raw + 64, dtype=torch.uint8, device=dev)
        res = codec.decode_batch(src_t, src_t.numel(), h_t, n, 1, expected_crc=exp_crc, out_vals=vals_t)
        codec.sync()
        d = res.desc_np()
        assert (d["status"] == 0).all()
        voff = res.val_off_np()
        assert int(voff[-1]) == raw and (np.diff(voff) == 1024).all()
        # every decoded value is the generator's input (regenerated per table on the GPU)
        for t in range(T):
            want = synth.values_gpu("dict", R, 1024, device=dev, seed=synth.table_seed(synth.SEED, t) + 1)
            got = vals_t[t * R * 1024:(t + 1) * R * 1024].view(R, 1024)
            assert torch.equal(got, want), t
        whole = _digest(d)
        summed = 0
        tv = torch.empty(R * 1024 + 64, dtype=torch.uint8, device=dev)
        for t in range(T):
            rows = slice(t * R, (t + 1) * R)
            ht = h[rows].copy()
            b0 = int(ht["offset"][0])
            b1 = int(h["offset"][(t + 1) * R]) if t + 1 < T else src_t.numel()
            ht["offset"] -= np.uint64(b0)
            r = codec.decode_batch(src_t[b0:b1], b1 - b0, handles_tensor(ht, dev), R, 1,
                                   expected_crc=exp_crc[rows], out_vals=tv)
            summed = _add(summed, _digest(r.desc_np()))
        assert summed == whole
        for t in range(T):
            _check_table_vs_restatement(src_t, h, exp_crc, d, t, snappy=True, vals_t=vals_t, voff=voff)
        del src_t, h_t, exp_crc, vals_t, res
    torch.cuda.empty_cache()
