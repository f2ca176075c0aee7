"""Synthetic bithash workloads built directly in HBM.

The reference's tests draw keys/values from utils.FuncRandBytes' alphabet
(internal/utils/func.go:22-30) with an unseeded math/rand; here a seeded
torch generator stands in, so inputs are reproducible.  Records are laid out
exactly as Writer.add writes them (block2.go:73-105): tables of
TableMaxSize=128 MiB split after the add that crosses the limit
(bithash_writer.go:47-67), each data region followed by the 12-byte zero
terminator (writer.go:393-407).  The per-table tail (conflict / indexhash /
meta / footer) is not materialised: the decode path never reads it.
"""
import numpy as np
import torch

ALPHABET = b"1qaz2wsx3edc4rfv5tgb6yhn7ujm8ik9ol0pabcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
TABLE_MAX = 128 << 20
SEED = 0xB17A105DB


def records_per_table(rec_len, table_max=TABLE_MAX):
    return -(-table_max // rec_len)      # the add that reaches >= table_max stays in the table


def _alpha(device):
    return torch.tensor(list(ALPHABET), dtype=torch.uint8, device=device)


def _rand_alpha(g, shape, device, alpha):
    idx = torch.randint(0, len(ALPHABET), shape, generator=g, device=device, dtype=torch.int64)
    return alpha[idx]


def uniform_tables(n, key_len=32, val_len=1024, device="cuda", seed=SEED, table_max=TABLE_MAX, first_file_num=1,
                   chunk=1 << 16):
    """n records of (key_len, val_len) packed into 128 MiB tables on `device`.

    Returns (src uint8 tensor, handles numpy HANDLE_DT, meta dict)."""
    from ._lib import HANDLE_DT
    device = torch.device(device)
    klen = key_len + 8
    L = 12 + klen + val_len
    R = records_per_table(L, table_max)
    ntab = -(-n // R)
    tbytes = R * L + 12
    total = (ntab - 1) * tbytes + (n - (ntab - 1) * R) * L + 12
    src = torch.zeros(total, dtype=torch.uint8, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    alpha = _alpha(device)
    hdr = np.zeros(12, dtype=np.uint8)
    for t in range(ntab):
        r0, r1 = t * R, min(n, (t + 1) * R)
        view = src[t * tbytes:t * tbytes + (r1 - r0) * L].view(r1 - r0, L)
        hdr[:] = np.frombuffer(np.array([klen, val_len, first_file_num + t], dtype="<u4").tobytes(), dtype=np.uint8)
        view[:, :12] = torch.from_numpy(hdr.copy()).to(device)
        for c0 in range(0, r1 - r0, chunk):
            c1 = min(r1 - r0, c0 + chunk)
            m = c1 - c0
            view[c0:c1, 12:12 + key_len] = _rand_alpha(g, (m, key_len), device, alpha)
            seq = torch.arange(r0 + c0 + 1, r0 + c1 + 1, device=device, dtype=torch.int64)
            tr = (seq << 8) | 1
            view[c0:c1, 12 + key_len:12 + klen] = tr.view(torch.uint8).view(m, 8)
            view[c0:c1, 12 + klen:] = _rand_alpha(g, (m, val_len), device, alpha)
    h = np.zeros(n, dtype=HANDLE_DT)
    i = np.arange(n, dtype=np.uint64)
    h["offset"] = (i // R) * np.uint64(tbytes) + (i % R) * np.uint64(L)
    h["length"] = L
    meta = dict(n=n, rec_len=L, records_per_table=R, tables=ntab, table_bytes=tbytes, src_bytes=total,
                block_bytes=n * L)
    return src, h, meta


def table_seed(seed, t):
    """Generator seed of table t: a table's bytes depend only on (seed, t), so a
    table decodes to the same descriptors whichever rank materialises it."""
    return (int(seed) * 1_000_003 + 7919 * int(t)) & ((1 << 63) - 1)


def table_set(table_ids, records_per_table, key_len=32, val_len=1024, device="cuda", seed=SEED, first_file_num=1,
              chunk=1 << 16):
    """The tables `table_ids` of a fixed corpus (table t holds
    records t*R+1 .. (t+1)*R as seqNums, file number first_file_num + t),
    concatenated in the order given.  Returns (src uint8 tensor, handles HANDLE_DT,
    meta); table j of the list starts at j * table_bytes."""
    from ._lib import HANDLE_DT
    device = torch.device(device)
    klen = key_len + 8
    L = 12 + klen + val_len
    R = int(records_per_table)
    tbytes = R * L + 12
    src = torch.zeros(len(table_ids) * tbytes, dtype=torch.uint8, device=device)
    alpha = _alpha(device)
    hdr = np.zeros(12, dtype=np.uint8)
    for j, t in enumerate(table_ids):
        g = torch.Generator(device=device)
        g.manual_seed(table_seed(seed, t))
        view = src[j * tbytes:j * tbytes + R * L].view(R, L)
        hdr[:] = np.frombuffer(np.array([klen, val_len, first_file_num + t], dtype="<u4").tobytes(), dtype=np.uint8)
        view[:, :12] = torch.from_numpy(hdr.copy()).to(device)
        for c0 in range(0, R, chunk):
            c1 = min(R, c0 + chunk)
            m = c1 - c0
            view[c0:c1, 12:12 + key_len] = _rand_alpha(g, (m, key_len), device, alpha)
            seq = torch.arange(t * R + c0 + 1, t * R + c1 + 1, device=device, dtype=torch.int64)
            view[c0:c1, 12 + key_len:12 + klen] = ((seq << 8) | 1).view(torch.uint8).view(m, 8)
            view[c0:c1, 12 + klen:] = _rand_alpha(g, (m, val_len), device, alpha)
    n = len(table_ids) * R
    h = np.zeros(n, dtype=HANDLE_DT)
    i = np.arange(n, dtype=np.uint64)
    h["offset"] = (i // R) * np.uint64(tbytes) + (i % R) * np.uint64(L)
    h["length"] = L
    meta = dict(n=n, rec_len=L, records_per_table=R, tables=len(table_ids), table_bytes=tbytes,
                src_bytes=int(src.numel()), block_bytes=n * L, table_ids=list(table_ids))
    return src, h, meta


def table_set_snappy(codec, table_ids, records_per_table, device="cuda", seed=SEED, val_len=1024, gen="dict"):
    """The snappy variant of table_set(): table t's records_per_table values
    (values_gpu(gen), seeded per table) encoded on the GPU by
    bhg_encode_batch (SnappyCompressor, fileNum 1 + t, seqNums t*R+1..) into one
    data region + 12-byte terminator each, concatenated in the order given.
    Returns (src uint8 tensor, handles HANDLE_DT, writer CRCs int32 tensor,
    raw value bytes)."""
    from ._lib import HANDLE_DT
    from .codec import EncodeBuffers
    device = torch.device(device)
    R = int(records_per_table)
    parts, hs, crcs = [], [], []
    base, raw = 0, 0
    for t in table_ids:
        ts = table_seed(seed, t)
        keys = keys_gpu(R, device=device, seed=ts).reshape(-1).contiguous()
        key_off = torch.arange(0, (R + 1) * 32, 32, dtype=torch.int64, device=device)
        tr = (torch.arange(t * R + 1, (t + 1) * R + 1, dtype=torch.int64, device=device) << 8) | 1
        vals = values_gpu(gen, R, val_len, device=device, seed=ts + 1).reshape(-1).contiguous()
        val_off = torch.arange(0, (R + 1) * val_len, val_len, dtype=torch.int64, device=device)
        out = torch.empty(R * 64 + vals.numel() * 7 // 6 + 64, dtype=torch.uint8, device=device)
        bufs = EncodeBuffers(R, 1, device)
        fns = torch.tensor([1 + t], dtype=torch.int32, device=device)
        codec.encode_batch(keys, key_off, tr, vals, val_off, R, 1, fns, 1, 0, 1 << 30, out, bufs,
                           vals_len=vals.numel())
        codec.sync()
        size = int(bufs.table_size[0].item())
        parts.append(out[:size + 12].clone())
        parts[-1][size:] = 0                               # writeData's empty record header
        h = np.zeros(R, dtype=HANDLE_DT)
        h["offset"] = bufs.pos.cpu().numpy().view(np.uint64) + np.uint64(base)
        h["length"] = bufs.bh_len.cpu().numpy().view(np.uint32)
        hs.append(h)
        crcs.append(bufs.crc.clone())
        base += size + 12
        raw += vals.numel()
        del keys, vals, out, bufs
    if not parts:
        return (torch.zeros(0, dtype=torch.uint8, device=device), np.zeros(0, dtype=HANDLE_DT),
                torch.zeros(0, dtype=torch.int32, device=device), 0)
    return torch.cat(parts), np.concatenate(hs), torch.cat(crcs), raw


def compressible_values(rng, n_vals, val_len, dict_size=4096, fresh=0.2):
    """Values of tokens (4-64 B) drawn from a seeded dictionary, ~20 % fresh
    random bytes -- the SURVEY §8d C3 generator (numpy, host)."""
    d = rng.integers(0, 256, size=dict_size, dtype=np.uint8)
    out = np.empty((n_vals, val_len), dtype=np.uint8)
    for i in range(n_vals):
        pos = 0
        row = out[i]
        while pos < val_len:
            if rng.random() < fresh:
                ln = int(rng.integers(1, 16))
                row[pos:pos + ln] = rng.integers(0, 256, size=min(ln, val_len - pos), dtype=np.uint8)
            else:
                ln = int(rng.integers(4, 64))
                st = int(rng.integers(0, dict_size - ln))
                m = min(ln, val_len - pos)
                row[pos:pos + m] = d[st:st + m]
            pos += ln
    return out


def compressible_values_gpu(n, val_len, device="cuda", seed=SEED, words=8, word_len=16, fresh_frac=0.25):
    """[n, val_len] uint8 values on the GPU: 16-byte chunks drawn from a per-value
    set of `words` random words, a quarter of the chunks fresh random bytes --
    snappy sees intra-value repetition (about 2:1 for 1 KiB values)."""
    device = torch.device(device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    nch = -(-val_len // word_len)
    out = torch.empty((n, nch * word_len), dtype=torch.uint8, device=device)
    chunk = 1 << 15
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        w = torch.randint(0, 256, (m, words, word_len), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
        pick = torch.randint(0, words, (m, nch), generator=g, device=device)
        fresh = torch.rand((m, nch), generator=g, device=device) < fresh_frac
        rnd = torch.randint(0, 256, (m, nch, word_len), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
        sel = torch.gather(w, 1, pick.unsqueeze(-1).expand(m, nch, word_len))
        sel = torch.where(fresh.unsqueeze(-1), rnd, sel)
        out[c0:c0 + m] = sel.reshape(m, nch * word_len)
    return out[:, :val_len]


# SURVEY §8(d)'s compressible value generator, on the GPU.  Tokens of 4..64 B: a fifth of them
# fresh random bytes, the rest entries of a seeded 4 KiB dictionary (cut into ~120 entries of
# 4..64 B) picked by a Zipf law over the entries' ranks.  snappy compresses each value alone, so
# only repeats INSIDE a value pay: with the survey's Zipf(1.1) the 1 KiB values compress to 0.83
# (restated golang/snappy, 300 values), so the exponent is raised to 1.8 to meet its ratio target
# of ~0.5 (1 KiB values: 0.46-0.62 over six dictionary seeds; the bench records the mean on-disk
# size of the batch it times).
DICT_BYTES = 4096
DICT_ZIPF = 1.8
DICT_FRESH = 0.2


def dict_values_gpu(n, val_len, device="cuda", seed=SEED, dict_bytes=DICT_BYTES, zipf=DICT_ZIPF, fresh=DICT_FRESH,
                    chunk_bytes=1 << 24):
    """[n, val_len] uint8 values on the GPU from the §8(d) token generator above."""
    device = torch.device(device)
    hr = np.random.default_rng(int(seed) & ((1 << 63) - 1))
    d = hr.integers(0, 256, dict_bytes, dtype=np.uint8)
    cuts = [0]
    while cuts[-1] < dict_bytes:
        cuts.append(min(dict_bytes, cuts[-1] + int(hr.integers(4, 65))))
    K = len(cuts) - 1
    tok_start = torch.tensor(cuts[:-1], dtype=torch.int64, device=device)
    tok_len = torch.tensor(np.diff(cuts), dtype=torch.int64, device=device)
    d_t = torch.from_numpy(d).to(device)
    prob = torch.tensor(1.0 / np.arange(1, K + 1) ** zipf, dtype=torch.float32, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) & ((1 << 63) - 1))
    T = -(-val_len // 4) + 1                      # tokens that can start inside a value (>= 4 B each)
    out = torch.empty((n, val_len), dtype=torch.uint8, device=device)
    m_chunk = max(1, chunk_bytes // max(val_len, 1))
    pos = torch.arange(val_len, device=device, dtype=torch.int64)
    for c0 in range(0, n, m_chunk):
        m = min(m_chunk, n - c0)
        is_fresh = torch.rand((m, T), generator=g, device=device) < fresh
        k = torch.multinomial(prob, m * T, replacement=True, generator=g).view(m, T)
        flen = torch.randint(4, 65, (m, T), generator=g, device=device)
        ln = torch.where(is_fresh, flen, tok_len[k])
        ends = torch.cumsum(ln, 1)
        starts = ends - ln
        t = torch.searchsorted(ends, pos.unsqueeze(0).expand(m, val_len).contiguous(), right=True)
        off = pos.unsqueeze(0) - torch.gather(starts, 1, t)
        fr = torch.gather(is_fresh, 1, t)
        # (a fresh token's dictionary index is unused: clamped into the dictionary)
        dbyte = d_t[(torch.gather(tok_start[k], 1, t) + off).clamp_(max=dict_bytes - 1)]
        rnd = torch.randint(0, 256, (m, val_len), generator=g, device=device, dtype=torch.int32).to(torch.uint8)
        out[c0:c0 + m] = torch.where(fr, rnd, dbyte)
    return out


VALUE_GENS = ("dict", "chunk16")


def values_gpu(gen, n, val_len, device="cuda", seed=SEED):
    """[n, val_len] compressible values: gen "dict" (the primary C3/C4/C5-snappy
    workload) or "chunk16" (compressible_values_gpu: 16-B chunks of 8 per-value words)."""
    if gen == "dict":
        return dict_values_gpu(n, val_len, device=device, seed=seed)
    if gen == "chunk16":
        return compressible_values_gpu(n, val_len, device=device, seed=seed)
    raise ValueError("value generator %r (one of %s)" % (gen, VALUE_GENS))


def kv_pairs_gpu(n, val_lens, device="cuda", seed=SEED, key_len=32, gen="dict"):
    """n (key, trailer, value) inputs of a BithashWriter.Add batch built in HBM:
    key_len-byte alphabet keys, seqNums 1..n, value i = the first val_lens[i]
    bytes of a compressible row (values_gpu(gen)).  Returns device
    tensors (keys, key_off[n+1], trailers, vals, val_off[n+1])."""
    device = torch.device(device)
    keys = keys_gpu(n, key_len=key_len, device=device, seed=seed)
    key_off = torch.arange(0, (n + 1) * key_len, key_len, dtype=torch.int64, device=device)
    tr = (torch.arange(1, n + 1, dtype=torch.int64, device=device) << 8) | 1
    val_lens = val_lens.to(device=device, dtype=torch.int64)
    maxlen = int(val_lens.max().item()) if n else 1
    val_off = torch.zeros(n + 1, dtype=torch.int64, device=device)
    val_off[1:] = torch.cumsum(val_lens, 0)
    parts = []
    chunk = max(1, min(1 << 16, (1 << 26) // max(maxlen, 1)))
    cols = torch.arange(maxlen, device=device)
    for c0 in range(0, n, chunk):          # ragged values: row-major masked_select = concatenation
        m = min(chunk, n - c0)
        raw = values_gpu(gen, m, maxlen, device=device, seed=seed + c0)
        parts.append(torch.masked_select(raw, cols.unsqueeze(0) < val_lens[c0:c0 + m].unsqueeze(1)))
    vals = torch.cat(parts) if parts else torch.zeros(1, dtype=torch.uint8, device=device)
    return keys.reshape(-1).contiguous(), key_off, tr, vals, val_off


def keys_gpu(n, key_len=32, device="cuda", seed=SEED + 1):
    device = torch.device(device)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return _rand_alpha(g, (n, key_len), device, _alpha(device))


def full_tables(codec, n, key_len=32, val_len=1024, seed=SEED, table_max=TABLE_MAX, first_file_num=1):
    """uniform_tables() closed into complete .bht files: every table's
    Writer.writeTable tail (conflict / indexhash / meta / footer) built on the
    GPU by bhg_table_tail from the records, their FNV-1 (one GPU decode pass)
    and table-relative handles; then NewReader's footer/meta parse on the host
    (table.open_table).

    Returns (src uint8 tensor of the concatenated files, TABLE_DT records,
    handles HANDLE_DT rebased to src, meta)."""
    from . import table as BT
    from ._lib import TABLE_DT
    from .codec import handles_tensor
    device = codec.device
    src0, h0, meta = uniform_tables(n, key_len, val_len, device=device, seed=seed, table_max=table_max,
                                    first_file_num=first_file_num)
    R, L, tb = meta["records_per_table"], meta["rec_len"], meta["table_bytes"]
    ntab = meta["tables"]
    h0_t = handles_tensor(h0, device)
    res = codec.decode_batch(src0, src0.numel(), h0_t, n)
    i = torch.arange(n, device=device, dtype=torch.int64)
    bh_off = ((i % R) * L).to(torch.int32)
    table = (i // R).to(torch.int32)
    fnv = res.desc.view(-1, 40)[:, 28:32].contiguous().view(torch.int32).reshape(-1)
    counts = [min(n, (t + 1) * R) - t * R for t in range(ntab)]
    data_end = torch.tensor([c * L for c in counts], dtype=torch.int64, device=device)
    tail, toff, tlen, _ = codec.table_tail(src0, h0_t, bh_off, fnv, table, None, n, ntab, data_end)
    codec.sync()
    toff, tlen = toff.cpu().numpy(), tlen.cpu().numpy()
    parts, recs = [], []
    base = 0
    h = h0.copy()
    for t in range(ntab):
        de = counts[t] * L
        f = torch.cat([src0[t * tb:t * tb + de], tail[int(toff[t]):int(toff[t]) + int(tlen[t])]])
        rec, _ = BT.open_table(f.cpu().numpy(), base=base)
        recs.append(rec)
        r0 = t * R
        h["offset"][r0:r0 + counts[t]] = np.uint64(base) + np.arange(counts[t], dtype=np.uint64) * np.uint64(L)
        parts.append(f)
        base += int(f.numel())
    src = torch.cat(parts)
    meta = dict(meta, src_bytes=base, table_files=[int(p.numel()) for p in parts])
    return src, np.array(recs, dtype=TABLE_DT), h, meta
