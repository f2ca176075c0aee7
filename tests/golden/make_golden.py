"""Generates the golden fixtures in tests/golden/ ("Golden fixtures to commit").

The reference ships no binary golden data for this path (no Go toolchain here
to run it either), so the fixtures are produced by the CPU restatement
(oracle/) after it has been pinned by the reference's own asserted tests
(tests/test_oracle_known_answers.py: K1-K4 sizes/counts/collisions) and, for
snappy, cross-checked against an independent implementation (pyarrow's C++
snappy: every stream we store must decompress to its raw bytes there, and
pyarrow-compressed streams must decode identically in the restatement).

Run from the repo root:  python tests/golden/make_golden.py
Outputs (all small; data only, no reference source):
  k2.bht                      K2 table file (100 keys + 12 FNV-1 collision keys, 2 KiB values)
  k2_scan.npy                 TableIterator handles over k2.bht (bho_scan_region mode 0)
  k1_manifest.json            K1 split sizes, sha256 of the three table files, rebuild offset
  rec_none.bin/.npz           256 C2-shaped records + edge records, handles, expected descriptors
  rec_snappy.bin/.npz         the same with snappy values, + decoded values and offsets
  snappy_edges.npz            raw <-> golang/snappy v0.0.4 encodings at the format's boundaries
                              (+ pyarrow/C++ snappy encodings of the same raw bytes)
  encode.npz                  encode_batch inputs/outputs for 64 records, NoCompressor and snappy,
                              64 KiB table_max (splits, positions, CRCs, FNV-1)
"""
import hashlib
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402
from oracle import table as T  # noqa: E402

ALPHA = b"1qaz2wsx3edc4rfv5tgb6yhn7ujm8ik9ol0pabcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
K2_KEYS = [b"l41khazkyppk4sBj7BhdQxpfMGF2bKH9", b"zZah6yQoo4ElihZfMVwragoejhuHaocb",
           b"yBZrxusPKQdo1rKauI6rtOfs5tjbySx6", b"l0asXWDhSamz5qncres4xJSsaUK2Jhtz",
           b"wmoVNuhDBJOblKUS8wiSXNNmTjvcxrc7", b"H7fyvszFYYZqM0NnmfmjRjPoslT1V4nu",
           b"NplhsekvJnBm7gJHge5qsgJcqb68GCJu", b"1gncjKqtxufeiqwGfdpVrJubtEabsOyl",
           b"AqLMVOYwsi67FbCqHr2aivuoyKZH1eiW", b"zSpkzpkG9xbvR4IgqNcfF24pdg351Any",
           b"tk0F3dTRD8BGqaPAekliaDiZvRojoTk1", b"dzurIotnFYUPynzW6V9DzyfdzTzs2chx"]


def alpha_bytes(rng, n):
    return bytes(rng.choice(ALPHA) for _ in range(n))


def k2_table():
    rng = random.Random(2)
    st = T.Store(64 << 20)
    kv = [(b"bithash_testkey_%d" % i, alpha_bytes(rng, 2048)) for i in range(100)]
    ckv = [(k, alpha_bytes(rng, 2048)) for k in K2_KEYS]
    s = st.flush_start()
    seq = 1
    for i, (k, v) in enumerate(kv):
        s.add(k, seq, v)
        seq += 1
        if i == 50:
            for ck, cv in ckv:
                s.add(ck, seq, cv)
                seq += 1
    s.compact = True
    s.finish()
    return bytes(st.files[1])


def k1_manifest():
    rng = random.Random(3)
    st = T.Store(1 << 20)
    s = st.flush_start()
    for i in range(1200):
        s.add(b"bithash_testkey_%d" % i, i + 1, alpha_bytes(rng, 2048))
    s.finish()
    w = st.mutable[-1]
    files = {fn: bytes(st.files[fn]) for fn in (1, 2)}
    files[3] = bytes(w.file)
    sizes = [T.open_table(files[fn])["data_bh"][1] - 12 for fn in (1, 2)]
    return {"seed": 3, "records": 1200, "value_len": 2048, "table_max": 1 << 20,
            "closed_data_sizes": sizes, "mutable_current_offset": w.current_offset,
            "sha256": {str(fn): hashlib.sha256(b).hexdigest() for fn, b in files.items()},
            "file_len": {str(fn): len(b) for fn, b in files.items()}}


def records(rng, codec):
    """256 C2-shaped records plus edge records (mixed sizes, ikeySize < 8,
    nil rules, zero/over-long handles), at arbitrary byte offsets."""
    specs = [(alpha_bytes(rng, 32), alpha_bytes(rng, 1024), 1 + i // 100) for i in range(256)]
    for kl in (0, 1, 7, 8, 9, 35, 36, 37, 48, 255):
        specs.append((alpha_bytes(rng, kl), alpha_bytes(rng, rng.randrange(0, 3000)), 77))
    buf = bytearray()
    hs = []
    for i, (k, v, fn) in enumerate(specs):
        buf += bytes(rng.randrange(256) for _ in range(rng.randrange(4)))
        val = O.snappy_encode(v) if codec else v
        rec = O.record_set(k, (i + 1) << 8 | 1, val, fn)
        hs.append((len(buf), len(rec), 0))
        buf += rec
    # readRecord nil rules / handle errors (block2.go:57-66, reader.go:234-258)
    buf += b"\x00" * 12                                 # ikeySize 0 -> nil
    hs.append((len(buf) - 12, 12, 0))
    hs.append((0, 0, 0))                                # zero length
    hs.append((0, 11, 0))                               # shorter than a header
    hs.append((len(buf) - 5, 100, 0))                   # runs past the end -> incomplete
    return bytes(buf), np.array(hs, dtype=O.HANDLE_DT)


def snappy_edges():
    import pyarrow as pa
    rng = random.Random(7)
    cases = []
    raw = []
    for n in (0, 1, 2, 15, 16, 17, 59, 60, 61, 62, 255, 256, 257, 65536, 65537):
        raw.append(bytes(rng.randrange(256) for _ in range(n)))
    # copies: lengths 4/11/12/64/65/67/68, offsets 2047/2048/65535, overlapping runs
    for ln in (4, 11, 12, 64, 65, 67, 68, 200):
        for offd in (1, 3, 8, 2047, 2048, 4096):
            p = bytes(rng.randrange(256) for _ in range(offd))
            raw.append(p + (p * (ln // max(1, offd) + 2))[:ln] + bytes(rng.randrange(256) for _ in range(5)))
    raw.append(b"a" * 100000)
    raw.append(alpha_bytes(rng, 5000))
    raw.append(bytes(rng.randrange(4) for _ in range(9000)))
    codec = pa.Codec("snappy")
    for r in raw:
        enc = O.snappy_encode(r)
        assert codec.decompress(enc, decompressed_size=len(r)).to_pybytes() == r
        assert O.snappy_decode(enc) == r
        pae = codec.compress(r).to_pybytes()
        assert O.snappy_decode(pae) == r
        cases.append((r, enc, pae))
    out = {}
    for j, name in enumerate(("raw", "go", "pyarrow")):
        out[name] = np.frombuffer(b"".join(c[j] for c in cases) or b"\0", dtype=np.uint8)
        out[name + "_off"] = np.concatenate([[0], np.cumsum([len(c[j]) for c in cases])]).astype(np.uint64)
    return out


def encode_case(rng):
    keys = [alpha_bytes(rng, rng.randrange(1, 60)) for _ in range(64)]
    vals = [alpha_bytes(rng, rng.randrange(0, 5000)) for _ in range(64)]
    trs = np.array([(i + 1) << 8 | 1 for i in range(64)], dtype=np.uint64)
    out = {}
    for codec in (0, 1):
        e = O.encode_batch(keys, trs, vals, codec=codec, file_nums=[11, 12, 13, 14], table_max=64 << 10)
        out.update({"c%d_%s" % (codec, k): np.asarray(v) for k, v in e.items() if k != "ntables"})
        out["c%d_ntables" % codec] = np.array([e["ntables"]])
    kb = np.frombuffer(b"".join(keys), dtype=np.uint8)
    vb = np.frombuffer(b"".join(vals), dtype=np.uint8)
    koff = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    voff = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.uint64)
    return dict(keys=kb, key_off=koff, vals=vb, val_off=voff, trailers=trs, **out)


def main():
    O.build()
    k2 = k2_table()
    open(os.path.join(HERE, "k2.bht"), "wb").write(k2)
    h, end = O.scan_region(k2, mode=0)
    np.save(os.path.join(HERE, "k2_scan.npy"), h)
    json.dump(k1_manifest(), open(os.path.join(HERE, "k1_manifest.json"), "w"), indent=1)
    for codec, name in ((0, "rec_none"), (1, "rec_snappy")):
        rng = random.Random(100 + codec)
        src, hs = records(rng, codec)
        desc, vals, voff = O.decode_batch(src, hs, codec=codec)
        open(os.path.join(HERE, name + ".bin"), "wb").write(src)
        extra = {}
        if codec:
            extra = dict(vals=np.asarray(vals)[:int(voff[-1])], val_off=np.asarray(voff))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), handles=hs, desc=desc, **extra)
    np.savez_compressed(os.path.join(HERE, "snappy_edges.npz"), **snappy_edges())
    np.savez_compressed(os.path.join(HERE, "encode.npz"), **encode_case(random.Random(55)))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
