"""LAB: time the wave-cooperative discovery stages (coop_lab.hip) on the C3 batch (1M x 1 KiB dict
values, snappy) next to the product decode of the same batch; element counts checked against a CPU
parse of 2,000 streams."""
import ctypes
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bitalosdb_amd.codec import BithashCodec, handles_tensor  # noqa: E402


def count_elements(st):
    i = 0
    while st[i] >= 0x80:
        i += 1
    i += 1
    c = 0
    while i < len(st):
        tag = st[i]
        ty = tag & 3
        if ty == 0:
            x = tag >> 2
            if x < 60:
                i += 2 + x
            else:
                nb = x - 59
                i += 1 + nb + int.from_bytes(bytes(st[i + 1:i + 1 + nb]), "little") + 1
        else:
            i += (2, 3, 5)[ty - 1]
        c += 1
    return c


def main():
    n = int(os.environ.get("COOP_N", "1000000"))
    dev = torch.device("cuda:0")
    codec = BithashCodec(0)
    val_lens = torch.full((n,), 1024, dtype=torch.int64, device=dev)
    src, h, meta, enc = bench._encode_tables(codec, n, val_lens, dev, 1234, 1, "dict")
    h_t = handles_tensor(h, dev)
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcoop.so"))
    lib.coop_run.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                             ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)

    def run(mode, wg):
        r = lib.coop_run(src.data_ptr(), src.numel(), h_t.data_ptr(), n, cnt.data_ptr(), mode, wg, s.cuda_stream)
        assert r == 0, r

    def timeit(fn, reps=30):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return float(np.median(ts)), float(np.min(ts))

    srcb = src.cpu().numpy()
    rng = np.random.default_rng(5)
    idx = rng.choice(n, 2000, replace=False)
    run(0, 8)
    torch.cuda.synchronize()
    got = cnt.cpu().numpy()
    bad = 0
    for i in idx:
        off, ln = int(h["offset"][i]), int(h["length"][i])
        rec = srcb[off:off + ln]
        k = int(np.frombuffer(rec[:4].tobytes(), dtype=np.uint32)[0])
        st = list(rec[12 + k:].tobytes())
        bad += count_elements(st) != int(got[i])
    print("element counts: %d of 2000 checked blocks differ; mean elements/block %.1f" % (bad, got.mean()))
    for mode, name in ((0, "discover+chain"), (1, "staging only")):
        for wg in (4, 8):
            med, best = timeit(lambda: run(mode, wg))
            print("%-16s wg/cu %d  median %.4f ms  best %.4f" % (name, wg, med, best))
    desc = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    voff = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
    vals = torch.empty(n * 1024 + 64, dtype=torch.uint8, device=dev)
    step = lambda: codec.decode_batch(src, src.numel(), h_t, n, 1, expected_crc=enc[-1].crc, out_desc=desc,
                                      out_vals=vals, out_val_off=voff)
    med, best = timeit(step)
    print("%-16s median %.4f ms  best %.4f (whole C3 step: header pass + scan + k_snappy_lds)" % ("product", med, best))


if __name__ == "__main__":
    main()
