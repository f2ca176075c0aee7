"""End-to-end host decode (bhg_decode_batch_host, NoCompressor) on the C2 batch
under each pinning combination; prints GiB/s of table bytes.  Lab only.
usage: python scripts/lab/e2e_lab.py  (BHG_HOST_ZEROCOPY=0 forces the staged paths)"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from bitalosdb_amd import synth  # noqa: E402
from bitalosdb_amd.codec import DESC_DT, BithashCodec  # noqa: E402


def main():
    c = BithashCodec(0)
    src_t, h, meta = synth.uniform_tables(1_000_000, device="cuda")
    src = src_t.cpu().numpy()
    n, L = len(h), meta["rec_len"]
    h = np.ascontiguousarray(h)
    desc = np.empty(n, dtype=DESC_DT)
    ref, _, _ = c.decode_host(src, h, out_desc=desc.copy())
    for name, pins in [("pageable", ()), ("src", ("src",)), ("src+desc", ("src", "desc")),
                       ("src+desc+handles", ("src", "desc", "h"))]:
        bufs = {"src": src, "desc": desc, "h": h}
        for k in pins:
            c.host_register(bufs[k])
        c.decode_host(src, h, out_desc=desc)
        reps, t = 5, time.perf_counter()
        for _ in range(reps):
            c.decode_host(src, h, out_desc=desc)
        s = (time.perf_counter() - t) / reps
        ok = np.array_equal(desc["crc"], ref["crc"]) and np.array_equal(desc["status"], ref["status"])
        for k in pins:
            c.host_unregister(bufs[k])
        print("%-18s %7.2f GiB/s  %.2f ms  zero_copy=%s  %s" % (name, n * L / s / 2 ** 30, s * 1e3,
              os.environ.get("BHG_HOST_ZEROCOPY", "1"), "ok" if ok else "MISMATCH"), flush=True)
    c.close()


if __name__ == "__main__":
    main()
