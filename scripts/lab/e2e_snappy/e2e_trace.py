"""Lab: the snappy end-to-end host path (bhg_decode_batch_host, pinned buffers) on the c3
workload (1M dict-value blocks), timed per call; run under rocprofv3 --kernel-trace
--memory-copy-trace to see how the chunk copies and kernels overlap.  argv[1] == "shuffle":
handles in random order (the whole-batch path); "pageable": no host buffer page-locked."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from bitalosdb_amd.codec import BithashCodec, DESC_DT  # noqa: E402

dev = torch.device("cuda:0")
codec = BithashCodec(0)
n = 1 << 20
val_lens = torch.full((n,), 1024, dtype=torch.int64, device=dev)
src, h, meta, enc = bench._encode_tables(codec, n, val_lens, dev, bench.synth_seed(0), 1, "dict")
ecrc = enc[-1].crc.cpu().numpy().view(np.uint32).copy()
if "shuffle" in sys.argv[1:]:
    perm = np.random.default_rng(3).permutation(n)
    h, ecrc = h[perm].copy(), ecrc[perm].copy()
host_src = src.cpu().numpy()
desc = np.empty(n, dtype=DESC_DT)
vals = np.empty(n * 1024 + 64, dtype=np.uint8)
bufs = () if "pageable" in sys.argv[1:] else (host_src, desc, vals, h, ecrc)
for b in bufs:
    codec.host_register(b)
disk = float(h["length"].astype(np.float64).sum())
for i in range(4):
    t = time.perf_counter()
    codec.decode_host(host_src, h, compressor=1, expected_crc=ecrc, out_desc=desc, out_vals=vals)
    dt = time.perf_counter() - t
    print("call %d: %.2f ms  %.2f GiB/s on disk" % (i, dt * 1e3, disk / dt / 2 ** 30), flush=True)
for b in bufs[::-1]:
    codec.host_unregister(b)
