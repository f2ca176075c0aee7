"""Lab: the NoCompressor end-to-end host path (bhg_decode_batch_host, pinned src / handles /
descriptors) on the C2 batch (1M 32 B / 1 KiB blocks), timed per call; run under rocprofv3
--kernel-trace --memory-copy-trace to see how the chunk copies and kernels overlap."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from bitalosdb_amd import synth  # noqa: E402
from bitalosdb_amd.codec import BithashCodec, DESC_DT  # noqa: E402

dev = torch.device("cuda:0")
codec = BithashCodec(0)
n = 1 << 20
src_t, h, meta = synth.uniform_tables(n, device=dev)
host_src = src_t.cpu().numpy()
desc = np.empty(n, dtype=DESC_DT)
bufs = (host_src, desc, h)
for b in bufs:
    codec.host_register(b)
for i in range(4):
    t = time.perf_counter()
    codec.decode_host(host_src, h, out_desc=desc)
    dt = time.perf_counter() - t
    print("call %d: %.2f ms  %.2f GiB/s" % (i, dt * 1e3, host_src.size / dt / 2 ** 30), flush=True)
for b in bufs[::-1]:
    codec.host_unregister(b)
