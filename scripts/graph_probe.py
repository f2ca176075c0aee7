"""Probe (development, not product): C2 step time with eager launches vs the
same K decode launches captured once into a HIP graph and replayed."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bitalosdb_amd import _lib, synth  # noqa: E402
from bitalosdb_amd.codec import BithashCodec, handles_tensor  # noqa: E402

K = 20
dev = torch.device("cuda", 0)
_lib.lib()
codec = BithashCodec(0)
with torch.cuda.stream(codec.stream):
    src_t, h, meta = synth.uniform_tables(1_000_000, device=dev)
    n = len(h)
    h_t = handles_tensor(h, dev)
    desc_t = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    ref = None

    def step(stream=None):
        codec.decode_batch(src_t, src_t.numel(), h_t, n, out_desc=desc_t, stream=stream)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ref = desc_t.clone()
    for rep in range(int(os.environ.get("EAGER_REPS", "3"))):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        torch.cuda.synchronize()
        print("eager  ms/step %.4f" % ((time.perf_counter() - t0) / K * 1e3), flush=True)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(K):
                step(stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    desc_t.zero_()
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        print("graph  ms/step %.4f" % ((time.perf_counter() - t0) / K * 1e3), flush=True)
    print("graph output equal:", bool(torch.equal(desc_t, ref)))
codec.close()
