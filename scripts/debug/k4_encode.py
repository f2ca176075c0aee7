"""Standalone repro of the K4-size encode (102,400 x 2 KiB, one 512 MiB table)."""
import faulthandler
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
faulthandler.enable()
from bitalosdb_amd.codec import BithashCodec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 102_400
tmax = int(sys.argv[2]) if len(sys.argv) > 2 else 512 << 20
c = BithashCodec(0)
rng = np.random.default_rng(4)
blob = rng.integers(0, 256, n * 2048, dtype=np.uint8).tobytes()
vals = [blob[i * 2048:(i + 1) * 2048] for i in range(n)]
keys = [b"bithash_testkey_%d" % i for i in range(n)]
trs = [((i + 1) << 8) | 1 for i in range(n)]
t0 = time.time()
print("encode start", flush=True)
res = c.encode(keys, trs, vals, file_nums=[1], table_max=tmax)
print("encode done", res["ntables"], res["summary"], time.time() - t0, flush=True)
