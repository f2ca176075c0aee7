# lab: dump the first 60 MB of the scanmix bench's table 0 (and its full length) for a host
# simulation of the segment walks' entry guesses
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
sys.argv = ["bench.py", "--config", "scanmix"]
import bench
from bitalosdb_amd import _lib, synth
from bitalosdb_amd.codec import BithashCodec
_lib.lib()
codec = BithashCodec(0)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev); g.manual_seed(bench.synth_seed(0) + 7)
n = 1_000_000
val_lens = torch.randint(64, 4097, (n,), generator=g, device=dev, dtype=torch.int64)
src, h, meta, bufs = bench._encode_tables(codec, n, val_lens, dev, bench.synth_seed(0), 0)
ts = bufs[-1].table_start.cpu().numpy().view(np.uint32)[:meta["ntables"]]
toff = [int(h["offset"][i]) for i in ts] + [meta["src_bytes"]]
t0, t1 = toff[0], toff[1]
np.save("gpurun_out/r5/seg/table0_head.npy", src[t0:t0 + 60_000_000].cpu().numpy())
np.save("gpurun_out/r5/seg/table0_meta.npy", np.array([t0, t1, len(toff) - 1], dtype=np.int64))
print("table0", t0, t1, t1 - t0, "tables", len(toff) - 1)
