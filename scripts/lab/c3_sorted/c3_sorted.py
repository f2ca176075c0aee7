"""Lab: how much of C3's tier-1 walk is group imbalance?  Decode the C3 batch with its handles in
write order and sorted by snappy element count (so a wave's 18 blocks walk alike); SORT=0/1."""
import ctypes, os, subprocess, sys, time
import numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
sys.path.insert(0, ROOT)
import bench
from bitalosdb_amd.codec import BithashCodec, handles_tensor
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/c3count.so"
subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(here, "count.c")])
lib = ctypes.CDLL(so)
dev = torch.device("cuda:0")
codec = BithashCodec(0)
n = 1_000_000
src, h, meta, enc = bench._encode_tables(codec, n, torch.full((n,), 1024, dtype=torch.int64, device=dev), dev, bench.synth_seed(0), 1, "dict")
ecrc = enc[-1].crc
host = src.cpu().numpy()
off = np.ascontiguousarray(h["offset"]); ln = np.ascontiguousarray(h["length"])
cnt = np.zeros(n, dtype=np.uint32)
lib.count_elements(host.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p), ln.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(n), cnt.ctypes.data_as(ctypes.c_void_p))
g = cnt[: n // 18 * 18].reshape(-1, 18).astype(np.float64)
print("elements mean %.2f std %.2f; group waste (18 x sum max / sum) %.3f" % (cnt.mean(), cnt.std(), 18 * g.max(1).sum() / g.sum()))
for mode in [int(x) for x in os.environ.get("MODES", "0 1 0 1").split()]:
    perm = np.argsort(cnt, kind="stable") if mode else np.arange(n)
    hh = h[perm]
    h_t = handles_tensor(hh, dev)
    ec = ecrc.view(torch.int32)[torch.from_numpy(perm.astype(np.int64)).to(dev)].contiguous().view(ecrc.dtype) if mode else ecrc
    desc = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    voff = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
    vals = torch.empty(n * 1024 + 64, dtype=torch.uint8, device=dev)
    step = lambda: codec.decode_batch(src, src.numel(), h_t, n, 1, expected_crc=ec, out_desc=desc, out_vals=vals, out_val_off=voff)
    for _ in range(5): step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20): step()
    torch.cuda.synchronize()
    d = desc.cpu().numpy().view(bench.DESC_DT)
    print("sorted" if mode else "write order", "ms/step %.4f" % ((time.perf_counter() - t) / 20 * 1e3), "ok", int((d["status"] == 0).sum()))
