#!/usr/bin/env python
"""Benchmark: GiB/s of bithash blocks decoded (device-resident), 32 B key / 1 KiB value.

One "step" = one pass of the hot path (bhg_decode_batch: CRC-32C + readRecord
validation + KV-record decode + FNV-1) over one batch of 1M synthetic blocks
already resident in HBM (BASELINE.json configs[1]).  N GPUs (torch.distributed
run, one rank per GPU) each decode their own tables: weak scaling, no
data-path collective.  Rank 0 prints one JSON line.

Extra legs (N=1, rank 0, outside the timed region):
  * cpu_baseline -- the C restatement (oracle/) on the host cores, bounded sample
  * e2e          -- the host-buffer path (H2D + kernel + D2H), recorded in DESIGN.md
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s bithash blocks decoded (device-resident), 32B key / 1KB value, 1 GPU"
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
ALGO_BYTES_PER_BLOCK = 16 + 1076 + 40   # handle + record + descriptor


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1_000_000, help="blocks per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    return ap.parse_args()


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model


def pmc_traffic():
    """Per-launch HBM bytes of the decode kernel from the committed rocprofv3
    --pmc summary (FETCH_SIZE x2 on gfx950 + WRITE_SIZE, KiB -> bytes)."""
    p = os.path.join(ROOT, "profiles", "pmc_decode_c2.json")
    if not os.path.exists(p):
        return None
    try:
        return float(json.load(open(p))["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from bitalosdb_amd import _lib, synth
    from bitalosdb_amd.codec import BithashCodec, handles_tensor
    _lib.lib()
    codec = BithashCodec(local)
    with torch.cuda.stream(codec.stream):      # every torch op and event on the codec's HIP stream
        run(a, world, rank, local, dev, codec)
    codec.close()
    if world > 1:
        dist.destroy_process_group()


def run(a, world, rank, local, dev, codec):
    import torch.distributed as dist
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    n = a.blocks
    # rank r owns its own tables (round-robin by table file: file numbers disjoint per rank)
    src_t, h, meta = synth.uniform_tables(n, device=dev, seed=synth.SEED + rank,
                                          first_file_num=1 + rank * 1000)
    h_t = handles_tensor(h, dev)
    desc_t = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    L = meta["rec_len"]

    def step():
        codec.decode_batch(src_t, src_t.numel(), h_t, n, out_desc=desc_t)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local])

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        starts[i].record()
        step()
        ends[i].record()
    torch.cuda.synchronize(dev)
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kern_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    avg_kern_ms = float(np.mean(kern_ms))

    # descriptors -> status histogram + digest (checked across ranks, outside the timed region)
    d = codec_desc = desc_t.view(-1, 40).cpu().numpy().reshape(-1).view(
        np.dtype([("key_off", "<u4"), ("key_len", "<u4"), ("val_off", "<u4"), ("val_len", "<u4"),
                  ("trailer", "<u8"), ("file_num", "<u4"), ("fnv1", "<u4"), ("crc", "<u4"),
                  ("status", "<u4")]))
    ok_blocks = int((d["status"] == 0).sum())
    digest = int(np.bitwise_xor.reduce(d["crc"].astype(np.uint64) * np.uint64(0x9E3779B1) ^ d["fnv1"]))
    stats = torch.tensor([elapsed, float(ok_blocks), float(n)], dtype=torch.float64, device=dev)
    if world > 1:
        mx = stats[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = float(mx.item())
        ok_total, n_total = float(sm[0].item()), float(sm[1].item())
    else:
        ok_total, n_total = float(ok_blocks), float(n)

    total_blocks = n_total * a.steps
    value = total_blocks * L / elapsed / 2 ** 30
    achieved = n * ALGO_BYTES_PER_BLOCK / (avg_kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic()
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded torch generator; FuncRandBytes alphabet keys/values; 128 MiB tables)",
        "config": {"workload": "BASELINE configs[1]: 1M uncompressed bithash blocks per GPU, CRC-verify + "
                               "KV-record decode, 32B key / 1KB value",
                   "blocks_per_gpu": n, "record_bytes": L, "tables_per_gpu": meta["tables"],
                   "codec": "none", "parallelism": "table-sharded x%d" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "kernel": "k_decode_lane<MODE_NONE,4,16,512,8,2>", "kernel_avg_ms": round(avg_kern_ms, 4),
                     "algorithmic_bytes_per_block": ALGO_BYTES_PER_BLOCK},
        "status_ok_blocks": int(ok_total),
        "digest_rank0": "%016x" % (digest & (2 ** 64 - 1)),
    }

    if rank == 0 and world == 1 and not a.no_e2e:
        # end-to-end: host buffers (pageable) -> H2D -> kernel -> D2H descriptors
        host_src = src_t.cpu().numpy()
        t = time.perf_counter()
        reps = 2
        for _ in range(reps):
            codec.decode_host(host_src, h)
        e2e_s = (time.perf_counter() - t) / reps
        out["e2e_host"] = {"value": round(n * L / e2e_s / 2 ** 30, 3), "unit": "GiB/s",
                           "note": "pageable host src (%.2f GB) + handles H2D, decode, 40 B/block D2H, synchronous"
                                   % (host_src.size / 1e9)}
    else:
        host_src = None

    if rank == 0 and world == 1 and not a.no_cpu:
        from oracle import oracle as O
        if host_src is None:
            host_src = src_t.cpu().numpy()
        threads = min(16, os.cpu_count() or 1)
        # parity on the measured batch (restatement vs device descriptors)
        exp, _, _ = O.decode_batch(host_src, h, nthreads=threads)
        parity = all(np.array_equal(exp[f], d[f]) for f in d.dtype.names)
        reps, t = 0, time.perf_counter()
        while True:
            O.decode_batch(host_src, h, nthreads=threads)
            reps += 1
            if time.perf_counter() - t >= a.cpu_seconds:
                break
        cpu_s = time.perf_counter() - t
        m1 = min(n, 200_000)
        t = time.perf_counter()
        O.decode_batch(host_src, h[:m1], nthreads=1)
        st_s = time.perf_counter() - t
        out["cpu_baseline"] = {
            "value": round(reps * n * L / cpu_s / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "C restatement of readData/readRecord + masked CRC-32C (SSE4.2) + FNV-1 over the same %d "
                      "blocks, %d passes in %.1f s on %d threads (%s); 1 thread: %.3f GiB/s"
                      % (n, reps, cpu_s, threads, cpu_info(), m1 * L / st_s / 2 ** 30)}
        out["parity_vs_restatement"] = "bit-exact" if parity else "MISMATCH"

    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
