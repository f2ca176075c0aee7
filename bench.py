#!/usr/bin/env python
"""Benchmark: GiB/s of bithash blocks decoded (device-resident), 32 B key / 1 KiB value.

One "step" = one pass of the hot path (bhg_decode_batch: CRC-32C verify
against the writer's CRCs + readRecord validation + KV-record decode + FNV-1)
over one batch of synthetic blocks already resident in HBM.

  N = 1 (default): BASELINE.json configs[1], 1M blocks.  Nested: `strong_c5`,
        the fixed 25 GB corpus (configs[4], 184 tables x 124,738 blocks) on this
        one GPU -- the base of the strong-scaling curve -- and `c1` (configs[0],
        100k blocks on the host CPU).
  N > 1: `bench.py --gpus N` starts N rank processes itself when no launcher
        did (torch.distributed.run works too); the line is the same 25 GB corpus
        with table t decoded by rank t mod N (strong scaling: value = corpus
        bytes / max-over-ranks time), RCCL only for the final reduction.
        Nested: `weak_c2`, 1M blocks per GPU (weak scaling).
  --config c1/c3/c4/c5/...: the other BASELINE configs and rows (see --help).

Extra legs (N=1, rank 0, outside the timed region):
  * cpu_baseline -- the C restatement (oracle/) on the host cores, bounded sample:
                    in-memory on every usable core, 1 thread, and pread-per-block
  * copy ceiling -- a measured device-to-device copy of the same bytes
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

DESC_DT = np.dtype([("key_off", "<u4"), ("key_len", "<u4"), ("val_off", "<u4"), ("val_len", "<u4"),
                    ("trailer", "<u8"), ("file_num", "<u4"), ("fnv1", "<u4"), ("crc", "<u4"), ("status", "<u4")])

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s bithash blocks decoded (device-resident), 32B key / 1KB value, 1 GPU"
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
ALGO_BYTES_PER_BLOCK = 16 + 1076 + 40   # handle + record + descriptor


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group: nccl (= RCCL, the real run) or gloo (rehearsal of the multi-rank "
                         "path with several ranks on one GPU; device = LOCAL_RANK mod visible GPUs)")
    ap.add_argument("--steps", type=int, default=20)
    # GPU clocks ramp over the first ~100 C2 launches (~30 ms of load; profiles/r1_s6_clock_ramp_probe.txt)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--ramp-ms", type=float, default=300.0,
                    help="untimed steps of the measured kernel for at least this long before the --warmup steps "
                         "(the MI355X clocks ramp over tens of ms of load); 0 disables; recorded in the line")
    ap.add_argument("--blocks", type=int, default=1_000_000, help="blocks per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--codec", default="none", choices=["none", "snappy"], help="c5 only")
    ap.add_argument("--values", default="dict", choices=["dict", "chunk16"], help="c3/c4/c5-snappy values: " +
                    "dict: SURVEY 8(d)'s token generator (the primary workload); chunk16: 16-B chunks of 8 per-value "
                    "random words")
    ap.add_argument("--no-secondary", action="store_true", help="c3/c4: skip the nested line of the other value "
                                                                  "generator")
    ap.add_argument("--c5-tables", type=int, default=184, help="c5 corpus size in 128 MiB tables")
    ap.add_argument("--bigval-n", type=int, default=7000,
                    help="bigval: values U[4 KiB, 256 KiB] + 1%% at 1-4 MiB (~1 GiB at 7,000)")
    ap.add_argument("--no-c5", action="store_true", help="N=1: skip the nested strong_c5 record")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the two rocprofv3 --pmc child passes that measure roofline.traffic (N=1, rank 0)")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "scan", "scanmix", "get",
                                                       "indexcrc", "tail", "mixdec", "bigval", "spawncheck"],
                    help="c1: 100k blocks on the host CPU; c2: uncompressed decode (BASELINE metric; at N > 1 "
                         "the line is the C5 strong-scaling corpus); c3: snappy decode; c4: encode; "
                         "c5: 25 GB corpus sharded round-robin by table over the GPUs (strong scaling); "
                         "scan/scanmix: table data-region scan over uniform / mixed-length tables; "
                         "get: batched Bithash.Get (HashIndex + conflict SeekGE + readData) over full tables; "
                         "indexcrc: per-table indexhash_checksum verify (masked CRC-32C of 1.51 MB per table); "
                         "tail: Writer.writeTable's tail (bhg_table_tail) for 1M records as 8 tables of 128 MiB "
                         "and as ONE table of 1M records (natural FNV-1 collisions -> a conflict block); "
                         "mixdec: decode of C4-shaped tables (1M pairs, values U[64, 4096] B), snappy line with "
                         "the NoCompressor line nested; "
                         "spawncheck: no GPU -- the --gpus N launch path alone (rank env, gloo rendezvous, "
                         "the all-reduce that reports ranks_seen, rank 0's JSON line), for CPU tests")
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


def usable_cores():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def copy_ceiling(src_t, dev, reps=5):
    """Measured device-to-device copy of the same bytes (read + write), GB/s."""
    dst = torch.empty_like(src_t)
    dst.copy_(src_t)
    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    for i in range(reps):
        e0[i].record()
        dst.copy_(src_t)
        e1[i].record()
    torch.cuda.synchronize(dev)
    ms = float(np.mean([x.elapsed_time(y) for x, y in zip(e0, e1)]))
    del dst
    return 2.0 * src_t.numel() / (ms * 1e-3) / 1e9, ms


# HBM traffic of a config's kernels, measured in the run: bench.py starts itself again (a child
# process; nothing is exec'd) under rocprofv3 --pmc for two short passes (the counter blocks do
# not fit one pass) and reads the L2->fabric request counters split by request size.  gfx950's
# FETCH_SIZE tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM section); the split counters
# need no correction: read = 32 n32 + 64 n64 + 128 n128, write = 32 (n - n64) + 64 n64.
PMC_PASSES = (("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"),
              ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"))


def measure_traffic(config_args, kernels, timeout_s=240):
    """{full kernel name: median HBM bytes per launch (read, write)} for every kernel whose name
    contains one of `kernels`, from two rocprofv3 --pmc passes of `bench.py <config_args> --steps 2
    --warmup 1`; None (with the reason) when the profiler is missing or a pass fails.  Each kernel
    listed runs once per step, so the sum over the result is the step's traffic."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if prof is None:
        return None, "rocprofv3 not found"
    env = dict(os.environ, BHG_TRAFFIC_CHILD="1", TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    per = {}   # (kernel, dispatch) -> {counter: value}
    with tempfile.TemporaryDirectory(prefix="bhg_pmc_", dir=env["TMPDIR"]) as td:
        for i, counters in enumerate(PMC_PASSES):
            out = os.path.join(td, "p%d" % i)
            cmd = [prof, "--pmc", *counters, "-d", out, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.join(ROOT, "bench.py"), *config_args, "--steps", "2", "--warmup", "1",
                   "--no-cpu", "--no-e2e", "--no-c5"]
            import signal
            errf = os.path.join(td, "p%d.err" % i)
            with open(errf, "wb") as ef:
                pr = subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=ef, start_new_session=True)
                try:
                    rc = pr.wait(timeout=timeout_s)
                except subprocess.TimeoutExpired:
                    os.killpg(pr.pid, signal.SIGKILL)    # the profiler and the bench under it
                    pr.wait()
                    return None, "pmc pass %d timed out" % i
            if rc != 0:
                return None, "pmc pass %d exit %d: %s" % (i, rc, open(errf, "rb").read()[-200:].decode(errors="replace"))
            for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
                for row in csv.DictReader(open(f)):
                    kn = row["Kernel_Name"]
                    if not any(k in kn for k in kernels):
                        continue
                    # keyed by the FULL kernel name (template arguments included): two instantiations
                    # of one template (k_snappy_enc<2048, ..> and <4096, ..>) are two kernels of the step
                    full = kn.split("(")[0].strip()
                    key = (full, i, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                    per.setdefault(key, {})[row["Counter_Name"]] = float(row["Counter_Value"])
    res = {}
    for full in sorted({kk for (kk, _, _) in per}):
        rd = [32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) +
              128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) for (kk, i, _), c in per.items() if kk == full and i == 0]
        wr = [32 * (c.get("TCC_EA0_WRREQ_sum", 0) - c.get("TCC_EA0_WRREQ_64B_sum", 0)) +
              64 * c.get("TCC_EA0_WRREQ_64B_sum", 0) for (kk, i, _), c in per.items() if kk == full and i == 1]
        if rd and wr:
            res[full] = {"read": float(np.median(rd)), "write": float(np.median(wr)), "launches": min(len(rd), len(wr)),
                         "name": full}
    if not res:
        return None, "no dispatch of %s in the pmc passes" % ",".join(kernels)
    return res, None


def traffic_fields(cfg_args, kernels, alg_bytes_per_launch, what):
    """roofline.traffic (+ ratio and provenance) for the dominant kernel(s): summed per-launch
    bytes of `kernels` from measure_traffic; null with the reason when not measurable."""
    if os.environ.get("BHG_TRAFFIC_CHILD") or os.environ.get("BHG_NO_TRAFFIC"):
        return {"traffic": None, "traffic_source": "not measured (profiling child or BHG_NO_TRAFFIC)"}
    res, err = measure_traffic(cfg_args, kernels)
    if res is None:
        return {"traffic": None, "traffic_source": "not measured: %s" % err}
    tot = sum(v["read"] + v["write"] for v in res.values())
    return {"traffic": round(tot), "traffic_ratio": round(tot / alg_bytes_per_launch, 4),
            "traffic_source": "measured in this run: bench.py %s under rocprofv3 --pmc (%s | %s), median per "
                              "launch of each kernel, summed over %s (each runs once per step); HBM bytes = 32/64/128-B read requests + 32/64-B write requests at "
                              "the L2 fabric interface; algorithmic bytes per launch %d (%s)" % (
                                  " ".join(cfg_args), " ".join(PMC_PASSES[0]), " ".join(PMC_PASSES[1]),
                                  ", ".join(v["name"] for v in res.values()), alg_bytes_per_launch, what),
            "traffic_by_kernel": {v["name"]: {"read": round(v["read"]), "write": round(v["write"]),
                                              "launches": v["launches"]} for v in res.values()}}


BACKEND = "nccl"
# a process group is up: N > 1, or the one-rank rehearsal of the N > 1 path (BHG_BENCH_PG1=1 at
# --gpus 1: RCCL init, barriers, all-reduces and all-gathers on one real GPU; the line is then the
# N > 1 line's shape, with its collectives run by a world of one)
PG = False


def dist_barrier(world, local):
    """Barrier of the N>1 bench (nccl: on the rank's device stream; gloo: host)."""
    if PG:
        import torch.distributed as dist
        if BACKEND == "nccl":
            dist.barrier(device_ids=[local])
        else:
            dist.barrier()


def dist_sum_(t, world):
    """In-place SUM all-reduce of a small tensor (gloo: through host memory)."""
    if PG:
        import torch.distributed as dist
        if BACKEND == "nccl":
            dist.all_reduce(t)
        else:
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`bench.py --gpus N` with no outer launcher: start N rank processes of this
    same command (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env), one per
    GPU, and exit with the worst exit code.  This process never touches the GPU
    (no HIP call happens before the children start), and the children are
    started, not exec'd."""
    import subprocess
    import threading
    port = _free_port()
    procs = []

    def forward(pipe):   # rank 0's stdout: the JSON line to stdout, library chatter (gloo) to stderr
        for line in iter(pipe.readline, b""):
            (sys.stdout if line.lstrip().startswith(b"{") else sys.stderr).buffer.write(line)
            (sys.stdout if line.lstrip().startswith(b"{") else sys.stderr).flush()

    fwd = None
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BHG_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
        if r == 0:
            fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
            fwd.start()
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
        failed = [rc for rc in rcs if rc not in (None, 0)]
        if failed:   # one rank died: the others would wait in a collective forever
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                try:
                    rcs[r] = p.wait(30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    rcs[r] = p.wait()
            break
        time.sleep(0.05)
    fwd.join(30)
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE %d" % (a.gpus, world), file=sys.stderr)
        sys.exit(2)
    import torch.distributed as dist
    if a.config == "spawncheck":
        return spawn_check(a, world, rank)
    global BACKEND, PG
    BACKEND = a.backend
    if a.backend == "gloo":   # rehearsal: ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
    PG = world > 1 or os.environ.get("BHG_BENCH_PG1") == "1"
    if PG:
        if world == 1:
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.cuda.set_device(local)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from bitalosdb_amd import _lib, synth
    from bitalosdb_amd.codec import BithashCodec, handles_tensor
    _lib.lib()
    codec = BithashCodec(local)
    with torch.cuda.stream(codec.stream):      # every torch op and event on the codec's HIP stream
        run(a, world, rank, local, dev, codec)
    codec.close()
    if PG:
        dist.destroy_process_group()


def spawn_check(a, world, rank):
    """--config spawncheck: the multi-rank launch path without a GPU.  Every rank joins a
    gloo group and all-reduces 1 and its rank; rank 0 prints what it saw."""
    import torch.distributed as dist
    from bitalosdb_amd import shard
    t = torch.tensor([1, rank], dtype=torch.int64)
    if world > 1:
        dist.init_process_group("gloo")
        dist.all_reduce(t)
    # the N > 1 line's self-describing fields, from the same helper c5_measure uses (dummy timings)
    sf = shard.scaling_fields(1.0 + 0.5 * rank, 0.5, torch.device("cpu"))
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"config": "spawncheck", "n_gpus": world, "ranks_seen": int(t[0]),
                          "rank_sum": int(t[1]), "spawned": os.environ.get("BHG_BENCH_SPAWNED") == "1",
                          "scaling_fields": sf}), flush=True)


def run(a, world, rank, local, dev, codec):
    if a.config == "c3":
        return run_c3(a, world, rank, local, dev, codec)
    if a.config == "c4":
        return run_c4(a, world, rank, local, dev, codec)
    if a.config in ("scan", "scanmix"):
        return run_scan(a, world, rank, local, dev, codec)
    if a.config == "get":
        return run_get(a, world, rank, local, dev, codec)
    if a.config == "indexcrc":
        return run_indexcrc(a, world, rank, local, dev, codec)
    if a.config == "tail":
        return run_tail(a, world, rank, local, dev, codec)
    if a.config == "bigval":
        return run_bigval(a, world, rank, local, dev, codec)
    if a.config == "mixdec":
        return run_mixdec(a, world, rank, local, dev, codec)
    if a.config == "c5":
        return run_c5(a, world, rank, local, dev, codec)
    if a.config == "c1":
        return run_c1(a, world, rank, local, dev, codec)
    if PG:
        # N > 1: the fixed 25 GB corpus split by table over the N GPUs (strong scaling), with
        # the per-GPU C2 batch (weak scaling) nested
        res = c5_measure(a, world, rank, local, dev, codec, "none", with_cpu=False)
        torch.cuda.empty_cache()
        weak = c2_measure(a, world, rank, local, dev, codec, with_extras=False)
        if rank == 0:
            res["weak_c2"] = {k: weak[k] for k in ("value", "unit", "ms_per_step", "scaling", "roofline",
                                                   "status_ok_blocks", "valid", "digest_all_ranks")}
            res["weak_c2"]["workload"] = weak["config"]["workload"]
            res["weak_c2"]["per_gpu_GiBps"] = round(weak["value"] / world, 3)
            print(json.dumps(res), flush=True)
        return
    out = c2_measure(a, world, rank, local, dev, codec, with_extras=True)
    if not a.no_c5:
        # the same fixed-corpus C5 measurement the N > 1 lines report, at N = 1: the base of the strong-scaling curve
        torch.cuda.empty_cache()
        s = c5_measure(a, world, rank, local, dev, codec, "none", with_cpu=False)
        out["strong_c5"] = {k: s[k] for k in ("metric", "value", "unit", "ms_per_step", "scaling", "per_gpu_GiBps",
                                              "roofline", "status_ok_blocks", "valid", "digest_all_ranks",
                                              "ranks_seen")}
        out["strong_c5"]["workload"] = s["config"]["workload"]
    if rank == 0:
        print(json.dumps(out), flush=True)


def c2_measure(a, world, rank, local, dev, codec, with_extras):
    """BASELINE configs[1] on this rank's GPU: 1M blocks of its own tables,
    CRC-verify + record decode, K timed steps.  Returns the bench line (dict)."""
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    n = a.blocks
    # rank r owns its own tables (round-robin by table file: file numbers disjoint per rank)
    src_t, h, meta = synth.uniform_tables(n, device=dev, seed=synth.SEED + rank,
                                          first_file_num=1 + rank * 1000)
    h_t = handles_tensor(h, dev)
    desc_t = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    L = meta["rec_len"]
    # the CRCs the writer recorded (crc.New(record).Value()), from the lane-per-range GPU primitive:
    # the timed step is the CRC-verify path (a mismatch would flip the block to BHG_ST_CRC_MISMATCH)
    exp_crc = codec.crc_batch(src_t, h_t, n)

    def step():
        codec.decode_batch(src_t, src_t.numel(), h_t, n, expected_crc=exp_crc, out_desc=desc_t)

    # the measured D2D copy ceiling of the same bytes (before the warm-up steps), then the stated
    # clock ramp (clock_ramp: --ramp-ms of untimed steps), then the --warmup steps
    copy_gbps, copy_ms = copy_ceiling(src_t, dev, reps=100)
    ramp = clock_ramp(a, dev, step)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    def barrier():
        dist_barrier(world, local)

    # timed region: K back-to-back steps, no per-step event markers in the stream
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # the kernel's launch duration for roofline.achieved: a separate pass of K steps, each
    # bracketed by HIP events on the stream the kernel runs on (torch's current stream)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    for i in range(a.steps):
        starts[i].record()
        step()
        ends[i].record()
    torch.cuda.synchronize(dev)
    kern_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    avg_kern_ms = float(np.mean(kern_ms))

    # descriptors -> status histogram + digest (checked across ranks, outside the timed region)
    d = codec_desc = desc_t.view(-1, 40).cpu().numpy().reshape(-1).view(
        np.dtype([("key_off", "<u4"), ("key_len", "<u4"), ("val_off", "<u4"), ("val_len", "<u4"),
                  ("trailer", "<u8"), ("file_num", "<u4"), ("fnv1", "<u4"), ("crc", "<u4"),
                  ("status", "<u4")]))
    ok_blocks = int((d["status"] == 0).sum())
    from bitalosdb_amd import shard
    digest = shard.block_digest(d["crc"], d["fnv1"], d["trailer"], d["status"])
    elapsed, ok_total, n_total, digest_all = shard.reduce_stats(elapsed, ok_blocks, n, digest, dev)

    total_blocks = n_total * a.steps
    value = total_blocks * L / elapsed / 2 ** 30
    achieved = n * (ALGO_BYTES_PER_BLOCK + 4) / (avg_kern_ms * 1e-3) / 1e9   # + the expected CRC read
    if rank == 0 and world == 1 and with_extras and not a.no_traffic:
        tf = traffic_fields(["--config", "c2", "--blocks", str(n)], ["k_decode_tile"],
                            n * (ALGO_BYTES_PER_BLOCK + 4), "handle 16 + record %d + descriptor 40 + expected CRC 4 "
                            "per block" % L)
    else:
        tf = {"traffic": None, "traffic_source": "measured only at N=1 on rank 0"}
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ramp": ramp,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded torch generator; FuncRandBytes alphabet keys/values; 128 MiB tables)",
        "config": {"workload": "BASELINE configs[1]: 1M uncompressed bithash blocks per GPU, CRC-verify "
                               "(expected_crc) + KV-record decode, 32B key / 1KB value",
                   "blocks_per_gpu": n, "record_bytes": L, "tables_per_gpu": meta["tables"],
                   "codec": "none", "parallelism": "table-sharded x%d" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), **tf,
                     "kernel": "k_decode_tile<8, 2>", "kernel_avg_ms": round(avg_kern_ms, 4),
                     "algorithmic_bytes_per_block": ALGO_BYTES_PER_BLOCK + 4,
                     "measured_copy_ceiling": {"GBps": round(copy_gbps, 1), "ms": round(copy_ms, 4),
                                               "what": "torch D2D copy of the same %d B (read + write), "
                                                       "100 reps run before the clock ramp and the warm-up "
                                                       "steps" % src_t.numel(),
                                               "frac_of_copy": round(achieved / copy_gbps, 4)}},
        "status_ok_blocks": int(ok_total),
        "valid": bool(ok_total == n_total),
        "digest_all_ranks": "%016x" % digest_all,
    }

    if rank == 0 and world == 1 and with_extras and not a.no_e2e:
        # end-to-end: host src -> H2D -> kernel -> D2H descriptors (bhg_decode_batch_host; handles are
        # sorted, so the 64 MiB-chunk 3-stream pipeline runs).  Pageable first, then the same buffer
        # page-locked with bhg_host_register (an mmap'd table file pinned once per mapping).
        host_src = src_t.cpu().numpy()
        from bitalosdb_amd.codec import DESC_DT
        host_desc = np.empty(n, dtype=DESC_DT)
        e2e = {}
        for mode in ("pageable", "pinned"):
            if mode == "pinned":   # an mmap'd table file, its handle list and a reused descriptor buffer, pinned once
                codec.host_register(host_src)
                codec.host_register(host_desc)
                codec.host_register(h)
            for _ in range(2):      # warm the ring buffers (the second call still ran ~15 % slow on the box)
                codec.decode_host(host_src, h, out_desc=host_desc)
            reps, t = 5, time.perf_counter()
            for _ in range(reps):
                got_host, _, _ = codec.decode_host(host_src, h, out_desc=host_desc)
            e2e_s = (time.perf_counter() - t) / reps
            e2e[mode] = round(n * L / e2e_s / 2 ** 30, 3)
            if mode == "pinned":
                codec.host_unregister(h)
                codec.host_unregister(host_desc)
                codec.host_unregister(host_src)
        host_ok = bool(np.array_equal(got_host["crc"], d["crc"]) and np.array_equal(got_host["status"], d["status"]))
        out["e2e_host"] = {"value": e2e["pinned"], "unit": "GiB/s", "pageable": e2e["pageable"],
                           "matches_device_path": host_ok,
                           "note": "host src (%.2f GB) + handles -> descriptors in host memory, 64 MiB chunks "
                                   "over 3 streams (H2D, decode, D2H overlapped), descriptor buffer reused.  value: "
                                   "src, handles and descriptors page-locked (bhg_host_register); pageable also "
                                   "given" % (host_src.size / 1e9)}
    else:
        host_src = None

    if rank == 0 and world == 1 and with_extras and not a.no_cpu:
        from oracle import oracle as O
        if host_src is None:
            host_src = src_t.cpu().numpy()
        threads = usable_cores()
        exp_host = exp_crc.cpu().numpy().view(np.uint32)
        # parity on the measured batch (restatement vs device descriptors, same expected CRCs)
        exp, _, _ = O.decode_batch(host_src, h, expected_crc=exp_host, nthreads=threads)
        parity = all(np.array_equal(exp[f], d[f]) for f in d.dtype.names)
        budget = a.cpu_seconds / 3
        reps, t = 0, time.perf_counter()
        while True:
            O.decode_batch(host_src, h, expected_crc=exp_host, nthreads=threads)
            reps += 1
            if time.perf_counter() - t >= budget:
                break
        cpu_s = time.perf_counter() - t
        m1 = min(n, 200_000)
        t = time.perf_counter()
        O.decode_batch(host_src, h[:m1], expected_crc=exp_host[:m1], nthreads=1)
        st_s = time.perf_counter() - t
        # Reader.readData's shape: one pread per block from the table file (page cache)
        import tempfile
        fd, path = tempfile.mkstemp(prefix="bhg_c2_", dir="/tmp")
        try:
            with os.fdopen(os.dup(fd), "wb") as f:
                host_src.tofile(f)
            preps, t = 0, time.perf_counter()
            while True:
                pd = O.decode_batch_pread(fd, h, expected_crc=exp_host, nthreads=threads)
                preps += 1
                if time.perf_counter() - t >= budget:
                    break
            pr_s = time.perf_counter() - t
            pread_ok = bool(np.array_equal(pd["crc"], d["crc"]) and np.array_equal(pd["status"], d["status"]))
        finally:
            os.close(fd)
            os.unlink(path)
        out["cpu_baseline"] = {
            "value": round(reps * n * L / cpu_s / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": "C restatement of readData/readRecord + masked CRC-32C verify (SSE4.2) + FNV-1 over the same "
                      "%d blocks in memory, %d passes in %.1f s on %d threads = every core this process may use "
                      "(os.cpu_count() %d; %s)" % (n, reps, cpu_s, threads, os.cpu_count() or 0, cpu_info()),
            "one_thread": round(m1 * L / st_s / 2 ** 30, 3),
            "pread_per_block": {"value": round(preps * n * L / pr_s / 2 ** 30, 3), "threads": threads,
                                "matches_device_path": pread_ok,
                                "note": "one pread() of bh.Length bytes per block from the table file in the page "
                                        "cache, as Reader.readData's ReadAt (reader.go:251)"}}
        out["parity_vs_restatement"] = "bit-exact" if parity else "MISMATCH"
        out["valid"] = bool(out["valid"] and parity)
        out["c1"] = c1_baseline(host_src, h, exp_host, L)
    return out


def c1_baseline(host_src, h, exp_host, L, m=100_000):
    """BASELINE configs[0] (C1): the reader on the host CPU over 100k uncompressed
    blocks -- the C restatement of readData/readRecord + CRC verify + FNV-1
    (1 thread and every usable core), plumbing only, no GPU.
    100k blocks are ~10 ms of work: the all-core figure decodes them 32 times per
    call (one 3.2M-handle batch, ~0.3 s), so per-call thread start-up is amortised."""
    from oracle import oracle as O
    hs, es = h[:m], exp_host[:m]
    res = {}
    for name, thr, rep in (("one_thread", 1, 1), ("all_cores", usable_cores(), 32)):
        hb = np.tile(hs, rep) if rep > 1 else hs
        eb = np.tile(es, rep) if rep > 1 else es
        reps, t = 0, time.perf_counter()
        while True:
            O.decode_batch(host_src, hb, expected_crc=eb, nthreads=thr)
            reps += 1
            if time.perf_counter() - t >= 1.0:
                break
        res[name] = round(reps * rep * m * L / (time.perf_counter() - t) / 2 ** 30, 3)
    return {"workload": "BASELINE configs[0]: %d uncompressed blocks (32B/1KB) decoded on the host" % m,
            "unit": "GiB/s", "value": res["one_thread"], "one_thread": res["one_thread"],
            "all_cores": res["all_cores"], "cores": usable_cores(), "kind": "port", "cpu": cpu_info(),
            "all_cores_note": "the 100k blocks 32 times per call (3.2M handles, >= 1 s of calls), so thread start-up "
                              "per call is amortised"}


def run_c1(a, world, rank, local, dev, codec):
    """BASELINE configs[0] as its own line: C1 on the host (1 thread = value, and
    every core), the GPU decode of the same 100k blocks beside it."""
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    n = 100_000
    src_t, h, meta = synth.uniform_tables(n, device=dev, seed=synth.SEED)
    h_t = handles_tensor(h, dev)
    exp_crc = codec.crc_batch(src_t, h_t, n)
    desc_t = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    el, kms = _timed(a, dev, lambda: codec.decode_batch(src_t, src_t.numel(), h_t, n, expected_crc=exp_crc,
                                                        out_desc=desc_t))
    host = src_t.cpu().numpy()
    c1 = c1_baseline(host, h, exp_crc.cpu().numpy().view(np.uint32), meta["rec_len"], m=n)
    d = desc_t.cpu().numpy().view(DESC_DT)
    from oracle import oracle as O
    e, _, _ = O.decode_batch(host, h, expected_crc=exp_crc.cpu().numpy().view(np.uint32), nthreads=usable_cores())
    out = {"metric": "GiB/s bithash blocks decoded on the host CPU (reference reader restated), 100k blocks",
           "value": c1["value"], "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(n * meta["rec_len"] / (c1["value"] * 2 ** 30) * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": c1["workload"]}, "cpu": c1,
           "gpu_same_blocks": {"value": round(n * meta["rec_len"] * a.steps / el / 2 ** 30, 3), "unit": "GiB/s",
                               "step_event_ms": round(kms, 4)},
           "parity_vs_restatement": "bit-exact" if all(np.array_equal(e[f], d[f]) for f in DESC_DT.names)
           else "MISMATCH"}
    if rank == 0:
        print(json.dumps(out), flush=True)


def _pack_values(vals_t):
    """[n, L] uint8 device tensor -> (flat bytes, u64 offsets[n+1]) device tensors."""
    n, L = vals_t.shape
    off = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=vals_t.device)
    return vals_t.reshape(-1).contiguous(), off


def _encode_inputs(n, val_lens, dev, seed, gen):
    """Keys/trailers/values for n pairs (values from the compressible generator `gen`)."""
    from bitalosdb_amd import synth
    return synth.kv_pairs_gpu(n, val_lens, device=dev, seed=seed, gen=gen)


def _encode_tables(codec, n, val_lens, dev, seed, compressor, gen="dict"):
    """Encode n pairs into bithash tables on the GPU; returns (src, handles, meta, raw_bytes)."""
    from bitalosdb_amd.codec import EncodeBuffers, HANDLE_DT
    keys, key_off, tr, vals, val_off = _encode_inputs(n, val_lens, dev, seed, gen)
    cap = int(n * 64 + vals.numel() * 7 // 6 + 64)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    maxt = 4096
    fns = torch.arange(1, maxt + 1, dtype=torch.int32, device=dev)
    bufs = EncodeBuffers(n, maxt, dev)
    codec.encode_batch(keys, key_off, tr, vals, val_off, n, compressor, fns, maxt, 0, 128 << 20, out, bufs)
    codec.sync()
    pos = bufs.pos.cpu().numpy().view(np.uint64)
    ln = bufs.bh_len.cpu().numpy().view(np.uint32)
    h = np.zeros(n, dtype=HANDLE_DT)
    h["offset"] = pos
    h["length"] = ln
    total = int(bufs.summary[0].item())
    return out[:total], h, dict(src_bytes=total, ntables=int(bufs.summary[1].item())), (keys, key_off, tr, vals, val_off, bufs)


def clock_ramp(a, dev, fn):
    """Untimed steps of the measured path for >= a.ramp_ms of wall time, before the --warmup steps:
    the clocks come out of idle over tens of ms of load, so without it a short --warmup (the driver
    runs --warmup 5) times part of the ramp.  Returns the record put in the JSON line."""
    if a.ramp_ms <= 0:
        return {"ms": 0.0, "steps": 0}
    torch.cuda.synchronize(dev)
    t0, k = time.perf_counter(), 0
    while True:
        for _ in range(8):
            fn()
        k += 8
        torch.cuda.synchronize(dev)
        if (time.perf_counter() - t0) * 1e3 >= a.ramp_ms:
            break
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": k,
            "what": "untimed steps of the measured kernel before the --warmup steps (clock ramp)"}


def _timed(a, dev, fn):
    a.ramp_record = clock_ramp(a, dev, fn)
    for _ in range(a.warmup):
        fn()
    torch.cuda.synchronize(dev)
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    t0 = time.perf_counter()
    for i in range(a.steps):
        starts[i].record()
        fn()
        ends[i].record()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    return el, float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)]))


def _secondary_gen(gen):
    from bitalosdb_amd import synth
    return [g for g in synth.VALUE_GENS if g != gen][0]


def run_c3(a, world, rank, local, dev, codec):
    """BASELINE configs[2]: 1M snappy blocks, full CRC (against the writer's CRCs) + decompress +
    decode, 32 B / 1 KiB.  The line is the --values generator (default: SURVEY 8(d)'s dictionary
    generator); the other generator is nested as a secondary line."""
    out = c3_measure(a, world, rank, local, dev, codec, a.values, extras=True)
    if not a.no_secondary:
        torch.cuda.empty_cache()
        g2 = _secondary_gen(a.values)
        sec = c3_measure(a, world, rank, local, dev, codec, g2, extras=False)
        out["secondary_values_" + g2] = {k: sec[k] for k in ("value", "unit", "ms_per_step", "roofline",
                                                              "status_ok_blocks")}
        out["secondary_values_" + g2].update(sec["config"])
    if rank == 0:
        print(json.dumps(out), flush=True)


def c3_measure(a, world, rank, local, dev, codec, gen, extras):
    n = a.blocks
    val_lens = torch.full((n,), 1024, dtype=torch.int64, device=dev)
    src, h, meta, enc = _encode_tables(codec, n, val_lens, dev, synth_seed(rank), 1, gen)
    exp_crc = enc[-1].crc                      # the writer's CRCs (crc.New(record).Value())
    from bitalosdb_amd.codec import handles_tensor
    h_t = handles_tensor(h, dev)
    desc = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    voff = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
    vals = torch.empty(n * 1024 + 64, dtype=torch.uint8, device=dev)
    step = lambda: codec.decode_batch(src, src.numel(), h_t, n, 1, expected_crc=exp_crc, out_desc=desc,
                                      out_vals=vals, out_val_off=voff)
    el, kms = _timed(a, dev, step)
    d = desc.cpu().numpy().view(DESC_DT)
    disk = float(h["length"].astype(np.float64).sum())
    out = {"metric": "GiB/s bithash blocks decoded (device-resident), snappy, 32B key / 1KB value, 1 GPU",
           "value": round(disk * a.steps / el / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ramp": a.ramp_record, "ms_per_step": round(el / a.steps * 1e3, 4),
           "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (GPU-encoded snappy tables, values: %s)" % gen,
           "config": {"workload": "BASELINE configs[2]: 1M snappy blocks, CRC-verify (expected_crc = the writer's "
                                  "CRCs) + decompress + decode",
                      "values": gen, "blocks_per_gpu": n, "mean_record_bytes": round(disk / n, 1),
                      "snappy_ratio": round((disk - n * 52.0) / (n * 1024.0), 4),
                      "decoded_GiBps": round(n * 1024 * a.steps / el / 2 ** 30, 3)},
           "status_ok_blocks": int((d["status"] == 0).sum())}
    out["valid"] = out["status_ok_blocks"] == n
    # SURVEY 8(d) C3 algorithmic bytes: handle 16 + record L + expected CRC 4 + desc 40 + 1 KiB decoded
    # value per block, over the whole step (header/CRC pass + scan + snappy kernel; kms = event-timed step)
    alg = n * (16 + 4 + 40 + 1024) + disk
    out["roofline"] = {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                       "traffic": None, "scope": "whole step (k_decode_stream<1> header/CRC pass + size scan + k_snappy_lds + k_snappy_rt)",
                       "step_event_ms": round(kms, 4)}
    if extras and rank == 0 and world == 1 and not a.no_traffic:
        out["roofline"].update(traffic_fields(["--config", "c3", "--blocks", str(n), "--values", gen,
                                               "--no-secondary"],
                                              ["k_decode_stream", "k_snappy_lds", "k_snappy_rt", "k_chunk_"], int(alg),
                                              "handle 16 + on-disk record + expected CRC 4 + descriptor 40 + 1 KiB "
                                              "value per block"))
    if extras and rank == 0 and world == 1 and not a.no_cpu:
        from oracle import oracle as O
        host = src.cpu().numpy()
        thr = usable_cores()
        ecrc = exp_crc.cpu().numpy().view(np.uint32)
        exp, ev, eo = O.decode_batch(host, h, codec=1, expected_crc=ecrc, nthreads=thr)
        got_v = vals.cpu().numpy()
        par = all(np.array_equal(exp[f], d[f]) for f in d.dtype.names) and \
            got_v[:int(eo[-1])].tobytes() == ev[:int(eo[-1])].tobytes()
        t = time.perf_counter()
        reps = 0
        while time.perf_counter() - t < a.cpu_seconds:
            O.decode_batch(host, h, codec=1, expected_crc=ecrc, nthreads=thr, out_val_off=eo)
            reps += 1
        cs = time.perf_counter() - t
        # one thread: the first 100k blocks (a bounded sample), same restated decode
        n1 = min(n, 100_000)
        h1 = h[:n1]
        disk1 = float(h1["length"].astype(np.float64).sum())
        t = time.perf_counter()
        reps1 = 0
        while time.perf_counter() - t < 2.0:
            O.decode_batch(host, h1, codec=1, expected_crc=ecrc[:n1], nthreads=1, out_val_off=eo[:n1 + 1])
            reps1 += 1
        cs1 = time.perf_counter() - t
        out["cpu_baseline"] = {"value": round(reps * disk / cs / 2 ** 30, 3), "unit": "GiB/s", "cores": thr,
                               "kind": "port", "one_thread": round(reps1 * disk1 / cs1 / 2 ** 30, 3),
                               "sample": "C restatement (readRecord + CRC verify + golang/snappy decode), "
                               "%d passes over the same %d blocks on %d threads = every core this process may use; "
                               "one_thread: the first %d blocks on 1 thread (%s)" % (reps, n, thr, n1, cpu_info())}
        out["parity_vs_restatement"] = "bit-exact" if par else "MISMATCH"
        out["valid"] = bool(out["valid"] and par)
    if extras and rank == 0 and world == 1 and not a.no_e2e:
        # end-to-end: host table bytes -> H2D -> header/CRC pass + scan + snappy -> D2H descriptors, value
        # offsets and the decoded values (bhg_decode_batch_host; snappy stages the whole src in HBM).
        # Caller-owned output buffers are reused; pageable first, then page-locked (bhg_host_register).
        host_src = src.cpu().numpy()
        ecrc_h = exp_crc.cpu().numpy().view(np.uint32).copy()
        host_desc = np.empty(n, dtype=DESC_DT)
        host_vals = np.empty(n * 1024 + 64, dtype=np.uint8)
        e2e = {}
        for mode in ("pageable", "pinned"):
            bufs = (host_src, host_desc, host_vals, h, ecrc_h)
            if mode == "pinned":
                for b in bufs:
                    codec.host_register(b)
            run = lambda: codec.decode_host(host_src, h, compressor=1, expected_crc=ecrc_h,
                                            out_desc=host_desc, out_vals=host_vals)
            run()
            run()
            reps, t = 5, time.perf_counter()
            for _ in range(reps):
                got_d, got_v, _ = run()
            e2e_s = (time.perf_counter() - t) / reps
            e2e[mode] = round(disk / e2e_s / 2 ** 30, 3)
            if mode == "pinned":
                for b in bufs[::-1]:
                    codec.host_unregister(b)
        d_vals = vals.cpu().numpy()
        nv = got_v.size
        host_ok = bool(all(np.array_equal(got_d[f], d[f]) for f in d.dtype.names)
                       and np.array_equal(got_v, d_vals[:nv]))
        out["e2e_host"] = {"value": e2e["pinned"], "unit": "GiB/s on disk", "pageable": e2e["pageable"],
                           "decoded_GiBps_pinned": round(e2e["pinned"] * n * 1024 / disk, 3),
                           "matches_device_path": host_ok,
                           "note": "host src (%.2f GB) + handles + expected CRCs -> descriptors, value offsets and "
                                   "%.2f GB of decoded values in host memory: 64 MiB src chunks, chunk k + 1's H2D "
                                   "under chunk k's values going back (a copy kernel into the mapped out_vals when "
                                   "it is page-locked, else into page-locked staging that host threads copy on), "
                                   "caller-owned output buffers reused.  value: "
                                   "all host buffers page-locked (bhg_host_register); pageable also given"
                                   % (host_src.size / 1e9, n * 1024 / 1e9)}
        out["valid"] = bool(out["valid"] and host_ok)
    return out


def run_c4(a, world, rank, local, dev, codec):
    """BASELINE configs[3]: encode 1M pairs, values U[64, 4096] B -> record-pack + snappy + CRC.
    The line is the --values generator; the other one is nested as a secondary line."""
    res = c4_measure(a, world, rank, local, dev, codec, a.values, extras=True)
    if not a.no_secondary:
        torch.cuda.empty_cache()
        g2 = _secondary_gen(a.values)
        sec = c4_measure(a, world, rank, local, dev, codec, g2, extras=False)
        res["secondary_values_" + g2] = {k: sec[k] for k in ("value", "unit", "ms_per_step", "roofline")}
        res["secondary_values_" + g2].update(sec["config"])
    if rank == 0:
        print(json.dumps(res), flush=True)


def c4_measure(a, world, rank, local, dev, codec, gen, extras):
    from bitalosdb_amd.codec import EncodeBuffers
    n = a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(synth_seed(rank) + 7)
    val_lens = torch.randint(64, 4097, (n,), generator=g, device=dev, dtype=torch.int64)
    keys, key_off, tr, vals, val_off = _encode_inputs(n, val_lens, dev, synth_seed(rank), gen)
    cap = int(n * 64 + vals.numel() * 7 // 6 + 64)
    out_t = torch.empty(cap, dtype=torch.uint8, device=dev)
    maxt = 4096
    fns = torch.arange(1, maxt + 1, dtype=torch.int32, device=dev)
    bufs = EncodeBuffers(n, maxt, dev)
    step = lambda: codec.encode_batch(keys, key_off, tr, vals, val_off, n, 1, fns, maxt, 0, 128 << 20, out_t, bufs)
    el, kms = _timed(a, dev, step)
    raw = float(vals.numel() + n * 32)
    total = int(bufs.summary[0].item())
    res = {"metric": "GiB/s KV input encoded (record-pack + snappy + CRC), values 64B-4KB, 1 GPU",
           "value": round(raw * a.steps / el / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ramp": a.ramp_record, "ms_per_step": round(el / a.steps * 1e3, 4),
           "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic compressible values (%s)" % gen,
           "config": {"workload": "BASELINE configs[3]: 1M KV pairs -> record-pack + compress + CRC",
                      "values": gen, "pairs_per_gpu": n, "input_bytes": int(raw), "output_bytes": total,
                      "snappy_ratio": round((total - n * 52.0) / float(vals.numel()), 4),
                      "tables": int(bufs.summary[1].item())}}
    # SURVEY 8(d) C4 algorithmic bytes: read key 32 + value v + 16 B (offsets, trailer); write the
    # records (52 + c each, = output_bytes) + handle 8 + FNV 4 + CRC 4; whole step (kms = event-timed)
    alg = raw + 16.0 * n + total + 16.0 * n
    res["roofline"] = {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "traffic": None,
                       "scope": "whole step (sizes, scan, k_snappy_enc, split, pack, crc)",
                       "step_event_ms": round(kms, 4),
                       "note": "k_snappy_enc is latency bound (DESIGN.md 4.3); snappy scratch traffic excluded"}
    if extras and rank == 0 and world == 1 and not a.no_traffic:
        res["roofline"].update(traffic_fields(["--config", "c4", "--blocks", str(n), "--values", gen,
                                               "--no-secondary"],
                                              ["k_enc_sizes", "k_snappy_enc", "k_enc_split", "k_enc_tsize",
                                               "k_enc_pack", "k_enc_meta", "k_enc_class", "k_snappy_maxlen",
                                               "k_chunk_"], int(alg),
                                              "key + value + 16 B in, records + handle/FNV/CRC out per pair; the "
                                              "snappy scratch written by k_snappy_enc and read by k_enc_pack is "
                                              "extra traffic"))
    if extras and rank == 0 and world == 1 and not a.no_cpu:
        from oracle import oracle as O
        vo = val_off.cpu().numpy().astype(np.uint64)
        vb = vals.cpu().numpy()
        kb = keys.cpu().numpy()
        ko = key_off.cpu().numpy().astype(np.uint64)
        trs = tr.cpu().numpy().astype(np.uint64)
        # parity on the first 20k pairs (one restated writer, reference-definition CRC)
        m = min(n, 20000)
        ks = [kb[32 * i:32 * i + 32].tobytes() for i in range(m)]
        vs = [vb[vo[i]:vo[i + 1]].tobytes() for i in range(m)]
        exp = O.encode_batch(ks, trs[:m], vs, codec=1, file_nums=list(range(1, 100)))
        got_out = out_t.cpu().numpy()
        par = got_out[:len(exp["out"])].tobytes() == exp["out"].tobytes()
        # baseline: every usable core (independent writers over contiguous pair ranges, all n pairs,
        # repeated for ~cpu_seconds / 2), and 1 thread over the first 100k pairs
        thr = usable_cores()
        reps, t = 0, time.perf_counter()
        while True:
            O.encode_batch_mt(kb, ko, trs, vb, vo, n, 1, 128 << 20, thr)
            reps += 1
            if time.perf_counter() - t >= a.cpu_seconds / 2:
                break
        cs = time.perf_counter() - t
        m1 = min(n, 100_000)
        t = time.perf_counter()
        O.encode_batch_mt(kb, ko, trs, vb, vo, m1, 1, 128 << 20, 1)
        c1s = time.perf_counter() - t
        raw1 = float(vo[m1] - vo[0]) + 32.0 * m1
        res["cpu_baseline"] = {"value": round(raw * reps / cs / 2 ** 30, 3), "unit": "GiB/s", "cores": thr,
                               "kind": "port", "one_thread": round(raw1 / c1s / 2 ** 30, 3),
                               "sample": "restated BithashWriter.Add + golang/snappy Encode + FNV-1 + masked CRC-32C "
                                         "(SSE4.2): all %d pairs, %d passes in %.1f s on %d threads = every usable "
                                         "core, one writer per contiguous pair range; one_thread: the first %d "
                                         "pairs on 1 thread (%s)" % (n, reps, cs, thr, m1, cpu_info())}
        res["parity_first_%d" % m] = "bit-exact" if par else "MISMATCH"
    return res


def run_mixdec(a, world, rank, local, dev, codec):
    """Decode of the C4-shaped tables (SURVEY 8(d) C4 value mix: 1M pairs, values U[64, 4096] B of
    the --values generator, as BithashWriter.Add writes them): the snappy line, with the
    NoCompressor decode of the same pairs nested.  Reader.readData decodes any value length
    (reader.go:233-272); this is the shape outside the 1 KiB benchmark values."""
    out = mixdec_measure(a, world, rank, local, dev, codec, 1, extras=True)
    torch.cuda.empty_cache()
    nc = mixdec_measure(a, world, rank, local, dev, codec, 0, extras=True)
    out["nocompressor"] = {k: nc[k] for k in ("value", "unit", "ms_per_step", "roofline", "status_ok_blocks",
                                               "parity_first_blocks", "valid")}
    out["nocompressor"].update(nc["config"])
    out["valid"] = bool(out["valid"] and nc["valid"])
    if rank == 0:
        print(json.dumps(out), flush=True)


def mixdec_measure(a, world, rank, local, dev, codec, compressor, extras):
    from bitalosdb_amd.codec import handles_tensor
    n = a.blocks
    g = torch.Generator(device=dev)
    g.manual_seed(synth_seed(rank) + 7)
    val_lens = torch.randint(64, 4097, (n,), generator=g, device=dev, dtype=torch.int64)
    src, h, meta, enc = _encode_tables(codec, n, val_lens, dev, synth_seed(rank), compressor, a.values)
    exp_crc = enc[-1].crc
    h_t = handles_tensor(h, dev)
    desc = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    dec_total = int(val_lens.sum().item())
    if compressor:
        voff = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
        vals = torch.empty(dec_total + 64, dtype=torch.uint8, device=dev)
        step = lambda: codec.decode_batch(src, src.numel(), h_t, n, 1, expected_crc=exp_crc, out_desc=desc,
                                          out_vals=vals, out_val_off=voff)
    else:
        step = lambda: codec.decode_batch(src, src.numel(), h_t, n, 0, expected_crc=exp_crc, out_desc=desc)
    el, kms = _timed(a, dev, step)
    d = desc.cpu().numpy().view(DESC_DT)
    disk = float(h["length"].astype(np.float64).sum())
    lens = val_lens.cpu().numpy()
    name = "snappy" if compressor else "NoCompressor"
    out = {"metric": "GiB/s bithash blocks decoded (device-resident), %s, C4 value mix 64B-4KB, 1 GPU" % name,
           "value": round(disk * a.steps / el / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ramp": a.ramp_record, "ms_per_step": round(el / a.steps * 1e3, 4),
           "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (GPU-encoded %s tables, values: %s)" % (name, a.values),
           "config": {"workload": "decode of the C4-shaped tables: 1M pairs, 32 B keys, values U[64, 4096] B, "
                                  "CRC-verify (the writer's CRCs) + %sdecode" % ("decompress + " if compressor else ""),
                      "codec": name, "values": a.values, "blocks_per_gpu": n, "mean_record_bytes": round(disk / n, 1),
                      "decoded_value_bytes": dec_total,
                      "decoded_GiBps": round(dec_total * a.steps / el / 2 ** 30, 3)},
           "status_ok_blocks": int((d["status"] == 0).sum())}
    if compressor:
        # k_snappy_lds takes blocks that decode to <= 1 KiB (bhg_snappy_dec.hip); the rest go to k_snappy_rt
        out["config"]["blocks_decoding_over_1KiB"] = int((lens > 1024).sum())
        out["config"]["share_over_1KiB"] = round(float((lens > 1024).mean()), 4)
    out["valid"] = out["status_ok_blocks"] == n
    alg = n * (16 + 4 + 40) + disk + (dec_total if compressor else 0)
    out["roofline"] = {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                       "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                       "traffic": None, "scope": "whole step (event-timed)", "step_event_ms": round(kms, 4),
                       "algorithmic": "handle 16 + record + expected CRC 4 + descriptor 40%s per block" %
                                      (" + decoded value" if compressor else "")}
    if extras and rank == 0 and world == 1:
        # parity: the first 20k blocks against the restated decode (oracle/bithash_oracle.c)
        from oracle import oracle as O
        m = min(n, 20000)
        host = src.cpu().numpy()
        ecrc = exp_crc.cpu().numpy().view(np.uint32)
        exp, ev, eo = O.decode_batch(host, h[:m], codec=compressor, expected_crc=ecrc[:m], nthreads=usable_cores())
        par = all(np.array_equal(exp[f], d[:m][f]) for f in d.dtype.names)
        if compressor:
            got_v = vals.cpu().numpy()
            par = par and got_v[:int(eo[-1])].tobytes() == ev[:int(eo[-1])].tobytes()
        out["parity_first_blocks"] = "%s (%d blocks)" % ("bit-exact" if par else "MISMATCH", m)
        out["valid"] = bool(out["valid"] and par)
    return out


def run_bigval(a, world, rank, local, dev, codec):
    """Values past the LDS tiers (missing #2): bithash holds every KKV value over 288 B
    (internal/consts/base.go:29) up to 256 MiB (bithash/writer.go:43), and golang/snappy cuts a value
    into 64-KiB blocks (internal/compress/compress.go:67-69, 83-85).  --bigval-n values of U[4 KiB,
    256 KiB] plus 1 % of U[1 MiB, 4 MiB] (~1 GiB at the default 7,000), 32-B keys, 128 MiB tables.
    Legs, each its own timed loop: snappy encode (the BithashWriter.Add batch), snappy decode of the
    tables it wrote, and the NoCompressor decode of the same pairs.  Parity: decoded values equal
    the encoder's input byte for byte; encoded bytes equal the restated writer on the first values."""
    from bitalosdb_amd.codec import EncodeBuffers, handles_tensor, HANDLE_DT
    n = a.bigval_n
    g = torch.Generator(device=dev)
    g.manual_seed(synth_seed(rank) + 11)
    lens = torch.randint(4096, (256 << 10) + 1, (n,), generator=g, device=dev, dtype=torch.int64)
    big = torch.rand(n, generator=g, device=dev) < 0.01
    lens = torch.where(big, torch.randint(1 << 20, (4 << 20) + 1, (n,), generator=g, device=dev, dtype=torch.int64), lens)
    keys, key_off, tr, vals, val_off = _encode_inputs(n, lens, dev, synth_seed(rank), a.values)
    raw = float(vals.numel() + 32 * n)
    maxt = 4096
    fns = torch.arange(1, maxt + 1, dtype=torch.int32, device=dev)
    lens_h = lens.cpu().numpy()
    cfg = {"values": a.values, "pairs_per_gpu": n, "value_bytes": int(vals.numel()),
           "values_over_64KiB": int((lens_h > 65536).sum()), "values_1_4MiB": int((lens_h >= 1 << 20).sum()),
           "largest_value": int(lens_h.max())}
    res = {"metric": "GiB/s bithash values > 4 KiB, encode and decode (device-resident), 1 GPU",
           "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic compressible values (%s), GPU-generated" % a.values, "config": cfg}
    legs = {}
    for compressor in (1, 0):
        name = "snappy" if compressor else "NoCompressor"
        cap = int(n * 64 + vals.numel() * 7 // 6 + 64)
        out_t = torch.empty(cap, dtype=torch.uint8, device=dev)
        bufs = EncodeBuffers(n, maxt, dev)
        enc = lambda: codec.encode_batch(keys, key_off, tr, vals, val_off, n, compressor, fns, maxt, 0, 128 << 20,
                                         out_t, bufs)
        if compressor:
            el, kms = _timed(a, dev, enc)
        else:
            enc()
            codec.sync()
        total = int(bufs.summary[0].item())
        st = bufs.status.cpu().numpy().view(np.uint32)
        if compressor:
            alg = raw + 16.0 * n + total + 16.0 * n
            legs["encode_snappy"] = {
                "value": round(raw * a.steps / el / 2 ** 30, 3), "unit": "GiB/s (key + value input)",
                "ms_per_step": round(el / a.steps * 1e3, 4), "ramp": a.ramp_record,
                "output_bytes": total, "snappy_ratio": round((total - 52.0 * n) / float(vals.numel()), 4),
                "status_ok": int((st == 0).sum()),
                "roofline": {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                             "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                             "scope": "whole step (event-timed)", "step_event_ms": round(kms, 4)}}
            if rank == 0 and world == 1:
                from oracle import oracle as O
                m = min(n, 48)
                vo = val_off[:m + 1].cpu().numpy().astype(np.uint64)
                vb = vals[:int(vo[m])].cpu().numpy()
                kb = keys[:32 * m].cpu().numpy()
                ks = [kb[32 * i:32 * i + 32].tobytes() for i in range(m)]
                vs = [vb[vo[i]:vo[i + 1]].tobytes() for i in range(m)]
                exp = O.encode_batch(ks, tr[:m].cpu().numpy().astype(np.uint64), vs, codec=1,
                                     file_nums=list(range(1, 100)))
                par = out_t[:len(exp["out"])].cpu().numpy().tobytes() == exp["out"].tobytes()
                legs["encode_snappy"]["parity_first_%d_values" % m] = "bit-exact" if par else "MISMATCH"
        pos = bufs.pos.cpu().numpy().view(np.uint64)
        ln = bufs.bh_len.cpu().numpy().view(np.uint32)
        h = np.zeros(n, dtype=HANDLE_DT)
        h["offset"] = pos
        h["length"] = ln
        h_t = handles_tensor(h, dev)
        src = out_t[:total]
        desc = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        exp_crc = bufs.crc
        if compressor:
            voff = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev)
            dvals = torch.empty(vals.numel() + 64, dtype=torch.uint8, device=dev)
            dec = lambda: codec.decode_batch(src, src.numel(), h_t, n, 1, expected_crc=exp_crc, out_desc=desc,
                                             out_vals=dvals, out_val_off=voff)
        else:
            dec = lambda: codec.decode_batch(src, src.numel(), h_t, n, 0, expected_crc=exp_crc, out_desc=desc)
        el, kms = _timed(a, dev, dec)
        d = desc.cpu().numpy().view(DESC_DT)
        disk = float(h["length"].astype(np.float64).sum())
        ok = int((d["status"] == 0).sum())
        if compressor:
            par = bool(torch.equal(dvals[:vals.numel()], vals)) and ok == n
        else:  # zero-copy views: the value bytes at val_off inside each record equal the input
            vo_rec = d["val_off"].astype(np.uint64) + h["offset"]
            par = ok == n and bool(np.array_equal(d["val_len"].astype(np.int64), lens_h))
            if par:
                idx = torch.from_numpy(vo_rec.astype(np.int64)).to(dev)
                par = bool(torch.equal(src[idx], vals[val_off[:-1]]))  # first byte of every value
        alg = n * (16 + 4 + 40) + disk + (vals.numel() if compressor else 0)
        legs["decode_" + name] = {
            "value": round(disk * a.steps / el / 2 ** 30, 3), "unit": "GiB/s (on-disk records)",
            "decoded_GiBps": round(vals.numel() * a.steps / el / 2 ** 30, 3),
            "ms_per_step": round(el / a.steps * 1e3, 4), "ramp": a.ramp_record, "status_ok": ok,
            "parity": "bit-exact (values == encoder input)" if par else "MISMATCH",
            "roofline": {"bound": "hbm", "achieved": round(alg / (kms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(alg / (kms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "scope": "whole step (event-timed)", "step_event_ms": round(kms, 4)}}
        del out_t, bufs, desc
        torch.cuda.empty_cache()
    res["legs"] = legs
    res["value"] = legs["decode_snappy"]["value"]
    res["ms_per_step"] = legs["decode_snappy"]["ms_per_step"]
    res["roofline"] = legs["decode_snappy"]["roofline"]
    res["valid"] = all(v.get("parity", "bit-exact").startswith("bit-exact") for v in legs.values()) and \
        legs["encode_snappy"].get("parity_first_48_values", "bit-exact") == "bit-exact"
    if rank == 0:
        print(json.dumps(res), flush=True)


C5_RECORDS_PER_TABLE = 124_738      # 128 MiB / 1076 B, the add that crosses the limit included


def run_c5(a, world, rank, local, dev, codec):
    out = c5_measure(a, world, rank, local, dev, codec, a.codec, with_cpu=True)
    if rank == 0:
        print(json.dumps(out), flush=True)


def c5_measure(a, world, rank, local, dev, codec, codec_name, with_cpu):
    """BASELINE configs[4]: a fixed 25 GB corpus of bithash table files (184
    tables x 124,738 blocks of 32 B key / 1 KiB value), table t decoded by
    rank t mod N (round-robin by table file).  Each rank decodes
    all of its tables in one bhg_decode_batch per step (CRC verify against
    the writer's CRCs + record decode, snappy decompress for --codec snappy);
    no data-path collective.  value = corpus bytes / max-over-ranks time:
    strong scaling, every N decodes the same 25 GB."""
    import torch.distributed as dist
    from bitalosdb_amd import shard, synth
    from bitalosdb_amd.codec import handles_tensor
    T, R = a.c5_tables, C5_RECORDS_PER_TABLE
    owned = shard.owned_tables(T, world, rank)
    snappy = codec_name == "snappy"
    t_build = time.perf_counter()
    if snappy:
        src_t, h, exp_crc, raw = synth.table_set_snappy(codec, owned, R, device=dev, seed=synth.SEED, gen=a.values)
    else:
        src_t, h, meta = synth.table_set(owned, R, device=dev, seed=synth.SEED, first_file_num=1)
        raw = len(h) * 1024
    n = len(h)
    h_t = handles_tensor(h, dev)
    if not snappy:
        exp_crc = codec.crc_batch(src_t, h_t, n)
    desc_t = torch.empty(max(n, 1) * 40, dtype=torch.uint8, device=dev)
    vals_t = torch.empty(max(n, 1) * 1024 + 64, dtype=torch.uint8, device=dev) if snappy else None
    voff_t = torch.empty((n + 1) * 8, dtype=torch.uint8, device=dev) if snappy else None
    torch.cuda.synchronize(dev)
    build_s = time.perf_counter() - t_build
    disk = float(h["length"].astype(np.float64).sum())

    def step():
        if n:
            codec.decode_batch(src_t, src_t.numel(), h_t, n, 1 if snappy else 0, expected_crc=exp_crc,
                               out_desc=desc_t, out_vals=vals_t, out_val_off=voff_t)

    ramp = clock_ramp(a, dev, step)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    def barrier():
        dist_barrier(world, local)

    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    for i in range(a.steps):
        e0[i].record()
        step()
        e1[i].record()
    torch.cuda.synchronize(dev)
    step_ms = float(np.mean([x.elapsed_time(y) for x, y in zip(e0, e1)])) if n else 0.0
    d = desc_t[:n * 40].cpu().numpy().view(DESC_DT)
    ok = int((d["status"] == 0).sum())
    digest = shard.block_digest(d["crc"], d["fnv1"], d["trailer"], d["status"])
    el_max, ok_total, n_total, digest_all = shard.reduce_stats(elapsed, ok, n, digest, dev)
    dt = torch.tensor([disk, raw], dtype=torch.float64, device=dev)
    dist_sum_(dt, world)
    disk_total, raw_total = float(dt[0].item()), float(dt[1].item())
    ranks = torch.ones(1, dtype=torch.int64, device=dev)
    dist_sum_(ranks, world)          # the world size the collective backend (RCCL for N > 1) reports
    value = disk_total * a.steps / el_max / 2 ** 30
    # per-GPU roofline of this rank's step: algorithmic bytes (handle + record + descriptor + expected CRC,
    # + decoded value bytes written for snappy) over the event-timed step
    algo = n * (16 + 40 + 4) + disk + (raw if snappy else 0)
    achieved = algo / (step_ms * 1e-3) / 1e9 if step_ms else 0.0
    out = {
        "metric": "GiB/s bithash table files decoded (device-resident), 25 GB corpus sharded by table, "
                  "32B key / 1KB value",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ramp": ramp,
        "ms_per_step": round(el_max / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (per-table seeded generator: a table's bytes do not depend on N)",
        "config": {"workload": "BASELINE configs[4]: %d tables x %d blocks (%.2f GB on disk), table t -> rank t "
                               "mod %d, CRC-verify + record decode%s" % (T, R, disk_total / 1e9, world,
                                                                        " + snappy decompress" if snappy else ""),
                   "codec": codec_name, "tables": T, "tables_this_rank": len(owned), "blocks_total": int(n_total),
                   "parallelism": "table-sharded x%d" % world, "corpus_build_s": round(build_s, 2)},
        "per_gpu_GiBps": round(value / world, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None, "scope": "rank 0, per GPU",
                     "step_avg_ms": round(step_ms, 4)},
        "status_ok_blocks": int(ok_total), "valid": bool(ok_total == n_total == T * R),
        "digest_all_ranks": "%016x" % digest_all, "ranks_seen": int(ranks.item()),
        "backend": BACKEND if PG else None,
    }
    if snappy:
        out["decoded_GiBps"] = round(raw_total * a.steps / el_max / 2 ** 30, 3)
        out["config"]["values"] = a.values
    if PG:
        out.update(shard.scaling_fields(elapsed, achieved / HBM_PEAK_GBPS, dev))
    if rank == 0 and world == 1 and with_cpu and not a.no_cpu and n:
        from oracle import oracle as O
        # parity + baseline on a bounded sample: the first table (the restatement decodes it bit for bit)
        first = np.nonzero(h["offset"] >= 0)[0][:R]
        hs = h[first]
        lo = int(hs["offset"].min())
        hi = int((hs["offset"] + hs["length"]).max())
        host = src_t[lo:hi].cpu().numpy()
        hr = hs.copy()
        hr["offset"] -= np.uint64(lo)
        ecrc = exp_crc[:R].cpu().numpy().view(np.uint32)
        threads = usable_cores()
        e, _, _ = O.decode_batch(host, hr, codec=1 if snappy else 0, expected_crc=ecrc, nthreads=threads)
        dd = d[:R]
        fields = [f for f in DESC_DT.names if not (snappy and f == "val_off")]
        par = all(np.array_equal(e[f], dd[f]) for f in fields)
        reps, t = 0, time.perf_counter()
        while time.perf_counter() - t < a.cpu_seconds:
            O.decode_batch(host, hr, codec=1 if snappy else 0, expected_crc=ecrc, nthreads=threads)
            reps += 1
        cs = time.perf_counter() - t
        out["cpu_baseline"] = {"value": round(reps * (hi - lo) / cs / 2 ** 30, 3), "unit": "GiB/s", "cores": threads,
                               "kind": "port", "sample": "C restatement over table 0 (%d blocks, %d B), %d passes on "
                                                         "%d threads (%s)" % (R, hi - lo, reps, threads, cpu_info())}
        out["parity_table0_vs_restatement"] = "bit-exact" if par else "MISMATCH"
        out["valid"] = bool(out["valid"] and par)
    return out


def run_scan(a, world, rank, local, dev, codec):
    """Row A4: bhg_scan_tables (TableIterator.findEntry header chase, table.go:358-395)
    over 1M records.  scan: uniform 32 B / 1 KiB records in 128 MiB tables (C2 data);
    scanmix: values U[64, 4096] B (the C4 input, NoCompressor) -- every record a
    different length, so the window chase does all the work."""
    from bitalosdb_amd import synth
    n = a.blocks
    if a.config == "scan":
        src, h, meta = synth.uniform_tables(n, device=dev, seed=synth_seed(rank))
        tb = meta["table_bytes"]
        toff = np.array([t * tb for t in range(meta["tables"])] + [meta["src_bytes"]], dtype=np.uint64)
        what = "uniform 1076 B records, 128 MiB tables (C2 data)"
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(synth_seed(rank) + 7)
        val_lens = torch.randint(64, 4097, (n,), generator=g, device=dev, dtype=torch.int64)
        src, h, meta, bufs = _encode_tables(codec, n, val_lens, dev, synth_seed(rank), 0)
        ts = bufs[-1].table_start.cpu().numpy().view(np.uint32)[:meta["ntables"]]
        toff = np.array([int(h["offset"][i]) for i in ts] + [meta["src_bytes"]], dtype=np.uint64)
        what = "values U[64, 4096] B, raw, 128 MiB tables (C4 input)"
    ntab = len(toff) - 1
    from bitalosdb_amd.codec import _u64_tensor
    toff_t = _u64_tensor(toff, dev)
    out_h, first, end = codec.scan_tables(src, toff_t, mode=0)
    codec.sync()
    got = out_h.cpu().numpy().view(np.uint8).reshape(-1).view(np.dtype([("offset", "<u8"), ("length", "<u4"), ("pad", "<u4")]))
    par = len(got) == n and bool((got["offset"] == h["offset"]).all() and (got["length"] == h["length"]).all())
    step = lambda: codec.scan_tables(src, toff_t, mode=0, max_out=n)
    el, kms = _timed(a, dev, step)
    scanned = float(toff[-1])
    res = {"metric": "GiB/s table data regions scanned (TableIterator header chase), 1 GPU",
           "value": round(scanned * a.steps / el / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ramp": a.ramp_record, "ms_per_step": round(el / a.steps * 1e3, 4),
           "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
           "config": {"workload": "row A4 table scan: " + what, "records_per_gpu": n, "tables": ntab,
                      "bytes": int(scanned), "Mrecords_per_s": round(n * a.steps / el / 1e6, 2)},
           "parity_vs_generator_handles": "bit-exact" if par else "MISMATCH"}
    if rank == 0 and world == 1 and not a.no_cpu:
        from oracle import oracle as O
        host = src.cpu().numpy()
        t = time.perf_counter()
        done = 0
        for ti in range(ntab):
            O.scan_region(host[int(toff[ti]):int(toff[ti + 1])], mode=0, max_records=n)
            done += int(toff[ti + 1] - toff[ti])
            if time.perf_counter() - t > a.cpu_seconds:
                break
        cs = time.perf_counter() - t
        res["cpu_baseline"] = {"value": round(done / cs / 2 ** 30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": "bho_scan_region over %d B of the same tables, 1 thread (%s)"
                                         % (done, cpu_info())}
    if rank == 0:
        print(json.dumps(res), flush=True)


def run_indexcrc(a, world, rank, local, dev, codec):
    """Row A6(ii): verify the indexhash_checksum of one GPU's share of the C5
    tables -- 23 tables (184 / 8), indexhash_data 1,510,000 B each (SURVEY
    8(d): 8 + 65536*4 + 10*124,738 B).  bhg_crc32c_masked_long (one workgroup
    per range) against bhg_crc32c_masked_batch (one lane per range), both
    checked against the restatement."""
    from bitalosdb_amd.codec import handles_tensor
    from oracle import oracle as O
    ntab, ln = 23, 8 + 65536 * 4 + 10 * 124738
    g = torch.Generator(device="cpu").manual_seed(0xB17A105DB + rank)
    host = torch.randint(0, 256, (ntab * ln,), dtype=torch.uint8, generator=g)
    src_t = host.to(dev)
    h = np.zeros(ntab, dtype=O.HANDLE_DT)
    h["offset"] = np.arange(ntab, dtype=np.uint64) * ln
    h["length"] = ln
    h_t = handles_tensor(h, dev)

    def timed(fn, steps):
        for _ in range(a.warmup):
            fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / steps, out

    t_long, got = timed(lambda: codec.crc_long(src_t, h_t, ntab), a.steps)
    t_lane, got2 = timed(lambda: codec.crc_batch(src_t, h_t, ntab), 2)
    hb = host.numpy().tobytes()
    exp = np.array([O.crc_masked(hb[i * ln:(i + 1) * ln]) for i in range(ntab)], dtype=np.uint32)
    got = got.cpu().numpy().view(np.uint32)
    got2 = got2.cpu().numpy().view(np.uint32)
    t0 = time.perf_counter()
    for i in range(ntab):
        O.crc_masked(hb[i * ln:(i + 1) * ln])
    t_cpu = time.perf_counter() - t0
    if rank == 0:
        out = {"metric": "GiB/s indexhash_data CRC-verified (per-table indexhash_checksum), 1 GPU",
               "value": round(ntab * ln / t_long / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": round(t_long * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic random indexhash bytes",
               "config": {"workload": "row A6(ii): 23 tables x 1,510,000 B indexhash_data (one GPU of C5)",
                          "kernel": "k_crc_long"},
               "lane_per_range_ms": round(t_lane * 1e3, 3),
               "parity_vs_restatement": "bit-exact" if (np.array_equal(got, exp) and np.array_equal(got2, exp))
               else "MISMATCH",
               "cpu_baseline": {"value": round(ntab * ln / t_cpu / 2 ** 30, 3), "unit": "GiB/s", "cores": 1,
                                "kind": "port", "sample": "C restatement (bytewise table CRC-32C, bho_crc_masked) over the same 23 ranges, %s"
                                % cpu_info()}}
        print(json.dumps(out))
    return 0


def run_tail(a, world, rank, local, dev, codec):
    """Rows A10 / f2: bhg_table_tail (conflict block, HashIndex, indexhash checksum, meta, footer)
    for 1M 32 B / 1 KiB records: as 8 tables of 128 MiB, and as one table holding all 1M records
    (its ~1M 32-bit khashes collide naturally: the conflict-run and dedupe kernels get work)."""
    from bitalosdb_amd import synth
    from bitalosdb_amd.codec import handles_tensor
    n = a.blocks
    res = {"metric": "ms per Writer.writeTable tail batch (bhg_table_tail), 1M records, 1 GPU", "unit": "ms",
           "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "higher_is_better": False, "scaling": "weak",
           "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform 32 B / 1 KiB records)"}
    for label, tmax in (("tables_128MiB", 128 << 20), ("one_table", 1 << 62)):
        src_t, h, meta = synth.uniform_tables(n, device=dev, seed=synth_seed(rank), table_max=tmax)
        h_t = handles_tensor(h, dev)
        d = codec.decode_batch(src_t, src_t.numel(), h_t, n)
        R, L = meta["records_per_table"], meta["rec_len"]
        i = torch.arange(n, device=dev, dtype=torch.int64)
        bh_off = ((i % R) * L).to(torch.int32)
        table = (i // R).to(torch.int32)
        fnv = d.desc.view(-1, 40)[:, 28:32].contiguous().view(torch.int32).reshape(-1)
        nt = meta["tables"]
        counts = [min(n, (t + 1) * R) - t * R for t in range(nt)]
        data_end = torch.tensor([c * L for c in counts], dtype=torch.int64, device=dev)
        tail, toff, tlen, stats = codec.table_tail(src_t, h_t, bh_off, fnv, table, None, n, nt, data_end)
        cap = int(toff[nt].item())
        el, kms = _timed(a, dev, lambda: codec.table_tail(src_t, h_t, bh_off, fnv, table, None, n, nt, data_end,
                                                          tail_cap=cap))
        st = stats.view(-1, 4).cpu().numpy()
        res[label] = {"tables": nt, "records": n, "ms_per_tail_batch": round(el / a.steps * 1e3, 4),
                      "event_ms": round(kms, 4), "conflict_keys": int(st[:, 1].sum()),
                      "index_items": int(st[:, 0].sum()), "tail_bytes": cap}
        del src_t, h_t, d, tail
        torch.cuda.empty_cache()
    res["value"] = res["one_table"]["ms_per_tail_batch"]
    res["ms_per_step"] = res["value"]
    res["config"] = {"workload": "row A10 / f2: table tail of 1M records (value = the one-table case)"}
    if rank == 0:
        print(json.dumps(res), flush=True)


def run_get(a, world, rank, local, dev, codec):
    """Batched point reads over complete .bht tables (row A12 + A11 + A2):
    1M random existing keys -> bhg_get_batch (FNV-1, HashIndex.Get64, conflict
    SeekGE) -> bhg_decode_batch (readData) on the returned handles."""
    import torch.distributed as dist
    from bitalosdb_amd import synth
    from bitalosdb_amd._lib import TABLE_DT
    n = a.blocks
    src_t, tabs, h, meta = synth.full_tables(codec, n, seed=synth.SEED + rank, first_file_num=1 + rank * 1000)
    R = meta["records_per_table"]
    rng = np.random.default_rng(7 + rank)
    q = rng.permutation(n).astype(np.int64)
    qt = torch.from_numpy(q).to(dev)
    off_t = torch.from_numpy(h["offset"].astype(np.int64)).to(dev)
    kpos = (off_t[qt] + 12).unsqueeze(1) + torch.arange(32, device=dev).unsqueeze(0)
    kb_t = src_t[kpos.reshape(-1)].contiguous()
    ko_t = torch.arange(0, 32 * n + 1, 32, dtype=torch.int64, device=dev)
    ti_t = torch.from_numpy((q // R).astype(np.int32)).to(dev)
    tab_t = torch.from_numpy(tabs.view(np.uint8).copy()).to(dev)
    out_h = torch.empty(2 * n, dtype=torch.int64, device=dev)
    out_s = torch.empty(n, dtype=torch.int32, device=dev)
    desc_t = torch.empty(n * 40, dtype=torch.uint8, device=dev)
    L = meta["rec_len"]

    def step(ev=None):
        codec.get_batch_dev(src_t, tab_t, len(tabs), kb_t, ko_t, ti_t, None, n, out_h, out_s)
        if ev is not None:
            ev.record()
        codec.decode_batch(src_t, src_t.numel(), out_h, n, out_desc=desc_t)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    e2 = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    dist_barrier(world, local)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        e0[i].record()
        step(e1[i])
        e2[i].record()
    torch.cuda.synchronize(dev)
    dist_barrier(world, local)
    elapsed = time.perf_counter() - t0
    get_ms = float(np.mean([x.elapsed_time(y) for x, y in zip(e0, e1)]))
    dec_ms = float(np.mean([x.elapsed_time(y) for x, y in zip(e1, e2)]))
    st = out_s.cpu().numpy()
    d = desc_t.view(-1, 40).cpu().numpy().reshape(-1).view(DESC_DT)
    seq_ok = bool(((d["trailer"] >> 8) == (q + 1).astype(np.uint64)).all())
    from bitalosdb_amd import shard
    elapsed, ok_total, n_total, _ = shard.reduce_stats(elapsed, int((st == 0).sum()), n, 0, dev)
    out = {
        "metric": "M Bithash.Get/s (batched HashIndex lookup + conflict SeekGE + readData), 32B key / 1KB value",
        "value": round(n_total * a.steps / elapsed / 1e6, 3), "unit": "Mget/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (full .bht tables, random key order)",
        "config": {"workload": "row A12: 1M random existing keys over %d tables of 128 MiB" % len(tabs),
                   "queries_per_gpu": n, "tables": len(tabs), "conflict_blocks": int((tabs["conflict_bh_len"] > 0).sum())},
        "kernels_ms": {"k_get": round(get_ms, 4), "decode": round(dec_ms, 4)},
        "value_GiBps": round(n_total * a.steps * L / elapsed / 2 ** 30, 3),
        "status_ok": int(ok_total), "every_get_returned_its_own_record": seq_ok,
    }
    if rank == 0 and world == 1 and not a.no_cpu:
        from oracle import table as T
        host = src_t.cpu().numpy()
        files = []
        for t in range(len(tabs)):
            b0 = int(tabs["base"][t])
            files.append(host[b0:b0 + meta["table_files"][t]].tobytes())
        from oracle import oracle as O
        opened = [T.open_table(f) for f in files]
        m = 20000
        kb = kb_t[:32 * m].cpu().numpy().tobytes()
        tsec = time.perf_counter()
        for i in range(m):
            t = int(q[i] // R)
            key = kb[32 * i:32 * i + 32]
            v = T.hash_index_get64(opened[t]["index_data"], O.fnv32(key))
            T._read_data(files[t], (v & 0xFFFFFFFF, v >> 32), 0)
        cpu_s = time.perf_counter() - tsec
        out["cpu_baseline"] = {"value": round(m / cpu_s / 1e6, 6), "unit": "Mget/s", "cores": 1, "kind": "port",
                               "sample": "%d gets through the Python restatement of HashIndex.Get64 + readData over "
                                         "opened in-memory tables, 1 thread (%s)" % (m, cpu_info())}
    if rank == 0:
        print(json.dumps(out), flush=True)


def synth_seed(rank):
    from bitalosdb_amd import synth
    return synth.SEED + rank


if __name__ == "__main__":
    main()
