"""N>1 path on CPU: world_size-2 gloo runs of the C5 sharding bench.py uses
over RCCL on the GPU node -- round-robin table ownership, each rank decoding
its own tables (the C restatement stands in for the GPU here), and the
MAX-time / SUM-count / digest reduction, which must equal one process
decoding every table."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from bitalosdb_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ntables = 9
    mine = shard.owned_tables(ntables, world, rank)
    # 100 blocks per table; each rank "decodes" its tables
    handles = np.zeros(ntables * 100, dtype=[("offset", "<u8"), ("length", "<u4"), ("pad", "<u4")])
    tab = np.repeat(np.arange(ntables), 100)
    sub = shard.shard_handles(handles, tab, world, rank)
    el, ok, n, dg = shard.reduce_stats(0.5 + rank, len(sub), len(sub), 1000 + rank, torch.device("cpu"))
    q.put((rank, mine, len(sub), el, ok, n, dg))
    dist.destroy_process_group()


N_TABLES, R = 9, 300


def _decode_digest(table_ids):
    """Materialise tables `table_ids` of the fixed corpus on the CPU and decode
    them with the restatement: (ok blocks, n blocks, digest)."""
    import torch
    from bitalosdb_amd import synth
    from oracle import oracle as O
    src, h, meta = synth.table_set(table_ids, R, key_len=32, val_len=200, device="cpu")
    d, _, _ = O.decode_batch(src.numpy(), h)
    return int((d["status"] == 0).sum()), len(h), shard.block_digest(d["crc"], d["fnv1"], d["trailer"], d["status"])


def _c5_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.owned_tables(N_TABLES, world, rank)
    ok, n, dg = _decode_digest(mine)
    el, ok_all, n_all, dg_all = shard.reduce_stats(0.25 * (rank + 1), ok, n, dg, torch.device("cpu"))
    q.put((rank, mine, n, el, ok_all, n_all, dg_all))
    dist.destroy_process_group()


def test_world2_gloo_c5_decode_digest():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_c5_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(2))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ok1, n1, dg1 = _decode_digest(list(range(N_TABLES)))         # one process, every table
    (r0, m0, nr0, el0, oka, na, dga), (r1, m1, nr1, el1, okb, nb, dgb) = res
    assert m0 == [0, 2, 4, 6, 8] and m1 == [1, 3, 5, 7]
    assert nr0 == 5 * R and nr1 == 4 * R
    assert el0 == el1 == 0.5
    assert oka == okb == ok1 == n1 == na == nb == N_TABLES * R
    assert dga == dgb == dg1


def test_world2_gloo_sharding():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (r0, m0, s0, el0, ok0, n0, d0), (r1, m1, s1, el1, ok1, n1, d1) = res
    assert m0 == [0, 2, 4, 6, 8] and m1 == [1, 3, 5, 7]
    assert s0 == 500 and s1 == 400
    assert el0 == el1 == 1.5                      # max over ranks
    assert ok0 == ok1 == n0 == n1 == 900          # sum over ranks
    assert d0 == d1 == 2001


def test_single_process_reduce():
    import torch
    el, ok, n, dg = shard.reduce_stats(1.25, 7, 8, (5 << 32) | 9, torch.device("cpu"))
    assert (el, ok, n, dg) == (1.25, 7, 8, (5 << 32) | 9)


def test_world1_group_runs_the_collectives():
    """bench.py's one-rank rehearsal (BHG_BENCH_PG1=1) keeps a process group of one up, and the
    shard reductions must run through it (not be skipped as 'single process') and return the
    rank's own values; here on gloo, on the GPU box on RCCL (profiles/r5/pg1/)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q))
    p.start()
    r, mine, s, el, ok, n, dg = q.get(timeout=120)
    p.join(60)
    assert p.exitcode == 0
    assert mine == list(range(9)) and s == 900
    assert (el, ok, n, dg) == (0.5, 900, 900, 1000)


def _bench(args, env_extra=None, timeout=180):
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, cwd=root,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_self_spawn_world2():
    """`bench.py --gpus 2` with no outer launcher (how the driver runs it): bench.py starts
    the two rank processes itself, they rendezvous over gloo and all-reduce, and rank 0's
    JSON line reports n_gpus 2 and ranks_seen 2 (--config spawncheck: the launch path
    without a GPU; the GPU lines run the same spawn_ranks / main code first)."""
    import json
    r = _bench(["--gpus", "2", "--backend", "gloo", "--config", "spawncheck"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    sf = d.pop("scaling_fields")
    assert d == {"config": "spawncheck", "n_gpus": 2, "ranks_seen": 2, "rank_sum": 1, "spawned": True}
    # the N > 1 line's self-describing fields (shard.scaling_fields, shared with c5_measure)
    assert sf["base_n1"] == "strong_c5" and "strong_c5" in sf["speedup_rule"]
    assert sf["rank_elapsed_s"]["per_rank"] == [1.0, 1.5]
    assert sf["rank_elapsed_s"]["max"] == 1.5 and sf["rank_elapsed_s"]["min"] == 1.0
    assert sf["rank_elapsed_s"]["imbalance"] == 1.5 and sf["per_gpu_frac"] == [0.5, 0.5]


def test_bench_gpus_must_match_world_size():
    """--gpus N under an outer launcher whose WORLD_SIZE differs is an error (exit 2)."""
    r = _bench(["--gpus", "2", "--config", "spawncheck"], {"WORLD_SIZE": "3", "RANK": "0"}, timeout=120)
    assert r.returncode == 2 and "--gpus 2 but WORLD_SIZE 3" in r.stderr
