"""Table-file sharding over the GPUs of one node.

Bithash tables (`<fileNum>.bht`) are immutable and self-contained, so decode
shards by table file with no data-path exchange: table t is owned by rank
t mod world (round-robin).  The only collective is a final reduction of
counters / timing over RCCL (backend "nccl") -- or gloo in the CPU tests.
"""
import numpy as np
import torch
import torch.distributed as dist


def table_owner(table_index, world):
    return table_index % world


def owned_tables(ntables, world, rank):
    return [t for t in range(ntables) if table_owner(t, world) == rank]


def shard_handles(handles, table_of_handle, world, rank):
    """Handles (HANDLE_DT array) whose table index belongs to `rank`."""
    mask = (np.asarray(table_of_handle) % world) == rank
    return handles[mask]


def block_digest(crc, fnv1, trailer, status):
    """Order- and partition-independent digest of decoded blocks: the 64-bit mix
    of each block's (crc, fnv1, trailer, status), summed as two independent
    32-bit lanes mod 2^32 -- per-rank digests add up (reduce_stats) to the
    single-process digest of the same blocks."""
    m = (np.asarray(crc, np.uint64) * np.uint64(0x9E3779B97F4A7C15)) ^ \
        (np.asarray(fnv1, np.uint64) << np.uint64(17)) ^ np.asarray(trailer, np.uint64) ^ \
        (np.asarray(status, np.uint64) << np.uint64(40))
    m = m * np.uint64(0xBF58476D1CE4E5B9)
    m ^= m >> np.uint64(31)
    lo = int((m & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64)) & 0xFFFFFFFF
    hi = int((m >> np.uint64(32)).sum(dtype=np.uint64)) & 0xFFFFFFFF
    return lo | (hi << 32)


def reduce_stats(elapsed_s, ok_blocks, n_blocks, digest, device):
    """MAX of elapsed, SUM of block counts, per-rank digests added as two 32-bit
    lanes mod 2^32 (block_digest); returns python values.  Runs outside the timed region."""
    multi = dist.is_available() and dist.is_initialized()  # a world of one too (the RCCL rehearsal)
    if multi and dist.get_backend() == "gloo":
        device = "cpu"   # gloo reduces host tensors
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    c = torch.tensor([ok_blocks, n_blocks, digest & 0xFFFFFFFF, digest >> 32], dtype=torch.int64, device=device)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    c = c.cpu().tolist()
    return float(t.item()), int(c[0]), int(c[1]), (int(c[2]) & 0xFFFFFFFF) | ((int(c[3]) & 0xFFFFFFFF) << 32)


def gather_floats(values, device):
    """Every rank's list of floats (all_gather; gloo through host tensors), rank order."""
    multi = dist.is_available() and dist.is_initialized()  # a world of one too (the RCCL rehearsal)
    if multi and dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if not multi:
        return [t.cpu().tolist()]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def scaling_fields(elapsed_s, frac, device):
    """Fields that make an N > 1 line self-describing: which N = 1 record its
    speed-up is taken against, every rank's timed elapsed (max / min: the imbalance of the
    round-robin table split) and every rank's roofline fraction."""
    g = gather_floats([elapsed_s, frac], device)
    el = [r[0] for r in g]
    return {"base_n1": "strong_c5",
            "speedup_rule": "speed-up at N = this line's value / the N = 1 BENCH line's nested strong_c5.value "
                            "(the same fixed corpus on one GPU), never / its top-level value (the 1M-block C2 batch)",
            "rank_elapsed_s": {"max": round(max(el), 6), "min": round(min(el), 6),
                               "imbalance": round(max(el) / min(el), 4) if min(el) > 0 else None,
                               "per_rank": [round(x, 6) for x in el]},
            "per_gpu_frac": [round(r[1], 4) for r in g]}
