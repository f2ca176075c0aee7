#!/usr/bin/env python
"""Per-launch HBM traffic of one kernel from scripts/profile_bench.sh output.

FETCH_SIZE x2 (gfx950 counts wide streaming reads at half their bytes,
/opt/skills/guides/MI355X_MICROARCH.md "HBM / rocprofv3"), WRITE_SIZE x1,
KiB -> bytes; plus the kernel's average duration from the trace pass.
usage: scripts/pmc_summary.py <gpurun_out/tag> <kernel-name-substring> [out.json] [--grid N]
(--grid keeps only dispatches of that total grid size in work-items, e.g. the
bench's main launches, not the end-to-end leg's chunk launches)"""
import csv
import glob
import json
import sys


def rows(pattern):
    for f in glob.glob(pattern, recursive=True):
        yield from csv.DictReader(open(f))


def main():
    args = [a for a in sys.argv[1:]]
    grid = None
    if "--grid" in args:
        k = args.index("--grid")
        grid = int(args[k + 1])
        del args[k:k + 2]
    d, kname = args[0], args[1]
    vals = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v = [float(r["Counter_Value"]) for r in rows(d + "/pmc_%s/**/*counter_collection.csv" % c)
             if kname in r["Kernel_Name"] and r["Counter_Name"] == c and (grid is None or int(r["Grid_Size"]) == grid)]
        vals[c] = (sum(v) / len(v), len(v)) if v else (None, 0)
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows(d + "/trace/**/*kernel_trace.csv")
            if kname in r["Kernel_Name"] and (grid is None or
                                              int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) == grid)]
    fetch, wr = vals["FETCH_SIZE"][0], vals["WRITE_SIZE"][0]
    out = {"kernel": kname, "launches": [vals["FETCH_SIZE"][1], vals["WRITE_SIZE"][1]],
           "fetch_size_kib": fetch, "write_size_kib": wr,
           "read_bytes_per_launch": None if fetch is None else fetch * 1024 * 2,
           "write_bytes_per_launch": None if wr is None else wr * 1024,
           "hbm_bytes_per_launch": None if fetch is None or wr is None else fetch * 2048 + wr * 1024,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1; KiB -> bytes",
           "trace_launches": len(durs), "trace_avg_ms": (sum(durs) / len(durs) / 1e6) if durs else None,
           "trace_min_ms": (min(durs) / 1e6) if durs else None, "grid_filter": grid, "source": d}
    s = json.dumps(out, indent=1)
    print(s)
    if len(args) > 2:
        open(args[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
