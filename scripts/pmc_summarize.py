#!/usr/bin/env python
"""Summarise rocprofv3 --pmc passes (FETCH_SIZE pass, WRITE_SIZE pass) for one
kernel into the per-launch HBM-traffic JSON that bench.py reports as
roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
reports half the bytes of a wide streaming read -> x2; WRITE_SIZE is exact for
16 B/lane stores.  Both counters are in KiB.

usage: scripts/pmc_summarize.py <fetch_csv> <write_csv> <kernel-substring> <out.json> [note]
"""
import csv
import json
import sys


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit("no %s rows for %r in %s" % (counter, kernel, path))
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    note = sys.argv[5] if len(sys.argv) > 5 else ""
    f_kib, nf = per_launch(fetch_csv, kernel, "FETCH_SIZE")
    w_kib, nw = per_launch(write_csv, kernel, "WRITE_SIZE")
    read_b = f_kib * 1024 * 2
    write_b = w_kib * 1024
    rec = {"kernel": kernel, "launches": [nf, nw], "fetch_size_kib": f_kib, "write_size_kib": w_kib,
           "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": read_b + write_b,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1; KiB -> bytes",
           "note": note}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
