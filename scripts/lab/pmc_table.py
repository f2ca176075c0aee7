#!/usr/bin/env python
"""Print mean per-dispatch counter values per kernel from rocprofv3 --pmc CSV dirs.
usage: scripts/lab/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][-60:]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
