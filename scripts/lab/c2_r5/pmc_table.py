"""Average of every counter per kernel over a rocprofv3 --pmc output tree (lab helper).
usage: pmc_table.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ks = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
last = None
for (k, c), v in sorted(acc.items()):
    if k != last:
        print(k)
        last = k
    print("   %-28s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
