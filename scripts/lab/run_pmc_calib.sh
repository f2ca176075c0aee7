#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-calib}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/p1 -o run --output-format csv -- ./scripts/lab/pmc_calib > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
cat $O/run.log | tail -2
python3 - "$O" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p1/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE": d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print("%-12s launches %d  FETCH_SIZE %.1f KiB = %.1f MB per launch (median)" % (k, len(v), sorted(v)[len(v)//2], sorted(v)[len(v)//2] * 1024 / 1e6))
PY
