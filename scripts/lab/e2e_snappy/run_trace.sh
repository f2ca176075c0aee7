#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
rm -rf $O/tr2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/tr2 -o run -- python3 -u scripts/lab/e2e_snappy/e2e_trace.py > $O/trace2_run.txt 2>&1; rc=$?
grep "call" $O/trace2_run.txt
python3 - <<'PY'
import csv, glob
O = "gpurun_out/e2e_snappy/tr2"
api = list(csv.DictReader(open(glob.glob(O + "/*hip_api_trace.csv")[0])))
keep = [r for r in api if r["Function"] in ("hipMemcpyAsync", "hipEventSynchronize", "hipEventRecord", "hipStreamSynchronize", "hipLaunchKernel", "hipMemsetAsync", "hipModuleLaunchKernel", "hipExtLaunchKernel")]
with open(O + "/../api_small.csv", "w") as f:
    w = csv.writer(f)
    w.writerow(["Function", "Thread_Id", "Start_Timestamp", "End_Timestamp"])
    for r in keep:
        w.writerow([r["Function"], r["Thread_Id"], r["Start_Timestamp"], r["End_Timestamp"]])
print(len(api), len(keep))
PY
rm -f $O/tr2/*hip_api_trace.csv
exit $rc
