#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
rm -rf $O/tr3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/lab/e2e_snappy/e2e_trace_c2.py > $O/c2_e2e_plain.txt 2>&1 || exit 1
grep call $O/c2_e2e_plain.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr3 -o run -- python3 -u scripts/lab/e2e_snappy/e2e_trace_c2.py > $O/trace3_run.txt 2>&1; rc=$?
grep "call" $O/trace3_run.txt
exit $rc
