#!/bin/bash
# whole-batch snappy host path (unsorted handles) with the copy kernel: tests, then timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_c_client.py -m gpu -x -v -k "host or client" --timeout 120 --timeout-method thread > $O/pytest_host3.txt 2>&1; rc=$?
tail -3 $O/pytest_host3.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u scripts/lab/e2e_snappy/e2e_trace.py shuffle > $O/e2e_unsorted.txt 2>&1 || exit 1
grep call $O/e2e_unsorted.txt
