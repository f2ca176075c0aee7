#!/bin/bash
# snappy decode walk change: decode / full-size / C5 tests (default build), then C3 A/B over scripts/lab/libvar builds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4c3b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/lab/run_c3var.sh ${1:-r4c3b}/var
