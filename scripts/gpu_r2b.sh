#!/bin/bash
# round-2 session-2 first GPU run: GPU tests + smoke, stream-kernel lab, default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r2b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
LAB_EXPECTED=1 timeout -k 10 120 scripts/lab/stream_lab 30 all > $O/stream_lab.txt 2>&1 || exit 1
LAB_EXPECTED=1 timeout -k 10 120 scripts/lab/stream_lab 30 stream_c4 1 > $O/stream_lab_shuffled.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_w5.json 2> $O/bench_w5.err || exit 1
echo done
