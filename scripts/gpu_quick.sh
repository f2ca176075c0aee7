#!/bin/bash
# quick validation of the current tree: GPU tests + smoke + the driver's default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-quick}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -2 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_c2_w5.json 2> $O/bench_c2_w5.err || exit 1
cat $O/bench_c2_w5.json
