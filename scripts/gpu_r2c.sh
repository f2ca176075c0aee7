#!/bin/bash
# GPU tests + smoke + default bench at the driver's warm-up (5) and at 100
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r2c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_w5.json 2> $O/bench_w5.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e > $O/bench_w100.json 2> $O/bench_w100.err || exit 1
python -c "
import json
for f in ['bench_w5','bench_w100']:
    d=json.load(open('$O/'+f+'.json'))
    print(f, d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])
"
