#!/bin/bash
# round-4 validation call: every GPU test (ADVICE fixes, the 8(d) generator at full size), then
# the C3 / C4 lines on both value generators (traffic measured in the run).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for c in c3 c4; do
  timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_$c.json')); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], r['frac'], r.get('traffic_ratio'), d['config'].get('snappy_ratio'), d.get('valid'), [ (k, v['value'], v['snappy_ratio']) for k, v in d.items() if k.startswith('secondary')])"
done
