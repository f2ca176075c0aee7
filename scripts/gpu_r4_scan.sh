#!/bin/bash
# scan change: all GPU tests, then the tail / c3 / c4 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4scan}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
for c in tail c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --no-secondary > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
done
python -c "
import json
d=json.load(open('$O/bench_tail.json')); print('tail 9 tables', d['tables_128MiB']['ms_per_tail_batch'], 'one table', d['one_table']['ms_per_tail_batch'])
for c in ('c3','c4'):
    d=json.load(open('$O/bench_'+c+'.json')); print(c, d['value'], d['ms_per_step'])"
