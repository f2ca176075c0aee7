#!/bin/bash
# round-4 last tree (after the snappy host pipeline): all GPU tests + smoke, the driver's default
# line (--warmup 5), the self-spawned 2-rank gloo rehearsal, the C3 line with its e2e_host leg,
# and rocprofv3 kernel stats of the default line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4final4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_c2_w5.json 2> $O/bench_c2_w5.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --warmup 5 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || exit 1
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
for f in $O/bench_*.json; do python -c "
import json; d=json.load(open('$f')); r=d.get('roofline',{})
print('$f'.split('/')[-1], d['n_gpus'], d['value'], d['unit'], d['ms_per_step'], r.get('frac'), d.get('valid'), d.get('e2e_host',{}).get('value'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c2 -o run --output-format csv \
  -- python3 bench.py --warmup 5 --no-cpu --no-e2e --no-c5 --no-traffic > $O/prof_c2.json 2> $O/prof_c2.err || { echo "rocprof failed"; exit 1; }
f=$(find $O/prof_c2 -name "*kernel_stats.csv" | head -1); cp $f $O/c2_kernel_stats.csv && rm -rf $O/prof_c2
head -3 $O/c2_kernel_stats.csv
