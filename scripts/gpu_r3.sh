#!/bin/bash
# round-3 GPU run: GPU tests (C5 full corpus + bit-31 addresses included) + smoke,
# the default bench line (C2 + nested strong_c5 + c1), the self-spawned 2-rank
# path rehearsed with gloo on the one GPU, C3 / C4 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_c2_w5.json 2> $O/bench_c2_w5.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --warmup 5 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || exit 1
for c in c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
for f in $O/bench_*.json; do python -c "
import json; d=json.load(open('$f')); r=d.get('roofline',{})
print('$f'.split('/')[-1], d['n_gpus'], d['value'], d['unit'], d['ms_per_step'], r.get('frac'), d.get('valid'), d.get('strong_c5',{}).get('value'))"; done
