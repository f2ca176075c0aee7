#!/bin/bash
# round-2 session-3 measurement run: GPU tests + smoke, C2 at the driver's warm-up and at 100,
# C3 / C4 / C5 (none, snappy) / Get legs, then rocprofv3 kernel stats + PMC of the C2 command
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r2s3v}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -2 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_c2_w5.json 2> $O/bench_c2_w5.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-e2e > $O/bench_c2_w100.json 2> $O/bench_c2_w100.err || exit 1
for c in c3 c4 get; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 300 python -u bench.py --config c5 --codec none > $O/bench_c5_none.json 2> $O/bench_c5_none.err || exit 1
timeout -k 10 300 python -u bench.py --config c5 --codec snappy --steps 3 --warmup 2 > $O/bench_c5_snappy.json 2> $O/bench_c5_snappy.err || exit 1
scripts/profile_bench.sh ${1:-r2s3v}_prof --warmup 5 --no-cpu --no-e2e || exit 1
for f in $O/bench_*.json; do python -c "
import json; d=json.load(open('$f')); r=d.get('roofline',{})
print('$f'.split('/')[-1], d['value'], d['unit'], d['ms_per_step'], r.get('frac'), r.get('kernel_avg_ms'), d.get('valid'))"; done
