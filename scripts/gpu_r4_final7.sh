#!/bin/bash
# round-4 last tree, every leg: all GPU tests + smoke, the driver's default line (--warmup 5:
# C2 + nested strong_c5 + c1), the self-spawned 2- and 4-rank gloo rehearsals, C3 / C4 / C5-snappy /
# Get / indexcrc / tail lines, rocprofv3 kernel stats of C2 / C3 / C4 (no counter passes: the
# device kernels are those of gpu_r4_final2.sh's run)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4final7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> $O/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --warmup 5 > $O/bench_c2_w5.json 2> $O/bench_c2_w5.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --warmup 5 > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err || exit 1
timeout -k 10 400 python -u bench.py --gpus 4 --backend gloo --warmup 5 > $O/bench_g4_gloo.json 2> $O/bench_g4_gloo.err || exit 1
for c in c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
timeout -k 10 300 python -u bench.py --config c5 --codec snappy --no-cpu > $O/bench_c5_snappy.json 2> $O/bench_c5_snappy.err || { echo "bench c5 snappy failed"; exit 1; }
for c in get indexcrc tail; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; exit 1; }
done
for f in $O/bench_*.json; do python -c "
import json; d=json.load(open('$f')); r=d.get('roofline',{})
print('$f'.split('/')[-1], d['n_gpus'], d['value'], d['unit'], d['ms_per_step'], r.get('frac'), r.get('traffic_ratio'), d.get('valid'), d.get('strong_c5',{}).get('value'))"; done
for c in c2 c3 c4; do
  w=""; [ $c = c2 ] && w="--warmup 5"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$c -o run --output-format csv \
    -- python3 bench.py --config $c $w --no-cpu --no-e2e --no-c5 --no-traffic --no-secondary > $O/prof_$c.json 2> $O/prof_$c.err || { echo "rocprof $c failed"; tail -5 $O/prof_$c.err; exit 1; }
  f=$(find $O/prof_$c -name "*kernel_stats.csv" | head -1); cp $f $O/${c}_kernel_stats.csv && rm -rf $O/prof_$c
done
echo "rocprof ok"
du -sh $O
