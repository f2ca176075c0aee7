#!/bin/bash
# round 6 GPU calls: TESTS (pytest files), SMOKE=1, AB=<n> (C2 --warmup 5 vs 100, with and without
# the clock ramp, n alternations), BENCH="<args>" (one extra bench line), PROF="<bench args>" (rocprof stats),
# ABENV=<var> ABARGS="<bench args>" ABN=<n>: the bench line with <var>=0 and =1, n alternations
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6/${TAG:-run}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python3 -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
  tail -3 $O/pytest.txt
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
if [ -n "$AB" ]; then
  for r in $(seq 1 $AB); do
    for v in "5 300" "100 300" "5 0" "100 0"; do
      set -- $v
      f=$O/ab_w$1_r$2_$r.json
      timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup $1 --ramp-ms $2 --no-cpu --no-e2e --no-traffic --no-c5 > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.load(open('$f')); print('w=$1 ramp=$2 run $r', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
    done
  done
fi
if [ -n "$BENCH" ]; then
  i=0
  while IFS= read -r args; do
    [ -z "$args" ] && continue
    i=$((i+1))
    f=$O/bench_$i.json
    timeout -k 10 400 python3 -u bench.py $args > $f 2> $f.err || { tail -20 $f.err; exit 1; }
    echo "bench $i ($args): $(tail -c 600 $f)"
  done <<< "$BENCH"
fi
if [ -n "$ABENV" ]; then
  for r in $(seq 1 ${ABN:-3}); do
    for v in ${ABVALS:-0 1}; do
      f=$O/abenv_${v}_$r.json
      env $ABENV=$v timeout -k 10 300 python3 -u bench.py $ABARGS > $f 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 -c "import json; d=json.load(open('$f')); print('$ABENV=$v run $r', d['value'], d['ms_per_step'])"
    done
  done
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $PROF > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
  head -12 $O/kernel_stats.csv | cut -c1-200
fi
echo done
