#!/bin/bash
# snappy decode change: decode / full-size / C5 GPU tests, then the C3 bench (dict + chunk16) and its rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4c3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -5 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); s=d['secondary_values_chunk16']; print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_ratio'), d['status_ok_blocks'], 'chunk16', s['value'], s['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c3 -o run --output-format csv \
  -- python3 bench.py --config c3 --no-cpu --no-e2e --no-c5 --no-traffic --no-secondary > $O/prof_c3.json 2> $O/prof_c3.err || { echo "rocprof failed"; exit 1; }
f=$(find $O/prof_c3 -name "*kernel_stats.csv" | head -1); cp $f $O/c3_kernel_stats.csv && rm -rf $O/prof_c3
python -c "
import csv
for r in csv.DictReader(open('$O/c3_kernel_stats.csv')):
    if 'bhg' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
