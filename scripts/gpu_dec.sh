#!/bin/bash
# decode paths: all decode/golden/fullsize GPU tests, then C2 (driver warm-up) and C3 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-dec}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_golden.py tests/test_gpu_get.py tests/test_gpu_tail.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 240 python -u bench.py --warmup 5 --no-cpu --no-e2e > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
timeout -k 10 240 python -u bench.py --config c3 --no-cpu --no-e2e > $O/c3_prod.json 2> $O/c3_prod.err || { tail -5 $O/c3_prod.err; exit 1; }
for v in ${VARIANTS:-}; do
  BHG_LIB_PATH=$PWD/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 240 python -u bench.py --config c3 --no-cpu --no-e2e > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --config c3 --no-cpu --no-e2e --steps 20 --warmup 20 > $O/c3_prof.json 2> $O/c3_prof.err || { tail -5 $O/c3_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/c3_kernel_stats.csv
for f in $O/c2.json $O/c3_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['value'], d.get('roofline',{}).get('kernel_avg_ms'))"; done
