#!/bin/bash
# C2 A/B: decode tests on the product library, then the C2 bench alternating product / variant libraries
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c2ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_golden.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --warmup 5 --no-cpu --no-e2e > $O/c2_prod_$r.json 2> $O/c2_prod_$r.err || { tail -5 $O/c2_prod_$r.err; exit 1; }
  for v in ${VARIANTS:-}; do
    BHG_LIB_PATH=$PWD/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 240 python -u bench.py --warmup 5 --no-cpu --no-e2e > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail -5 $O/c2_${v}_$r.err; exit 1; }
  done
done
for f in $O/c2_*.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f', d['ms_per_step'], d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d.get('valid'))"; done
