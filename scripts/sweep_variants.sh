#!/bin/bash
# decode-kernel variant sweep on the GPU box (one bench line per variant)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
for v in ${VARIANTS:-0 1 2 3 4 5 6}; do
  BHG_DECODE_VARIANT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $OUT/v$v.log 2>&1 || exit $?
  echo "variant $v: $(python -c "import json,sys; d=json.loads(open('$OUT/v$v.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])")"
done
