#!/bin/bash
# A/B of library builds on one box for bench lines without a roofline field: value and ms per run
# (lab helper).   VARS="base crc4" ARGS="--config indexcrc --warmup 5 --no-cpu" REPS=3 TAG=ab bash scripts/lab/ab_line.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5/${TAG:-ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 300 python3 -u bench.py $ARGS > $O/b_$v$rep.json 2> $O/b_$v$rep.err || { tail -5 $O/b_$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/b_$v$rep.json').read().strip().splitlines()[-1])
print('%-10s %d %10.3f %s ms %s' % ('$v', $rep, d['value'], d['unit'], d.get('ms_per_step')))" | tee -a $O/ab.txt
  done
done
