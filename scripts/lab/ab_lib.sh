#!/bin/bash
# A/B of library builds on one box: for each repetition and each variant under scripts/lab/libvar/,
# run the bench line given in ARGS with that .so; prints value / ms / frac per run (lab helper).
#   VARS="base longwin" ARGS="--warmup 5 --no-cpu --no-e2e --no-traffic --no-c5" REPS=3 TAG=ab
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5/${TAG:-ab}
mkdir -p $O
: > $O/ab.txt
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 300 python3 -u bench.py $ARGS > $O/b_$v$rep.json 2> $O/b_$v$rep.err || { tail -5 $O/b_$v$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_$v$rep.json')); n=d.get('nocompressor')
s='%-10s %d %10.3f %8.4f %7.4f' % ('$v', $rep, d['value'], d['ms_per_step'], d['roofline']['frac'])
if n: s += '   none %10.3f %8.4f %7.4f' % (n['value'], n['ms_per_step'], n['roofline']['frac'])
print(s)" | tee -a $O/ab.txt
  done
done
