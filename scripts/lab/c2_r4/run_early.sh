#!/bin/bash
# C3: the stream kernel's first handle load before its LDS table build ("searly") vs after
# ("sbase"), alternated 3 times on one box; both builds carry the tile kernel's early table fill
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c3_early
mkdir -p $O
: > $O/early.txt
for rep in 1 2 3; do
  for v in sbase searly; do
    BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 200 python3 -u bench.py --config c3 --no-cpu --no-e2e --no-traffic --no-secondary --steps 50 --warmup 10 > $O/b_$v$rep.json 2> $O/b_$v$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/b_$v$rep.json')); print('$v', $rep, d['value'], d['ms_per_step'], d['roofline']['frac'])" >> $O/early.txt
  done
done
cat $O/early.txt
