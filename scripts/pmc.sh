#!/bin/bash
# PMC passes for one bench configuration (each pass its own rocprofv3 run; no trace domains combined with --pmc)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-pmc}
shift
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$OUT/p$i -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-e2e > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $P"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $P"
done
