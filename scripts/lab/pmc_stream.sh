#!/bin/bash
# PMC passes over stream_lab kernels (one rocprofv3 run per pass; pmc only, no trace domains)
# usage: scripts/lab/pmc_stream.sh <outdir> <lab-filter> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-streampmc}
FILT=$2
shift 2
mkdir -p $OUT
export TMPDIR=/tmp
export LAB_WARM=30
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$OUT/p$i -o run --output-format csv \
    -- $GRAFT_REPO_ROOT/scripts/lab/stream_lab 3 $FILT > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $P"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $P"
done
