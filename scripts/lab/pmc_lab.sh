#!/bin/bash
# PMC passes over decode_lab kernels (one rocprofv3 run per pass; pmc only, no trace domains)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-labpmc}
FILT=$2
shift 2
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$OUT/p$i -o run --output-format csv \
    -- $GRAFT_REPO_ROOT/scripts/lab/decode_lab 3 $FILT > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $P"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $P"
done
