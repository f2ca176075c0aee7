#!/bin/bash
# rocprofv3 evidence for one bench.py command (run on the GPU box):
#   1. --kernel-trace --stats of the command itself      -> gpurun_out/<tag>/trace
#   2. --pmc FETCH_SIZE, then --pmc WRITE_SIZE (separate passes, no trace
#      domains, cpu/e2e legs off)                         -> gpurun_out/<tag>/pmc_{fetch,write}
# usage: scripts/profile_bench.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/trace" -o run --output-format csv \
  -- python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "trace run failed"; tail -5 "$OUT/bench.err"; exit 1; }
echo "trace ok"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/$OUT/pmc_$C" -o run --output-format csv \
    -- python3 bench.py --no-cpu --no-e2e "$@" > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" || { echo "pmc $C failed"; tail -5 "$OUT/pmc_$C.err"; exit 1; }
  echo "pmc $C ok"
done
