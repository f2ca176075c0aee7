#!/bin/bash
# snappy decode variants: parity tests, then C3 bench per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-snap}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -k "snappy" -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for v in ${VARIANTS:-2 3}; do
  BHG_SNAPPY_VARIANT=$v timeout -k 10 240 python -u bench.py --config c3 --no-cpu --no-e2e > $O/c3_v$v.json 2> $O/c3_v$v.err || { tail -5 $O/c3_v$v.err; exit 1; }
  echo "v$v: $(cut -c1-400 $O/c3_v$v.json)"
done
