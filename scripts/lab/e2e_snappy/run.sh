#!/bin/bash
# host copy threads for pageable snappy outputs: 4 / 8 / 12 / 16
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
mkdir -p $O
: > $O/hpool_threads.txt
for v in hp4 hp8 hp12 hp16; do
  echo "== $v" >> $O/hpool_threads.txt
  BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 200 python3 -u scripts/lab/e2e_snappy/e2e_trace.py pageable >> $O/hpool_threads.txt 2>&1 || exit 1
done
grep "==\|call" $O/hpool_threads.txt
