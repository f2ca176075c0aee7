#!/bin/bash
# k_copy_out grid sweep (workgroups per 4 CUs) on the pinned snappy e2e path
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
mkdir -p $O
: > $O/copy_out_grid.txt
for v in co1 co2 co4 co8 co16; do
  echo "== $v" >> $O/copy_out_grid.txt
  BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 200 python3 -u scripts/lab/e2e_snappy/e2e_trace.py >> $O/copy_out_grid.txt 2>&1 || exit 1
done
grep "==\|call [23]" $O/copy_out_grid.txt
