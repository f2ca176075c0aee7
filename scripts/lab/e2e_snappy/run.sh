#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
mkdir -p $O
for cb in 16777216 33554432 67108864 134217728; do
  echo "chunk $cb"
  BHG_HOST_CHUNK_BYTES=$cb timeout -k 10 200 python3 -u scripts/lab/e2e_snappy/e2e_trace.py > $O/e2e_cb$cb.txt 2>&1 || exit 1
  grep call $O/e2e_cb$cb.txt | tail -2
done
