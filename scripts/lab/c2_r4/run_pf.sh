#!/bin/bash
# tile-kernel prefetch variants (PF 0..3) on the C2 layout: bit-exactness vs the product and event timings
set -o pipefail
cd "$GRAFT_REPO_ROOT/scripts/lab/c2_r4" || exit 1
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-pf}
mkdir -p $O
timeout -k 10 120 ./dma_lab 60 > $O/pf_lab.txt 2>&1 || { cat $O/pf_lab.txt; exit 1; }
timeout -k 10 120 ./dma_lab 60 >> $O/pf_lab.txt 2>&1 || { cat $O/pf_lab.txt; exit 1; }
cat $O/pf_lab.txt
