#!/bin/bash
# stream-kernel knock-outs at three batch sizes (per-tile cost vs prologue)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sko}
mkdir -p $O
for N in 1000000 262144 131072; do
  echo "== n=$N" >> $O/stream_ko.txt
  LAB_N=$N LAB_EXPECTED=1 timeout -k 10 100 scripts/lab/stream_lab 30 =stream_c4,=ko_nodesc,=ko_noztab,=ko_all,=ko_all_nodesc >> $O/stream_ko.txt 2>&1 || exit 1
done
