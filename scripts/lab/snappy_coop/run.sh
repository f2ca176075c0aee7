#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-coop}
mkdir -p $O
timeout -k 10 300 python -u scripts/lab/snappy_coop/coop_run.py > $O/coop.txt 2>&1; rc=$?
cat $O/coop.txt
exit $rc
