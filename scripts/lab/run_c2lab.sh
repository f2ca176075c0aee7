#!/bin/bash
# C2 decode lab: stream_lab at three batch sizes + the decode GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c2lab}
FILT=${2:-=stream_c4,=ko_all}
mkdir -p $O
for N in 1000000 131072; do
  echo "== n=$N" >> $O/lab.txt
  LAB_N=$N LAB_EXPECTED=1 timeout -k 10 100 scripts/lab/stream_lab 30 $FILT >> $O/lab.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
cat $O/lab.txt
exit $rc
