#!/bin/bash
# decode parity tests, then the C2 bench repeated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c2t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash scripts/gpu_c2.sh ${1:-c2t}
