#!/bin/bash
# all GPU tests + smoke on the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4tests}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
tail -1 $O/smoke.txt
exit $rc
