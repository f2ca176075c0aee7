#!/bin/bash
# C3 end-to-end host path (bhg_decode_batch_host, snappy, pipelined): GPU tests, then the c3 bench
# line with its e2e_host leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4c3e2e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -v -k "host" --timeout 120 --timeout-method thread > $O/pytest_host.txt 2>&1; rc=$?
tail -3 $O/pytest_host.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c3 --no-secondary --no-traffic > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench c3 failed"; tail -5 $O/bench_c3.err; exit 1; }
python -c "
import json
d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['valid'], d.get('parity_vs_restatement')); print(json.dumps(d.get('e2e_host')))"
