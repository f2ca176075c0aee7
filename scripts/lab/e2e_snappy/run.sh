#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/e2e_snappy
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_c_client.py -m gpu -x -v -k "host or client" --timeout 120 --timeout-method thread > $O/pytest_host.txt 2>&1; rc=$?
tail -3 $O/pytest_host.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --no-secondary --no-traffic --no-cpu > $O/bench_c3_staged.json 2> $O/bench_c3_staged.err || exit 1
python -c "
import json; d=json.load(open('$O/bench_c3_staged.json')); print(d['value'], json.dumps(d.get('e2e_host')))"
