#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3c3b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.txt
tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/trace" -o run --output-format csv \
  -- python3 bench.py --config c3 --no-cpu --warmup 10 > $O/bench_c3_prof.json 2> $O/bench_c3_prof.err || exit 1
python -c "
import json; d=json.load(open('$O/bench_c3_prof.json')); r=d.get('roofline',{})
print('c3', d['value'], d['ms_per_step'], r.get('frac'), r.get('step_event_ms'), d['status_ok_blocks'])"
find $O/trace -name '*kernel_stats.csv' -exec grep -E "snappy|chunk" {} \; | cut -c1-200
bash scripts/pmc_c3.sh ${1:-r3c3b}/pmc
