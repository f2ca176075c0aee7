#!/bin/bash
# long-range CRC + table tail change: crc_long / tail / encode / compaction / get GPU tests, then the
# indexcrc and tail benches and the tail's kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4tail}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_crc_long.py tests/test_gpu_tail.py tests/test_gpu_encode.py tests/test_gpu_compaction.py tests/test_gpu_get.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for c in indexcrc tail; do
  timeout -k 10 300 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
done
python -c "
import json
d=json.load(open('$O/bench_indexcrc.json')); print('indexcrc', d['value'], d['unit'], d['ms_per_step'])
d=json.load(open('$O/bench_tail.json')); print('tail 9 tables', d['tables_128MiB']['ms_per_tail_batch'], 'one table', d['one_table']['ms_per_tail_batch'])"
bash scripts/gpu_r4_tailprof.sh ${1:-r4tail}/prof
