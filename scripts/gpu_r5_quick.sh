#!/bin/bash
# round 5: decode GPU tests + C2 (driver-shaped) + the C4-mix decode, one call
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-quick}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_decode.py tests/test_gpu_fullsize.py} > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --warmup 5 --no-cpu --no-e2e --no-traffic --no-c5 > $O/bench_c2_$r.json 2> $O/bench_c2_$r.err || { tail -20 $O/bench_c2_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2_$r.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
if [ -n "$MIX" ]; then
timeout -k 10 300 python3 -u bench.py --config mixdec --steps 10 --warmup 5 > $O/bench_mixdec.json 2> $O/bench_mixdec.err || { tail -20 $O/bench_mixdec.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_mixdec.json')); n=d['nocompressor']
print('mix snappy', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_first_blocks'])
print('mix none', n['value'], n['ms_per_step'], n['roofline']['frac'], n['parity_first_blocks'])"
fi
