#!/bin/bash
# round 6, the 8-wave role shapes of k_snappy_lds_multi: GPU tests, smoke, mixdec / C3 / bigval lines and
# the mixdec kernel stats on the working tree; then the 12-wave shapes (scripts/lab/var/m12) against it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6/m8
mkdir -p $O
line() {
  local nm=$1; shift
  timeout -k 10 400 python3 -u bench.py "$@" > $O/bench_$nm.json 2> $O/bench_$nm.err || { tail -20 $O/bench_$nm.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$nm.json').read().strip().splitlines()[-1]); print('$nm', d['value'], d['unit'], d.get('ms_per_step'), (d.get('nocompressor') or {}).get('value'))"
}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
line mixdec --config mixdec --steps 10 --warmup 5 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_mixdec -o run --output-format csv -- python3 bench.py --config mixdec --steps 10 --warmup 5 --no-cpu > $O/prof_mixdec.json 2> $O/prof_mixdec.err &&
cp $(find $O/prof_mixdec -name "run_kernel_stats.csv" | head -1) $O/mixdec_kernel_stats.csv && rm -rf $O/prof_mixdec &&
line c3 --config c3 --warmup 5 &&
line bigval --config bigval --warmup 1 --steps 3 &&
TAG=m12 ABN=2 VARS="old m12" ARGS="--config mixdec --no-cpu" bash scripts/lab/var/run.sh
