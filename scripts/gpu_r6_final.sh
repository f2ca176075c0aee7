#!/bin/bash
# round 6 closing measurements on the committed tree, in two parts (one gpurun call each):
#   PART=a: GPU tests, smoke, the driver-shaped C2 line, C2 kernel stats, C2 SQ counters
#   PART=b: C3 / C4 / C5-snappy / mixdec / Get / bigval / tail / indexcrc / scan / scanmix lines, kernel stats, the
#           one-rank RCCL rehearsal of the N > 1 line, C3 + C4 SQ counters, gloo x2
#   PART=c: part b from the tail line on; PART=d: from the RCCL rehearsal line on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6/final
mkdir -p $O
stats() {  # stats <name> <bench args...>: rocprofv3 kernel stats of one bench line
  local nm=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$nm -o run --output-format csv -- python3 bench.py "$@" > $O/prof_$nm.json 2> $O/prof_$nm.err || { tail -20 $O/prof_$nm.err; return 1; }
  cp $(find $O/prof_$nm -name "run_kernel_stats.csv" | head -1) $O/${nm}_kernel_stats.csv && rm -rf $O/prof_$nm
}
line() {  # line <name> <bench args...>
  local nm=$1; shift
  timeout -k 10 500 python3 -u bench.py "$@" > $O/bench_$nm.json 2> $O/bench_$nm.err || { tail -20 $O/bench_$nm.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$nm.json').read().strip().splitlines()[-1]); print('$nm', d['value'], d['unit'], d.get('ms_per_step'), d.get('roofline', {}).get('frac'))"
}
if [ "$PART" = a ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
  line c2_w5 --warmup 5 &&
  stats c2 --warmup 5 --no-cpu --no-e2e --no-traffic --no-c5 &&
  ARGS="--warmup 5" PMC_ROUND=r6 TAG=final/pmc_c2 KERNEL=k_decode_tile bash scripts/pmc_bench.sh
else
  [ "$PART" = c ] || [ "$PART" = d ] || {
  line c3 --config c3 --warmup 5 &&
  stats c3 --config c3 --warmup 5 --no-cpu --no-e2e --no-secondary &&
  line c4 --config c4 --warmup 5 &&
  stats c4 --config c4 --warmup 5 --no-cpu --no-e2e --no-secondary &&
  line c5_snappy --config c5 --codec snappy --warmup 2 &&
  line mixdec --config mixdec --steps 10 --warmup 5 &&
  stats mixdec --config mixdec --steps 10 --warmup 5 &&
  line get --config get --warmup 5 &&
  line bigval --config bigval --warmup 1 --steps 3 &&
  stats bigval --config bigval --warmup 1 --steps 3 --no-cpu; } &&
  { [ "$PART" = d ] || {
  line tail --config tail --warmup 5 &&
  line indexcrc --config indexcrc --warmup 5 &&
  line scan --config scan --warmup 5 &&
  line scanmix --config scanmix --warmup 2 --steps 5; }; } &&
  { export BHG_BENCH_PG1=1; line pg1_nccl --steps 5 --warmup 2; r=$?; unset BHG_BENCH_PG1; [ $r = 0 ]; } &&
  line g2_gloo --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu --no-e2e --no-c5 &&
  ARGS="--config c3 --no-secondary" PMC_ROUND=r6 TAG=final/pmc_c3 KERNEL=k_ bash scripts/pmc_bench.sh &&
  ARGS="--config c4 --no-secondary" PMC_ROUND=r6 TAG=final/pmc_c4 KERNEL=k_snappy_enc bash scripts/pmc_bench.sh
fi
