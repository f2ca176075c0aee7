#!/bin/bash
# GPU-box driver: parity tests, bench, rocprofv3 kernel-trace summary.
# usage: bash scripts/gpu_run.sh <tag> [steps...]   (each GPU step under its own timeout, chained)
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$TAG
mkdir -p $OUT
nproc > $OUT/nproc.txt
grep -m1 "model name" /proc/cpuinfo > $OUT/cpu.txt
shift
STEPS=${@:-"test bench prof"}
for s in $STEPS; do
  case $s in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest rc=$rc" >> $OUT/pytest_gpu.log; tail -3 $OUT/pytest_gpu.log
      [ $rc -eq 0 ] || exit $rc ;;
    testf)
      timeout -k 10 600 python -m pytest ${TESTF:-tests} -m gpu -x -q > $OUT/pytest_f.log 2>&1; rc=$?
      echo "pytest rc=$rc" >> $OUT/pytest_f.log; tail -15 $OUT/pytest_f.log
      [ $rc -eq 0 ] || exit $rc ;;
    scan)
      timeout -k 10 300 python bench.py --config scan --steps 10 --warmup 2 > $OUT/bench_scan.log 2>&1 || exit $?
      cat $OUT/bench_scan.log
      timeout -k 10 300 python bench.py --config scanmix --steps 10 --warmup 2 > $OUT/bench_scanmix.log 2>&1 || exit $?
      cat $OUT/bench_scanmix.log ;;
    get)
      timeout -k 10 600 python bench.py --config get --steps 10 --warmup 2 > $OUT/bench_get.log 2>&1 || exit $?
      cat $OUT/bench_get.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
      cat $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || exit $?
      cat $OUT/bench.log ;;
    benchq)
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $OUT/benchq.log 2>&1 || exit $?
      cat $OUT/benchq.log ;;
    prof)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv \
        -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e > $OUT/prof.log 2>&1 || exit $?
      find $OUT/prof -name "*stats*" | head ;;
    c3)
      timeout -k 10 600 python bench.py --config c3 --steps 10 --warmup 2 --cpu-seconds 8 > $OUT/bench_c3.log 2>&1 || exit $?
      cat $OUT/bench_c3.log ;;
    c4)
      timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 1 > $OUT/bench_c4.log 2>&1 || exit $?
      cat $OUT/bench_c4.log ;;
    profc3)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/profc3 -o run --output-format csv \
        -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 5 --warmup 1 --no-cpu > $OUT/profc3.log 2>&1 || exit $?
      find $OUT/profc3 -name "*stats*" | head ;;
    profc4)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/profc4 -o run --output-format csv \
        -- python3 $GRAFT_REPO_ROOT/bench.py --config c4 --steps 3 --warmup 1 --no-cpu > $OUT/profc4.log 2>&1 || exit $?
      find $OUT/profc4 -name "*stats*" | head ;;
    pmc)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$OUT/pmc1 -o run --output-format csv \
        -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $OUT/pmc1.log 2>&1 || exit $?
      timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$OUT/pmc2 -o run --output-format csv \
        -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $OUT/pmc2.log 2>&1 || exit $?
      python scripts/pmc_summarize.py $OUT/pmc1/run_counter_collection.csv $OUT/pmc2/run_counter_collection.csv \
        "${PMC_KERNEL:-k_decode_tile<8>}" $OUT/pmc_decode_c2.json "C2 1M x 1076 B blocks; run $TAG" ;;
  esac
done
echo done
