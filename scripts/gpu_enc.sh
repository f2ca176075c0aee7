#!/bin/bash
# snappy encode: parity tests on the product library, then the C4 bench (+ variants), rocprof kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-enc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_gpu_tail.py tests/test_gpu_compaction.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
# 1 = some test failed (keep going to the benches); anything else (timeout, abort, fault) ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -30 $O/pytest.txt; exit $rc; }
grep -E "FAILED|ERROR" $O/pytest.txt | head -20
tail -2 $O/pytest.txt
timeout -k 10 240 python -u bench.py --config c4 --no-cpu --no-e2e > $O/c4_prod.json 2> $O/c4_prod.err || { tail -5 $O/c4_prod.err; exit 1; }
echo "prod: $(cut -c1-300 $O/c4_prod.json)"
for v in ${VARIANTS:-}; do
  BHG_LIB_PATH=$PWD/scripts/lab/libvar/$v/libbithashgpu.so timeout -k 10 240 python -u bench.py --config c4 --no-cpu --no-e2e --no-traffic > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  echo "$v: $(cut -c1-300 $O/c4_$v.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --config c4 --no-cpu --no-e2e --no-traffic --steps 5 --warmup 2 > $O/c4_rocprof.json 2> $O/c4_rocprof.err || { tail -5 $O/c4_rocprof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/c4_kernel_stats.csv
