#!/bin/bash
# snappy decode: GPU snappy tests on the default build, then bench c3 per scripts/lab/libvar/<name> build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c3var}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_golden.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or c3 or golden" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for d in scripts/lab/libvar/*/; do
  nm=$(basename $d)
  BHG_LIB_PATH=$PWD/$d/libbithashgpu.so timeout -k 10 200 python -u bench.py --config c3 --no-cpu --steps 10 --warmup 3 > $O/c3_$nm.json 2> $O/c3_$nm.err || { echo "bench $nm failed"; tail -3 $O/c3_$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_$nm.json')); print('$nm', d['value'], d['ms_per_step'], d.get('parity_vs_restatement', d.get('valid')))"
done
