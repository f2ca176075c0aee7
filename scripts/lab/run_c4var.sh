#!/bin/bash
# snappy encode: GPU encode tests on the default build, then bench c4 per scripts/lab/libvar/<name> build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c4var}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_golden.py tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread -k "encode or c4 or golden or two_threads" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for d in scripts/lab/libvar/*/; do
  nm=$(basename $d)
  BHG_LIB_PATH=$PWD/$d/libbithashgpu.so timeout -k 10 200 python -u bench.py --config c4 --no-cpu --steps 5 --warmup 2 > $O/c4_$nm.json 2> $O/c4_$nm.err || { echo "bench $nm failed"; tail -3 $O/c4_$nm.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_$nm.json')); print('$nm', d['value'], d['ms_per_step'], d.get('parity_vs_restatement', d.get('valid')))"
done
