#!/bin/bash
# combined A/B: decode + encode parity tests on the product library, then C2 and C4 bench lines
# alternating product / variant libraries (scripts/lab/libvar/<v>), traffic on the first C2 line only
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_decode.py tests/test_golden.py tests/test_gpu_fullsize.py tests/test_gpu_encode.py tests/test_gpu_tail.py tests/test_gpu_compaction.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
line() {  # $1 tag, $2 lib (or ""), rest: bench args
  local tag=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export BHG_LIB_PATH=$PWD/scripts/lab/libvar/$lib/libbithashgpu.so; else unset BHG_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-c5 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); r=d.get('roofline',{})
print('$tag', d['ms_per_step'], d['value'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traffic'), r.get('traffic_ratio'))"
  unset BHG_LIB_PATH
}
for c in ${CONFIGS:-c2 c4}; do
  w=""; [ $c = c2 ] && w="--warmup 5"
  line ${c}_prod_t "" --config $c $w
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in ${VARIANTS:-}; do line ${c}_${v}_$r $v --config $c $w --no-traffic; done
    line ${c}_prod_$r "" --config $c $w --no-traffic
  done
done
