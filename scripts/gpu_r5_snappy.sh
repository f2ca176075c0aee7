#!/bin/bash
# round 5: snappy decode tiers -- decode tests, kernel stats of mixdec and C3, SQ counters of the tiers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-snappy}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_fullsize.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for c in mixdec c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 5 --no-secondary > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
f=$(find $O/prof_$c -name "run_kernel_stats.csv" | head -1); cp $f $O/kstats_$c.csv; rm -rf $O/prof_$c
python3 -c "
import csv; [print('$c', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3)) for r in csv.DictReader(open('$O/kstats_$c.csv')) if 'bhg::' in r['Name']]"
done
ARGS="--config mixdec" TAG=${TAG:-snappy}/pmc KERNEL=k_snappy bash scripts/pmc_bench.sh
