#!/bin/bash
# kernel stats (and optionally SQ counters) of one bench line under a lab library variant (lab helper)
#   V=wave ARGS="--config mixdec --steps 10 --warmup 5" TAG=pv KERNEL=k_snappy PMC=1 bash scripts/lab/prof_var.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-pv}
mkdir -p $O
export BHG_LIB_PATH=$GRAFT_REPO_ROOT/scripts/lab/libvar/$V/libbithashgpu.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
f=$(find $O/prof -name "run_kernel_stats.csv" | head -1); cp $f $O/kstats.csv; rm -rf $O/prof
python3 -c "
import csv; [print('$V', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs'])/1e3)) for r in csv.DictReader(open('$O/kstats.csv')) if 'bhg::' in r['Name']]"
if [ -n "$PMC" ]; then ARGS="$ARGS" TAG=${TAG:-pv}/pmc KERNEL=${KERNEL:-k_} bash scripts/pmc_bench.sh; fi
