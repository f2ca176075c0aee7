#!/bin/bash
# round 5: the decode of C4-shaped tables (bench.py --config mixdec) and its kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5/${TAG:-mixdec}
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --config mixdec --steps 10 --warmup 5 > $O/bench_mixdec.json 2> $O/bench_mixdec.err || { tail -20 $O/bench_mixdec.err; exit 1; }
cat $O/bench_mixdec.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config mixdec --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/mixdec_kernel_stats.csv
head -12 $O/mixdec_kernel_stats.csv
