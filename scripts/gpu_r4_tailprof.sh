#!/bin/bash
# rocprofv3 kernel stats of the table-tail bench (9 x 128 MiB tables and one 1M-record table)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-tailprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv \
  -- python3 bench.py --config tail --steps 10 --warmup 5 > $O/tail.json 2> $O/tail.err || { echo "rocprof failed"; tail -5 $O/tail.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/tail_kernel_stats.csv && rm -rf $O/prof
python -c "
import csv
rows=[r for r in csv.DictReader(open('$O/tail_kernel_stats.csv'))]
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us avg', round(float(r['TotalDurationNs'])/1e6,2), 'ms total')"
