#!/bin/bash
# rocprofv3 kernel stats of bench configs (product library): one short run per config
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-stats}
mkdir -p $O
export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$c -o run --output-format csv -- python3 bench.py --config $c --no-cpu --no-e2e --no-c5 --no-traffic --steps 5 --warmup 2 > $O/${c}_rocprof.json 2> $O/${c}_rocprof.err || { tail -5 $O/${c}_rocprof.err; exit 1; }
  f=$(find $O/prof_$c -name "*kernel_stats.csv" | head -1); cp $f $O/${c}_kernel_stats.csv
  python3 -c "
import csv
rows=[r for r in csv.DictReader(open('$O/${c}_kernel_stats.csv')) if 'bhg' in r['Name']]
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]: print('$c', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
