#!/bin/bash
# C2 bench repeated (variance check)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-c2}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-e2e ${BENCH_ARGS:-} > $O/c2_$r.json 2> $O/c2_$r.err || { tail -5 $O/c2_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2_$r.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['roofline']['frac'])"
done
