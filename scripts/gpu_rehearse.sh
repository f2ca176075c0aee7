#!/bin/bash
# multi-rank rehearsal on the one-GPU box: `bench.py --gpus N --backend gloo` self-spawns N ranks
# that share GPU 0 (the C5 strong-scaling line), plus the encoder GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-reh}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for N in ${NS:-4 8}; do
  timeout -k 10 400 python -u bench.py --gpus $N --backend gloo --warmup 3 --steps 5 > $O/bench_g${N}_gloo.json 2> $O/bench_g${N}_gloo.err || { echo "N=$N failed"; tail -20 $O/bench_g${N}_gloo.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_g${N}_gloo.json'))
print($N, d['n_gpus'], d.get('ranks_seen'), d['value'], d['ms_per_step'], d.get('valid'), d.get('digest_all_ranks'), d.get('status_ok_blocks'))"
done
