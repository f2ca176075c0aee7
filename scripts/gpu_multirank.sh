#!/bin/bash
# rehearsal of the N>1 bench path on a one-GPU box: 2 ranks (gloo process group, both on GPU 0)
# for the default C2 line and the C5 strong-scaling line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-mr}
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --backend gloo --steps 10 --warmup 5 > $O/c2_g2.json 2> $O/c2_g2.err || { tail -20 $O/c2_g2.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --backend gloo --config c5 --steps 3 --warmup 2 > $O/c5_g2.json 2> $O/c5_g2.err || { tail -20 $O/c5_g2.err; exit 1; }
cat $O/c2_g2.json $O/c5_g2.json
