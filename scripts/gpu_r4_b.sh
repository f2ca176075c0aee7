#!/bin/bash
# round-4 call b: the LDS-DMA C2 lab kernel beside the product, then the encode path with the
# CRC fused into k_enc_pack (encode / compaction / tail / full-size GPU tests + the C4 line)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 scripts/lab/c2_r4/dma_lab 30 > $O/dma_lab.txt 2>&1; echo "dma_lab rc=$?" >> $O/dma_lab.txt
cat $O/dma_lab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_get.py tests/test_gpu_encode.py tests/test_gpu_compaction.py tests/test_gpu_tail.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $O/pytest_enc.txt 2>&1; rc=$?
tail -3 $O/pytest_enc.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c4 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { echo "bench c4 failed"; tail -5 $O/bench_c4.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_c4.json')); r=d['roofline']
print('c4', d['value'], d['ms_per_step'], r['frac'], r.get('traffic_ratio'), [(k, v['value']) for k, v in d.items() if k.startswith('secondary')])
print(json.dumps({k: v for k, v in r.get('traffic_by_kernel', {}).items()}))"
timeout -k 10 300 python -u bench.py --config tail --steps 5 --warmup 2 > $O/bench_tail.json 2> $O/bench_tail.err || { echo "bench tail failed"; tail -5 $O/bench_tail.err; exit 1; }
cat $O/bench_tail.json
