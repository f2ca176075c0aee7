# lab A/B of the tile kernel's lanes per record (BHG_TILE_LPR 8 / 16) + parity with 16
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/lpr; mkdir -p $O
BHG_TILE_LPR=16 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py > $O/pytest_16.txt 2>&1 || { tail -30 $O/pytest_16.txt; exit 1; }
tail -n 1 $O/pytest_16.txt
for r in 1 2 3; do for v in 8 16; do
  f=$O/mixdec_${v}_$r.json
  BHG_TILE_LPR=$v timeout -k 10 200 python3 -u bench.py --config mixdec --no-cpu > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); x=d['nocompressor']; print('mixdec NoComp LPR=$v run $r', x['value'], x['ms_per_step'], x['roofline']['frac'])"
done; done
for v in 8 16; do
  f=$O/c2_${v}.json
  BHG_TILE_LPR=$v timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-e2e --no-traffic --no-c5 > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('c2 LPR=$v', d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
