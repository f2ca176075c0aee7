# lab A/B of the LDS tier shapes (BHG_SL_H: 0 product, 1 tier 2 halved, 2 both halved) + parity at H=2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/slh; mkdir -p $O
BHG_SL_H=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decode.py -k snappy > $O/pytest_h2.txt 2>&1 || { tail -30 $O/pytest_h2.txt; exit 1; }
tail -n 2 $O/pytest_h2.txt
BHG_SL_H=2 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "mixed or c3" > $O/pytest_h2f.txt 2>&1 || { tail -30 $O/pytest_h2f.txt; exit 1; }
tail -n 2 $O/pytest_h2f.txt
for r in 1 2; do for v in 0 1 2; do for c in c3 mixdec; do
  f=$O/${c}_${v}_$r.json
  BHG_SL_H=$v timeout -k 10 200 python3 -u bench.py --config $c --no-cpu > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('$c H=$v run $r', d['value'], d['ms_per_step'])"
done; done; done
