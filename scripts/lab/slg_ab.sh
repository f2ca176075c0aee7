set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/slg; mkdir -p $O
BHG_SL_G=24 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_decode.py -k snappy > $O/pytest24.txt 2>&1 || { tail -30 $O/pytest24.txt; exit 1; }
tail -2 $O/pytest24.txt
BHG_SL_G=24 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "mixed or c3" > $O/pytest24f.txt 2>&1 || { tail -30 $O/pytest24f.txt; exit 1; }
tail -2 $O/pytest24f.txt
for r in 1 2; do for v in 11 24 14 22; do for c in c3 mixdec; do
  f=$O/${c}_${v}_$r.json
  BHG_SL_G=$v timeout -k 10 200 python3 -u bench.py --config $c --no-cpu > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('$c G=$v run $r', d['value'], d['ms_per_step'])"
done; done; done
