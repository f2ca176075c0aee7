# lab A/B of the snappy header pass's window / chain shape (BHG_STREAM_CFG) + parity for each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/stream; mkdir -p $O
for v in 1 2 3; do
  BHG_STREAM_CFG=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_decode.py -k "snappy or crc" > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  echo "cfg $v: $(tail -n 1 $O/pytest_$v.txt)"
done
BHG_STREAM_CFG=3 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_fullsize.py -k "c3 or mixed" > $O/pytest_3f.txt 2>&1 || { tail -30 $O/pytest_3f.txt; exit 1; }
echo "cfg 3 fullsize: $(tail -n 1 $O/pytest_3f.txt)"
for r in 1 2; do for v in 0 1 2 3; do for c in c3 mixdec; do
  f=$O/${c}_${v}_$r.json
  BHG_STREAM_CFG=$v timeout -k 10 200 python3 -u bench.py --config $c --no-cpu > $f 2> $f.err || { tail -5 $f.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('$c cfg=$v run $r', d['value'], d['ms_per_step'])"
done; done; done
