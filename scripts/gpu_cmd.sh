cd $GRAFT_REPO_ROOT
O=gpurun_out/t14
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_get.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do for st in 1 0; do
echo "stage $st" >> $O/lab.txt
BHG_TILE_STAGE=$st timeout -k 10 120 scripts/lab/decode_lab 30 =none >> $O/lab.txt 2>&1 || exit $?
done; done
cat $O/lab.txt
