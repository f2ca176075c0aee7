cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t10
mkdir -p $O
BHG_SNAPPY_VARIANT=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for sv in 4 2; do
BHG_SNAPPY_VARIANT=$sv timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > $O/c3_$sv.log 2>&1 || exit $?
echo "sv $sv $(grep -o '"ms_per_step": [0-9.]*' $O/c3_$sv.log)"
done
BHG_SNAPPY_VARIANT=4 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/p4 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/p4.log 2>&1 || exit $?
python - $O/p4/run_counter_collection.csv <<'PY'
import csv,sys
v=[float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if "k_snappy_rt" in r["Kernel_Name"]]
print("  FETCH GB/launch (x2 corrected):", round(2*sum(v)/len(v)*1024/1e9,3) if v else None)
PY
