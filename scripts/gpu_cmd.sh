cd $GRAFT_REPO_ROOT
O=gpurun_out/t8
mkdir -p $O
for w in 1 2 4 8; do
BHG_LANE_WGS_PER_CU=$w BHG_SNAPPY_VARIANT=2 timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > $O/c3_$w.log 2>&1 || exit $?
echo "wgs/cu $w"; grep '^{' $O/c3_$w.log | cut -c150-330
done
