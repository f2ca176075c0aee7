set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 || exit $?
cat gpurun_out/bench1.log
