cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t4
for d in 0 1 2 3 0; do
  echo "tile diag $d" >> gpurun_out/t4/lab.txt
  BHG_TILE_DIAG=$d timeout -k 10 120 scripts/lab/decode_lab 30 =none >> gpurun_out/t4/lab.txt 2>&1 || exit $?
done
cat gpurun_out/t4/lab.txt
