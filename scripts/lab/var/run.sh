# lab: alternate bench lines over variant libraries: VARS="old segmin16 ..." (old = the working tree's
# library), ARGS="<bench args>", ABN alternations; output gpurun_out/r6/$TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/${TAG:-var}; mkdir -p $O
for r in $(seq 1 ${ABN:-2}); do
  for v in $VARS; do
    f=$O/${v}_$r.json
    if [ $v = old ]; then unset BHG_LIB_PATH; else export BHG_LIB_PATH=scripts/lab/var/$v/lib/libbithashgpu.so; fi
    timeout -k 10 300 python3 -u bench.py $ARGS > $f 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json; d=json.load(open('$f')); print('$v run $r', d['value'], d['ms_per_step'])"
  done
done
