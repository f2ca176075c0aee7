# lab A/B: the working tree's library (new) against HEAD's (scripts/lab/abprev), alternating runs of
# the bench lines in $LINES (one per line), ABN alternations; output under gpurun_out/r6/$TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6/${TAG:-libab}; mkdir -p $O
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  for r in $(seq 1 ${ABN:-3}); do
    for v in new old; do
      f=$O/l${i}_${v}_$r.json
      if [ $v = old ]; then export BHG_LIB_PATH=scripts/lab/abprev/lib/libbithashgpu.so; else unset BHG_LIB_PATH; fi
      timeout -k 10 300 python3 -u bench.py $args > $f 2> $f.err || { tail -5 $f.err; exit 1; }
      python3 -c "import json; d=json.load(open('$f')); x=d.get('nocompressor'); print('line $i ($args) $v run $r', d['value'], d['ms_per_step'], (x or {}).get('value'))"
    done
  done
done <<< "$LINES"
