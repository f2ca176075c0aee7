#!/bin/bash
# snappy decode: bench c3 (dict values, CRC-verified, parity-checked) per scripts/lab/libvar/<name> build, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c3var}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for d in scripts/lab/libvar/*/; do
  nm=$(basename $d)
  BHG_LIB_PATH=$PWD/$d/libbithashgpu.so timeout -k 10 200 python -u bench.py --config c3 --no-cpu --no-traffic --steps 20 --warmup 20 > $O/c3_${nm}_$rep.json 2> $O/c3_${nm}_$rep.err || { echo "bench $nm failed"; tail -3 $O/c3_${nm}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_${nm}_$rep.json')); s=d.get('secondary_values_chunk16',{}); print('$nm', d['value'], d['ms_per_step'], d.get('parity_vs_restatement'), d.get('status_ok_blocks'), 'chunk16', s.get('value'), s.get('ms_per_step'))"
done
done
