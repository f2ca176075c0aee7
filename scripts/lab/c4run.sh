#!/bin/bash
# local helper: one gpurun of scripts/gpu_enc.sh <name> (encode tests + C4 bench), then a summary
cd /root/repo || exit 1
N=$1; shift
timeout 1500 /usr/local/graft/bin/gpurun --timeout 1000 -- "VARIANTS=\"$*\" bash scripts/gpu_enc.sh $N" > /tmp/gr_$N.log 2>&1
grep "status=" /tmp/gr_$N.log | cut -c1-160
[ -d gpurun_out/$N ] || exit 3
tail -1 gpurun_out/$N/pytest.txt; grep FAILED gpurun_out/$N/pytest.txt | head -5
for f in gpurun_out/$N/c4_*.json; do
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$f'.split('/')[-1], d['value'], d['ms_per_step'])
" 2>/dev/null
done
