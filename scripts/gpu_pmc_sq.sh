#!/bin/bash
# SQ counter passes (instruction mix, waits, LDS) of the kernels of the given bench configs,
# each --pmc pass its own rocprofv3 run with no trace domains: scripts/gpu_pmc_sq.sh <tag> c2 c4 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
for c in "$@"; do
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/pmc_${c}_p$i -o run --output-format csv \
      -- python3 bench.py --config $c --no-cpu --no-e2e --no-c5 --no-traffic --steps 1 --warmup 1 > $O/pmc_${c}_p$i.log 2>&1 || { echo "pmc $c $i failed"; tail -5 $O/pmc_${c}_p$i.log; exit 1; }
  done
  python3 scripts/lab/pmc_table.py $O/pmc_${c}_p1 $O/pmc_${c}_p2 > $O/pmc_${c}_sq.txt 2>&1 || true
done
echo "pmc ok"
