#!/bin/bash
# SQ counters (two passes) + FETCH/WRITE of the C3 snappy decode kernels (bench --config c3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-c3pmc}
mkdir -p $O
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/p$i -o run --output-format csv -- python3 bench.py --config c3 --no-cpu --steps 2 --warmup 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 scripts/lab/pmc_table.py $O/p1 $O/p2 $O/p3 $O/p4 | grep -A 20 "k_snappy"
