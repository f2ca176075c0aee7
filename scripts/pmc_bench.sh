#!/bin/bash
# SQ counter passes (2 x 8 SQ counters) of one bench.py line; one rocprofv3 run per pass.
#   ARGS="--config c4 --no-secondary" TAG=pmc_c4 bash scripts/pmc_bench.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${PMC_ROUND:-r5}/${TAG:-pmc}
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $O/p$i -o run --output-format csv -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu --no-e2e --no-traffic --no-c5 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 scripts/lab/c2_r5/pmc_table.py $O ${KERNEL:-k_} > $O/summary.txt
rm -rf $O/p1 $O/p2   # the raw counter CSVs of every kernel: too large to merge back
cat $O/summary.txt
