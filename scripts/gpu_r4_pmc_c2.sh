#!/bin/bash
# SQ counter passes of the C2 kernel (k_decode_tile<8, 2, 2>), each --pmc pass its own run, no trace domains
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-pmc_c2}
mkdir -p $O
export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/pmc_c2_p$i -o run --output-format csv \
    -- python3 bench.py --config c2 --no-cpu --no-e2e --no-c5 --no-traffic --steps 3 --warmup 2 > $O/pmc_c2_p$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $O/pmc_c2_p$i.log; exit 1; }
done
python3 scripts/lab/pmc_table.py $O/pmc_c2_p1 $O/pmc_c2_p2 > $O/pmc_c2_sq.txt 2>&1 || true
rm -rf $O/pmc_c2_p1 $O/pmc_c2_p2
grep -A17 "k_decode_tile" $O/pmc_c2_sq.txt | head -20
