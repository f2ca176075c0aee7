#!/bin/bash
# SQ counters of the snappy decode (bench c3) for each scripts/lab/libvar/<name> build; pmc only
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-cfgpmc}
mkdir -p $O
export TMPDIR=/tmp
for d in scripts/lab/libvar/*/; do
  nm=$(basename $d)
  i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "GRBM_GUI_ACTIVE FETCH_SIZE"; do
    i=$((i+1))
    BHG_LIB_PATH=$PWD/$d/libbithashgpu.so timeout -s KILL 150 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/${nm}_p$i -o run --output-format csv -- python3 bench.py --config ${CFG:-c3} --no-cpu --steps 1 --warmup 1 > $O/${nm}_p$i.log 2>&1 || { echo "pass $nm $i failed"; tail -5 $O/${nm}_p$i.log; exit 1; }
  done
  echo "== $nm"
  python3 scripts/lab/pmc_table.py $O/${nm}_p1 $O/${nm}_p2 $O/${nm}_p3 | grep -A 20 "${KSEL:-k_snappy}"
done
