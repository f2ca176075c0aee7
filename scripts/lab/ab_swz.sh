#!/bin/bash
# C4 hash-slot swizzle: encode tests, A/B, SQ counters of the swizzled encoder (lab helper)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r5/swz
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_encode.py tests/test_gpu_fullsize.py tests/test_gpu_tail.py > gpurun_out/r5/swz/pytest.txt 2>&1 || { tail -30 gpurun_out/r5/swz/pytest.txt; exit 1; }
tail -1 gpurun_out/r5/swz/pytest.txt
VARS="swz0 swz1" ARGS="--config c4 --warmup 5 --no-secondary" REPS=3 TAG=swz/ab bash scripts/lab/ab_lib.sh &&
ARGS="--config c4 --no-secondary" TAG=swz/pmc KERNEL=k_snappy_enc bash scripts/pmc_bench.sh
