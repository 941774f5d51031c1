#!/bin/bash
# PMC counters of the GEMM kernels (counters only with --kernel-trace/--stats; no sys/runtime traces).
set -o pipefail
TAG=${1:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-include-regex "sim_gemm|coef" -d $OUT/p1 -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1 > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex "sim_gemm|coef" -d $OUT/p2 -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1 > $OUT/p2.log 2>&1
echo rc=$?
