#!/bin/bash
# Barrier-interval clock stamps (ABL=32) and the no-DMA ablation (ABL=1) of the forward GEMM at
# BASELINE config 5, fp16 vs fp8 (diagnostic build). usage: tools/gpu_stamps8.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-stamps8}; mkdir -p $OUT
export TMPDIR=/tmp
for c in fp16 fp8; do
  NTXENT_GEMM_ABL=32 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 8192 --dim 1024 --compute $c --iters 1 --warmup 1 2> $OUT/stamps_$c.log > /dev/null || exit 1
  grep "mode=0" $OUT/stamps_$c.log | head -1 | cut -c1-1500
  NTXENT_GEMM_ABL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/noload_$c -o run --output-format csv -- build/bin/ntxent_bench_abl --batch 8192 --dim 1024 --compute $c --iters 10 --warmup 2 > $OUT/noload_$c.log 2>&1 || exit 1
  grep -h "sim_gemm" $(find $OUT/noload_$c -name "*kernel_stats.csv") | awk -F'",' '{print $1, $2}' | cut -c1-160
done
