#!/bin/bash
# BASELINE config 4 (B=1024/view, d=8192): forward GEMM time vs the stream-K split factor p
# (diagnostic build: NTXENT_SK_SPLIT), plus the item timeline at the default p.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-cfg4}; mkdir -p $OUT
export TMPDIR=/tmp
for P in 2 3 4 5 7; do
  NTXENT_SK_SPLIT=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p$P -o run --output-format csv -- build/bin/ntxent_bench_abl --batch 1024 --dim 8192 --iters 10 --warmup 2 > $OUT/p$P.log 2>&1 || exit 1
  echo "p=$P $(grep -h 'Li0ELi0ELi1' $(find $OUT/p$P -name '*kernel_stats.csv') | awk -F'",' '{print $2}' | cut -d, -f3) ns fwd; $(tail -1 $OUT/p$P.log | cut -c1-140)"
done
NTXENT_GEMM_ABL=64 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 1024 --dim 8192 --iters 2 --warmup 1 2>&1 | grep TIMELINE | head -1 | cut -c1-400
