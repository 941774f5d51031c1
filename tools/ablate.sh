#!/bin/bash
# GEMM ablations (timing only): rocprof kernel stats of the C++ bench under NTXENT_GEMM_DEBUG bits.
set -o pipefail
TAG=${1:-abl}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for D in 0 1 2 4 6; do
  NTXENT_GEMM_DEBUG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/d$D -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 10 --warmup 2 > $OUT/d$D.log 2>&1 || exit 1
done
echo ok
