#!/bin/bash
# A/B: forward tile order (NTXENT_TILE_ORDER) x LDS-DMA cache policy (NTXENT_GEMM_DEBUG bits 8-10).
set -o pipefail
TAG=${1:-feed}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for ORD in 0 1; do for CP in 0 1 2 3 4; do
  D=$((CP << 8))
  NTXENT_TILE_ORDER=$ORD NTXENT_GEMM_DEBUG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/o${ORD}c${CP} -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 10 --warmup 2 > $OUT/o${ORD}c${CP}.log 2>&1 || exit 1
done; done
echo ok
