#!/bin/bash
# Barrier-interval clock stamps (block 0, waves 0 and 4) of the DzE and Dz GEMMs.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzestamps}; mkdir -p $OUT
NTXENT_GEMM_ABL=32 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 1 --warmup 0 --exp > $OUT/stamps_exp.log 2>&1 || { echo fail; tail $OUT/stamps_exp.log; exit 1; }
NTXENT_GEMM_ABL=32 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 1 --warmup 0 --no-exp > $OUT/stamps_noexp.log 2>&1 || { echo fail; exit 1; }
grep "STAMPS mode=3" $OUT/stamps_exp.log | head -1 | cut -c1-900
grep "STAMPS mode=2" $OUT/stamps_noexp.log | head -1 | cut -c1-900
