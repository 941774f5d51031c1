#!/bin/bash
# Per-block GEMM item timelines (diagnostic build, NTXENT_GEMM_ABL=64): main-loop cycles per
# K-step, epilogue phases, fixups, for the headline and BASELINE config 5 (fp16 vs fp8).
# usage: tools/gpu_timeline.sh TAG   (after `bash tools/ablate_ct.sh build` on the host)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-timeline}; mkdir -p $OUT
run() { NTXENT_GEMM_ABL=64 timeout -k 10 120 build/bin/ntxent_bench_abl "$@" --iters 2 --warmup 1 2>&1 | grep TIMELINE | head -2; }
echo "== headline fp16" ; run --batch 4096 --dim 2048 | tee $OUT/head.log
echo "== cfg5 fp16"     ; run --batch 8192 --dim 1024 --compute fp16 | tee $OUT/cfg5_fp16.log
echo "== cfg5 fp8"      ; run --batch 8192 --dim 1024 --compute fp8 | tee $OUT/cfg5_fp8.log
echo "== cfg4 fp16"     ; run --batch 1024 --dim 8192 | tee $OUT/cfg4.log
