#!/bin/bash
# fp8 path: GPU tests + native bench of BASELINE config 5 (B=8192, d=1024) fp8 vs fp16.
set -o pipefail
TAG=${1:-fp8}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1 || { echo "cpp tests failed"; tail -20 $OUT/cpp_tests.log; exit 1; }
for C in fp8 fp16; do
  timeout -k 10 200 build/bin/ntxent_bench --batch 8192 --dim 1024 --compute $C --iters 20 --warmup 3 > $OUT/cfg5_$C.log 2>&1 || { echo "bench $C failed"; exit 1; }
  timeout -k 10 200 build/bin/ntxent_bench --batch 4096 --dim 2048 --compute $C --iters 20 --warmup 3 > $OUT/head_$C.log 2>&1 || { echo "bench $C failed"; exit 1; }
done
echo done
