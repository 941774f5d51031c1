#!/bin/bash
# Native runtime on the GPU: C++ tests, C++ bench (eager + hipGraph), pytest -m gpu.
set -o pipefail
TAG=${1:-native}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1 || { echo "cpp tests failed"; tail -20 $OUT/cpp_tests.log; exit 1; }
timeout -k 10 200 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 20 --warmup 3 --graph --json $OUT/cpp_bench.json > $OUT/cpp_bench.log 2>&1 || { echo "cpp bench failed"; tail $OUT/cpp_bench.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
echo done
