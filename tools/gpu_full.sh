#!/bin/bash
# Full GPU check: pytest -m gpu, C++ tests, harness (quick), headline bench + rocprof stats.
set -o pipefail
TAG=${1:-full}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1 || { echo "cpp tests failed"; tail -20 $OUT/cpp_tests.log; exit 1; }
timeout -k 10 300 python bench/harness.py --quick --out-dir $OUT/harness > $OUT/harness.log 2>&1 || { echo "harness failed"; tail -20 $OUT/harness.log; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail $OUT/bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo done
