#!/bin/bash
# Full GPU check of the current tree: C++ tests, pytest -m gpu, bench.py x2, rocprofv3 kernel
# stats + trace of bench.py, native bench at the headline and BASELINE configs 2/4/5.
# usage: tools/gpu_check.sh TAG [quick]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-check}; mkdir -p $OUT
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1 || { echo "cpp tests failed"; tail -30 $OUT/cpp_tests.log; exit 1; }
tail -2 $OUT/cpp_tests.log
if [ "$2" != "quick" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
fi
for i in 1 2; do
timeout -k 10 200 python bench.py > $OUT/bench$i.log 2>&1 || { echo "bench failed"; tail $OUT/bench$i.log; exit 1; }
tail -1 $OUT/bench$i.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
cp $(find $OUT/prof -name "*kernel_trace.csv" | head -1) $OUT/kernel_trace.csv
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg5f8 --batch 8192 --dim 1024 --compute fp8"; do
  set -- $c; t=$1; shift
  timeout -k 10 120 build/bin/ntxent_bench "$@" --iters 30 --warmup 5 > $OUT/$t.log 2>&1 || { echo "native $t failed"; tail $OUT/$t.log; exit 1; }
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
done
echo done
