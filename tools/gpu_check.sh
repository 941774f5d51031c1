#!/bin/bash
# GPU check of the current tree: C++ tests, the whole pytest -m gpu suite (no -x: every
# failure is listed), bench.py x2, rocprofv3 kernel stats of bench.py, native bench at the
# BASELINE configs. usage: tools/gpu_check.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp NTXENT_GPU_CHECK=1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-check}; mkdir -p $OUT
timeout -k 10 400 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1 || { echo "cpp tests failed"; tail -30 $OUT/cpp_tests.log; exit 1; }
tail -1 $OUT/cpp_tests.log
if [ "$2" != "skip-tests" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --durations 15 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest_gpu.log | tail -2
grep -E "^(FAILED|ERROR)" $OUT/pytest_gpu.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
fi
for i in 1 2; do
timeout -k 10 200 python bench.py > $OUT/bench$i.log 2>&1 || { echo "bench failed"; tail $OUT/bench$i.log; exit 1; }
tail -1 $OUT/bench$i.log | cut -c1-220
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python tools/show_prof.py $OUT/kernel_stats.csv 12
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg5f8 --batch 8192 --dim 1024 --compute fp8"; do
  set -- $c; t=$1; shift
  timeout -k 10 120 build/bin/ntxent_bench "$@" --iters 30 --warmup 10 > $OUT/$t.log 2>&1 || { echo "native $t failed"; tail $OUT/$t.log; exit 1; }
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
done
echo done
