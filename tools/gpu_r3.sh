#!/bin/bash
# Round-3 GPU check: C++ tests, new-feature tests first (fail fast), the whole GPU suite,
# bench.py x2, native headline/configs (A/B switches given in $AB, e.g. "--no-dzsym"),
# rocprofv3 kernel stats of bench.py.
# usage: tools/gpu_r3.sh TAG [FIRST_TESTS] [quick]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r3}; mkdir -p $OUT
FIRST=${2:-}
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "cpp tests failed rc=$rc"; grep -E "FAIL|W=" $OUT/cpp_tests.log | head -20; [ $rc -ge 124 ] && exit 1; }
grep -E "W=|passed" $OUT/cpp_tests.log | tail -12
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python -u -m pytest $FIRST -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest_first.log 2>&1 || { echo "first tests failed"; tail -40 $OUT/pytest_first.log; exit 1; }
  grep -E "DZSYM|passed|failed" $OUT/pytest_first.log | tail -12
fi
if [ "$3" != "quick" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for i in 1 2; do
  timeout -k 10 200 python bench.py > $OUT/bench$i.log 2>&1 || { echo "bench failed"; tail $OUT/bench$i.log; exit 1; }
  tail -1 $OUT/bench$i.log | cut -c1-190
done
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg5f8 --batch 8192 --dim 1024 --compute fp8"; do
  set -- $c; t=$1; shift
  for v in "" $AB; do
    timeout -k 10 120 build/bin/ntxent_bench "$@" $v --iters 40 --warmup 10 > $OUT/$t$v.log 2>&1 || { echo "native $t $v failed"; tail $OUT/$t$v.log; exit 1; }
    echo "$t $v: $(grep -A1 'fwd+bwd' $OUT/$t$v.log | tail -1 | cut -c1-150)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python tools/show_prof.py $OUT/kernel_stats.csv 9
echo done
