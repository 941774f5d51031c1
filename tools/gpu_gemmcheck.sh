#!/bin/bash
# Quick GEMM regression check on the GPU box: kernel tests + production parity + fp8 tests, then
# the native bench at the headline and BASELINE configs 2/4/5 (fp16 + fp8) with rocprof stats.
# usage: tools/gpu_gemmcheck.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-gemmcheck}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_production.py tests/test_gpu_fp8.py -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; grep -E "^FAILED" $OUT/pytest.log | head
[ $rc -le 1 ] || exit 1
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 > $OUT/$t.log 2>&1 || { echo "$t failed"; tail -3 $OUT/$t.log; return 1; }
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(tail -1 $OUT/$t.log | cut -c1-150)"
  grep -h "sim_gemm" $OUT/kstats_$t.csv | awk -F'",' '{print "   ", $1, $2}' | cut -d, -f1,4 | cut -c1-140
}
run head --batch 4096 --dim 2048 && run cfg2 --batch 4096 --dim 512 && run cfg4 --batch 1024 --dim 8192 && \
run cfg5_fp16 --batch 8192 --dim 1024 --compute fp16 && run cfg5_fp8 --batch 8192 --dim 1024 --compute fp8
timeout -k 10 300 build/bin/ntxent_tests > $OUT/cpp_tests.log 2>&1; echo "cpp tests rc=$?: $(tail -1 $OUT/cpp_tests.log)"; grep FAIL $OUT/cpp_tests.log | head
