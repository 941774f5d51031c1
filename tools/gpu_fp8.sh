#!/bin/bash
# fp8 (block-scaled MX) forward + parity tests + config-5 fp8 vs fp16 on the native bench, with
# rocprofv3 kernel stats of both (same box, same call). usage: tools/gpu_fp8.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-fp8}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_production.py -v -s --timeout 200 --timeout-method thread > $OUT/pytest_fp8_prod.log 2>&1; rc=$?
grep -E "PARITY|PASS|FAIL|Error|passed|failed" $OUT/pytest_fp8_prod.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit 1; }
for c in fp16 fp8; do
  timeout -k 10 120 build/bin/ntxent_bench --batch 8192 --dim 1024 --compute $c --iters 30 > $OUT/cfg5_$c.log 2>&1 || { echo "bench $c failed"; tail $OUT/cfg5_$c.log; exit 1; }
  tail -2 $OUT/cfg5_$c.log
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- build/bin/ntxent_bench --batch 8192 --dim 1024 --compute $c --iters 10 > $OUT/prof_$c.log 2>&1 || { echo "rocprof $c failed"; tail $OUT/prof_$c.log; exit 1; }
  f=$(find $OUT/prof_$c -name "*kernel_stats.csv" | head -1); cp $f $OUT/kstats_cfg5_$c.csv
  cut -d, -f1-4 $OUT/kstats_cfg5_$c.csv | head -8
done
timeout -k 10 120 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 30 > $OUT/head.log 2>&1 && tail -1 $OUT/head.log
echo done
