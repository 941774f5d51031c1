set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/trab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do for b in new old; do
  BIN=build/bin/ntxent_bench; [ $b = old ] && BIN=build/bin/ntxent_bench_old
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_${b}_$rep -o run --output-format csv -- $BIN --batch 4096 --dim 2048 --iters 20 --warmup 5 > $OUT/${b}_$rep.log 2>&1 || exit 1
  f=$(find $OUT/p_${b}_$rep -name '*kernel_stats.csv' | head -1)
  echo "$b r$rep: $(grep -h lse_transpose $f | cut -d, -f4)"
done; done
