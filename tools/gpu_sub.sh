#!/bin/bash
# 64x64 diagonal sub-tiles vs 16-row strips: GPU tests + rocprof A/B (headline, cfg2, cfg5).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sub}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_kernels.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
prof() {
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 5 > $OUT/$t.log 2>&1 || return 1
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
  grep -h -E "diag_sub|diag_strip" $OUT/kstats_$t.csv | cut -d, -f1,4 | sed 's/"_ZN6ntxent3dev//' | cut -c1-90 || true
}
for rep in 1 2; do
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
  set -- $c; t=$1; shift
  prof ${t}_r$rep "$@" && prof ${t}_strips_r$rep "$@" --no-subtiles || exit 1
done
done
echo done
