#!/bin/bash
# Split-K dZ A/B at BASELINE config 2 (and the headline as a no-change control) + GPU tests.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-splitkdz}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_kernels.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
prof() {
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 5 > $OUT/$t.log 2>&1 || return 1
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
  grep -h -E "Li2ELi0ELi1E|sk_dz" $OUT/kstats_$t.csv | cut -d, -f1,4 | sed 's/"_ZN6ntxent3dev//' | cut -c1-90 || true
}
for rep in 1 2; do
prof cfg2_r$rep --batch 4096 --dim 512 && prof cfg2_off_r$rep --batch 4096 --dim 512 --no-splitk || exit 1
done
prof cfg2x1024 --batch 4096 --dim 1024 && prof cfg2x1024_off --batch 4096 --dim 1024 --no-splitk || exit 1
echo done
