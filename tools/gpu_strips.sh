#!/bin/bash
# Diagonal-strip remainder vs stream-K split: GPU tests (production parity + strips A/B), then
# rocprofv3 kernel stats of the native bench with and without strips at the headline and
# BASELINE configs 2 and 5. usage: tools/gpu_strips.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-strips}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_production.py tests/test_gpu_kernels.py -m gpu -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep PARITY $OUT/pytest.log | tail -12
prof() {  # tag, args
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 3 > $OUT/$t.log 2>&1 || return 1
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
}
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
  set -- $c; t=$1; shift
  prof ${t} "$@" && prof ${t}_nostrips "$@" --no-strips || exit 1
done
timeout -k 10 200 python bench.py > $OUT/bench1.log 2>&1 || { echo "bench failed"; tail $OUT/bench1.log; exit 1; }
tail -1 $OUT/bench1.log | cut -c1-250
echo done
