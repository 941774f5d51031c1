#!/bin/bash
# Generic native A/B: rocprof kernel stats of ntxent_bench for a config with and without a flag.
# usage: tools/gpu_ab.sh TAG "FLAG" "KERNEL_REGEX" [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; mkdir -p $OUT
FLAG="$2"; KRE="$3"
if [ -n "$4" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$4" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
fi
prof() {  # tag, args
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 3 > $OUT/$t.log 2>&1 || return 1
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
  grep -h -E "$KRE" $OUT/kstats_$t.csv | cut -d, -f1,4 | sed 's/"_ZN6ntxent3dev//' | cut -c1-90 || true
}
for rep in 1 2; do
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512"; do
  set -- $c; t=$1; shift
  prof ${t}_r$rep "$@" && prof ${t}_off_r$rep "$@" $FLAG || exit 1
done
done
echo done
