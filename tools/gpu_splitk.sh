#!/bin/bash
# Split-K + reduce forward (tile-starved launches) vs the stream-K fixup: GPU tests and rocprof
# of BASELINE config 4 with and without it. usage: tools/gpu_splitk.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-splitk}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_production.py -m gpu -x -q -s -k "splitk or wide or strips" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log; grep PARITY $OUT/pytest.log | tail -8
prof() {  # tag, args
  local t=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 3 > $OUT/$t.log 2>&1 || return 1
  cp $(find $OUT/p_$t -name '*kernel_stats.csv' | head -1) $OUT/kstats_$t.csv
  echo "$t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-150)"
  grep -h "Li0ELi0ELi1E\|sk_reduce\|fp8e4m3ELi0ELi0" $OUT/kstats_$t.csv | cut -d, -f1,4 | sed 's/"_ZN6ntxent3dev//' | cut -c1-90
}
prof cfg4 --batch 1024 --dim 8192 && prof cfg4_nosplitk --batch 1024 --dim 8192 --no-splitk && \
prof cfg4f8 --batch 1024 --dim 8192 --compute fp8 && prof cfg4f8_nosplitk --batch 1024 --dim 8192 --compute fp8 --no-splitk || exit 1
echo done
