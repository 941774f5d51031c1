#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of the native bench at the BASELINE configs.
# usage: tools/gpu_cfgprof.sh TAG [extra ntxent_bench flags]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-cfgprof}; shift; EXTRA="$*"; mkdir -p $OUT
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg5f8 --batch 8192 --dim 1024 --compute fp8"; do
  set -- $c $EXTRA; t=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$t -o run --output-format csv -- build/bin/ntxent_bench "$@" --iters 20 --warmup 10 > $OUT/$t.log 2>&1 || { echo "rocprof $t failed"; tail -5 $OUT/$t.log; exit 1; }
  cp $(find $OUT/$t -name "*kernel_stats.csv" | head -1) $OUT/${t}_kernel_stats.csv
  echo "== $t: $(grep -A1 'fwd+bwd' $OUT/$t.log | tail -1 | cut -c1-120)"
  python tools/show_prof.py $OUT/${t}_kernel_stats.csv 10
done
