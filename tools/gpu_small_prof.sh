#!/bin/bash
# Kernel durations of the small path (rocprofv3 kernel trace) at three sweep points.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-smallprof}; mkdir -p $OUT
for cfg in "32 64" "256 256" "1024 256"; do
  set -- $cfg
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p_$1_$2 -o run -- build/bin/ntxent_bench --batch $1 --dim $2 --iters 20 --warmup 2 > $OUT/p_$1_$2.log 2>&1 || { echo "prof $cfg failed"; tail $OUT/p_$1_$2.log; exit 1; }
  echo "== B=$1 D=$2"; python tools/show_prof.py $(find $OUT/p_$1_$2 -name "*kernel_stats.csv" | head -1) 6
done
