#!/bin/bash
# Same-box A/B of two native bench binaries (rocprof kernel averages, interleaved twice).
# usage: tools/gpu_binab.sh BIN_A BIN_B [bench args...]
set -o pipefail
A=$1; B=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/binab; mkdir -p $OUT
export TMPDIR=/tmp
for X in $A $B $A $B; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$X -o run --output-format csv -- build/bin/$X --batch 4096 --dim 2048 --iters 20 --warmup 3 "$@" > $OUT/$X.log 2>&1 || exit 1
  echo "$X $(tail -1 $OUT/$X.log | cut -c1-150)"
  python tools/show_prof.py $OUT/$X/run_kernel_stats.csv 3
done
