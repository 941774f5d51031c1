#!/bin/bash
# Buffer-placement A/B with per-kernel times: for each NTXENT_SKEW (KiB offsets of
# zq,zqt,sc,cbuf,slabs) run bench.py under rocprofv3 and print ms/step + GEMM averages.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/skewprof; mkdir -p $OUT
i=0
for S in "$@"; do
  i=$((i+1))
  NTXENT_SKEW=$S timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python bench.py --steps 30 --warmup 5 > $OUT/b$i.log 2>&1 || { echo "failed $S"; tail -3 $OUT/b$i.log; exit 1; }
  echo "skew=$S"
  python tools/show_prof.py $OUT/p$i/run_kernel_stats.csv 4
done
