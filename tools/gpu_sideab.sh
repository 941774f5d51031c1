#!/bin/bash
# Same-box A/B: transpose on a side stream beside the forward GEMM (1) or serial (0).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/sideab; mkdir -p $OUT
i=0
for S in 1 0 1 0; do
  i=$((i+1))
  NTXENT_SIDE_TRANSPOSE=$S timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/p$i -o run --output-format csv -- python bench.py --steps 30 --warmup 5 > $OUT/b$i.log 2>&1 || exit 1
  NTXENT_SIDE_TRANSPOSE=$S timeout -k 10 150 python bench.py --steps 40 --warmup 5 > $OUT/c$i.log 2>&1 || exit 1
  echo "side=$S $(grep -o '"ms_per_step": [0-9.]*' $OUT/c$i.log)"
  python tools/show_prof.py $OUT/p$i/run_kernel_stats.csv 3
done
