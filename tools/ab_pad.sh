#!/bin/bash
# A/B of the leading-dimension pad (NTXENT_LD_PAD) on the headline shape: rocprof kernel stats.
set -o pipefail
TAG=${1:-pad}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for P in 0 64 128 32; do
  NTXENT_LD_PAD=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p$P -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 10 --warmup 2 > $OUT/p$P.log 2>&1 || exit 1
done
echo ok
