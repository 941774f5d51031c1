#!/bin/bash
# small-path backward column-split sweep (native bench, fwd+bwd ms)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-splits}; mkdir -p $OUT
for b in 128 256 512 1024; do for d in 64 256; do for s in 1 2 4 8; do
  timeout -k 10 60 build/bin/ntxent_bench --batch $b --dim $d --iters 50 --warmup 3 --small-splits $s > $OUT/s_${b}_${d}_${s}.log 2>&1 || { echo "fail $b $d $s"; tail -3 $OUT/s_${b}_${d}_${s}.log; exit 1; }
  echo "B=$b D=$d splits=$s $(tail -1 $OUT/s_${b}_${d}_${s}.log | awk -F'|' '{print $2 "|" $4}')"
done; done; done
