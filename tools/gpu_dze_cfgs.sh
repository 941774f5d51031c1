#!/bin/bash
# Native bench fwd+bwd: exponential (--exp) vs coefficient backward over d (B = 4096/view) and B.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzecfg}; mkdir -p $OUT
for cfg in "4096 256" "4096 512" "4096 1024" "4096 2048" "2048 512" "1024 8192"; do
  set -- $cfg
  for F in --exp --no-exp; do
    timeout -k 10 120 build/bin/ntxent_bench --batch $1 --dim $2 --iters 30 --warmup 5 $F > $OUT/b$1_d$2$F.log 2>&1 || { echo "fail $cfg $F"; exit 1; }
    echo "B=$1 d=$2 $F: $(grep -E '^ +[0-9]+ +[0-9]+ ' $OUT/b$1_d$2$F.log | head -1 | cut -c1-160)"
  done
done
