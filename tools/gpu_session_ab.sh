#!/bin/bash
# Same-call A/B of the native bench: working tree (new) vs build/bin/ntxent_bench_old (an older
# revision's complete build), interleaved, headline + BASELINE configs 2 / 4 / 5 (fp16, fp8).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-session_ab}; mkdir -p $OUT
for rep in 1 2; do
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg5f8 --batch 8192 --dim 1024 --compute fp8"; do
  set -- $c; t=$1; shift
  for b in new old; do
    BIN=build/bin/ntxent_bench; [ $b = old ] && BIN=build/bin/ntxent_bench_old
    timeout -k 10 120 $BIN "$@" --iters 40 --warmup 60 > $OUT/${t}_${b}_$rep.log 2>&1 || { echo "$t $b failed"; exit 1; }
    echo "$t $b r$rep: $(grep -A1 'fwd+bwd' $OUT/${t}_${b}_$rep.log | tail -1 | awk -F'|' '{print $4}')"
  done
done
done
echo done
