#!/bin/bash
# A/B of the GEMM operand LDS-DMA cache policy (tools/build_variant.sh builds), interleaved rounds.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/aux; mkdir -p $OUT
for r in 1 2; do
  for v in "" _aux1 _aux2 _aux3 _aux16; do
    for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
      set -- $c; t=$1; shift
      timeout -k 10 120 build/bin/ntxent_bench$v "$@" --iters 40 --warmup 10 > $OUT/$t$v.log 2>&1 || { echo "fail $t$v"; tail -3 $OUT/$t$v.log; exit 1; }
      echo "r$r $t$v: $(grep -A1 'fwd+bwd' $OUT/$t$v.log | tail -1 | cut -c24-150)"
    done
  done
done
