#!/bin/bash
# Same-box A/B of an environment toggle on the native bench (fwd+bwd ms at the BASELINE configs),
# interleaved twice. usage: tools/gpu_ab_env.sh TAG VAR "VALUE_A VALUE_B" [configs...]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; mkdir -p $OUT
VAR=$2; VALS=${3:-"0 1"}
shift 3
CFGS=${@:-"head cfg2 cfg4 cfg5"}
args() { case $1 in head) echo "--batch 4096 --dim 2048";; cfg2) echo "--batch 4096 --dim 512";; cfg4) echo "--batch 1024 --dim 8192";;
  cfg5) echo "--batch 8192 --dim 1024 --compute fp16";; cfg5f8) echo "--batch 8192 --dim 1024 --compute fp8";; esac; }
for round in 1 2; do
  for v in $VALS; do
    for c in $CFGS; do
      env $VAR=$v timeout -k 10 120 build/bin/ntxent_bench $(args $c) --iters 30 --warmup 10 > $OUT/${c}_${VAR}${v}_r$round.log 2>&1 || { echo "bench $c $VAR=$v failed"; tail $OUT/${c}_${VAR}${v}_r$round.log; exit 1; }
      echo "r$round $VAR=$v $c: $(grep -A1 'fwd+bwd' $OUT/${c}_${VAR}${v}_r$round.log | tail -1 | cut -c1-120)"
    done
  done
done
