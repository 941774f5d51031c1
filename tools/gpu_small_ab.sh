#!/bin/bash
# Small-path A/B (2N <= 2048, d <= 256: one forward + one backward launch) of a variant binary
# against the default: bitwise gradient digest, then fwd+bwd ms in two interleaved rounds.
# usage: tools/gpu_small_ab.sh TAG VARIANT
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-small_ab}; mkdir -p $OUT
V=$2
CFGS=("s512x256 --batch 512 --dim 256" "s1024x128 --batch 1024 --dim 128" "s256x64 --batch 256 --dim 64")
for r in 1 2; do
  for c in "${CFGS[@]}"; do
    set -- $c; t=$1; shift
    for v in base $V; do
      bin=build/bin/ntxent_bench; [ $v = base ] || bin=build/bin/ntxent_bench_$v
      timeout -k 10 60 $bin "$@" --iters 200 --warmup 50 --grad-digest > $OUT/r${r}_${t}_$v.log 2>&1 || { echo "fail $t $v"; tail -5 $OUT/r${r}_${t}_$v.log; exit 1; }
      fb=$(grep -A1 'fwd+bwd' $OUT/r${r}_${t}_$v.log | tail -1 | awk -F'|' '{print $4}' | awk '{print $1}')
      echo "r$r $t $v fwdbwd=$fb $(grep 'grad digest' $OUT/r${r}_${t}_$v.log)"
    done
  done
done
echo done
