#!/bin/bash
# Interleaved A/B of an environment switch on bench.py in one process tree (same box).
# usage: tools/gpu_ab.sh VAR VAL_A VAL_B [rounds] [bench.py args...]
set -o pipefail
VAR=$1; A=$2; B=$3; N=${4:-3}; shift 4
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab; mkdir -p $OUT
for i in $(seq $N); do
  for V in $A $B; do
    env $VAR=$V timeout -k 10 120 python bench.py --steps 40 --warmup 5 "$@" > $OUT/b.log 2>&1 || { echo "bench failed"; tail -3 $OUT/b.log; exit 1; }
    echo "$VAR=$V $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
