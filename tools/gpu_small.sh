#!/bin/bash
# Reference forward-latency sweep (B {32..1024} x D {64,128,256}, host fp64 check) with the fused
# one-launch small forward (default) and with the prep launch (--small-fuse-rows 0), plus graphs.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-small}; mkdir -p $OUT
for v in "" "--small-fuse-rows 0" "--graph"; do
  t=$(echo "fused$v" | tr -d ' -')
  timeout -k 10 240 build/bin/ntxent_bench --check $v --iters 200 --warmup 20 > $OUT/$t.log 2>&1 || { echo "sweep $v failed"; tail $OUT/$t.log; exit 1; }
  echo "== $t"; grep -E "^ +[0-9]+ +[0-9]+ " $OUT/$t.log | awk '{print $1, $2, $4, "fwd", $6, "bwd", $11, "fb", $16, "graph", $21}'
  grep -iE "check|max" $OUT/$t.log | tail -3
done
