#!/bin/bash
# One GPU iteration: numerics quick-check, rocprof kernel stats of the headline bench, C++ bench.
# usage: tools/gpu_round.sh TAG  (outputs under gpurun_out/TAG/)
set -o pipefail
TAG=${1:-run}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/gpu_quick.py > $OUT/quick.log 2>&1 || { echo "quick failed"; tail -5 $OUT/quick.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; exit 1; }
if [ -x build/bin/ntxent_bench ]; then
  timeout -k 10 200 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 20 --warmup 3 > $OUT/cpp_bench.log 2>&1 || echo "cpp bench failed"
fi
echo done
