#!/bin/bash
# BASELINE.json configs + reference sweeps on one MI355X (native bench, bench.py, python harness).
set -o pipefail
TAG=${1:-cfg}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B=build/bin/ntxent_bench
timeout -k 10 200 $B --batch 4096 --dim 512 --iters 50 --warmup 5 --graph --json $OUT/cfg2.json > $OUT/cfg2.log 2>&1 || exit 1
timeout -k 10 200 $B --batch 1024 --dim 8192 --iters 50 --warmup 5 --graph --json $OUT/cfg4.json > $OUT/cfg4.log 2>&1 || exit 1
timeout -k 10 200 $B --batch 8192 --dim 1024 --compute fp8 --iters 30 --warmup 3 --json $OUT/cfg5.json > $OUT/cfg5.log 2>&1 || exit 1
timeout -k 10 200 $B --batch 4096 --dim 2048 --iters 50 --warmup 5 --graph --json $OUT/head.json > $OUT/head.log 2>&1 || exit 1
timeout -k 10 300 $B --iters 100 --warmup 1 --check --json $OUT/refsweep.json > $OUT/refsweep.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $OUT/bench.log 2>&1 || exit 1
timeout -k 10 600 python bench/harness.py --out-dir $OUT/harness > $OUT/harness.log 2>&1 || exit 1
echo done
