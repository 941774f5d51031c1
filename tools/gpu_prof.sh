#!/bin/bash
# rocprofv3 kernel statistics of the headline bench (bench.py) plus the BASELINE.json configs
# on the native bench. usage: tools/gpu_prof.sh TAG
set -o pipefail
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "prof failed"; tail -5 $OUT/prof.log; exit 1; }
python tools/show_prof.py $OUT/prof/run_kernel_stats.csv 9
B=build/bin/ntxent_bench
timeout -k 10 120 $B --batch 4096 --dim 2048 --iters 50 --warmup 5 --graph --json $OUT/head.json > $OUT/head.log 2>&1 || exit 1
timeout -k 10 120 $B --batch 4096 --dim 512 --iters 50 --warmup 5 --graph --json $OUT/cfg2.json > $OUT/cfg2.log 2>&1 || exit 1
timeout -k 10 120 $B --batch 1024 --dim 8192 --iters 50 --warmup 5 --graph --json $OUT/cfg4.json > $OUT/cfg4.log 2>&1 || exit 1
timeout -k 10 120 $B --batch 8192 --dim 1024 --compute fp8 --iters 30 --warmup 3 --json $OUT/cfg5.json > $OUT/cfg5.log 2>&1 || exit 1
for f in head cfg2 cfg4 cfg5; do tail -1 $OUT/$f.log; done
