#!/bin/bash
# Round-2 baseline on the GPU box: smoke, GPU tests, 1-GPU bench (with fp32 secondary),
# the built-in launcher rehearsed with 2 ranks on one GPU (gloo), and a rocprofv3 kernel-stat
# capture of the headline step. usage: tools/gpu_r2_base.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r2base}; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench1.log 2>&1 || { echo "bench1 failed"; tail $OUT/bench1.log; exit 1; }
tail -1 $OUT/bench1.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --share-gpu > $OUT/bench_launch2.log 2>&1 || { echo "launcher N=2 failed"; tail -20 $OUT/bench_launch2.log; exit 1; }
tail -1 $OUT/bench_launch2.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
echo done
