#!/bin/bash
# Small-problem path on the GPU box: its tests, the kernel tests, and the reference sweep on
# the native bench with and without the small path. usage: tools/gpu_small.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-small}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_small.log 2>&1 || { echo "small tests failed"; tail -40 $OUT/pytest_small.log; exit 1; }
tail -1 $OUT/pytest_small.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_kernels.log 2>&1 || { echo "kernel tests failed"; tail -40 $OUT/pytest_kernels.log; exit 1; }
tail -1 $OUT/pytest_kernels.log
timeout -k 10 200 build/bin/ntxent_bench --iters 50 --check > $OUT/refsweep_small.log 2>&1 || { echo "sweep failed"; tail -20 $OUT/refsweep_small.log; exit 1; }
timeout -k 10 200 build/bin/ntxent_bench --iters 50 --graph > $OUT/refsweep_graph.log 2>&1 || { echo "sweep graph failed"; tail -20 $OUT/refsweep_graph.log; exit 1; }
timeout -k 10 200 build/bin/ntxent_bench --iters 50 --no-small > $OUT/refsweep_large.log 2>&1 || { echo "sweep large failed"; tail -20 $OUT/refsweep_large.log; exit 1; }
awk -F"|" "NR>2 && NF>4 {print \$1 \"|\" \$4 \"|\" \$5}" $OUT/refsweep_graph.log
echo done
