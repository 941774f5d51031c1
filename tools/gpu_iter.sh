#!/bin/bash
# One build->measure iteration on the GPU box: GPU tests, GEMM item timelines (diagnostic
# build), native bench and bench.py. usage: tools/gpu_iter.sh TAG [pytest-args...]
set -o pipefail
TAG=${1:-iter}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
if [ -x build/bin/ntxent_bench_abl ]; then
  NTXENT_GEMM_ABL=64 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 3 --warmup 2 > $OUT/timeline.log 2>&1 || { echo "timeline failed"; tail -5 $OUT/timeline.log; exit 1; }
  grep TIMELINE $OUT/timeline.log | tail -2 | cut -c1-400
fi
timeout -k 10 120 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 30 --warmup 5 > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 120 python bench.py > $OUT/benchpy.log 2>&1 || { echo "bench.py failed"; tail -5 $OUT/benchpy.log; exit 1; }
tail -1 $OUT/benchpy.log | cut -c1-220
