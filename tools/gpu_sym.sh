#!/bin/bash
# Symmetric data-parallel mode on one MI355X: emulated W-rank numerics, W gloo processes sharing
# the GPU, per-rank compute cost vs the all-gather mode, and a 2-rank bench rehearsal.
set -o pipefail
TAG=${1:-sym}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fp8.py -k "symmetric" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_sym.log 2>&1 || { echo "sym tests failed"; tail -40 $OUT/pytest_sym.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiproc.py -k "symmetric-symmetric" -x -v --timeout 240 --timeout-method thread > $OUT/pytest_sym_mp.log 2>&1 || { echo "sym multiproc failed"; tail -40 $OUT/pytest_sym_mp.log; exit 1; }
timeout -k 10 300 python tools/sym_cost.py --iters 5 > $OUT/sym_cost.log 2>&1 || { echo "sym cost failed"; tail -20 $OUT/sym_cost.log; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --share-gpu --negatives symmetric > $OUT/bench_gloo2.log 2>&1 || { echo "gloo bench failed"; tail -20 $OUT/bench_gloo2.log; exit 1; }
echo done
