#!/bin/bash
# Rehearsal of the driver's round-end GPU steps: smoke(), pytest -m gpu, 1-GPU bench, and the
# N-rank bench path rehearsed on one GPU (gloo, then RCCL over sockets; all ranks on cuda:0).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-roundend}; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 200 python bench.py > $OUT/bench1.log 2>&1 || { echo "bench1 failed"; tail $OUT/bench1.log; exit 1; }
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2955$N bench.py --gpus $N --steps 3 --warmup 1 --backend gloo --share-gpu > $OUT/bench_gloo$N.log 2>&1 || { echo "gloo bench N=$N failed"; tail -20 $OUT/bench_gloo$N.log; exit 1; }
done
for N in 2 4; do  # RCCL itself (per-rank host ids, socket transport on one GPU)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2966$N bench.py --gpus $N --steps 3 --warmup 1 --backend nccl --share-gpu > $OUT/bench_rccl$N.log 2>&1 || { echo "rccl bench N=$N failed"; tail -20 $OUT/bench_rccl$N.log; exit 1; }
done
echo done
