#!/bin/bash
# RCCL at W > 1 on the 1-GPU box (per-rank NCCL_HOSTID, socket transport): probe, the
# multi-process RCCL tests against the fp64 oracle, and bench.py's N-rank path over RCCL.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-rccl_shared}; mkdir -p $OUT
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 tools/rccl_two_ranks_one_gpu.py > $OUT/probe.log 2>&1 || { echo "probe failed"; tail -20 $OUT/probe.log; exit 1; }
grep '^{' $OUT/probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -k rccl -x -v --timeout 280 --timeout-method thread > $OUT/pytest_rccl.log 2>&1 || { echo "rccl tests failed"; tail -30 $OUT/pytest_rccl.log; exit 1; }
tail -1 $OUT/pytest_rccl.log
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2966$N bench.py --gpus $N --steps 3 --warmup 1 --backend nccl --share-gpu > $OUT/bench_rccl$N.log 2>&1 || { echo "rccl bench N=$N failed"; tail -20 $OUT/bench_rccl$N.log; exit 1; }
  grep '^{' $OUT/bench_rccl$N.log | cut -c1-400
done
echo done
