#!/bin/bash
# World-size-8 rehearsal on the 1-GPU box (8 ranks share cuda:0; RCCL over its socket transport
# with per-rank NCCL_HOSTID): bench.py's launcher + symmetric / all-gather data-parallel step and the
# native Engine's RcclComm at N = 8, then the per-rank compute floor of config 3 (tools/sym_cost.py,
# one rank's kernels at W = 1, 2, 4, 8 with the gathered buffers filled locally) and the host-side
# enqueue cost of the autograd step (tools/bench_overhead.py).
# usage: tools/gpu_w8.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-w8}; mkdir -p $OUT
for neg in symmetric allgather; do
  timeout -k 10 300 python bench.py --gpus 8 --backend nccl --share-gpu --batch 512 --dim 256 --steps 3 --warmup 1 \
      --prewarm-steps 2 --negatives $neg --timeout 240 > $OUT/bench8_$neg.log 2>&1 || { echo "bench N=8 $neg failed"; tail -30 $OUT/bench8_$neg.log; exit 1; }
  echo "bench.py N=8 $neg: $(grep '^{' $OUT/bench8_$neg.log | cut -c1-300)"
  timeout -k 10 300 python bench.py --gpus 8 --impl native --backend nccl --share-gpu --batch 512 --dim 256 --steps 3 \
      --warmup 1 --prewarm-steps 2 --negatives $neg --timeout 240 > $OUT/bench8_native_$neg.log 2>&1 || { echo "native N=8 $neg failed"; tail -30 $OUT/bench8_native_$neg.log; exit 1; }
  echo "bench.py --impl native N=8 $neg: $(grep '^{' $OUT/bench8_native_$neg.log | cut -c1-300)"
  timeout -k 10 300 python tools/cpp_rccl_procs.py --gpus 8 --shared-gpu --negatives $neg --batch 512 --dim 128 \
      --timeout 200 > $OUT/cpp8_$neg.log 2>&1 || { echo "cpp N=8 $neg failed"; tail -30 $OUT/cpp8_$neg.log; exit 1; }
  tail -2 $OUT/cpp8_$neg.log
done
timeout -k 10 400 python tools/sym_cost.py --worlds 1,2,4,8 --iters 5 > $OUT/sym_cost.log 2>&1 || { echo "sym_cost failed"; tail -20 $OUT/sym_cost.log; exit 1; }
cat $OUT/sym_cost.log | tail -12
timeout -k 10 200 python tools/bench_overhead.py > $OUT/overhead.log 2>&1 || { echo "overhead failed"; tail -20 $OUT/overhead.log; exit 1; }
cat $OUT/overhead.log
echo done
