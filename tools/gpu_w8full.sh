#!/bin/bash
# Config-3 size (B = 4096/rank, d = 2048) rehearsal of the W = 8 data-parallel paths on the 1-GPU
# box (verdict r4, item 1): 8 ranks share cuda:0, RCCL over its socket transport.
#   part "a": bench.py --gpus 8 (torch path, symmetric + all-gather), tools/w8_full_check.py
#             (symmetric vs all-gather vs an fp32 torch oracle, per-rank peak HBM)
#   part "b": bench.py --gpus 8 --impl native (symmetric + all-gather), then the W = 2 kernel-trace
#             overlap at CU reserves 0 / 8 / 16 (tools/overlap_trace.py)
# usage: tools/gpu_w8full.sh TAG a|b
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-w8full}; mkdir -p $OUT
B="--batch 4096 --dim 2048"
if [ "$2" = "a" ]; then
for neg in symmetric allgather; do
  timeout -k 10 300 python bench.py --gpus 8 --backend nccl --share-gpu $B --steps 2 --warmup 1 \
      --prewarm-steps 1 --negatives $neg --timeout 280 > $OUT/bench8_$neg.log 2>&1 || { echo "bench N=8 $neg failed"; tail -30 $OUT/bench8_$neg.log; exit 1; }
  echo "bench.py N=8 $neg: $(grep '^{' $OUT/bench8_$neg.log | cut -c1-200)"
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29711 tools/w8_full_check.py $B --json-out $OUT/w8_full_check.json > $OUT/w8_full_check.log 2>&1 || { echo "w8_full_check failed"; tail -30 $OUT/w8_full_check.log; exit 1; }
cat $OUT/w8_full_check.json | cut -c1-600
fi
if [ "$2" = "b" ]; then
for neg in symmetric allgather; do
  timeout -k 10 300 python bench.py --gpus 8 --impl native --backend nccl --share-gpu $B --steps 2 --warmup 1 \
      --prewarm-steps 1 --negatives $neg --timeout 280 > $OUT/bench8_native_$neg.log 2>&1 || { echo "native N=8 $neg failed"; tail -30 $OUT/bench8_native_$neg.log; exit 1; }
  echo "bench.py --impl native N=8 $neg: $(grep '^{' $OUT/bench8_native_$neg.log | cut -c1-200)"
done
timeout -k 10 600 python tools/overlap_trace.py run --out $OUT/ov --world 2 --reserves 0,8,16 --timeout 180 > $OUT/ov.log 2>&1 || { echo "overlap trace failed"; tail -30 $OUT/ov.log; exit 1; }
python tools/overlap_trace.py analyze $OUT/ov --json $OUT/overlap.json | tee $OUT/overlap.md
find $OUT/ov -name "*.csv" ! -name "*kernel_trace.csv" -delete
fi
echo done
