#!/bin/bash
# Comm/compute overlap on one GPU (tools/overlap_proxy.py): which stream / HW-queue setup lets
# the RCCL kernel run under the persistent GEMM; kernel trace of each variant.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ovl}; mkdir -p $OUT
for v in "current 4" "new 4" "high 4" "current 8" "new 8" "high 16"; do
  set -- $v; gs=$1; q=$2
  GPU_MAX_HW_QUEUES=$q timeout -k 10 150 python tools/overlap_proxy.py --gemm-stream $gs --reserves 0,8,16,32 --iters 10 --json $OUT/${gs}_q$q.json > $OUT/${gs}_q$q.log 2>&1 || { echo "proxy $gs q$q failed"; tail -5 $OUT/${gs}_q$q.log; exit 1; }
  echo "== stream=$gs GPU_MAX_HW_QUEUES=$q"; grep -E "^reserve" $OUT/${gs}_q$q.log
done
for v in "current 4" "high 16"; do
  set -- $v; gs=$1; q=$2
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace_${gs}_q$q -o run --output-format csv -- python tools/overlap_proxy.py --gemm-stream $gs --iters 3 --reserves 16 > $OUT/trace_${gs}_q$q.log 2>&1 || { echo "trace $gs failed"; tail -5 $OUT/trace_${gs}_q$q.log; exit 1; }
done
echo done
