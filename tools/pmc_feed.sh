#!/bin/bash
# PMC counters of the GEMM feed path (counters only with --kernel-trace; no sys/runtime traces).
set -o pipefail
TAG=${1:-pmcfeed}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1"
i=0
for SET in "TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES" \
           "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_STALL_INFLIGHT_MAX" \
           "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCC_TAG_STALL" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $SET --kernel-include-regex "sim_gemm" -d $OUT/s$i -o run --output-format csv -- $B > $OUT/s$i.log 2>&1 || { echo "set $i failed"; tail -5 $OUT/s$i.log; }
done
echo done
