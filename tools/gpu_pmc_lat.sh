#!/bin/bash
# Is the GEMM operand staging latency- or bandwidth-bound? L2 (TCC) hit rate and the average
# vector-L1 -> L2 read latency (TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ) per kernel of the
# headline step (native bench). One pass per counter group, --kernel-trace only.
set -o pipefail
TAG=${1:-pmc_lat}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
have() { grep -qw "$1" $OUT/counters.txt; }
pick() { local out=""; for c in "$@"; do have $c && out="$out $c"; done; echo $out; }
P1=$(pick TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum)
P2=$(pick TA_BUSY_avr TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE)
echo "pass1: $P1" > $OUT/passes.txt; echo "pass2: $P2" >> $OUT/passes.txt
grep -iE "latency|TA_BUSY|PENDING|STALL" $OUT/counters.txt | head -40 > $OUT/candidates.txt
BENCH="build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P1 -d $OUT/p1 -o run --output-format csv -- $BENCH > $OUT/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P2 -d $OUT/p2 -o run --output-format csv -- $BENCH > $OUT/p2.log 2>&1
echo rc=$?
cat $OUT/passes.txt
