#!/bin/bash
# Hardware counters of the headline step's kernels (native bench, B=4096/view, d=2048):
#   pass 1  MFMA busy / MFMA instruction counts / LDS bank conflicts (SQ block)
#   pass 2  HBM bytes read (FETCH_SIZE) + GPU busy clocks
#   pass 3  HBM bytes written (WRITE_SIZE)
# Counters only with --kernel-trace (never with sys/runtime traces). Each pass keeps to the
# per-block limits (<= 8 SQ, <= 4 TCC, <= 2 GRBM) and only names counters `rocprofv3 -L` lists.
set -o pipefail
TAG=${1:-pmc_mfma}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
have() { grep -qw "$1" $OUT/counters.txt; }
pick() { local out=""; for c in "$@"; do have $c && out="$out $c"; done; echo $out; }
P1=$(pick SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU)
P2=$(pick FETCH_SIZE GRBM_GUI_ACTIVE)
P3=$(pick WRITE_SIZE GRBM_COUNT)
echo "pass1: $P1" > $OUT/passes.txt; echo "pass2: $P2" >> $OUT/passes.txt; echo "pass3: $P3" >> $OUT/passes.txt
BENCH="build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P1 -d $OUT/p1 -o run --output-format csv -- $BENCH > $OUT/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P2 -d $OUT/p2 -o run --output-format csv -- $BENCH > $OUT/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P3 -d $OUT/p3 -o run --output-format csv -- $BENCH > $OUT/p3.log 2>&1
echo rc=$?
