#!/bin/bash
# Which port binds the GEMMs? Hardware counters of the headline step (native bench,
# B=4096/view, d=2048), one pass per counter group (--kernel-trace --pmc only):
#   pass a  wave-state split (WAVE_CYCLES = ACTIVE + WAIT + WAIT_INST), MFMA busy, VMEM/LDS activity
#   pass b  texture-address / data / L1 unit busy and stall cycles, L2 hit/miss
#   pass c  LDS array cycles, bank conflicts, LDS / VMEM FIFO-full stalls
# usage: [BIN=build/bin/ntxent_bench_<variant>] tools/gpu_pmc_diag.sh TAG ["native bench args"]
set -o pipefail
TAG=${1:-pmc_diag}
ARGS=${2:-"--batch 4096 --dim 2048"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_TA_BUSY"
PB="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
PC="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_LDS GRBM_GUI_ACTIVE"
echo "a: $PA" > $OUT/passes.txt; echo "b: $PB" >> $OUT/passes.txt; echo "c: $PC" >> $OUT/passes.txt
BENCH="${BIN:-build/bin/ntxent_bench} $ARGS --iters 3 --warmup 1"
for p in a b c; do
  eval "C=\$P$(echo $p | tr a-c A-C)"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $OUT/$p -o run --output-format csv -- $BENCH > $OUT/$p.log 2>&1 || { echo "pass $p failed"; tail -5 $OUT/$p.log; exit 1; }
  cp $(find $OUT/$p -name "*counter_collection.csv" | head -1) $OUT/${p}_counters.csv
done
echo pmc done
