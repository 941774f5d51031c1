#!/bin/bash
# tools/l2_bound_probe.py timings, then per-list counters (MFMA busy, L2 hit/miss, L1->L2 latency).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-l2_bound}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/l2_bound_probe.py > $OUT/timing.log 2>&1 || { tail -20 $OUT/timing.log; exit 1; }
cat $OUT/timing.log
PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_TA_BUSY"
PB="TA_TA_BUSY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for L in plan512 same512 zero512; do
  for p in a b; do
    eval "C=\$P$(echo $p | tr a-b A-B)"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $OUT/${L}_$p -o run --output-format csv -- python3 tools/l2_bound_probe.py --only $L --iters 1 --warm 3 > $OUT/${L}_$p.log 2>&1 || { echo "pass $L $p failed"; tail -5 $OUT/${L}_$p.log; exit 1; }
    cp $(find $OUT/${L}_$p -name "*counter_collection.csv" | head -1) $OUT/${L}_${p}_counters.csv
  done
done
echo l2 bound done
