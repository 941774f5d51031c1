#!/bin/bash
# Coefficient-free dZ GEMM: native bench exp vs --no-exp, then compile-time ablations of the DzE
# main loop (rocprofv3 kernel stats per variant). usage: tools/gpu_dze_abl.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzeabl}; mkdir -p $OUT
timeout -k 10 120 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 30 --warmup 5 --exp > $OUT/native_exp.log 2>&1 || { echo "native failed"; tail $OUT/native_exp.log; exit 1; }
timeout -k 10 120 build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 30 --warmup 5 --no-exp > $OUT/native_noexp.log 2>&1 || { echo "native noexp failed"; exit 1; }
grep -iE "fwd\+bwd|backward|forward" $OUT/native_exp.log | head -4; echo ---; grep -iE "fwd\+bwd|backward|forward" $OUT/native_noexp.log | head -4
for A in ${ABLS:-0 1 2 4 128 129 130 6 134}; do
  NTXENT_GEMM_ABL=$A timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/a$A -o run --output-format csv -- build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 10 --warmup 2 --exp > $OUT/a$A.log 2>&1 || { echo "abl $A failed"; exit 1; }
  f=$(find $OUT/a$A -name "*kernel_stats.csv" | head -1)
  python3 - $f $A <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'Li3E' in r['Name']: print(f"ABL {sys.argv[2]:>4}: DzE {float(r['AverageNs'])/1000:8.1f} us")
PY
done
