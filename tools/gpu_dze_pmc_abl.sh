#!/bin/bash
# LDS bank conflicts of the DzE GEMM per compile-time ablation (which LDS access conflicts).
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzepmcabl}; mkdir -p $OUT
for A in ${ABLS:-0 128 2 130}; do
  NTXENT_GEMM_ABL=$A timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $OUT/a$A -o run --output-format csv -- build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 2 --warmup 1 --exp > $OUT/a$A.log 2>&1 || { echo "pmc $A failed"; tail -5 $OUT/a$A.log; exit 1; }
  f=$(find $OUT/a$A -name "*counter_collection.csv" | head -1)
  python3 - $f $A <<'PY'
import csv,sys,collections
acc=collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if 'Li3E' in r['Kernel_Name']: acc[r['Counter_Name']]+=float(r['Counter_Value'])
print('ABL', sys.argv[2], {c: f"{v:.3g}" for c,v in acc.items()})
PY
done
