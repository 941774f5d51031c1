#!/bin/bash
# LDS bank-conflict / activity counters of the dZ GEMMs: exponential (DzE) vs coefficient (Dz) path.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzepmc}; mkdir -p $OUT
for V in exp noexp; do
  F="--exp"; [ $V = noexp ] && F="--no-exp"
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/$V -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1 $F > $OUT/$V.log 2>&1 || { echo "pmc $V failed"; tail -5 $OUT/$V.log; exit 1; }
  f=$(find $OUT/$V -name "*counter_collection.csv" | head -1)
  python3 - $f $V <<'PY'
import csv,sys,collections
acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=r['Kernel_Name']
    if 'sim_gemm' not in k and 'coef' not in k: continue
    acc[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,d in acc.items():
    print(sys.argv[2], k[:60], {c: f"{v:.3g}" for c,v in d.items()})
PY
done
