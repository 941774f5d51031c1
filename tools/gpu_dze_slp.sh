#!/bin/bash
# DzE GEMM and the other GEMMs with and without SLP vectorisation (ablation builds), ABL 0 and 128.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzeslp}; mkdir -p $OUT
for B in ntxent_bench_abl ntxent_bench_abl_noslp; do
for A in 0 128; do
  NTXENT_GEMM_ABL=$A timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$B$A -o run --output-format csv -- build/bin/$B --batch 4096 --dim 2048 --iters 10 --warmup 2 --exp > $OUT/$B$A.log 2>&1 || { echo "$B $A failed"; exit 1; }
  f=$(find $OUT/$B$A -name "*kernel_stats.csv" | head -1)
  python3 - $f "$B ABL $A" <<'PY'
import csv,sys
d={r['Name'][:40]: float(r['AverageNs'])/1000 for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], {k: round(v,1) for k,v in d.items() if 'gemm' in k or 'norm' in k})
PY
done; done
