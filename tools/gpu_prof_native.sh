#!/bin/bash
# rocprofv3 kernel stats of the native bench at named configs. usage: tools/gpu_prof_native.sh TAG cfg...
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-profn}; mkdir -p $OUT
shift
args() { case $1 in head) echo "--batch 4096 --dim 2048";; cfg2) echo "--batch 4096 --dim 512";; cfg4) echo "--batch 1024 --dim 8192";;
  cfg5) echo "--batch 8192 --dim 1024 --compute fp16";; cfg5f8) echo "--batch 8192 --dim 1024 --compute fp8";; esac; }
for c in "$@"; do
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/$c -o run --output-format csv -- build/bin/ntxent_bench $(args $c) --iters 20 --warmup 5 > $OUT/$c.log 2>&1 || { echo "prof $c failed"; tail -5 $OUT/$c.log; exit 1; }
  cp $(find $OUT/$c -name "*kernel_stats.csv" | head -1) $OUT/${c}_kernel_stats.csv
  echo "== $c: $(grep -A1 'fwd+bwd' $OUT/$c.log | tail -1 | cut -c1-140)"
  python tools/show_prof.py $OUT/${c}_kernel_stats.csv 12
done
