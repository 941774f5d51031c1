#!/bin/bash
# Same-call A/B of build/bin/ntxent_bench (working tree) vs build/bin/ntxent_bench_old
# (tools/build_ab_old.sh REV), interleaved rounds; rocprofv3 kernel averages of the GEMMs.
# usage: tools/gpu_binab.sh TAG [rounds]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-binab}; mkdir -p $OUT
R=${2:-3}
for rep in $(seq 1 $R); do
for b in new old; do
  BIN=build/bin/ntxent_bench; [ $b = old ] && BIN=build/bin/ntxent_bench_old
  for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
    set -- $c; t=$1; shift
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_${t}_${b}_$rep -o run --output-format csv -- $BIN "$@" --iters 20 --warmup 5 > $OUT/${t}_${b}_$rep.log 2>&1 || { echo "$t $b failed"; exit 1; }
    f=$(find $OUT/p_${t}_${b}_$rep -name '*kernel_stats.csv' | head -1)
    echo "$t $b r$rep: fwdbwd=$(grep -A1 'fwd+bwd' $OUT/${t}_${b}_$rep.log | tail -1 | awk -F'|' '{print $4}' | awk '{print $1}') fwdgemm=$(grep -h 'Li0ELi0ELi1E' $f | cut -d, -f4) dz=$(grep -h 'Li2ELi0ELi1E' $f | cut -d, -f4)"
  done
done
done
echo done
