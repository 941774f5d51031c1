#!/bin/bash
# Variant builds (tools/build_variant.sh) against the default binary: bitwise gradient digest at
# the BASELINE shapes (layout / prefetch variants must not change a bit), then per-kernel times
# under rocprofv3 in two interleaved rounds.
# usage: tools/gpu_variants.sh TAG "v1 v2 ..." [kernel-name regex]
#   a variant "+flag" is the default binary run with --flag (a runtime option instead of a build)
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-variants}; mkdir -p $OUT
VARS=$2; PAT=${3:-sim_gemm|coef|diag_up|sk_}
CFGS=("head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg5 --batch 8192 --dim 1024 --compute fp16" "cfg4 --batch 1024 --dim 8192")
for c in "${CFGS[@]}"; do
  set -- $c; t=$1; shift
  for v in base $VARS; do
    bin=build/bin/ntxent_bench; ex=""; [ $v = base ] || bin=build/bin/ntxent_bench_$v
    case $v in +*) bin=build/bin/ntxent_bench; ex="--${v#+}";; esac
    timeout -k 10 120 $bin "$@" $ex --iters 3 --warmup 1 --grad-digest > $OUT/dig_${t}_$v.log 2>&1 || { echo "digest $t $v failed"; tail -5 $OUT/dig_${t}_$v.log; exit 1; }
    echo "$t $v $(grep 'grad digest' $OUT/dig_${t}_$v.log)"
  done
done
for r in 1 2; do
  for c in "${CFGS[@]}"; do
    set -- $c; t=$1; shift
    for v in base $VARS; do
      bin=build/bin/ntxent_bench; ex=""; [ $v = base ] || bin=build/bin/ntxent_bench_$v
      case $v in +*) bin=build/bin/ntxent_bench; ex="--${v#+}";; esac
      d=$OUT/r${r}_${t}_$v
      timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- $bin "$@" $ex --iters 30 --warmup 10 > $d.log 2>&1 || { echo "fail $t $v"; tail -5 $d.log; exit 1; }
      ks=$(find $d -name "*kernel_stats.csv" | head -1)
      fb=$(grep -A1 'fwd+bwd' $d.log | tail -1 | awk -F'|' '{print $4}' | awk '{print $1}')
      echo "r$r $t $v fwdbwd=$fb: $(python3 -c "
import csv,re
for x in csv.DictReader(open('$ks')):
    if re.search('$PAT', x['Name']): print(re.sub(r'void ntxent::dev::|<|>|\(.*','',x['Name'])[:34], round(float(x['AverageNs'])/1e3,1), end=' | ')
")"
    done
  done
done
echo done
