#!/bin/bash
# Forward-GEMM kernel time per variant (rocprofv3 kernel stats of the native bench), for
# ablation / A/B builds made by tools/build_variant.sh or by hand (build/bin/ntxent_bench_<v>).
# usage: tools/gpu_abl.sh TAG "v1 v2 ..." ["cfg args" ...]   (v = "" for build/bin/ntxent_bench,
#        "base:--flag" passes a flag to the base binary)
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-abl}; mkdir -p $OUT
VARS=$2; shift 2
CFGS=("$@"); [ ${#CFGS[@]} -gt 0 ] || CFGS=("head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512")
for r in 1 2; do
  for c in "${CFGS[@]}"; do
    set -- $c; t=$1; shift
    for v in $VARS; do
      bin=build/bin/ntxent_bench; flag=""
      case $v in base) ;; base:*) flag=${v#base:} ;; *) bin=build/bin/ntxent_bench_$v ;; esac
      d=$OUT/r${r}_${t}_${v//[:-]/_}
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- $bin "$@" $flag --iters 30 --warmup 10 > $d.log 2>&1 || { echo "fail $t $v"; tail -5 $d.log; exit 1; }
      ks=$(find $d -name "*kernel_stats.csv" | head -1)
      echo "r$r $t $v: $(python3 tools/show_prof.py $ks 3 | awk '{printf "%s %s | ", substr($1,17,32), $5}')"
    done
  done
done
