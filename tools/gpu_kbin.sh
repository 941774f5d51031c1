#!/bin/bash
# Per-kernel time of selected kernels (name pattern) across variant binaries of the native bench
# (build/bin/ntxent_bench_<v>, "base" = build/bin/ntxent_bench, "base:--flag" passes a flag),
# rocprofv3 kernel stats, two interleaved rounds.
# usage: tools/gpu_kbin.sh TAG PATTERN "v1 v2 ..." ["cfg args" ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-kbin}; mkdir -p $OUT
PAT=$2; VARS=$3; shift 3
CFGS=("$@"); [ ${#CFGS[@]} -gt 0 ] || CFGS=("head --batch 4096 --dim 2048")
for r in 1 2; do
  for c in "${CFGS[@]}"; do
    set -- $c; t=$1; shift
    for v in $VARS; do
      bin=build/bin/ntxent_bench; flag=""
      case $v in base) ;; base:*) flag=${v#base:} ;; *) bin=build/bin/ntxent_bench_$v ;; esac
      d=$OUT/r${r}_${t}_${v//[:-]/_}
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- $bin "$@" $flag --iters 30 --warmup 10 > $d.log 2>&1 || { echo "fail $t $v"; tail -5 $d.log; exit 1; }
      ks=$(find $d -name "*kernel_stats.csv" | head -1)
      echo "r$r $t $v: $(python3 -c "
import csv,re
for x in csv.DictReader(open('$ks')):
    if re.search('$PAT', x['Name']): print(x['Name'][17:45], round(float(x['AverageNs'])/1e3,1), end=' | ')
")"
    done
  done
done
