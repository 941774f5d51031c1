#!/bin/bash
# Per-kernel time of selected kernels (name pattern) across A/B flag sets of the native bench,
# rocprofv3 kernel stats, interleaved rounds.
# usage: tools/gpu_kgrep.sh TAG PATTERN "flagsA|flagsB|..." ["cfg args" ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-kgrep}; mkdir -p $OUT
PAT=$2; IFS='|' read -ra FLAGS <<< "$3"; shift 3
CFGS=("$@"); [ ${#CFGS[@]} -gt 0 ] || CFGS=("head --batch 4096 --dim 2048")
for r in 1 2; do
  for c in "${CFGS[@]}"; do
    set -- $c; t=$1; shift
    for i in "${!FLAGS[@]}"; do
      f=${FLAGS[$i]}; d=$OUT/r${r}_${t}_$i
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- build/bin/ntxent_bench "$@" $f --iters 30 --warmup 10 > $d.log 2>&1 || { echo "fail $t $f"; tail -5 $d.log; exit 1; }
      ks=$(find $d -name "*kernel_stats.csv" | head -1)
      echo "r$r $t [$f]: $(python3 -c "
import csv,sys,re
for x in csv.DictReader(open('$ks')):
    if re.search('$PAT', x['Name']): print(x['Name'][17:45], round(float(x['AverageNs'])/1e3,1), end=' | ')
")"
    done
  done
done
