#!/bin/bash
# Where does dz_sym's GEMM lose time? A: --dzsym (upper C, mirrored steps read transposed, B from
# Zq by transposed reads); B: --dzsym with NTXENT_DZSYM_NOMIR=1 (full mirrored C read directly,
# B still from Zq); C: default (full C, B = Z^T by ds_read_b128). Two rounds, then kernel stats.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/dzexp; mkdir -p $OUT
for r in 1 2; do
for v in A B C; do
  case $v in A) E=""; F="--dzsym";; B) E="NTXENT_DZSYM_NOMIR=1"; F="--dzsym";; C) E=""; F="";; esac
  for c in "head --batch 4096 --dim 2048" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
    set -- $c; t=$1; shift
    env $E timeout -k 10 120 build/bin/ntxent_bench "$@" $F --iters 40 --warmup 10 > $OUT/$t$v.log 2>&1 || { echo fail; exit 1; }
    echo "$v $t: $(grep -A1 'fwd+bwd' $OUT/$t$v.log | tail -1 | cut -c40-150)"
  done
done; done
for v in A B C; do
  case $v in A) E=""; F="--dzsym";; B) E="NTXENT_DZSYM_NOMIR=1"; F="--dzsym";; C) E=""; F="";; esac
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 $F --iters 10 --warmup 3 > $OUT/p$v.log 2>&1 || exit 1
  cp $(find $OUT/p$v -name "*kernel_stats.csv" | head -1) $OUT/p${v}_kernel_stats.csv
  echo $v; python tools/show_prof.py $OUT/p${v}_kernel_stats.csv 4
done
