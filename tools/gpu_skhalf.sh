#!/bin/bash
# fp16 split-K slabs: split-K GPU tests, then a same-call A/B of config 4 (B = 1024/view, d = 8192,
# split-K forward) and config 2 (B = 4096, d = 512, split-K dZ): default (fp16 slabs) vs
# --no-sk-half --no-sk-dz-half, interleaved rounds, rocprofv3 kernel averages.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-skhalf}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fwdstream.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
for rep in 1 2 3; do
for v in half f32; do
  F=""; [ $v = f32 ] && F="--no-sk-half --no-sk-dz-half"
  for c in "cfg4 --batch 1024 --dim 8192" "cfg2 --batch 4096 --dim 512"; do
    set -- $c; t=$1; shift
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/p_${t}_${v}_$rep -o run --output-format csv -- build/bin/ntxent_bench "$@" $F --iters 50 --warmup 10 > $OUT/${t}_${v}_$rep.log 2>&1 || { echo "$t $v failed"; tail $OUT/${t}_${v}_$rep.log; exit 1; }
    f=$(find $OUT/p_${t}_${v}_$rep -name '*kernel_stats.csv' | head -1)
    echo "$t $v r$rep: fwdbwd=$(grep -A1 'fwd+bwd' $OUT/${t}_${v}_$rep.log | tail -1 | awk -F'|' '{print $4}' | awk '{print $1}') fwd=$(grep -h 'Li0ELi1EEEvNS0_9SimParamsE' $f | cut -d, -f4) skr=$(grep -h 'sk_reduce' $f | cut -d, -f4) dz=$(grep -h 'Li2ELi1EEEvNS0_9SimParamsE' $f | cut -d, -f4) skdz=$(grep -h 'sk_dz_reduce' $f | cut -d, -f4)"
  done
done
done
for v in half f32; do  # without the profiler
  F=""; [ $v = f32 ] && F="--no-sk-half --no-sk-dz-half"
  timeout -k 10 120 build/bin/ntxent_bench --batch 1024 --dim 8192 $F --iters 100 --warmup 20 > $OUT/plain_cfg4_$v.log 2>&1 || exit 1
  timeout -k 10 120 build/bin/ntxent_bench --batch 4096 --dim 512 $F --iters 100 --warmup 20 > $OUT/plain_cfg2_$v.log 2>&1 || exit 1
  echo "plain $v: cfg4 $(grep -A1 'fwd+bwd' $OUT/plain_cfg4_$v.log | tail -1 | awk -F'|' '{print $4}') cfg2 $(grep -A1 'fwd+bwd' $OUT/plain_cfg2_$v.log | tail -1 | awk -F'|' '{print $4}')"
done
echo done
