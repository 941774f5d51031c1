set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/dzexp; mkdir -p $OUT
for r in 1 2; do
for v in "A" "B" "C"; do
  case $v in A) E=""; F="";; B) E="NTXENT_DZSYM_NOMIR=1"; F="";; C) E=""; F="--no-dzsym";; esac
  for c in "head --batch 4096 --dim 2048" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
    set -- $c; t=$1; shift
    env $E timeout -k 10 120 build/bin/ntxent_bench "$@" $F --iters 40 --warmup 10 > $OUT/$t$v.log 2>&1 || { echo fail; exit 1; }
    echo "$v $t: $(grep -A1 'fwd+bwd' $OUT/$t$v.log | tail -1 | cut -c40-150)"
  done
done; done
for v in A B; do
  case $v in A) E="";; B) E="NTXENT_DZSYM_NOMIR=1";; esac
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 10 --warmup 3 > $OUT/p$v.log 2>&1 || exit 1
  echo $v; python tools/show_prof.py $(find $OUT/p$v -name "*kernel_stats.csv" | head -1) 3
done
mkdir -p gpurun_out/ovl2
for gs in current new high; do
  timeout -k 10 120 python tools/overlap_proxy.py --gemm-stream $gs --reserves 0,16 --iters 10 > gpurun_out/ovl2/$gs.log 2>&1 || { echo "proxy $gs failed"; tail -5 gpurun_out/ovl2/$gs.log; exit 1; }
  grep -E "reserve|GPU_MAX" gpurun_out/ovl2/$gs.log
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python tools/overlap_proxy.py --gemm-stream new --reserves 0,16 --iters 10 > gpurun_out/ovl2/q8new.log 2>&1 && grep -E "reserve|GPU_MAX" gpurun_out/ovl2/q8new.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ovl2/trace_new -o run --output-format csv -- python tools/overlap_proxy.py --gemm-stream new --iters 3 --reserves 16 > gpurun_out/ovl2/trace_new.log 2>&1
echo done
