set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/bf16cmp; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do for c in fp16 bf16; do for cfg in "head --batch 4096 --dim 2048" "cfg5 --batch 8192 --dim 1024"; do
 set -- $cfg; t=$1; shift
 d=$OUT/r${r}_${t}_$c
 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- build/bin/ntxent_bench "$@" --compute $c --iters 30 --warmup 10 > $d.log 2>&1 || { echo fail; tail -5 $d.log; exit 1; }
 ks=$(find $d -name "*kernel_stats.csv" | head -1)
 fb=$(grep -A1 'fwd+bwd' $d.log | tail -1 | awk -F'|' '{print $4}' | awk '{print $1}')
 echo "r$r $t $c fwdbwd=$fb $(python3 tools/show_prof.py $ks 3 | tr '\n' ' ')"
done; done; done
