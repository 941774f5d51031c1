#!/bin/bash
# Forward-GEMM time vs the stream-K split factor p (diagnostic build: NTXENT_SK_SPLIT) at the
# headline shape and BASELINE configs 2, 4, 5. usage: tools/gpu_sksweep.sh TAG
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sksweep}; mkdir -p $OUT
export TMPDIR=/tmp
sweep() {  # tag, shape args
  local t=$1; shift
  for P in 1 2 3 4 6 8; do
    NTXENT_SK_SPLIT=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/${t}_p$P -o run --output-format csv -- build/bin/ntxent_bench_abl "$@" --iters 10 --warmup 2 > $OUT/${t}_p$P.log 2>&1 || return 1
    echo "$t p=$P fwd_gemm_ns=$(grep -h 'Li0ELi0ELi1E\|fp8e4m3, 0, 0, 1' $(find $OUT/${t}_p$P -name '*kernel_stats.csv') | head -1 | awk -F'",' '{print $2}' | cut -d, -f3)"
  done
}
sweep head --batch 4096 --dim 2048 && sweep cfg4 --batch 1024 --dim 8192 && sweep cfg2 --batch 4096 --dim 512 && \
sweep cfg5 --batch 8192 --dim 1024 --compute fp16 && sweep cfg5f8 --batch 8192 --dim 1024 --compute fp8
