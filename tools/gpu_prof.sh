#!/bin/bash
# rocprofv3 kernel stats of bench.py (N = 1) + the top kernels. usage: tools/gpu_prof.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-prof}; mkdir -p $OUT
shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off "$@" > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python tools/show_prof.py $OUT/kernel_stats.csv 10
