#!/bin/bash
# dz_sym A/B: correctness tests, native bench (default vs --no-dzsym) at the headline and
# configs 2/4/5, kernel stats + LDS counters of the dz_sym kernel.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-dzab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dzsym.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in "head --batch 4096 --dim 2048" "cfg2 --batch 4096 --dim 512" "cfg4 --batch 1024 --dim 8192" "cfg5 --batch 8192 --dim 1024 --compute fp16"; do
  set -- $c; t=$1; shift
  for r in 1 2; do for v in "" "--no-dzsym"; do
    timeout -k 10 120 build/bin/ntxent_bench "$@" $v --iters 40 --warmup 10 > $OUT/$t$v.log 2>&1 || { echo "native $t $v failed"; tail $OUT/$t$v.log; exit 1; }
    echo "$t $v: $(grep -A1 'fwd+bwd' $OUT/$t$v.log | tail -1 | cut -c40-150)"
  done; done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 10 --warmup 3 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python tools/show_prof.py $(find $OUT/prof -name "*kernel_stats.csv" | head -1) 8
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- build/bin/ntxent_bench --batch 4096 --dim 2048 --iters 3 --warmup 1 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
python3 - $(find $OUT/pmc -name "*counter_collection.csv" | head -1) <<'PY'
import csv,sys,collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if 'gemm' in r['Kernel_Name'] or 'dz_sym' in r['Kernel_Name']:
        agg[r['Kernel_Name'][:48]][r['Counter_Name']].append(float(r['Counter_Value']))
for n,d in agg.items():
    g=sum(d['GRBM_GUI_ACTIVE'])/len(d['GRBM_GUI_ACTIVE'])/8
    print(n, ' '.join(f"{k}={sum(v)/len(v):.3g}" for k,v in sorted(d.items())), f"mfma_busy={sum(d['SQ_VALU_MFMA_BUSY_CYCLES'])/len(d['SQ_VALU_MFMA_BUSY_CYCLES'])/(1024*g):.3f}")
PY
echo done
