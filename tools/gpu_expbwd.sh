#!/bin/bash
# Coefficient-free backward: its GPU tests, then bench.py x2 and a rocprofv3 kernel-stat capture.
# usage: tools/gpu_expbwd.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-expbwd}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_expbwd.py -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest_expbwd.log 2>&1 || { echo "pytest failed"; grep -E "PARITY|PASS|FAIL|Error|error" $OUT/pytest_expbwd.log | tail -30; exit 1; }
grep -E "PARITY|passed|failed" $OUT/pytest_expbwd.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --secondary-fp32 off --steps 30 > $OUT/bench$i.log 2>&1 || { echo "bench failed"; tail $OUT/bench$i.log; exit 1; }
  tail -1 $OUT/bench$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['step_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --secondary-fp32 off > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
cp $(find $OUT/prof -name "*kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:9]:
    print(f"{float(r['AverageNs'])/1000:8.1f} us  x{r['Calls']:>3}  {r['Name'][:70]}")
PY
