#!/bin/bash
# Final-bench evidence: smoke(), then bench.py x5 back-to-back on one box (the driver's command),
# one JSON line each, and their median. usage: tools/gpu_final_bench.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-final_bench}; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench$i.json 2> $OUT/bench$i.err || { echo "bench $i failed"; tail $OUT/bench$i.err; exit 1; }
  echo "run $i: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])" $OUT/bench$i.json)"
done
python - "$OUT" <<'PY' | tee $OUT/summary.txt
import json, statistics, sys, glob
ms = [json.loads(open(f).read().strip().splitlines()[-1])["ms_per_step"] for f in sorted(glob.glob(sys.argv[1] + "/bench*.json"))]
print("ms_per_step:", ms, "median", statistics.median(ms), "min", min(ms), "max", max(ms))
PY
