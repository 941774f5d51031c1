#!/bin/bash
# Round 6, verdict item 1/2: the data-parallel step's host cost and the config-3 shape on one GPU.
#   1. the RCCL multi-process tests (engine and torch implementations) + the config-3 W = 4 test
#   2. bench.py --gpus N --backend nccl --share-gpu at B = 4096, d = 2048 for N = 2, 4, 8, both
#      negatives modes, dist-impl engine (the default) and torch: host_enqueue_ms_per_step
#   3. cProfile of the torch symmetric path's host side at N = 8 (where its time goes)
# usage: tools/gpu_r6_dist.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6dist}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiproc.py -k "rccl" -v -rA --durations 10 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_rccl.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest_rccl.log | tail -2
grep -E "^(FAILED|ERROR)" $OUT/pytest_rccl.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
B="--batch 4096 --dim 2048 --steps 5 --warmup 1 --prewarm-steps 2 --backend nccl --share-gpu --timeout 280"
for N in 2 4 8; do
  for neg in symmetric allgather; do
    for impl in engine torch; do
      hp=""
      if [ $N = 8 ] && [ $impl = torch ]; then hp="--host-profile $OUT/hostprof_${neg}_w8.txt"; fi
      timeout -k 10 300 python bench.py --gpus $N $B --negatives $neg --dist-impl $impl $hp --json-out $OUT/b${N}_${neg}_${impl}.json > $OUT/b${N}_${neg}_${impl}.log 2>&1 || { echo "bench N=$N $neg $impl failed"; tail -30 $OUT/b${N}_${neg}_${impl}.log; exit 1; }
      python - $OUT/b${N}_${neg}_${impl}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config"]
print(f"N={d['n_gpus']} {c['negatives']:9s} {c['dist_impl']:6s} host_enqueue={d['host_enqueue_ms_per_step']:.3f} ms  socket ms/step={d['ms_per_step']:.1f}  loss={d['loss']:.8f} peak={d['peak_hbm_mb']}")
PY
    done
  done
done
echo done
