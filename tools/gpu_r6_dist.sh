#!/bin/bash
# Round 6, verdict items 1/2: the data-parallel step's host cost and the config-3 shape on one GPU.
#   1. pytest selection ($2, default: the RCCL multi-process tests incl. the config-3 W = 4 test)
#   2. bench.py (N = 1) twice: headline regression check
#   3. bench.py --gpus N --backend nccl --share-gpu at B = 4096, d = 2048 for N in $3 (default
#      "2 8"), both negatives modes, dist-impl engine (the default) and torch:
#      host_enqueue_ms_per_step; cProfile of the torch path's host side at N = 8
# usage: tools/gpu_r6_dist.sh TAG [PYTEST_ARGS] [NS]
set -o pipefail
export TMPDIR=/tmp NTXENT_GPU_CHECK=1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6dist}; mkdir -p $OUT
SEL=${2:-"tests/test_gpu_multiproc.py -k rccl"}
NS=${3:-"2 8"}
eval timeout -k 10 900 python -u -m pytest $SEL -v -rA --durations 10 --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $OUT/pytest.log | tail -2
grep -E "^(FAILED|ERROR)" $OUT/pytest.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 1; fi
for i in 1 2; do
timeout -k 10 200 python bench.py > $OUT/bench$i.log 2>&1 || { echo "bench failed"; tail $OUT/bench$i.log; exit 1; }
tail -1 $OUT/bench$i.log | cut -c1-200
done
B="--batch 4096 --dim 2048 --steps 5 --warmup 1 --prewarm-steps 2 --backend nccl --share-gpu --timeout 280"
for N in $NS; do
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
