#!/bin/bash
# Buffer placement / data A/B on bench.py (NTXENT_SKEW = KiB offsets of zq,zqt,sc,cbuf,slabs).
# usage: tools/gpu_skew.sh TAG [bench.py args --] [skew ...]
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-skew}
mkdir -p $OUT
shift
ARGS=()
if [[ " $* " == *" -- "* ]]; then
  while [ "$1" != "--" ]; do ARGS+=("$1"); shift; done
  shift
fi
SKEWS=("$@")
[ ${#SKEWS[@]} -eq 0 ] && SKEWS=("0,0,0,0,0" "0,1024,0,1344,0" "0,0,0,0,0")
for S in "${SKEWS[@]}"; do
  NTXENT_SKEW=$S timeout -k 10 120 python bench.py --steps 40 --warmup 5 "${ARGS[@]}" > $OUT/b.log 2>&1 || { echo "bench failed"; tail -3 $OUT/b.log; exit 1; }
  echo "$S ${ARGS[*]} $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
