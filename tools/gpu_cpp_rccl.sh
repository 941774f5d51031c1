#!/bin/bash
# Native RcclComm at W > 1 on the 1-GPU box: ntxent_bench as N processes (--proc-rank, per-rank
# NCCL_HOSTID, socket transport), each rank's loss checked against the --emulate run.
set -o pipefail
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-cpp_rccl}; mkdir -p $OUT
for c in "2 symmetric 1024 256" "2 allgather 1024 256" "3 symmetric 512 128" "4 symmetric 2048 512"; do
  set -- $c
  timeout -k 10 200 python tools/cpp_rccl_procs.py --gpus $1 --negatives $2 --batch $3 --dim $4 --shared-gpu > $OUT/procs_$1_$2.log 2>&1 || { echo "cpp rccl $c failed"; tail -20 $OUT/procs_$1_$2.log; exit 1; }
  cat $OUT/procs_$1_$2.log
done
echo done
