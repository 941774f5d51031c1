#!/bin/bash
# Compile-time GEMM main-loop ablations (diagnostic build; production kernels untouched).
#   host:  bash tools/ablate_ct.sh build        -> build/bin/ntxent_bench_abl
#   GPU:   bash tools/ablate_ct.sh run TAG      -> rocprof kernel stats per ablation
# NTXENT_GEMM_ABL bits: 1 no DMA, 2 no LDS operand reads, 4 no MFMA.
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = "build" ]; then
  INC=$ROOT/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/include
  mkdir -p $ROOT/build/abl
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 ${ABL_EXTRA_FLAGS} -DNTXENT_ABLATION_KERNELS -I$INC \
    -c $ROOT/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/ntxent_kernels.hip -o $ROOT/build/abl/k.o || exit 1
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $ROOT/build/ntxent_bench.o $ROOT/build/abl/k.o $ROOT/build/small_kernels.o $ROOT/build/engine.o \
    $ROOT/build/rccl_comm.o $ROOT/build/trace.o -o $ROOT/build/bin/ntxent_bench_abl -L/opt/rocm/lib -lrccl -ldl \
    -Wl,-rpath,/opt/rocm/lib || exit 1
  echo built
  exit 0
fi
TAG=${2:-ablct}
if [ "$1" = "stamps" ]; then
  OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
  NTXENT_GEMM_ABL=32 timeout -k 10 120 build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 2 --warmup 1 > $OUT/stamps.log 2>&1
  exit $?
fi
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for A in ${ABLS:-0 1 2 3 4 5 6}; do
  NTXENT_GEMM_ABL=$A timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/a$A -o run --output-format csv -- build/bin/ntxent_bench_abl --batch 4096 --dim 2048 --iters 10 --warmup 2 > $OUT/a$A.log 2>&1 || exit 1
done
echo ok
