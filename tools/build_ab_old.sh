#!/bin/bash
# Build build/bin/ntxent_bench_old from the kernels of git revision $1 (default HEAD) for a
# same-call A/B against the working tree's build/bin/ntxent_bench.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
TMP=$(mktemp -d)
git -C $ROOT archive $REV cuda-nt-xent-mpi-nccl-simclr_amd/csrc | tar -x -C $TMP
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -fPIC -O3 -I$TMP/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/include \
  -c $TMP/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/ntxent_kernels.hip -o $ROOT/build/k_old.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 $ROOT/build/ntxent_bench.o $ROOT/build/k_old.o $ROOT/build/small_kernels.o \
  $ROOT/build/engine.o $ROOT/build/rccl_comm.o $ROOT/build/trace.o -o $ROOT/build/bin/ntxent_bench_old \
  -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
rm -rf $TMP
echo built build/bin/ntxent_bench_old from $REV
