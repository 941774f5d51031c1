#!/bin/bash
# Experiment build: build/bin/ntxent_bench_<tag> with extra device-compile flags for the kernels
# (e.g. tools/build_variant.sh aux2 -DNTXENT_GEMM_DMA_AUX=2). Needs a normal build first.
set -e
TAG=$1; shift
cd "$(dirname "$0")/.."
HIPCC=/opt/rocm/bin/hipcc
INC=cuda-nt-xent-mpi-nccl-simclr_amd/csrc/include
$HIPCC --offload-arch=gfx950 -std=c++17 -fPIC -I$INC -O3 "$@" -c cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/ntxent_kernels.hip -o build/ntxent_kernels_$TAG.o
$HIPCC --offload-arch=gfx950 -std=c++17 -fPIC -I$INC -O3 "$@" -c cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/small_kernels.hip -o build/small_kernels_$TAG.o
$HIPCC --offload-arch=gfx950 build/ntxent_bench.o build/ntxent_kernels_$TAG.o build/small_kernels_$TAG.o build/engine.o build/engine_sym.o build/rccl_comm.o build/trace.o -o build/bin/ntxent_bench_$TAG -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
echo built build/bin/ntxent_bench_$TAG
