#!/bin/bash
# Build build/bin/ntxent_bench_<TAG> from git revision REV (kernels, runtime and bench all from that
# revision): same-box A/B of the current tree against an earlier one (tools/gpu_variants.sh TAG).
# usage: tools/build_rev.sh TAG REV
set -e
TAG=$1; REV=$2
cd "$(dirname "$0")/.."
ROOT=$PWD
T=$(mktemp -d /tmp/rev_XXXX)
git archive "$REV" cuda-nt-xent-mpi-nccl-simclr_amd/csrc bench | tar -x -C $T
HIPCC=/opt/rocm/bin/hipcc
INC=$T/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/include
for k in ntxent_kernels small_kernels; do
  $HIPCC --offload-arch=gfx950 -std=c++17 -fPIC -I$INC -O3 -c $T/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/$k.hip -o $T/$k.o &
done
for r in engine engine_sym rccl_comm trace; do
  $HIPCC -x c++ -D__HIP_PLATFORM_AMD__=1 -std=c++17 -fPIC -I/opt/rocm/include -I$INC -O2 -c $T/cuda-nt-xent-mpi-nccl-simclr_amd/csrc/runtime/$r.cpp -o $T/$r.o &
done
$HIPCC -x c++ -D__HIP_PLATFORM_AMD__=1 -std=c++17 -fPIC -I/opt/rocm/include -I$INC -O2 -c $T/bench/ntxent_bench.cpp -o $T/bench.o &
wait
$HIPCC --offload-arch=gfx950 $T/bench.o $T/ntxent_kernels.o $T/small_kernels.o $T/engine.o $T/engine_sym.o $T/rccl_comm.o $T/trace.o \
  -o $ROOT/build/bin/ntxent_bench_$TAG -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
rm -rf $T
echo built build/bin/ntxent_bench_$TAG from $REV
