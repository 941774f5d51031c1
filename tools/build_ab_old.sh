#!/bin/bash
# Build build/bin/ntxent_bench_old (or _$2) entirely from git revision $1 (default HEAD): kernels,
# runtime and the bench itself, so a same-call A/B against the working tree's
# build/bin/ntxent_bench survives API changes between the revisions.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
TAG=${2:-old}
TMP=$(mktemp -d)
git -C $ROOT archive $REV cuda-nt-xent-mpi-nccl-simclr_amd/csrc bench | tar -x -C $TMP
C=$TMP/cuda-nt-xent-mpi-nccl-simclr_amd/csrc
HIPCC=/opt/rocm/bin/hipcc
HOST="$HIPCC -x c++ -D__HIP_PLATFORM_AMD__=1 -std=c++17 -fPIC -I/opt/rocm/include -I$C/include -O2"
pids=()
for k in ntxent_kernels small_kernels; do
  $HIPCC --offload-arch=gfx950 -std=c++17 -fPIC -O3 -I$C/include -c $C/kernels/$k.hip -o $TMP/$k.o & pids+=($!)
done
objs="$TMP/ntxent_kernels.o $TMP/small_kernels.o"
for s in $C/runtime/engine.cpp $C/runtime/engine_sym.cpp $C/runtime/rccl_comm.cpp $C/runtime/trace.cpp; do
  [ -f $s ] || continue
  o=$TMP/$(basename $s .cpp).o; objs="$objs $o"
  $HOST -c $s -o $o & pids+=($!)
done
$HOST -c $TMP/bench/ntxent_bench.cpp -o $TMP/ntxent_bench.o & pids+=($!)
for p in "${pids[@]}"; do wait $p; done
$HIPCC --offload-arch=gfx950 $TMP/ntxent_bench.o $objs -o $ROOT/build/bin/ntxent_bench_$TAG \
  -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
rm -rf $TMP
echo built build/bin/ntxent_bench_$TAG from $REV
