// Compile-only probe: instantiates dz_sym_kernel alone (fast -Rpass-analysis / ISA iteration).
#include "../../cuda-nt-xent-mpi-nccl-simclr_amd/csrc/kernels/dz_sym.h"
template __global__ void ntxent::dev::dz_sym_kernel<_Float16>(const ntxent::dev::SimParams);
