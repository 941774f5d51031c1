// Microbenchmark: issue rate of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3, uniform vs per-lane
// E8M0 scales) against v_mfma_f32_16x16x32_f16, one wave per SIMD, 8 independent accumulators,
// cycles from s_memtime. Build: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));

template <int MODE>
__global__ __launch_bounds__(256) void k(const int* in, float* out, unsigned long long* cyc, int iters) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = in[(l * 8 + i) & 1023]; b[i] = in[(l * 8 + i + 5) & 1023]; }
  h8 ha = __builtin_bit_cast(h8, a.lo), hb = __builtin_bit_cast(h8, b.lo);
  const int sa = MODE == 1 ? 127 : 120 + (l & 7), sb = MODE == 1 ? 127 : 121 + (l & 3);
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (MODE == 0) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, acc[j], 0, 0, 0);
      else acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, sa, 0, sb);
    }
  }
  asm volatile("s_nop 0" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  int* in; float* out; unsigned long long* cyc;
  hipMalloc(&in, 4096); hipMalloc(&out, 256 * 1024 * 4); hipMalloc(&cyc, 8);
  int h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (i * 2654435761u) & 0x3f3f3f3f;  // small finite fp8/fp16 patterns
  hipMemcpy(in, h, 4096, hipMemcpyHostToDevice);
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[3] = {"f16 16x16x32", "mx fp8 16x16x128 scale=127", "mx fp8 16x16x128 per-lane scales"};
  for (int m = 0; m < 3; ++m) {
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0, 0);
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, in, out, cyc, iters);
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double flop = 256.0 * 4 * iters * 8 * (m == 0 ? 16384.0 : 65536.0);
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-36s %.1f s_memtime ticks per MFMA, %.3f ms, %.1f TFLOP/s (1 wave per SIMD, all CUs)\n", names[m],
           (double)c / (iters * 8.0), ms, flop / (ms * 1e-3) / 1e12);
  }
  return 0;
}
