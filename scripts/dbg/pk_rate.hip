// Microbenchmark: throughput of v_pk_fma_f32 vs v_fma_f32 on gfx950 (DESIGN.md §4.5 note).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v2f __attribute__((ext_vector_type(2)));
template <bool PK>
__global__ __launch_bounds__(256) void k(float* out, float a, float b, int iters) {
  if constexpr (PK) {
    v2f acc[8];
    for (int i = 0; i < 8; ++i) acc[i] = v2f{threadIdx.x * 1e-3f + i, i * 0.5f};
    const v2f va{a, a}, vb{b, b};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_elementwise_fma(acc[i], va, vb);
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
  } else {
    float acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 1e-3f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = fmaf(acc[i], a, b);
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}
int main() {
  float* d;
  const int blocks = 256 * 8;
  hipMalloc(&d, blocks * 256 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int pk = 0; pk < 2; ++pk) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (pk) hipLaunchKernelGGL(k<true>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f, iters);
      else hipLaunchKernelGGL(k<false>, dim3(blocks), dim3(256), 0, 0, d, 0.999f, 0.001f, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flops = 2.0 * 16 * iters * (double)blocks * 256;
      printf("%s: %.3f ms, %.1f TFLOP/s\n", pk ? "v_pk_fma_f32 (8 x 2 lanes)" : "v_fma_f32 (16)", ms,
             flops / ms / 1e9);
    }
  }
  return 0;
}
