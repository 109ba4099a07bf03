// VALU issue-rate probe (gfx950): independent v_fma_f32 chains vs v_pk_fma_f32 chains vs
// v_fmac_f32_dpp, timed with HIP events; prints wave-instructions per SIMD-cycle for each.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float* out, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n"
        "v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(s));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

typedef float v2f __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pk(float* out, float s) {
  v2f a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
      a7 = a0 + 7;
  v2f ss = {s, s};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %1, %1, %8, %8\n v_pk_fma_f32 %2, %2, %8, %8\n"
        "v_pk_fma_f32 %3, %3, %8, %8\n v_pk_fma_f32 %4, %4, %8, %8\n v_pk_fma_f32 %5, %5, %8, %8\n"
        "v_pk_fma_f32 %6, %6, %8, %8\n v_pk_fma_f32 %7, %7, %8, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(ss));
  }
  v2f t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

__global__ __launch_bounds__(256) void k_add(float* out, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
        "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(s));
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ __launch_bounds__(256) void k_pkadd(float* out, float s) {
  v2f a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
      a7 = a0 + 7;
  v2f ss = {s, s};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %1, %1, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %3, %3, %8\n"
        "v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8\n"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
        : "v"(ss));
  }
  v2f t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

template <class K>
static void run(const char* name, K kern, float* d, int blocks, int per_cu) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
  hipEventRecord(a, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  ms /= 5;
  int cu = 0, clk = 0;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  const double waves = (double)blocks * 4;
  const double instrs = waves * ITERS * 8;
  const double simd_cycles = (double)cu * 4 * (ms * 1e-3) * clk * 1e3;
  printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_instr_per_simd_cycle\": %.3f, \"clock_khz\": %d}\n",
         name, per_cu, ms, instrs / simd_cycles, clk);
}

int main() {
  int cu = 0;
  hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* d;
  hipMalloc(&d, (size_t)cu * 16 * 256 * sizeof(float));
  for (int per : {1, 2, 4}) {
    const int blocks = cu * per;  // 4 waves per block: `per` waves per SIMD
    run("v_fma_f32", k_fma, d, blocks, per);
    run("v_pk_fma_f32", k_pk, d, blocks, per);
    run("v_add_f32", k_add, d, blocks, per);
    run("v_pk_add_f32", k_pkadd, d, blocks, per);
  }
  hipFree(d);
  return 0;
}
