// VALU issue cost per instruction form on gfx950 (8 independent chains per wave, 2 and 4 waves
// per SIMD): ns per wave-instruction per SIMD.  Generated once, committed as source.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_rate2 valu_rate2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITERS = 2048;
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_fma_vvv_distinct(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fma_f32 %0, %0, %8, %9\nv_fma_f32 %1, %1, %8, %9\nv_fma_f32 %2, %2, %8, %9\nv_fma_f32 %3, %3, %8, %9\nv_fma_f32 %4, %4, %8, %9\nv_fma_f32 %5, %5, %8, %9\nv_fma_f32 %6, %6, %8, %9\nv_fma_f32 %7, %7, %8, %9" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_fma_v_same(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fma_f32 %0, %0, %8, %8\nv_fma_f32 %1, %1, %8, %8\nv_fma_f32 %2, %2, %8, %8\nv_fma_f32 %3, %3, %8, %8\nv_fma_f32 %4, %4, %8, %8\nv_fma_f32 %5, %5, %8, %8\nv_fma_f32 %6, %6, %8, %8\nv_fma_f32 %7, %7, %8, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_fma_v_inline(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fma_f32 %0, %0, 0.5, 1.0\nv_fma_f32 %1, %1, 0.5, 1.0\nv_fma_f32 %2, %2, 0.5, 1.0\nv_fma_f32 %3, %3, 0.5, 1.0\nv_fma_f32 %4, %4, 0.5, 1.0\nv_fma_f32 %5, %5, 0.5, 1.0\nv_fma_f32 %6, %6, 0.5, 1.0\nv_fma_f32 %7, %7, 0.5, 1.0" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_fmac_vv(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fmac_f32 %0, %8, %9\nv_fmac_f32 %1, %8, %9\nv_fmac_f32 %2, %8, %9\nv_fmac_f32 %3, %8, %9\nv_fmac_f32 %4, %8, %9\nv_fmac_f32 %5, %8, %9\nv_fmac_f32 %6, %8, %9\nv_fmac_f32 %7, %8, %9" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_fmac_v_inline(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fmac_f32 %0, 0.5, %8\nv_fmac_f32 %1, 0.5, %8\nv_fmac_f32 %2, 0.5, %8\nv_fmac_f32 %3, 0.5, %8\nv_fmac_f32 %4, 0.5, %8\nv_fmac_f32 %5, 0.5, %8\nv_fmac_f32 %6, 0.5, %8\nv_fmac_f32 %7, 0.5, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_mul_vv(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mul_f32 %0, %0, %8\nv_mul_f32 %1, %1, %8\nv_mul_f32 %2, %2, %8\nv_mul_f32 %3, %3, %8\nv_mul_f32 %4, %4, %8\nv_mul_f32 %5, %5, %8\nv_mul_f32 %6, %6, %8\nv_mul_f32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_mul_inline(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mul_f32 %0, 0.5, %0\nv_mul_f32 %1, 0.5, %1\nv_mul_f32 %2, 0.5, %2\nv_mul_f32 %3, 0.5, %3\nv_mul_f32 %4, 0.5, %4\nv_mul_f32 %5, 0.5, %5\nv_mul_f32 %6, 0.5, %6\nv_mul_f32 %7, 0.5, %7" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_add_vv(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_f32 %0, %0, %8\nv_add_f32 %1, %1, %8\nv_add_f32 %2, %2, %8\nv_add_f32 %3, %3, %8\nv_add_f32 %4, %4, %8\nv_add_f32 %5, %5, %8\nv_add_f32 %6, %6, %8\nv_add_f32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_sub_vv(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_sub_f32 %0, %0, %8\nv_sub_f32 %1, %1, %8\nv_sub_f32 %2, %2, %8\nv_sub_f32 %3, %3, %8\nv_sub_f32 %4, %4, %8\nv_sub_f32 %5, %5, %8\nv_sub_f32 %6, %6, %8\nv_sub_f32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_add_vv_e64neg(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_f32_e64 %0, %0, -%8\nv_add_f32_e64 %1, %1, -%8\nv_add_f32_e64 %2, %2, -%8\nv_add_f32_e64 %3, %3, -%8\nv_add_f32_e64 %4, %4, -%8\nv_add_f32_e64 %5, %5, -%8\nv_add_f32_e64 %6, %6, -%8\nv_add_f32_e64 %7, %7, -%8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_mov(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_mov_b32 %0, %8\nv_mov_b32 %1, %8\nv_mov_b32 %2, %8\nv_mov_b32 %3, %8\nv_mov_b32 %4, %8\nv_mov_b32 %5, %8\nv_mov_b32 %6, %8\nv_mov_b32 %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_fmac_dpp(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_fmac_f32_dpp %0, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %1, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %2, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %3, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %4, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %5, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %6, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_fmac_f32_dpp %7, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_add_dpp(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_f32_dpp %0, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %1, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %2, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %3, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %4, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %5, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %6, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\nv_add_f32_dpp %7, %8, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
__global__ __launch_bounds__(256) void k_pk_fma_distinct(float* out, float s) {
  v2f a[8]; for (int i = 0; i < 8; ++i) a[i] = v2f{(float)threadIdx.x + i, 1.f}; v2f b = {s, s}, c = {s*2, s};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_fma_f32 %0, %0, %8, %9\nv_pk_fma_f32 %1, %1, %8, %9\nv_pk_fma_f32 %2, %2, %8, %9\nv_pk_fma_f32 %3, %3, %8, %9\nv_pk_fma_f32 %4, %4, %8, %9\nv_pk_fma_f32 %5, %5, %8, %9\nv_pk_fma_f32 %6, %6, %8, %9\nv_pk_fma_f32 %7, %7, %8, %9" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_pk_add(float* out, float s) {
  v2f a[8]; for (int i = 0; i < 8; ++i) a[i] = v2f{(float)threadIdx.x + i, 1.f}; v2f b = {s, s}, c = {s*2, s};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_add_f32 %0, %0, %8\nv_pk_add_f32 %1, %1, %8\nv_pk_add_f32 %2, %2, %8\nv_pk_add_f32 %3, %3, %8\nv_pk_add_f32 %4, %4, %8\nv_pk_add_f32 %5, %5, %8\nv_pk_add_f32 %6, %6, %8\nv_pk_add_f32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_pk_mul(float* out, float s) {
  v2f a[8]; for (int i = 0; i < 8; ++i) a[i] = v2f{(float)threadIdx.x + i, 1.f}; v2f b = {s, s}, c = {s*2, s};
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_pk_mul_f32 %0, %0, %8\nv_pk_mul_f32 %1, %1, %8\nv_pk_mul_f32 %2, %2, %8\nv_pk_mul_f32 %3, %3, %8\nv_pk_mul_f32 %4, %4, %8\nv_pk_mul_f32 %5, %5, %8\nv_pk_mul_f32 %6, %6, %8\nv_pk_mul_f32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  v2f t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}
__global__ __launch_bounds__(256) void k_add_u32(float* out, float s) {
  float a[8]; for (int i = 0; i < 8; ++i) a[i] = (float)threadIdx.x + i; float b = s, c = s * 2;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile("v_add_u32 %0, %0, %8\nv_add_u32 %1, %1, %8\nv_add_u32 %2, %2, %8\nv_add_u32 %3, %3, %8\nv_add_u32 %4, %4, %8\nv_add_u32 %5, %5, %8\nv_add_u32 %6, %6, %8\nv_add_u32 %7, %7, %8" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]) : "v"(b), "v"(c));
  }
  float t = a[0]; for (int i = 1; i < 8; ++i) t += a[i]; out[blockIdx.x * 256 + threadIdx.x] = t;
}
template <class K>
static void run(const char* name, K kern, float* d, int blocks, int per) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
  hipEventRecord(a, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1.0001f);
  hipEventRecord(b, 0); hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b); ms /= 5;
  int cu = 0; hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  const double instrs = (double)blocks * 4 * ITERS * 8;
  const double ns_per = ms * 1e6 / (instrs / (cu * 4.0));
  printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f}\n", name, per, ms, ns_per);
}
int main() {
  int cu = 0; hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* d; hipMalloc(&d, (size_t)cu * 16 * 256 * sizeof(float));
  for (int per : {2, 4}) {
    run("fma_vvv_distinct", k_fma_vvv_distinct, d, cu * per, per);
    run("fma_v_same", k_fma_v_same, d, cu * per, per);
    run("fma_v_inline", k_fma_v_inline, d, cu * per, per);
    run("fmac_vv", k_fmac_vv, d, cu * per, per);
    run("fmac_v_inline", k_fmac_v_inline, d, cu * per, per);
    run("mul_vv", k_mul_vv, d, cu * per, per);
    run("mul_inline", k_mul_inline, d, cu * per, per);
    run("add_vv", k_add_vv, d, cu * per, per);
    run("sub_vv", k_sub_vv, d, cu * per, per);
    run("add_vv_e64neg", k_add_vv_e64neg, d, cu * per, per);
    run("mov", k_mov, d, cu * per, per);
    run("fmac_dpp", k_fmac_dpp, d, cu * per, per);
    run("add_dpp", k_add_dpp, d, cu * per, per);
    run("pk_fma_distinct", k_pk_fma_distinct, d, cu * per, per);
    run("pk_add", k_pk_add, d, cu * per, per);
    run("pk_mul", k_pk_mul, d, cu * per, per);
    run("add_u32", k_add_u32, d, cu * per, per);
  }
  hipFree(d);
  return 0;
}
