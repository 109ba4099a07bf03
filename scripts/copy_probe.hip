// copy_probe.hip — which float4 copy shape reaches the chip's practical HBM rate?
// (the library's one-shot copy measured 5.5 TB/s against the guide's
// 6.29 TB/s float4 copy.)  Variants, each over 2 GiB (src) -> 2 GiB (dst), rotating over
// buffer pairs so every timed launch starts cold, median of 15, HIP events:
//   oneshot U     : one-shot grid, each thread U float4 loads then U stores (the library's, U 4)
//   persist U W   : W workgroups per CU, grid-stride over chunks of U float4 per thread
//   nt            : nontemporal loads and stores (slc/nt bits via the builtins)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/copy_probe scripts/copy_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4f ld(const v4f* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_oneshot(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t base = (size_t)blockIdx.x * TPB * U + threadIdx.x;
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + base + u * TPB);
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(y + base + u * TPB, v[u]);
}

template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_persist(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t chunk = (size_t)TPB * U;
  const size_t nchunks = n / chunk;
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const size_t base = c * chunk + threadIdx.x;
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + base + u * TPB);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(y + base + u * TPB, v[u]);
  }
}

// contiguous range per workgroup (like the library's persistent kernels), U float4 per thread
template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_range(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t chunk = (size_t)TPB * U;
  const size_t nchunks = n / chunk;
  const size_t c0 = nchunks * blockIdx.x / gridDim.x, c1 = nchunks * (blockIdx.x + 1) / gridDim.x;
  for (size_t c = c0; c < c1; ++c) {
    const size_t base = c * chunk + threadIdx.x;
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + base + u * TPB);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(y + base + u * TPB, v[u]);
  }
}

// per-wave contiguous: wave w of the block moves U KiB contiguous (instruction u = next KiB)
template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_wavecont(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t base = ((size_t)blockIdx.x * TPB + (threadIdx.x & ~63u)) * U + (threadIdx.x & 63u);
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + base + u * 64);
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(y + base + u * 64, v[u]);
}
template <int U, bool NTL, int TPB>
__global__ __launch_bounds__(TPB) void k_readonly(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t base = (size_t)blockIdx.x * TPB * U + threadIdx.x;
  v4f s = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) s += ld<NTL>(x + base + u * TPB);
  if (s.x == 12345.f) y[blockIdx.x] = s;
}
template <int U, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_writeonly(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t base = (size_t)blockIdx.x * TPB * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) st<NTS>(y + base + u * TPB, v4f{1.f, 2.f, 3.f, 4.f});
}

// persistent, chunks handed out in address order by a ticket counter (one atomic per chunk
// per workgroup): does keeping the chip's in-flight window narrow recover the one-shot rate?
template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_ticket(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n,
                                                unsigned* ctr) {
  __shared__ unsigned tk[2];
  const size_t chunk = (size_t)TPB * U;
  const unsigned nchunks = (unsigned)(n / chunk);
  if (threadIdx.x == 0) tk[0] = atomicAdd(ctr, 1u);
  __syncthreads();
  unsigned c = tk[0];
  int par = 0;
  while (c < nchunks) {
    // next ticket taken before this chunk's loads (it lands while they fly)
    if (threadIdx.x == 0) tk[par ^ 1] = atomicAdd(ctr, 1u);
    const size_t base = c * chunk + threadIdx.x;
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + base + u * TPB);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(y + base + u * TPB, v[u]);
    __syncthreads();
    par ^= 1;
    c = tk[par];
  }
}

// persistent grid-stride with the next chunk's loads issued before this chunk's stores
// (the software pipeline of the library's persistent kernels)
template <int U, bool NTL, bool NTS, int TPB>
__global__ __launch_bounds__(TPB) void k_persist_pf(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  const size_t chunk = (size_t)TPB * U;
  const size_t nchunks = n / chunk;
  size_t c = blockIdx.x;
  if (c >= nchunks) return;
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NTL>(x + c * chunk + threadIdx.x + u * TPB);
  for (; c < nchunks; c += gridDim.x) {
    const size_t nx = c + gridDim.x < nchunks ? c + gridDim.x : c;
    v4f w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = ld<NTL>(x + nx * chunk + threadIdx.x + u * TPB);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NTS>(y + c * chunk + threadIdx.x + u * TPB, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = w[u];
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t bytes = (size_t)1 << 31;
  const size_t n = bytes / 16;
  constexpr int SETS = 3;
  v4f *xs[SETS], *ys[SETS];
  for (int i = 0; i < SETS; ++i) {
    if (hipMalloc(&xs[i], bytes) != hipSuccess || hipMalloc(&ys[i], bytes) != hipSuccess) return 1;
    hipMemset(xs[i], 0, bytes);
    hipMemset(ys[i], 0, bytes);
  }
  hipDeviceSynchronize();
  int cur = 0;
  unsigned* ctr;
  if (hipMalloc(&ctr, 4) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, int u, int nt, int per_cu, int tpb, auto launch) {
    for (int w = 0; w < 3; ++w) {
      cur = (cur + 1) % SETS;
      launch(xs[cur], ys[cur]);
    }
    std::vector<float> ts;
    for (int r = 0; r < 15; ++r) {
      cur = (cur + 1) % SETS;
      hipEventRecord(e0);
      launch(xs[cur], ys[cur]);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    printf("{\"kind\": \"%s\", \"U\": %d, \"nt\": %d, \"wg_per_cu\": %d, \"tpb\": %d, \"us\": %.1f, "
           "\"TBps\": %.3f, \"best_TBps\": %.3f}\n",
           name, u, nt, per_cu, tpb, med * 1e3, 2.0 * bytes / (med * 1e-3) / 1e12,
           2.0 * bytes / (ts[0] * 1e-3) / 1e12);
    fflush(stdout);
  };
#define ONESHOT(U, NTL, NTS, TPB)                                                                  \
  run("oneshot", U, NTL * 2 + NTS, 0, TPB, [&](const v4f* x, v4f* y) {                               \
    k_oneshot<U, NTL, NTS, TPB><<<(unsigned)(n / (TPB * U)), TPB>>>(x, y, n);                        \
  });
#define PERSIST(K, U, NTL, NTS, TPB, W)                                                            \
  run(#K, U, NTL * 2 + NTS, W, TPB, [&](const v4f* x, v4f* y) {                                      \
    K<U, NTL, NTS, TPB><<<(unsigned)(W * cus), TPB>>>(x, y, n);                                      \
  });
#define TICKET(U, NTL, NTS, W)                                                                      \
  run("ticket", U, NTL * 2 + NTS, W, 256, [&](const v4f* x, v4f* y) {                                \
    hipMemsetAsync(ctr, 0, 4, 0);                                                                    \
    k_ticket<U, NTL, NTS, 256><<<(unsigned)(W * cus), 256>>>(x, y, n, ctr);                          \
  });
  ONESHOT(1, true, true, 256)
  PERSIST(k_persist, 1, true, true, 256, 4) PERSIST(k_persist, 1, true, true, 256, 8)
  PERSIST(k_persist, 4, true, true, 256, 2) PERSIST(k_persist, 4, true, true, 256, 4)
  PERSIST(k_persist_pf, 1, true, true, 256, 4) PERSIST(k_persist_pf, 1, true, true, 256, 8)
  PERSIST(k_persist_pf, 4, true, true, 256, 2) PERSIST(k_persist_pf, 4, true, true, 256, 3)
  PERSIST(k_persist_pf, 4, true, true, 256, 4) PERSIST(k_persist_pf, 8, true, true, 256, 2)
  PERSIST(k_range, 4, true, true, 256, 2) PERSIST(k_range, 4, true, true, 256, 4)
  return 0;
}
