// bw_probe.hip — what HBM rate can a kernel with the C2 analysis's traffic mix reach on this
// box?  (the analysis reads 134 MB and writes 2 x 153 MB per step.)
//
// Streams float4 (16 B per lane per access) through buffers far larger than the Infinity
// Cache (rotating sets), grid-stride, and prints one JSON line per (mix, store kind, workgroups per CU):
//   read      : sum of x (one 4-B store per workgroup)
//   write     : y = const
//   copy      : y = x
//   r1w2      : y = x, z = 2 x   (the analysis's 1 : 2.3 read : write mix)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/bw_probe scripts/bw_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(v4f* p, v4f v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__global__ __launch_bounds__(256) void k_read(const v4f* __restrict__ x, size_t n, float* out) {
  v4f s = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += x[i];
  const float t = s.x + s.y + s.z + s.w;
  if (t == 12345.f) out[blockIdx.x] = t;  // never true for the zero-filled input: no store traffic
}
template <bool NT>
__global__ __launch_bounds__(256) void k_write(v4f* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    st<NT>(y + i, v4f{1.f, 2.f, 3.f, 4.f});
}
template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4f* __restrict__ x, v4f* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st<NT>(y + i, x[i]);
}
// n_in reads, 2 n_in x (8/7) writes spread over two outputs: each thread reads one v4f and
// writes 8/7 v4f to each output on average (7 readers of 8 write an extra one)
template <bool NT>
__global__ __launch_bounds__(256) void k_r1w2(const v4f* __restrict__ x, v4f* __restrict__ y,
                                               v4f* __restrict__ z, size_t n_in) {
  const size_t n_out = n_in / 7 * 8;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n_out; i += (size_t)gridDim.x * 256) {
    const v4f v = i < n_in ? x[i] : v4f{0, 0, 0, 0};
    st<NT>(y + i, v);
    st<NT>(z + i, v * 2.f);
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t n_in = (134217728ull / 16);  // 134 MB of input (2^24 complex samples)
  const size_t n_out = n_in / 7 * 8;        // 153 MB each output
  // SETS rotating buffer sets (2.6 GB): every timed launch touches data the previous
  // launches left cold, far outside the 256 MB Infinity Cache
  constexpr int SETS = 6;
  v4f *xs[SETS], *ys[SETS], *zs[SETS];
  float* o;
  for (int i = 0; i < SETS; ++i) {
    hipMalloc(&xs[i], n_in * 16);
    hipMalloc(&ys[i], n_out * 16);
    hipMalloc(&zs[i], n_out * 16);
    hipMemset(xs[i], 0, n_in * 16);
    hipMemset(ys[i], 0, n_out * 16);
    hipMemset(zs[i], 0, n_out * 16);
  }
  hipMalloc(&o, 1 << 20);
  int cur = 0;
  v4f *x = xs[0], *y = ys[0], *z = zs[0];
  auto next = [&]() {
    cur = (cur + 1) % SETS;
    x = xs[cur];
    y = ys[cur];
    z = zs[cur];
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* mix, bool nt, int per_cu, double bytes, auto launch) {
    const int grid = per_cu * cus;
    for (int w = 0; w < 3; ++w) {
      next();
      launch(grid);
    }
    std::vector<float> ts;
    for (int r = 0; r < 20; ++r) {
      next();
      hipEventRecord(e0);
      launch(grid);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const float med = ts[ts.size() / 2];
    printf("{\"mix\": \"%s\", \"nt\": %d, \"wg_per_cu\": %d, \"MB\": %.1f, \"us\": %.2f, \"TBps\": %.3f}\n", mix,
           (int)nt, per_cu, bytes / 1e6, med * 1e3, bytes / (med * 1e-3) / 1e12);
    fflush(stdout);
  };
  for (int per_cu : {2, 4, 8, 16}) {
    run("read", false, per_cu, n_in * 16.0, [&](int g) { k_read<<<g, 256>>>(x, n_in, o); });
    run("write", false, per_cu, n_out * 16.0, [&](int g) { k_write<false><<<g, 256>>>(y, n_out); });
    run("write", true, per_cu, n_out * 16.0, [&](int g) { k_write<true><<<g, 256>>>(y, n_out); });
    run("copy", false, per_cu, n_in * 32.0, [&](int g) { k_copy<false><<<g, 256>>>(x, y, n_in); });
    run("copy", true, per_cu, n_in * 32.0, [&](int g) { k_copy<true><<<g, 256>>>(x, y, n_in); });
    run("r1w2", false, per_cu, n_in * 16.0 + 2 * n_out * 16.0,
        [&](int g) { k_r1w2<false><<<g, 256>>>(x, y, z, n_in); });
    run("r1w2", true, per_cu, n_in * 16.0 + 2 * n_out * 16.0,
        [&](int g) { k_r1w2<true><<<g, 256>>>(x, y, z, n_in); });
  }
  return 0;
}
