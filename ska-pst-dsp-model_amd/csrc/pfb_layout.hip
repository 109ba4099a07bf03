// pfb_layout.hip — data-format kernels either side of the PFB path and their C ABI
// (include/pfb_api.h, "data formats" section):
//
//   * DADA unpack / pack: the file's TFP order (time, channel, polarisation, re/im;
//     NBIT 8/16/32/64) <-> the engine's [pol][t][chan] complex float32
//     (reshape_dada_data.m:23-30, DADARead.m:58-83, write_dada_data.m:32-50), and the
//     LowCBF heap order (reshape_low_cbf_data.m:14-43);
//   * corner turn (batched transpose) and channel gather with a selection map: the data
//     movement of the two-stage cascades (TwoStageFilterBank.m:92-110,
//     TwoStageInverseFilterBank.m:124-150);
//   * the FilterBank quantisation hooks round(rms / std(x) * x)
//     (FilterBank.m:75-83,106-113): a device reduction for var(x, 0, "all") followed
//     by the scale-and-round pass, with no host round trip (graph-capturable).
//
// All of these move bytes and do almost no arithmetic: each is HBM-bound, so they are
// written as coalesced streaming kernels (one read and one write per sample; the
// transpose stages 32x32 tiles through LDS so both sides stay coalesced).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <limits>
#include <type_traits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

#include "pfb_api.h"

pfb_status pfb_set_error(pfb_status s, const char* msg);  // pfb_api.hip

namespace {

#define LCHK(expr)                                                                          \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) {                                                                 \
      char m_[512];                                                                         \
      snprintf(m_, sizeof(m_), "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,   \
               __LINE__);                                                                   \
      return pfb_set_error(e_ == hipErrorOutOfMemory ? PFB_ERR_OOM : PFB_ERR_HIP, m_);     \
    }                                                                                       \
  } while (0)

pfb_status bad(const char* msg) { return pfb_set_error(PFB_ERR_INVALID_ARG, msg); }

constexpr int TPB = 256;

unsigned blocks_for(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

// Matlab cast(single -> intN): round half away from zero, saturate, NaN -> 0
template <class T>
__device__ __forceinline__ T to_sample(float v) {
  if constexpr (std::is_same<T, float>::value) {
    return v;
  } else if constexpr (std::is_same<T, double>::value) {
    return (double)v;
  } else {
    constexpr float lo = (float)std::numeric_limits<T>::min();
    constexpr float hi = (float)std::numeric_limits<T>::max();
    if (v != v) return (T)0;
    const float r = roundf(v);
    return (T)fminf(fmaxf(r, lo), hi);
  }
}

// ---------------------------------------------------------------- DADA unpack / pack
// One thread per (t, c): reads the P (x NDIM) adjacent file samples of its (t, c) and
// writes one complex sample into each polarisation's [t][chan] plane.
template <class T, int NDIM, bool LOWCBF>
__global__ void __launch_bounds__(TPB) dada_unpack_kernel(const T* __restrict__ in, int64_t n_dat,
                                                          int C, int P, float2* __restrict__ out,
                                                          int64_t ops) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n_dat * C) return;
  const int64_t t = i / C;
  const int c = (int)(i - t * C);
  for (int p = 0; p < P; ++p) {
    int64_t e;
    if constexpr (LOWCBF) {
      // heap of 32 samples: [heap][chan][pol][sample] (reshape_low_cbf_data.m:31-41)
      e = (((t >> 5) * C + c) * P + p) * 32 + (t & 31);
    } else {
      e = (t * C + c) * P + p;  // reshape(data, n_pol, n_chan, []) of TFP
    }
    const float re = (float)in[e * NDIM];
    const float im = NDIM == 2 ? (float)in[e * NDIM + 1] : 0.f;
    out[p * ops + i] = make_float2(re, im);
  }
}

template <class T>
__global__ void __launch_bounds__(TPB) dada_pack_kernel(const float2* __restrict__ in, int64_t ips,
                                                        int64_t n_dat, int C, int P,
                                                        T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n_dat * C) return;
  for (int p = 0; p < P; ++p) {
    const float2 v = in[p * ips + i];
    const int64_t e = i * P + p;  // (t * C + c) * P + p
    out[2 * e] = to_sample<T>(v.x);
    out[2 * e + 1] = to_sample<T>(v.y);
  }
}

// TFP order, complex samples, P = 1 or 2: element (t, c) = i of the file is the P x 2
// values at i * P * 2 whatever C is (reshape_dada_data.m), so a thread takes 4 adjacent
// i: one run of 8 P sizeof(T) bytes in (16 B for NBIT 8 dual-pol) as 16-byte loads, and
// per polarisation 4 samples = 2 x 16-byte stores out (the generic kernel issues one
// byte load per value and one 8-byte store per sample).  Needs 16-B aligned buffers
// and an even pol stride (checked by the launcher).
template <class T, int P>
__global__ void __launch_bounds__(TPB) dada_unpack_tfp4_kernel(const T* __restrict__ in, int64_t n,
                                                               float2* __restrict__ out, int64_t ops) {
  constexpr int V = 4;
  constexpr int NV = V * P * 2;                 // values per thread
  constexpr int BYTES = NV * (int)sizeof(T);    // 8 P sizeof(T): a multiple of 8
  const int64_t i0 = ((int64_t)blockIdx.x * TPB + threadIdx.x) * V;
  if (i0 >= n) return;
  T vals[NV];
  if (i0 + V <= n) {
    const char* src = reinterpret_cast<const char*>(in + i0 * P * 2);
    if constexpr (BYTES % 16 == 0) {
#pragma unroll
      for (int k = 0; k < BYTES / 16; ++k) {
        const uint4 w = reinterpret_cast<const uint4*>(src)[k];
        __builtin_memcpy(reinterpret_cast<char*>(vals) + 16 * k, &w, 16);
      }
    } else {
      const uint2 w = *reinterpret_cast<const uint2*>(src);
      __builtin_memcpy(vals, &w, 8);
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float4* o = reinterpret_cast<float4*>(out + p * ops + i0);
#pragma unroll
      for (int h = 0; h < V / 2; ++h) {
        const int a = (2 * h) * P * 2 + 2 * p, b = (2 * h + 1) * P * 2 + 2 * p;
        o[h] = make_float4((float)vals[a], (float)vals[a + 1], (float)vals[b], (float)vals[b + 1]);
      }
    }
  } else {
    for (int64_t i = i0; i < n; ++i)
      for (int p = 0; p < P; ++p) {
        const int64_t e = i * P + p;
        out[p * ops + i] = make_float2((float)in[2 * e], (float)in[2 * e + 1]);
      }
  }
}

template <class T>
hipError_t launch_unpack(const void* in, int ndim, bool lowcbf, int64_t n_dat, int C, int P,
                         float2* out, int64_t ops, hipStream_t s) {
  const unsigned g = blocks_for(n_dat * C);
  const T* src = static_cast<const T*>(in);
  const bool aligned = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0) && (P == 1 || ops % 2 == 0);
  // (NBIT 32/64 keep the generic kernel: its 4- and 8-byte value loads already coalesce)
  if (sizeof(T) <= 2 && ndim == 2 && !lowcbf && aligned && (P == 1 || P == 2)) {
    const int64_t n = n_dat * C;
    const unsigned g4 = blocks_for((n + 3) / 4);
    if (P == 2) hipLaunchKernelGGL((dada_unpack_tfp4_kernel<T, 2>), g4, TPB, 0, s, src, n, out, ops);
    else hipLaunchKernelGGL((dada_unpack_tfp4_kernel<T, 1>), g4, TPB, 0, s, src, n, out, ops);
    return hipGetLastError();
  }
  if (ndim == 2) {
    if (lowcbf) hipLaunchKernelGGL((dada_unpack_kernel<T, 2, true>), g, TPB, 0, s, src, n_dat, C, P, out, ops);
    else hipLaunchKernelGGL((dada_unpack_kernel<T, 2, false>), g, TPB, 0, s, src, n_dat, C, P, out, ops);
  } else {
    if (lowcbf) hipLaunchKernelGGL((dada_unpack_kernel<T, 1, true>), g, TPB, 0, s, src, n_dat, C, P, out, ops);
    else hipLaunchKernelGGL((dada_unpack_kernel<T, 1, false>), g, TPB, 0, s, src, n_dat, C, P, out, ops);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------- gather / transpose
// out[o][t][j] = in[o][t][src(j)], src(j) = src0 + j + (j >= split ? shift : 0)
// (strides in complex samples): a contiguous channel range, or the two-stage
// "chomp" that drops the oversampled channels in the middle (TwoStageFilterBank.m:104-105)
__global__ void __launch_bounds__(TPB) gather_kernel(const float2* __restrict__ in, int64_t ios,
                                                     int64_t irs, float2* __restrict__ out,
                                                     int64_t oos, int64_t ors, int64_t n_rows,
                                                     int n_sel, int src0, int split, int shift) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n_rows * n_sel) return;
  const int64_t o = blockIdx.y;
  const int64_t t = i / n_sel;
  const int j = (int)(i - t * n_sel);
  const int src = src0 + j + (j >= split ? shift : 0);
  out[o * oos + t * ors + j] = in[o * ios + t * irs + src];
}

// out[o][c][r] = in[o][r][c] through a padded 32 x 32 LDS tile (both sides coalesced)
__global__ void __launch_bounds__(TPB) transpose_kernel(const float2* __restrict__ in, int64_t ios,
                                                        int64_t irs, int64_t n_rows, int64_t n_cols,
                                                        float2* __restrict__ out, int64_t oos,
                                                        int64_t ors) {
  __shared__ float2 tile[32][33];
  const int64_t r0 = (int64_t)blockIdx.x * 32, c0 = (int64_t)blockIdx.y * 32;
  const int64_t o = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const float2* src = in + o * ios;
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = r0 + k, c = c0 + tx;
    if (r < n_rows && c < n_cols) tile[k][tx] = src[r * irs + c];
  }
  __syncthreads();
  float2* dst = out + o * oos;
  for (int k = ty; k < 32; k += 8) {
    const int64_t c = c0 + k, r = r0 + tx;
    if (r < n_rows && c < n_cols) dst[c * ors + r] = tile[tx][k];
  }
}

// ---------------------------------------------------------------- quantisation
// stats[0..2] += (sum re, sum im, sum |x|^2) in double over n_pol rows of n samples
// (grid: x = grid-stride over one row, y = polarisation; 16-byte loads of two samples)
__global__ void __launch_bounds__(TPB) moments_kernel(const float2* __restrict__ x, int64_t ps,
                                                      int64_t n, int n_pol, double* stats) {
  double sr = 0, si = 0, s2 = 0;
  const float2* row = x + blockIdx.y * ps;
  const bool vec = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
  const int64_t n2 = vec ? n / 2 : 0;
  const int64_t stride = (int64_t)gridDim.x * TPB;
  for (int64_t i0 = (int64_t)blockIdx.x * TPB + threadIdx.x; i0 < n2; i0 += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)  // four loads in flight per thread
      v[u] = i0 + u * stride < n2 ? reinterpret_cast<const float4*>(row)[i0 + u * stride]
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sr += (double)v[u].x + (double)v[u].z;
      si += (double)v[u].y + (double)v[u].w;
      s2 += (double)v[u].x * v[u].x + (double)v[u].y * v[u].y + (double)v[u].z * v[u].z +
            (double)v[u].w * v[u].w;
    }
  }
  for (int64_t i = 2 * n2 + (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
    const float2 v = row[i];
    sr += v.x;
    si += v.y;
    s2 += (double)v.x * v.x + (double)v.y * v.y;
  }
  __shared__ double red[3][TPB / 64];
  for (int off = 32; off > 0; off >>= 1) {
    sr += __shfl_down(sr, off, 64);
    si += __shfl_down(si, off, 64);
    s2 += __shfl_down(s2, off, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = sr;
    red[1][w] = si;
    red[2][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0, c = 0;
    for (int k = 0; k < TPB / 64; ++k) {
      a += red[0][k];
      b += red[1][k];
      c += red[2][k];
    }
    atomicAdd(&stats[0], a);
    atomicAdd(&stats[1], b);
    atomicAdd(&stats[2], c);
  }
}

// y = round(single(scale) * x) (Matlab round: half away from zero), scale = rms/std or 1;
// stats[3] receives the scale (thread 0 of block (0, 0)) for the host to read back
__global__ void __launch_bounds__(TPB) quantize_kernel(const float2* __restrict__ x, int64_t ips,
                                                       float2* __restrict__ y, int64_t ops, int64_t n,
                                                       int n_pol, double rms, double* stats) {
  double scale = 1.0;
  if (rms > 0) {
    const double cnt = (double)n * n_pol;
    const double m2 = (stats[0] * stats[0] + stats[1] * stats[1]) / cnt;
    const double var = (stats[2] - m2) / (cnt - 1.0);  // var(x, 0, "all")
    scale = rms / sqrt(var);
  }
  const float sf = (float)scale;  // single * double -> single (Matlab mixed-class rule)
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) stats[3] = scale;
  const float2* xr = x + blockIdx.y * ips;
  float2* yr = y + blockIdx.y * ops;
  const int64_t stride = (int64_t)gridDim.x * TPB;
  // 16-byte loads and stores (two samples) when both rows are 16-B aligned; the loads of
  // a thread's 4 iterations issue before its stores
  const bool vec = ((reinterpret_cast<uintptr_t>(xr) | reinterpret_cast<uintptr_t>(yr)) & 15) == 0;
  const int64_t n2 = vec ? n / 2 : 0;
  const float4* x4 = reinterpret_cast<const float4*>(xr);
  float4* y4 = reinterpret_cast<float4*>(yr);
  for (int64_t i0 = (int64_t)blockIdx.x * TPB + threadIdx.x; i0 < n2; i0 += 4 * stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * stride < n2) v[u] = x4[i0 + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * stride < n2)
        y4[i0 + u * stride] = make_float4(roundf(sf * v[u].x), roundf(sf * v[u].y), roundf(sf * v[u].z),
                                          roundf(sf * v[u].w));
  }
  for (int64_t i = 2 * n2 + (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
    const float2 v = xr[i];
    yr[i] = make_float2(roundf(sf * v.x), roundf(sf * v.y));
  }
}

// per-device scratch for the moments (4 doubles), allocated once per device
struct Scratch {
  std::mutex mu;
  std::vector<double*> per_dev;
};
Scratch g_scratch;

hipError_t stats_buffer(double** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_scratch.mu);
  if ((int)g_scratch.per_dev.size() <= dev) g_scratch.per_dev.resize(dev + 1, nullptr);
  if (!g_scratch.per_dev[dev]) {
    e = hipMalloc(&g_scratch.per_dev[dev], 4 * sizeof(double));
    if (e != hipSuccess) return e;
  }
  *out = g_scratch.per_dev[dev];
  return hipSuccess;
}

// Bandwidth probe (the achievable HBM rate beside the 8 TB/s spec): one float4
// per thread, nontemporal load and store, one-shot grid of 256-thread workgroups.  Round 6
// (scripts/copy_probe.hip, profiles/r06_copy_probe.jsonl, 2 GiB -> 2 GiB): this shape moves
// 6.5-6.6 TB/s (read + write); four float4 per thread 5.6-5.8, persistent grid-stride or
// contiguous-range loops 4.7-5.5 — the dispatcher's in-order workgroups keep the chip's
// requests in flight in one narrow window of addresses.  (Round 5's four-per-thread form
// measured 5.5 TB/s, which made every kernel look closer to the ceiling than it was.)
typedef float copy_v4f __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(TPB) copy_kernel(const copy_v4f* __restrict__ src,
                                                   copy_v4f* __restrict__ dst, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n4) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// n_pol rows of n samples, dst + q dps <- src + q sps (device to device): the strided
// copies of the stream objects' carry buffers (hipMemcpy2D rejects row pitches of a few MB)
__global__ void __launch_bounds__(TPB) copy_rows_kernel(float2* __restrict__ dst, int64_t dps,
                                                        const float2* __restrict__ src, int64_t sps,
                                                        int64_t n) {
  const int64_t q = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB)
    dst[q * dps + i] = src[q * sps + i];
}

unsigned grid_stride_blocks(int64_t total) {
  return (unsigned)std::min<int64_t>(std::max<int64_t>((total + TPB - 1) / TPB, 1), 4096);
}

}  // namespace

extern "C" {

pfb_status pfb_dada_unpack(const void* in, int32_t nbit, int32_t ndim, int32_t order,
                           int64_t n_dat, int32_t n_chan, int32_t n_pol, pfb_cf32* out,
                           int64_t out_pol_stride, void* stream) {
  if (n_dat < 0 || n_chan <= 0 || n_pol <= 0) return bad("pfb_dada_unpack: bad sizes");
  if (ndim != 1 && ndim != 2) return bad("pfb_dada_unpack: NDIM must be 1 or 2");
  if (order != PFB_DADA_TFP && order != PFB_DADA_LOWCBF)
    return bad("pfb_dada_unpack: unknown sample order");
  if (order == PFB_DADA_LOWCBF && n_dat % 32) return bad("pfb_dada_unpack: LowCBF data are heaps of 32 samples");
  if (out_pol_stride < n_dat * n_chan) return bad("pfb_dada_unpack: polarisation stride too small");
  if (n_dat == 0) return PFB_OK;
  if (!in || !out) return bad("pfb_dada_unpack: null buffer");
  hipStream_t s = (hipStream_t)stream;
  const bool lc = order == PFB_DADA_LOWCBF;
  float2* o = (float2*)out;
  switch (nbit) {
    case 8: LCHK((launch_unpack<int8_t>(in, ndim, lc, n_dat, n_chan, n_pol, o, out_pol_stride, s))); break;
    case 16: LCHK((launch_unpack<int16_t>(in, ndim, lc, n_dat, n_chan, n_pol, o, out_pol_stride, s))); break;
    case 32: LCHK((launch_unpack<float>(in, ndim, lc, n_dat, n_chan, n_pol, o, out_pol_stride, s))); break;
    case 64: LCHK((launch_unpack<double>(in, ndim, lc, n_dat, n_chan, n_pol, o, out_pol_stride, s))); break;
    default: return bad("pfb_dada_unpack: NBIT must be 8, 16, 32 or 64");
  }
  return PFB_OK;
}

pfb_status pfb_dada_pack(const pfb_cf32* in, int64_t in_pol_stride, int64_t n_dat, int32_t n_chan,
                         int32_t n_pol, void* out, int32_t nbit, void* stream) {
  if (n_dat < 0 || n_chan <= 0 || n_pol <= 0) return bad("pfb_dada_pack: bad sizes");
  if (in_pol_stride < n_dat * n_chan) return bad("pfb_dada_pack: polarisation stride too small");
  if (n_dat == 0) return PFB_OK;
  if (!in || !out) return bad("pfb_dada_pack: null buffer");
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = blocks_for(n_dat * n_chan);
  const float2* src = (const float2*)in;
  switch (nbit) {
    case 8: hipLaunchKernelGGL(dada_pack_kernel<int8_t>, g, TPB, 0, s, src, in_pol_stride, n_dat, n_chan, n_pol, (int8_t*)out); break;
    case 16: hipLaunchKernelGGL(dada_pack_kernel<int16_t>, g, TPB, 0, s, src, in_pol_stride, n_dat, n_chan, n_pol, (int16_t*)out); break;
    case 32: hipLaunchKernelGGL(dada_pack_kernel<float>, g, TPB, 0, s, src, in_pol_stride, n_dat, n_chan, n_pol, (float*)out); break;
    case 64: hipLaunchKernelGGL(dada_pack_kernel<double>, g, TPB, 0, s, src, in_pol_stride, n_dat, n_chan, n_pol, (double*)out); break;
    default: return bad("pfb_dada_pack: NBIT must be 8, 16, 32 or 64");
  }
  LCHK(hipGetLastError());
  return PFB_OK;
}

pfb_status pfb_gather_channels(const pfb_cf32* in, int64_t in_outer_stride, int64_t in_row_stride,
                               pfb_cf32* out, int64_t out_outer_stride, int64_t out_row_stride,
                               int64_t n_outer, int64_t n_rows, int32_t n_sel, int32_t src0,
                               int32_t split, int32_t shift, void* stream) {
  if (n_outer < 0 || n_rows < 0 || n_sel < 0) return bad("pfb_gather_channels: negative size");
  if (n_outer > 65535) return bad("pfb_gather_channels: n_outer > 65535");
  if (n_outer == 0 || n_rows == 0 || n_sel == 0) return PFB_OK;
  if (!in || !out) return bad("pfb_gather_channels: null buffer");
  const int64_t lo = std::min<int64_t>(src0, (int64_t)src0 + std::min(split, n_sel) + shift);
  const int64_t hi = (int64_t)src0 + n_sel - 1 + (split < n_sel ? shift : 0);
  if (lo < 0 || (n_rows > 1 && hi >= in_row_stride))
    return bad("pfb_gather_channels: source channel outside the input row");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(blocks_for(n_rows * n_sel), (unsigned)n_outer);
  hipLaunchKernelGGL(gather_kernel, grid, TPB, 0, s, (const float2*)in, in_outer_stride,
                     in_row_stride, (float2*)out, out_outer_stride, out_row_stride, n_rows, n_sel,
                     src0, split, shift);
  LCHK(hipGetLastError());
  return PFB_OK;
}

pfb_status pfb_corner_turn(const pfb_cf32* in, int64_t in_outer_stride, int64_t in_row_stride,
                           int64_t n_outer, int64_t n_rows, int64_t n_cols, pfb_cf32* out,
                           int64_t out_outer_stride, int64_t out_row_stride, void* stream) {
  if (n_outer < 0 || n_rows < 0 || n_cols < 0) return bad("pfb_corner_turn: negative size");
  if (n_outer > 65535 || (n_cols + 31) / 32 > 65535) return bad("pfb_corner_turn: too many columns/batches");
  if (n_outer == 0 || n_rows == 0 || n_cols == 0) return PFB_OK;
  if (!in || !out) return bad("pfb_corner_turn: null buffer");
  dim3 grid((unsigned)((n_rows + 31) / 32), (unsigned)((n_cols + 31) / 32), (unsigned)n_outer);
  hipLaunchKernelGGL(transpose_kernel, grid, TPB, 0, (hipStream_t)stream, (const float2*)in,
                     in_outer_stride, in_row_stride, n_rows, n_cols, (float2*)out, out_outer_stride,
                     out_row_stride);
  LCHK(hipGetLastError());
  return PFB_OK;
}

pfb_status pfb_quantize(const pfb_cf32* in, int64_t in_pol_stride, int64_t n, int32_t n_pol,
                        double rms, pfb_cf32* out, int64_t out_pol_stride, double* scale,
                        void* stream) {
  if (n < 0 || n_pol <= 0) return bad("pfb_quantize: bad sizes");
  if (in_pol_stride < n || out_pol_stride < n) return bad("pfb_quantize: polarisation stride too small");
  if (scale) *scale = 1.0;
  if (n == 0) return PFB_OK;
  if (!in || !out) return bad("pfb_quantize: null buffer");
  if (rms > 0 && n * (int64_t)n_pol < 2) return bad("pfb_quantize: var() of a single sample");
  hipStream_t s = (hipStream_t)stream;
  double* st = nullptr;
  LCHK(stats_buffer(&st));
  if (n_pol > 65535) return bad("pfb_quantize: n_pol > 65535");
  const dim3 g(std::max(1u, grid_stride_blocks(n * n_pol) / (unsigned)n_pol), (unsigned)n_pol);
  if (rms > 0) {
    LCHK(hipMemsetAsync(st, 0, 3 * sizeof(double), s));
    // few workgroups (each ends in three double atomics on one cache line, which serialise
    // in L2): ~4 per CU in total, every thread streaming many 16-byte loads
    const dim3 gm(std::max(1u, std::min(g.x, 1024u / (unsigned)n_pol)), (unsigned)n_pol);
    hipLaunchKernelGGL(moments_kernel, gm, TPB, 0, s, (const float2*)in, in_pol_stride, n, n_pol, st);
    LCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(quantize_kernel, g, TPB, 0, s, (const float2*)in, in_pol_stride, (float2*)out,
                     out_pol_stride, n, n_pol, rms, st);
  LCHK(hipGetLastError());
  if (scale) {
    LCHK(hipMemcpyAsync(scale, st + 3, sizeof(double), hipMemcpyDeviceToHost, s));
    LCHK(hipStreamSynchronize(s));
  }
  return PFB_OK;
}

pfb_status pfb_device_copy(void* dst, const void* src, int64_t n_bytes, void* stream) {
  if (!dst || !src || n_bytes < 0 || (n_bytes & 63) || (((uintptr_t)dst | (uintptr_t)src) & 15))
    return bad("pfb_device_copy: 16-B aligned pointers and a multiple of 64 bytes required");
  const int64_t n4 = n_bytes / 16;
  if (!n4) return PFB_OK;
  const int64_t blocks = (n4 + TPB - 1) / TPB;
  if (blocks > INT32_MAX) return bad("pfb_device_copy: more than 2^31 - 1 workgroups");
  const dim3 g((unsigned)blocks);
  hipLaunchKernelGGL(copy_kernel, g, TPB, 0, (hipStream_t)stream, (const copy_v4f*)src,
                     (copy_v4f*)dst, n4);
  LCHK(hipGetLastError());
  return PFB_OK;
}

}  // extern "C"

namespace pfb {
hipError_t launch_copy_rows(float2* dst, int64_t dps, const float2* src, int64_t sps, int64_t n, int n_pol,
                            hipStream_t s) {
  if (n <= 0 || n_pol <= 0) return hipSuccess;
  const unsigned gx = (unsigned)std::min<int64_t>(std::max<int64_t>((n + TPB - 1) / TPB, 1), 1024);
  hipLaunchKernelGGL(copy_rows_kernel, dim3(gx, (unsigned)n_pol), dim3(TPB), 0, s, dst, dps, src, sps, n);
  return hipGetLastError();
}
}  // namespace pfb
