// pfb_common.hpp — pieces shared by the kernel translation units (pfb_analysis.hip,
// pfb_rowfft.hip, pfb_synth.hip): workgroup size, store/load functors, the XCD-aware
// tile order, the row-FFT kernel template and launch helpers.
#pragma once

#include <hip/hip_ext.h>

#include "pfb_device.hpp"
#include "pfb_kernels.hpp"
#include "pfb_pair.hpp"

#include <algorithm>
#include <cstdlib>

namespace pfb {

constexpr int NT = 256;  // threads per workgroup (4 wave64)

// Cache policy (the buffer instructions' aux operand; gfx950: 1 = sc0, 2 = nt, 16 = sc1) of
// the C2 round trip's streams: analysis input loads, channelised-row stores, stage-1 row
// stores and loads, synthesis output stores.  Compile-time; a variant library is built with
// -DPFB_AUX_*=... (scripts/gpu_aux_ab.sh).  Measured (cache-policy A/B):
// nontemporal stores of the two products nobody re-reads (channelised rows, synthesis
// output) 1.5-2.7 % faster per pipelined step; nt on the stage-1 rows (re-read by the
// synthesis while partly Infinity-Cache resident) or on the input loads is slower.
#ifndef PFB_AUX_IN
#define PFB_AUX_IN 0
#endif
#ifndef PFB_AUX_CHAN
#define PFB_AUX_CHAN 2
#endif
#ifndef PFB_AUX_ZST
#define PFB_AUX_ZST 0
#endif
#ifndef PFB_AUX_ZLD
#define PFB_AUX_ZLD 0
#endif
#ifndef PFB_AUX_OUT
#define PFB_AUX_OUT 2
#endif
// strided channelised rows (a two-stage cascade's assembled stage-2 output): nt, the
// cascade 0.200-0.203 -> 0.192-0.195 ms (profiles/r04_v7_twostage_cache_policy_ab.jsonl);
// nt on the channel-major stage-1 product that stage 2 reads next: no consistent change
#ifndef PFB_AUX_STRIDED
#define PFB_AUX_STRIDED 2
#endif
constexpr int kAuxStrided = PFB_AUX_STRIDED;
// channel-major channelised rows (a cascade's stage-1 product, read by stage 2 next)
#ifndef PFB_AUX_COLMAJOR
#define PFB_AUX_COLMAJOR 0
#endif
constexpr int kAuxColMajor = PFB_AUX_COLMAJOR;
// LowCBF (PST filterbank) output rows: a product, as the channelised rows
#ifndef PFB_AUX_LCBF
#define PFB_AUX_LCBF PFB_AUX_CHAN
#endif
constexpr int kAuxLcbf = PFB_AUX_LCBF;
// the same for the C3 (SKA-Mid, N > 256) kernels' streams, nontemporal (1) or default (0):
// the FIR's stage-1 rows (PFB_NT_FIRZ), the row FFT's rows (RowStore, PFB_NT_ROW), the
// synth_wave512 output (PFB_NT_W5).  Measured: the C3 round trip 0.960/0.967 -> 0.936/0.954
// ms with ROW + W5 (profiles/r04_v5_cache_policy_ab.jsonl); per stream
// (profiles/r04_v9_c3_cache_policy_ab.jsonl, two boxes): all three nt 0.960-0.968 / 0.955-
// 0.961 against 0.974-0.988 / 0.961-0.972 with the FIR rows at the default policy — the
// 613 MB of rows exceed the Infinity Cache, and the row FFT that reads them runs 258-261
// instead of 282-289 us
#ifndef PFB_NT_FIRZ
#define PFB_NT_FIRZ 1
#endif
#ifndef PFB_NT_ROW
#define PFB_NT_ROW 1
#endif
#ifndef PFB_NT_W5
#define PFB_NT_W5 1
#endif
constexpr bool kNtFirZ = PFB_NT_FIRZ != 0, kNtRow = PFB_NT_ROW != 0, kNtW5 = PFB_NT_W5 != 0;
// and their loads: the FIR's input (PFB_NTL_FIR), the row FFT's rows (PFB_NTL_ROW), the
// synth_wave512 stage-1 rows (PFB_NTL_W5): none faster than the default policy
// (profiles/r04_v9_c3_load_policy_ab.jsonl)
#ifndef PFB_NTL_FIR
#define PFB_NTL_FIR 0
#endif
#ifndef PFB_NTL_ROW
#define PFB_NTL_ROW 0
#endif
#ifndef PFB_NTL_W5
#define PFB_NTL_W5 0
#endif
constexpr bool kNtlFir = PFB_NTL_FIR != 0, kNtlRow = PFB_NTL_ROW != 0, kNtlW5 = PFB_NTL_W5 != 0;
template <bool NT>
__device__ __forceinline__ float2 ld_nt(const float2* p) {
  if constexpr (NT) return __builtin_bit_cast(float2, __builtin_nontemporal_load(reinterpret_cast<const v2f*>(p)));
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st_nt(float2* p, float2 v) {
  if constexpr (NT) __builtin_nontemporal_store(__builtin_bit_cast(v2f, v), reinterpret_cast<v2f*>(p));
  else *p = v;
}
constexpr int kAuxIn = PFB_AUX_IN, kAuxChan = PFB_AUX_CHAN, kAuxZst = PFB_AUX_ZST, kAuxZld = PFB_AUX_ZLD,
              kAuxOut = PFB_AUX_OUT;

// ======================================================================= functors
struct AnalysisStore {
  static constexpr bool kIsLds = false;
  float2* out;
  int64_t K, Ktot, k0;  // K: end of the launch's rows; Ktot: rows of the whole call
  int N, sds, padded;
  float scale;
  int64_t k_lo = 0;     // first row of the launch (rows below it belong to another launch)
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const int64_t kg = k0 + row;
    if (kg < K && kg >= k_lo) {
      int64_t t = kg;
      if (padded) {
        // circular -sds shift (polyphase_analysis_padded.m:156); 0 <= kg < Ktot, so one
        // wrap suffices unless sds exceeds the row count (tiny inputs)
        t = kg - sds;
        while (t < 0) t += Ktot;
      }
      out[t * N + c] = cscale(v, scale);
    }
  }
};

// Row store through a range-checked buffer descriptor: rows [lo, records / (8 N)) of
// the descriptor's base are written, others dropped by the hardware (an out-of-range
// offset) — no branch per store, so the wave's vmcnt count stays path-independent and
// a later wait for a prefetch never has to wait for these stores too.
// Workgroup barrier of the wave synthesis kernels' block loops; TM bit 3 (a compile-time
// timing variant of the experiments build, results invalid) makes it a wave barrier — the
// barriers' share of a block's time
template <int TM>
__device__ __forceinline__ void wave_wg_sync() {
  if constexpr ((TM & 8) != 0) __builtin_amdgcn_wave_barrier();
  else __syncthreads();
}

struct BufRowStore {
  static constexpr bool kIsLds = false;
  __amdgpu_buffer_rsrc_t r;
  int lo, N;
  float scale;
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const uint32_t off = row >= lo ? (uint32_t)((row * N + c) * 8) : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, cscale(v, scale)), r, off, 0, kAuxChan);
  }
  // rows [k0, k0 + T) of a [row][N] array at `base`, valid rows [k_lo, k_hi)
  __device__ __forceinline__ static BufRowStore rows(float2* base, int64_t k0, int T, int64_t k_lo,
                                                      int64_t k_hi, int N, float scale) {
    const int64_t hi = min(max(k_hi - k0, (int64_t)0), (int64_t)T);
    const int lo = (int)min(max(k_lo - k0, (int64_t)0), (int64_t)T);
    return BufRowStore{make_rsrc_u(base + k0 * N, (uint32_t)(hi * N * 8)), lo, N, scale};
  }
};


// Rows [k0, k0 + T) of a strided channelised product (AnalysisArgs::out_rs): bin c of
// row `row` at base + row * rs + j(c) * cs, valid rows [lo, hi) and kept bins only — the
// rest are sent out of the descriptor's range (dropped).  Channel-major output (rs = 1,
// cs = series length) is the per-channel series a cascade's second stage reads; rs =
// nch1 nch2, cs = 1 with the chomp is TwoStageFilterBank's assembled output.
struct StridedRowStore {
  static constexpr bool kIsLds = false;
  __amdgpu_buffer_rsrc_t r;
  int lo, hi, rs, cs, split, shift, nsel;
  float scale;
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    // (bitwise, not short-circuit: the && chains compiled into divergent branches, two
    // exec-mask round trips per store)
    int j = c;
    bool ok = (row >= lo) & (row < hi);
    if (nsel > 0) {  // uniform
      j = c < split ? c : c - shift;
      ok = ok & ((c < split) | (c >= split + shift)) & (j < nsel);
    }
    const uint32_t off = ok ? (uint32_t)((row * rs + j * cs) * 8) : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, cscale(v, scale)), r, off, 0, kAuxStrided);
  }
  // the host checks that (T rs + jn cs) * 8 fits one descriptor (pfb_api.hip)
  __device__ __forceinline__ static StridedRowStore rows(float2* base, int64_t k0, int T, int64_t k_lo,
                                                          int64_t k_hi, int rs, int cs, int split,
                                                          int shift, int nsel, int N, float scale) {
    const int hi = (int)min(max(k_hi - k0, (int64_t)0), (int64_t)T);
    const int lo = (int)min(max(k_lo - k0, (int64_t)0), (int64_t)T);
    const int jn = nsel > 0 ? nsel : N;
    const uint32_t bytes = hi > 0 ? (uint32_t)(((int64_t)(hi - 1) * rs + (int64_t)(jn - 1) * cs + 1) * 8) : 0u;
    return StridedRowStore{make_rsrc_u(base + k0 * rs, bytes), lo, hi, rs, cs, split, shift, nsel, scale};
  }
};

// LowCBF output rows (216 of the 256 FFT bins, fftshifted): bin f of row `row` is channel
// c = (f - 148) mod 256 of output row k0 + row when c < 216 (polyphase_analysis_lowcbf.m /
// PSTFilterbank.m:35-44); other bins and rows outside [k_lo, k_hi) are dropped by the
// buffer range check.
struct LcbfRowStore {
  static constexpr bool kIsLds = false;
  __amdgpu_buffer_rsrc_t r;
  int lo;
  float scale;
  __device__ __forceinline__ void store(int row, int f, float2 v) const {
    const int c = (f + 108) & 255;
    const uint32_t off = (row >= lo && c < 216) ? (uint32_t)((row * 216 + c) * 8) : 0xFFFFFFF0u;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, cscale(v, scale)), r, off, 0, kAuxLcbf);
  }
  __device__ __forceinline__ static LcbfRowStore rows(float2* base, int64_t k0, int T, int64_t k_lo,
                                                       int64_t k_hi, float scale) {
    const int64_t hi = min(max(k_hi - k0, (int64_t)0), (int64_t)T);
    const int lo = (int)min(max(k_lo - k0, (int64_t)0), (int64_t)T);
    return LcbfRowStore{make_rsrc_u(base + k0 * 216, (uint32_t)(hi * 216 * 8)), lo, scale};
  }
};

// Row loader of the first FFT pass.  Rows past the end are clamped to the last valid
// row (their results are never stored), so every load is unconditional and the
// compiler can issue them back to back.
// Element (row, c) of a [row][N] array, or of its 2-row-run layout (run = true: rows 2g and
// 2g + 1 of column c at [g][c][0 / 1], i.e. 128-B lines of 2 rows x 8 columns) — the stage-1
// rows of the SKA-Mid round trip (FIR -> row FFT / synth_wave512_kernel)
__host__ __device__ __forceinline__ int64_t z_index(int64_t row, int c, int N, bool run) {
  return run ? (((row >> 1) * N + c) << 1) + (row & 1) : row * N + c;
}

template <bool PERM, bool GAIN>
struct RowLoad {
  static constexpr bool kIsLds = false;
  const float2* in;
  int64_t r0, last;
  int N;
  const int* perm;
  const float* cgain;
  int run;  // 2-row-run input layout (z_index)
  __device__ __forceinline__ float2 load(int row, int i) const {
    const int64_t r = min(r0 + row, last);
    const int c = PERM ? perm[i] : i;
    float2 v = ld_nt<kNtlRow>(in + z_index(r, c, N, run));
    if constexpr (GAIN) v = cscale(v, cgain[c]);  // taper acts on input rows (before re-ordering)
    return v;
  }
};

struct RowStore {
  static constexpr bool kIsLds = false;
  float2* out;
  int64_t r0, n_rows;
  int N;
  int64_t sds;
  int remap;
  float scale;
  int64_t row_base, n_total;  // output row = row_base + r (circularly shifted by -sds mod n_total)
  int zs;  // rows in runs of 2^zs per column (the wave synthesis' stage-1 row layout); 0: [row][c]
  int nt;  // nontemporal stores (PFB_NT_ROW) — 0: default policy, for rows read right after
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const int64_t r = r0 + row;
    if (r < n_rows) {
      int64_t t = row_base + r;
      if (remap) {  // row_base + r < n_total: one wrap (more only for tiny inputs)
        t -= sds;
        while (t < 0) t += n_total;
      }
      const int64_t i = zs ? ((((t >> zs) * N + c) << zs) + (t & ((1 << zs) - 1))) : t * N + c;
      if (nt) st_nt<kNtRow>(out + i, cscale(v, scale));
      else out[i] = cscale(v, scale);
    }
  }
};

// XCD-aware tile order: workgroups b and b+8 share an XCD (and its L2); give them
// consecutive tiles so the halo of one tile is an L2 hit for its neighbour.
// Bijective for any grid size (cdna_hip_programming.md, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_tile(int b, int nwg) {
  const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// ======================================================================= row FFT
struct RowFftArgs {
  const float2* in;
  int64_t in_pol_stride;
  float2* out;
  int64_t out_pol_stride;
  int64_t n_rows;
  const int* perm;
  const float* cgain;
  const float2* tw;
  float scale;
  int64_t sds;
  int remap;
  int64_t row_base;  // global index of row 0 (output row = row_base + r, then the remap)
  int64_t n_total;   // rows of the whole call (remap modulus)
  int zs = 0;        // output rows in runs of 2^zs per column (RowStore::zs)
  int nt = 1;        // RowStore::nt (the 4096-point kernel's rows are always nontemporal)
  int in_run = 0;    // input rows in 2-row runs per column (z_index), the SKA-Mid stage-1 rows
  int rev = 0;       // perm is the index reversal (N - i) mod N (the 4096-point pair kernel
                     // computes it instead of holding 16 column offsets per thread)
};

template <int N>
struct RowShape {
  static constexpr int ROWS = (N >= 4096) ? 1 : 4096 / N;
  static constexpr int RS = lds_row(N);
};

template <int N, int DIR, bool PERM, bool GAIN>
__global__ __launch_bounds__(NT) void row_fft_kernel(RowFftArgs a) {
  constexpr int ROWS = RowShape<N>::ROWS;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int pol = blockIdx.y;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  RowLoad<PERM, GAIN> ld{a.in + pol * a.in_pol_stride, r0, a.n_rows - 1, N, a.perm, a.cgain, a.in_run};
  RowStore st{a.out + pol * a.out_pol_stride, r0, a.n_rows, N, a.sds, a.remap, a.scale,
              a.row_base, a.n_total, a.zs, a.nt};
  LdsRows rows(smem, RowShape<N>::RS);
  // twiddle table -> LDS behind the rows (ordered before pass 2 by its barrier)
  float2* tw = smem + ROWS * RowShape<N>::RS;
  constexpr int TPT = (N + NT - 1) / NT;
  float2 twv[TPT];
#pragma unroll
  for (int i = 0; i < TPT; ++i) {
    const int m = threadIdx.x + i * NT;
    twv[i] = a.tw[m < N ? m : 0];
  }
#pragma unroll
  for (int i = 0; i < TPT; ++i)
    if (threadIdx.x + i * NT < N) tw[tw_slot(threadIdx.x + i * NT)] = twv[i];
  block_fft<N, DIR, ROWS, NT>(ld, st, rows, tw, threadIdx.x);
}

// All passes of FFTPlan<N> after the first (one row, LDS -> ... -> `last`).
template <int N, int DIR, class Last, class TW, int R0, int... Rest>
__device__ __forceinline__ void run_rest(const LdsRows& lds, const Last& last, const TW& tw, int tid,
                                         Radices<R0, Rest...>) {
  static_assert(sizeof...(Rest) > 0, "transform has a single pass");
  run_passes_impl<N, DIR, 1, NT, false, R0, Rest...>(lds, last, lds, tw, tid);
}

// Persistent row FFT for one-row-per-workgroup sizes (N >= 4096 with radix-16 first
// pass): each workgroup walks a contiguous range of rows (XCD-aware order), stages the
// twiddle table in LDS once, keeps the permutation / gain of its thread's 16 first-pass
// columns in registers, and loads row r + 1 into registers while it transforms row r.
// (The one-shot kernel re-read the 32 KB table from L2 for every one of the 73 400 C3
// rows and waited for each row's loads with nothing in flight.)
// (Two rows prefetched ahead and a half twiddle table were measured no faster, rounds 2
// and 4, and retired.)
template <int N>
constexpr size_t row_fft_persist_lds() {
  return ((size_t)RowShape<N>::RS + tw_slots(N)) * sizeof(float2);
}
template <int N, int DIR, bool PERM, bool GAIN>
__global__ __launch_bounds__(NT) void row_fft_persist_kernel(RowFftArgs a) {
  static_assert(RowShape<N>::ROWS == 1, "one row per workgroup");
  constexpr int R = FirstPassOf<N, 1, NT>::R, NB = N / R;
  static_assert(NB == NT, "one first-pass butterfly per thread");
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int pol = blockIdx.y;
  const int w = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t q0 = a.n_rows * w / gridDim.x, q1 = a.n_rows * (w + 1) / gridDim.x;
  if (q0 >= q1) return;
  const int tid = threadIdx.x;
  LdsRows rows(smem, RowShape<N>::RS);
  float2* tw = smem + RowShape<N>::RS;
  for (int m = tid; m < N; m += NT) tw[tw_slot(m)] = a.tw[m];
  const float2* in = a.in + pol * a.in_pol_stride;
  int col[R];
  float g[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = tid + r * NB;
    col[r] = PERM ? a.perm[i] : i;
    g[r] = GAIN ? a.cgain[col[r]] : 1.f;
  }
  float2 pf[R];
  auto load_row = [&](int64_t row) {
#pragma unroll
    for (int r = 0; r < R; ++r) pf[r] = ld_nt<kNtlRow>(in + z_index(row, col[r], N, a.in_run));
  };
  load_row(q0);
  vm_drain();
#pragma unroll 1
  for (int64_t row = q0; row < q1; ++row) {
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = GAIN ? cscale(pf[r], g[r]) : pf[r];
    load_row(min(row + 1, q1 - 1));  // unconditional: past the end re-reads the last row
    __syncthreads();  // tables / the previous row's last pass done with the LDS row
    // first pass (radix R, stride 1): no twiddles, outputs j R + r
    sdft<R, DIR>(v);
#pragma unroll
    for (int r = 0; r < R; ++r) rows.store(0, tid * R + r, v[r]);
    __syncthreads();
    RowStore st{a.out + pol * a.out_pol_stride, row, a.n_rows, N, a.sds, a.remap, a.scale,
                a.row_base, a.n_total, a.zs, a.nt};
    run_rest<N, DIR>(rows, st, (const float2*)tw, tid, typename FFTPlan<N>::type{});
  }
}

// ======================================================================= launchers
// Launch through hipExtLaunchKernelGGL when the profiler has armed events (they are
// consumed by this launch), else a plain launch.
template <class K, class... Args>
inline hipError_t launch_kernel(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
  LaunchEvents& ev = armed_launch_events();
  if (ev.start && ev.stop) {
    hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)lds, s, ev.start, ev.stop, 0, args...);
    ev = LaunchEvents{};
    launched_kernel_name() = hipKernelNameRefByPtr(reinterpret_cast<const void*>(kern), s);
  } else {
    hipLaunchKernelGGL(kern, grid, block, lds, s, args...);
  }
  return hipGetLastError();
}
template <class K>
inline hipError_t set_lds(K kernel, size_t bytes) {
  if (bytes > 65536) {
    return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
  }
  return hipSuccess;
}

inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}


// non-power-of-two channel counts of the synthesis stage-1 IFFT: the critically
// sampled / combined inputs of the two-stage inversion (nch2 = N de/nu, times combine;
// TwoStageInverseFilterBank.m:102-118)
inline bool mixed_chan_supported(int N) {
  switch (N) {
    case 14: case 28: case 56: case 112: case 192: case 216: case 224: case 384: case 432:
    case 448: case 768: case 864: case 896: case 1536: case 1792: case 3072: case 3584:
      return true;
    default:
      return false;
  }
}

inline bool pow2_supported(int N) {
  return N == 8 || N == 16 || N == 32 || N == 64 || N == 128 || N == 256 || N == 512 ||
         N == 1024 || N == 2048 || N == 4096;
}


// N-point row FFT over n_rows rows (pfb_rowfft.hip); DIR -1 forward, +1 inverse.
template <int DIR>
hipError_t dispatch_row_fft(int N, const RowFftArgs& r, int n_pol, hipStream_t s);

}  // namespace pfb
