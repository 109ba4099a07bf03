// pfb_kernels.hip — hand-written CDNA4 (gfx950) kernels of the PFB round trip.
//
//   analysis_fused_kernel  polyphase_analysis.m:83-121 / polyphase_analysis_padded.m:106-156
//                          one workgroup = T output rows of one polarisation: the input
//                          span is staged in LDS once, the taps of the thread's polyphase
//                          arm live in registers, the circular phase shift is applied as
//                          the LDS write address and the N-point FFT runs in LDS; the last
//                          Stockham pass writes the rows straight to HBM (coalesced).
//   fir_generic_kernel +   same maths for N > 256 (SKA-Mid 4096 channels): a FIR kernel
//   row_fft_kernel         writes the shifted polyphase sums, a row FFT kernel transforms.
//   row_fft_kernel         also synthesis stage 1 (inverse DFT across channels per row).
//   synth_block_kernel     synthesis stage 2 (polyphase_synthesis.m:163-316, re-ordered;
//                          see DESIGN.md): per block x 16 output phases t0, Nf-point FFT
//                          over time, kept-bin selection with deripple and four-step
//                          twiddle, W-point inverse FFT, overlap-discard, 1/L*de/nu.
#include "pfb_device.hpp"
#include "pfb_kernels.hpp"

namespace pfb {

constexpr int NT = 256;  // threads per workgroup (4 wave64)

// ======================================================================= functors
struct AnalysisStore {
  static constexpr bool kIsLds = false;
  float2* out;
  int64_t K, k0;
  int N, sds, padded;
  float scale;
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const int64_t kg = k0 + row;
    if (kg < K) {
      int64_t t = kg;
      if (padded) {
        t = (kg - sds) % K;
        if (t < 0) t += K;
      }
      out[t * N + c] = cscale(v, scale);
    }
  }
};

// Row loader of the first FFT pass.  Rows past the end are clamped to the last valid
// row (their results are never stored), so every load is unconditional and the
// compiler can issue them back to back.
template <bool PERM, bool GAIN>
struct RowLoad {
  static constexpr bool kIsLds = false;
  const float2* in;
  int64_t r0, last;
  int N;
  const int* perm;
  const float* cgain;
  __device__ __forceinline__ float2 load(int row, int i) const {
    const int64_t r = min(r0 + row, last);
    const int c = PERM ? perm[i] : i;
    float2 v = in[r * N + c];
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
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const int64_t r = r0 + row;
    if (r < n_rows) {
      int64_t t = r;
      if (remap) {
        t = (r - sds) % n_rows;
        if (t < 0) t += n_rows;
      }
      out[t * N + c] = cscale(v, scale);
    }
  }
};

// ======================================================================= analysis
template <int N, int PMAX, int TDIV = 1>
struct AnaShape {
  static constexpr int T = 4096 / N / TDIV; // output rows per workgroup
  static constexpr int RS = lds_row(N);     // padded LDS row (float2)
  static constexpr int KSTEP = NT / N;      // rows covered by one thread sweep
  static constexpr int KPT = T / KSTEP;     // rows per thread (= 16)
  // input span S = M (T-1) + P N <= N (T-1) + PMAX N samples, staged as float4 pairs
  static constexpr int SMAX = N * (T - 1) + PMAX * N;
  static constexpr int CH = (SMAX / 2 + NT - 1) / NT;  // float4 chunks per thread
};

// XCD-aware tile order: workgroups b and b+8 share an XCD (and its L2); give them
// consecutive tiles so the halo of one tile is an L2 hit for its neighbour.
// Bijective for any grid size (cdna_hip_programming.md, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_tile(int b, int nwg) {
  const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Stage x[base, base + S) into LDS (zero outside [0, n_dat)).  Interior tiles issue
// all of their 16-byte loads back to back before the first LDS write.
template <int CH>
__device__ __forceinline__ void stage_span(float2* smem, const float2* __restrict__ x,
                                           int64_t base, int S, int64_t n_dat, int tid) {
  const int S2 = (S + 1) >> 1;
  const bool interior = base >= 0 && base + 2 * (int64_t)S2 <= n_dat &&
                        ((reinterpret_cast<uintptr_t>(x + base) & 15) == 0);
  if (interior) {
    const float4* __restrict__ src = reinterpret_cast<const float4*>(x + base);
    float4 v[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = src[min(tid + i * NT, S2 - 1)];
    // unconditional (clamped) stores: a guarded store lets the compiler sink each load
    // into its branch and wait for it there, serialising the HBM latency
#pragma unroll
    for (int i = 0; i < CH; ++i) reinterpret_cast<float4*>(smem)[min(tid + i * NT, S2 - 1)] = v[i];
  } else {
    for (int s = tid; s < S; s += NT) {
      const int64_t g = base + s;
      smem[s] = (g >= 0 && g < n_dat) ? x[g] : make_float2(0.f, 0.f);
    }
  }
}

// PMAX = compile-time tap phases; EXACT means P == PMAX (no clamping needed).
template <int N, int PMAX, int VARIANT, int TDIV, bool EXACT>
__global__ __launch_bounds__(NT) void analysis_fused_kernel(AnalysisArgs a) {
  static_assert(NT % N == 0, "fused analysis needs N | 256");
  using S_ = AnaShape<N, PMAX, TDIV>;
  constexpr int T = S_::T;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int tid = threadIdx.x;
  const int pol = blockIdx.y;
  const int64_t k0 = (int64_t)xcd_tile(blockIdx.x, gridDim.x) * T;
  const int M = a.M, P = a.P;
  const int PN = P * N;
  const int S = M * (T - 1) + PN;
  const float2* __restrict__ x = a.in + pol * a.in_pol_stride;

  // 1. this thread's polyphase arm n: taps f[m N + n] in registers (taps are padded
  //    with zero rows to PMAX on the device, so the loads are unconditional)
  const int n = tid % N;
  const int kk0 = tid / N;
  float tr[PMAX];
#pragma unroll
  for (int m = 0; m < PMAX; ++m) tr[m] = a.taps[m * N + n];
  // 2. stage the input span of the T rows (Bunton: x[k0 M + s]; padded: x[k0 M - PN + s],
  //    zero history before t = 0, polyphase_analysis_padded.m:101-102)
  const int64_t base = (VARIANT == kBunton) ? k0 * M : k0 * M - PN;
  stage_span<S_::CH>(smem, x, base, S, a.n_dat, tid);
  __syncthreads();

  // 3. FIR: Bunton u_k[n] = sum_m f[mN+n] x[kM + mN + n]        (polyphase_analysis.m:105-115)
  //         padded y_q[n] = sum_p f[pN+n] x[qM - 1 - pN - n]      (polyphase_analysis_padded.m:118-126)
  //    Branch-free: taps are zero for m >= P and the LDS read index is clamped to the
  //    row's last phase (a sample of the row's own window, so 0 * x is exact even for
  //    non-finite x); a guarded read would serialise every LDS access.
  float2 u[S_::KPT];
#pragma unroll
  for (int e = 0; e < S_::KPT; ++e) {
    const int k = kk0 + e * S_::KSTEP;
    float ax = 0.f, ay = 0.f;
    if constexpr (VARIANT == kBunton) {
      const float2* p = smem + k * M + n;
#pragma unroll
      for (int m = 0; m < PMAX; ++m) {
        const int mm = EXACT ? m : min(m, P - 1);
        const float2 v = p[mm * N];
        ax = fmaf(tr[m], v.x, ax);
        ay = fmaf(tr[m], v.y, ay);
      }
    } else {
      const float2* p = smem + k * M + PN - 1 - n;
#pragma unroll
      for (int m = 0; m < PMAX; ++m) {
        const int mm = EXACT ? m : min(m, P - 1);
        const float2 v = p[-mm * N];
        ax = fmaf(tr[m], v.x, ax);
        ay = fmaf(tr[m], v.y, ay);
      }
    }
    u[e] = make_float2(ax, ay);
  }
  // twiddle table -> LDS, behind the FFT rows (the staged span is dead after the FIR)
  const float2 twv = a.twN[tid & (N - 1)];
  __syncthreads();
  if (tid < N) smem[T * S_::RS + tid] = twv;

  // 4. circular shift folded into the LDS write address
  //    Bunton: v[(n + r) mod N] = u[n], r = (M k) mod N               (polyphase_analysis.m:102-105)
  //    padded: z[(n - idx) mod N] = y[n], idx barrel index             (polyphase_analysis_padded.m:132-144)
  LdsRows rows(smem, S_::RS);
#pragma unroll
  for (int e = 0; e < S_::KPT; ++e) {
    const int k = kk0 + e * S_::KSTEP;
    const int64_t kg = k0 + k;
    int pos;
    if constexpr (VARIANT == kBunton) {
      const int r = (int)((kg * M) % N);
      pos = (n + r) % N;
    } else {
      const int b = (int)(kg % a.nu);
      const int idx = (b == 0) ? 0 : (int)(((int64_t)(a.nu - b) * (N - M)) % N);
      pos = (n - idx + N) % N;
    }
    rows.store(k, pos, u[e]);
  }
  __syncthreads();

  // 5. N-point DFT of every row; Bunton N*fft (forward), padded N^2*ifft (inverse dir.)
  AnalysisStore st{a.out + pol * a.out_pol_stride, a.K, k0, N, a.sds, VARIANT == kPadded,
                   (float)N};
  block_fft<N, (VARIANT == kBunton) ? -1 : +1, T, NT>(rows, st, rows, smem + T * S_::RS, tid);
}

template <int VARIANT>
__global__ __launch_bounds__(NT) void fir_generic_kernel(AnalysisArgs a) {
  const int pol = blockIdx.y;
  const int N = a.N, M = a.M, P = a.P;
  const int64_t idx = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (idx >= a.K * N) return;
  const int64_t k = idx / N;
  const int n = (int)(idx - k * N);
  const float2* __restrict__ x = a.in + pol * a.in_pol_stride;
  float ax = 0.f, ay = 0.f;
  for (int m = 0; m < P; ++m) {
    const float f = a.taps[m * N + n];
    int64_t g;
    if constexpr (VARIANT == kBunton) g = k * M + (int64_t)m * N + n;
    else g = k * M - 1 - (int64_t)m * N - n;
    if (g >= 0 && g < a.n_dat) {
      const float2 v = x[g];
      ax = fmaf(f, v.x, ax);
      ay = fmaf(f, v.y, ay);
    }
  }
  int pos;
  if constexpr (VARIANT == kBunton) {
    pos = (int)((n + (k * M) % N) % N);
  } else {
    const int b = (int)(k % a.nu);
    const int ix = (b == 0) ? 0 : (int)(((int64_t)(a.nu - b) * (N - M)) % N);
    pos = (n - ix + N) % N;
  }
  a.scratch[(int64_t)pol * a.K * N + k * N + pos] = make_float2(ax, ay);
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
  RowLoad<PERM, GAIN> ld{a.in + pol * a.in_pol_stride, r0, a.n_rows - 1, N, a.perm, a.cgain};
  RowStore st{a.out + pol * a.out_pol_stride, r0, a.n_rows, N, a.sds, a.remap, a.scale};
  LdsRows rows(smem, RowShape<N>::RS);
  // twiddle table -> LDS behind the rows (ordered before pass 2 by its barrier)
  float2* tw = smem + ROWS * RowShape<N>::RS;
  constexpr int TPT = (N + NT - 1) / NT;
  float2 twv[TPT];
#pragma unroll
  for (int i = 0; i < TPT; ++i) twv[i] = a.tw[(threadIdx.x + i * NT) & (N - 1)];
#pragma unroll
  for (int i = 0; i < TPT; ++i)
    if (threadIdx.x + i * NT < N) tw[threadIdx.x + i * NT] = twv[i];
  block_fft<N, DIR, ROWS, NT>(ld, st, rows, tw, threadIdx.x);
}

// ======================================================================= synthesis block
template <int NF, int W, int TG>
struct SynthShape {
  static constexpr int RSF = lds_row(NF) | 1;  // odd row stride: conflict-free column writes
  static constexpr int RSW = lds_row(W) | 1;
  static constexpr int RSMAX = RSF > RSW ? RSF : RSW;
  static constexpr int TWOFF = TG * RSMAX;  // twiddle tables (NF + W) + window behind the rows
  static constexpr size_t lds_bytes = (size_t)(TWOFF + NF + W) * sizeof(float2) + NF * sizeof(float);
};

template <int NF, int W, int TG>
__global__ __launch_bounds__(NT) void synth_block_kernel(SynthBlockArgs a) {
  using SS = SynthShape<NF, W, TG>;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int tid = threadIdx.x;
  const int t0 = blockIdx.x * TG;
  const int bl = blockIdx.y;
  const int pol = blockIdx.z;
  const int N = a.N;
  const float2* __restrict__ Z = a.Z + pol * a.z_pol_stride + (int64_t)bl * a.keep * N + t0;

  // 1. temporal taper + transpose: row i <- Z[tau][t0 + i]   (polyphase_synthesis.m:176-185)
  static_assert((TG * NF) % NT == 0, "tile must be a multiple of the workgroup");
  constexpr int LPT = TG * NF / NT;
  float2* twF = smem + SS::TWOFF;        // Nf twiddles, then W twiddles, then the window
  float2* twWl = twF + NF;
  float* win = reinterpret_cast<float*>(twWl + W);
  float2 zv[LPT];
#pragma unroll
  for (int e = 0; e < LPT; ++e) {
    const int idx = tid + e * NT;
    zv[e] = Z[(int64_t)(idx / TG) * N + (idx % TG)];
  }
  // twiddle tables of both transforms and the temporal window -> LDS
  constexpr int TF = (NF + W + NT - 1) / NT;
  constexpr int TW_ = (NF + NT - 1) / NT;
  float2 twv[TF];
  float wv[TW_];
#pragma unroll
  for (int i = 0; i < TF; ++i) {
    const int j = min(tid + i * NT, NF + W - 1);
    twv[i] = (j < NF) ? a.twNf[j] : a.twW[j - NF];
  }
#pragma unroll
  for (int i = 0; i < TW_; ++i) wv[i] = a.window[min(tid + i * NT, NF - 1)];
#pragma unroll
  for (int i = 0; i < TF; ++i)
    if (tid + i * NT < NF + W) twF[tid + i * NT] = twv[i];
#pragma unroll
  for (int i = 0; i < TW_; ++i)
    if (tid + i * NT < NF) win[tid + i * NT] = wv[i];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < LPT; ++e) {
    const int idx = tid + e * NT;
    const int tau = idx / TG;
    smem[(idx % TG) * SS::RSF + lpad(tau)] = cscale(zv[e], win[tau]);
  }
  __syncthreads();
  // 2. Nf-point forward FFT over time for every t0 row
  LdsRows rowsF(smem, SS::RSF);
  block_fft<NF, -1, TG, NT>(rowsF, rowsF, rowsF, twF, tid);
  __syncthreads();

  // 3. keep W bins (fftshift + discard, :188,240), deripple gain (:242-251), four-step
  //    twiddle e^{+2 pi i t0 expo / L} (carries the spans-Nyquist W/2 stitch shift);
  //    gain x twiddle come from one [t0][j'] table so the lookup is coalesced
  //    kept bin of slot j': spans Nyquist -> signed frequency j' (j' < W/2) or
  //    j' - W (j' >= W/2); critical -> fftshift(...)(d2 + j')
  constexpr int SEL = (TG * W + NT - 1) / NT;
  float2 sv[SEL];
#pragma unroll
  for (int e = 0; e < SEL; ++e) {
    const int idx = tid + e * NT;
    if (idx < TG * W) {
      const int i = idx / W;
      const int jp = idx - i * W;
      int src;
      if (a.spans) src = (jp < W / 2) ? jp : jp + NF - W;
      else src = (jp < W / 2) ? jp + NF - W / 2 : jp - W / 2;
      sv[e] = cmul(rowsF.load(i, src), a.tw4[(int64_t)(t0 + i) * W + jp]);  // coalesced
    }
  }
  __syncthreads();
  LdsRows rowsW(smem, SS::RSW);
#pragma unroll
  for (int e = 0; e < SEL; ++e) {
    const int idx = tid + e * NT;
    if (idx < TG * W) {
      const int i = idx / W;
      rowsW.store(i, idx - i * W, sv[e]);
    }
  }
  __syncthreads();
  // 4. W-point inverse FFT per t0 row
  block_fft<W, +1, TG, NT>(rowsW, rowsW, rowsW, twWl, tid);
  __syncthreads();

  // 5. overlap-discard (:302) and scale 1/L * de/nu (:285), y[t0 + N t1]
  const int nt1 = a.t1_hi - a.t1_lo;
  float2* __restrict__ o =
      a.out + pol * a.out_pol_stride + (a.block0 + bl) * (int64_t)a.Lkeep - a.Lov;
  const int64_t limit = a.out_limit - (a.block0 + bl) * (int64_t)a.Lkeep + a.Lov;
  for (int idx = tid; idx < TG * nt1; idx += NT) {
    const int i = idx % TG;
    const int t1 = a.t1_lo + idx / TG;
    const int64_t t = t0 + i + (int64_t)N * t1;
    if (t < limit) o[t] = cscale(rowsW.load(i, t1), a.scale);
  }
}

// ======================================================================= launchers
template <class K>
static hipError_t set_lds(K kernel, size_t bytes) {
  if (bytes > 65536) {
    return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
  }
  return hipSuccess;
}

template <int N, int PMAX, int VARIANT, int TDIV, bool EXACT = false>
static hipError_t launch_fused(const AnalysisArgs& a, hipStream_t s) {
  using S_ = AnaShape<N, PMAX, TDIV>;
  const size_t span = (size_t)a.M * (S_::T - 1) + (size_t)a.P * N;
  const size_t rows = (size_t)S_::T * S_::RS + N;  // FFT rows + twiddle table
  const size_t bytes = ((span + 1 > rows) ? span + 1 : rows) * sizeof(float2);
  auto kern = analysis_fused_kernel<N, PMAX, VARIANT, TDIV, EXACT>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((a.K + S_::T - 1) / S_::T), (unsigned)a.n_pol);
  hipLaunchKernelGGL(kern, grid, dim3(NT), bytes, s, a);
  return hipGetLastError();
}

template <int N, int VARIANT>
static hipError_t launch_fused_p(const AnalysisArgs& a, hipStream_t s) {
  // exact instantiations for the configured tap counts (SKA-Low 13 and 12 phases,
  // the 'test' config 11); other P use the clamped PMAX 16/32 kernels
  if (a.P == 13) {
    if (a.tile_div == 2) return launch_fused<N, 13, VARIANT, 2, true>(a, s);
    return launch_fused<N, 13, VARIANT, 1, true>(a, s);
  }
  if (a.P == 12) return launch_fused<N, 12, VARIANT, 1, true>(a, s);
  if (a.P == 11) return launch_fused<N, 11, VARIANT, 1, true>(a, s);
  if (a.P <= 16) return launch_fused<N, 16, VARIANT, 1>(a, s);
  return launch_fused<N, 32, VARIANT, 1>(a, s);
}

template <int N>
static hipError_t launch_fused_v(const AnalysisArgs& a, hipStream_t s) {
  if (a.variant == kBunton) return launch_fused_p<N, kBunton>(a, s);
  return launch_fused_p<N, kPadded>(a, s);
}

template <int N, int DIR, bool PERM, bool GAIN>
static hipError_t launch_row_fft_t(const RowFftArgs& r, int n_pol, hipStream_t s) {
  constexpr int ROWS = RowShape<N>::ROWS;
  const size_t bytes = ((size_t)ROWS * RowShape<N>::RS + N) * sizeof(float2);
  auto kern = row_fft_kernel<N, DIR, PERM, GAIN>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((r.n_rows + ROWS - 1) / ROWS), (unsigned)n_pol);
  hipLaunchKernelGGL(kern, grid, dim3(NT), bytes, s, r);
  return hipGetLastError();
}

template <int N, int DIR>
static hipError_t launch_row_fft(const RowFftArgs& r, int n_pol, hipStream_t s) {
  if constexpr (DIR > 0) {
    if (r.perm && r.cgain) return launch_row_fft_t<N, DIR, true, true>(r, n_pol, s);
    if (r.perm) return launch_row_fft_t<N, DIR, true, false>(r, n_pol, s);
    if (r.cgain) return launch_row_fft_t<N, DIR, false, true>(r, n_pol, s);
  }
  return launch_row_fft_t<N, DIR, false, false>(r, n_pol, s);
}

template <int DIR>
static hipError_t dispatch_row_fft(int N, const RowFftArgs& r, int n_pol, hipStream_t s) {
  switch (N) {
    case 8: return launch_row_fft<8, DIR>(r, n_pol, s);
    case 16: return launch_row_fft<16, DIR>(r, n_pol, s);
    case 32: return launch_row_fft<32, DIR>(r, n_pol, s);
    case 64: return launch_row_fft<64, DIR>(r, n_pol, s);
    case 128: return launch_row_fft<128, DIR>(r, n_pol, s);
    case 256: return launch_row_fft<256, DIR>(r, n_pol, s);
    case 512: return launch_row_fft<512, DIR>(r, n_pol, s);
    case 1024: return launch_row_fft<1024, DIR>(r, n_pol, s);
    case 2048: return launch_row_fft<2048, DIR>(r, n_pol, s);
    case 4096: return launch_row_fft<4096, DIR>(r, n_pol, s);
    default: return hipErrorInvalidValue;
  }
}

static bool pow2_supported(int N) {
  return N == 8 || N == 16 || N == 32 || N == 64 || N == 128 || N == 256 || N == 512 ||
         N == 1024 || N == 2048 || N == 4096;
}

bool analysis_supported(int N, int P, int variant, bool* fused) {
  (void)variant;
  const bool f = (N >= 8 && N <= 256 && pow2_supported(N) && P <= 32);
  if (fused) *fused = f;
  return pow2_supported(N);
}

hipError_t launch_analysis(const AnalysisArgs& a, hipStream_t s) {
  if (a.K <= 0) return hipSuccess;
  bool fused = false;
  if (!analysis_supported(a.N, a.P, a.variant, &fused)) return hipErrorInvalidValue;
  if (fused) {
    switch (a.N) {
      case 8: return launch_fused_v<8>(a, s);
      case 16: return launch_fused_v<16>(a, s);
      case 32: return launch_fused_v<32>(a, s);
      case 64: return launch_fused_v<64>(a, s);
      case 128: return launch_fused_v<128>(a, s);
      case 256: return launch_fused_v<256>(a, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (!a.scratch) return hipErrorInvalidValue;
  // generic: FIR into scratch, then row FFT (with the padded circular time shift)
  const int64_t total = a.K * a.N;
  dim3 grid((unsigned)((total + NT - 1) / NT), (unsigned)a.n_pol);
  if (a.variant == kBunton) hipLaunchKernelGGL(fir_generic_kernel<kBunton>, grid, dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(fir_generic_kernel<kPadded>, grid, dim3(NT), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  RowFftArgs r{a.scratch, a.K * a.N, a.out, a.out_pol_stride, a.K, nullptr, nullptr, a.twN,
               (float)a.N, a.sds, a.variant == kPadded};
  if (a.variant == kBunton) return dispatch_row_fft<-1>(a.N, r, a.n_pol, s);
  return dispatch_row_fft<+1>(a.N, r, a.n_pol, s);
}

bool chan_ifft_supported(int N) { return pow2_supported(N); }

hipError_t launch_chan_ifft(const ChanIfftArgs& c, hipStream_t s) {
  if (c.n_rows <= 0) return hipSuccess;
  RowFftArgs r{c.in, c.in_pol_stride, c.out, c.out_pol_stride, c.n_rows, c.perm, c.cgain, c.twN,
               1.0f, 0, 0};
  return dispatch_row_fft<+1>(c.N, r, c.n_pol, s);
}

template <int NF, int W, int TG>
static hipError_t launch_sb(const SynthBlockArgs& a, hipStream_t s) {
  using SS = SynthShape<NF, W, TG>;
  auto kern = synth_block_kernel<NF, W, TG>;
  hipError_t e = set_lds(kern, SS::lds_bytes);
  if (e != hipSuccess) return e;
  if (a.N % TG != 0) return hipErrorInvalidValue;
  dim3 grid((unsigned)(a.N / TG), (unsigned)a.n_blocks, (unsigned)a.n_pol);
  hipLaunchKernelGGL(kern, grid, dim3(NT), SS::lds_bytes, s, a);
  return hipGetLastError();
}

template <int NF, int W>
static hipError_t launch_sb_tg(const SynthBlockArgs& a, hipStream_t s) {
  if (a.N >= 16) return launch_sb<NF, W, 16>(a, s);
  return launch_sb<NF, W, 8>(a, s);
}

#define PFB_SYNTH_SIZES(X) \
  X(128, 112)              \
  X(128, 96)               \
  X(256, 224)              \
  X(256, 192)              \
  X(256, 216)              \
  X(512, 448)              \
  X(1024, 896)

bool synth_block_supported(int Nf, int W) {
#define X(a_, b_) if (Nf == a_ && W == b_) return true;
  PFB_SYNTH_SIZES(X)
#undef X
  return false;
}

hipError_t launch_synth_block(const SynthBlockArgs& a, hipStream_t s) {
  if (a.n_blocks <= 0) return hipSuccess;
#define X(a_, b_) \
  if (a.Nf == a_ && a.W == b_) return (a_ >= 1024) ? launch_sb<a_, b_, 8>(a, s) : launch_sb_tg<a_, b_>(a, s);
  PFB_SYNTH_SIZES(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace pfb
