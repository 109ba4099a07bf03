// pfb_spectral.hip — synthesis with a non-identity SPECTRAL taper
// (polyphase_synthesis.m:282 `FFFF = spectral_taper(FFFF, length(FFFF), input_overlap)`,
// set through InverseFilterBank.frequency_taper, InverseFilterBank.m:48-61 /
// TwoStageInverseFilterBank.m:57-70; the 'hann' handle is PFBWindow.m:70-100).
//
// The taper multiplies the stitched L-point spectrum element-wise, T[c][j] =
// H[(c W + j - W/2) mod L] (spans Nyquist) or H[c W + j] (critical): not separable in
// (channel c, kept bin j), so it cannot commute past the channel IFFT the way the
// re-ordered synthesis moves it.  This path keeps Matlab's order and
// factors only the final L-point IFFT (four-step, i = c W + j, t = t0 + N t1):
//   1. X[b][c][t]  = chan[b keep + t][c]                      (tile transpose)
//   2. F[b][c][f]  = FFT_Nf(window x X[b][c][:])[f]              (window on the transpose)
//   3. A[b][j][c]  = F[b][perm c][(d2 + j + Nf/2) mod Nf] g[j] cgain[perm c] T[c][j]
//   4. A1[b][j][t0] = sum_c A[b][j][c] e^{+2 pi i c t0 / N}     (row IFFT over c)
//   5. B[b][t0][j] = A1[b][j][t0]                              (tile transpose)
//   6. y[t0 + N t1] = (de/nu)/L e^{-i pi t0/N} (-1)^{t1} sum_j e^{2 pi i j t1/W}
//                     e^{2 pi i j t0/L} B[b][t0][j]            (row IFFT over j, spans)
//      kept t1 in [Lov/N, W - Lov/N) -> out[b Lkeep + t0 + N t1 - Lov].
// (e^{-i pi t/N} is the W/2 roll of the spans-Nyquist stitch, see DESIGN.md Appendix.)
// The numerical path is float32 like the rest; twiddles of step 6 in double.
#include "pfb_common.hpp"

namespace pfb {

// out[o][c][r] = in[o][r][c] x gain[r] (gain optional) for r < rows, c < cols (32 x 32 LDS tiles)
__global__ __launch_bounds__(256) void tile_transpose_kernel(const float2* __restrict__ in, int64_t ios,
                                                              int64_t irs, float2* __restrict__ out,
                                                              int64_t oos, int64_t ors, int rows, int cols,
                                                              const float* __restrict__ gain) {
  __shared__ float2 tile[32][33];
  const int64_t o = blockIdx.z;
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r0 + ty + 8 * k, c = c0 + tx;
    if (r < rows && c < cols) {
      const float2 v = in[o * ios + (int64_t)r * irs + c];
      tile[ty + 8 * k][tx] = gain ? cscale(v, gain[r]) : v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + ty + 8 * k, r = r0 + tx;
    if (r < rows && c < cols) out[o * oos + (int64_t)c * ors + r] = tile[tx][ty + 8 * k];
  }
}

// step 3: A[b][j][c] = F[b][perm c][src(j)] x gains x taper, 32 (j) x 32 (c) tiles
__global__ __launch_bounds__(256) void spec_select_kernel(SpectralArgs a, const float2* __restrict__ F,
                                                           float2* __restrict__ A) {
  __shared__ float2 tile[32][33];
  const int64_t b = blockIdx.z;
  const int j0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int W = a.W, N = a.N, Nf = a.Nf, W2 = a.W / 2, d2 = (a.Nf - a.W) / 2;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + ty + 8 * k, j = j0 + tx;
    if (c < N && j < W) {
      const int pc = a.perm ? a.perm[c] : c;
      const int f = (d2 + j + Nf / 2) % Nf;
      float gain = a.gainj[j] * (a.cgain ? a.cgain[pc] : 1.f);
      int64_t i = (int64_t)c * W + j - (a.spans ? W2 : 0);
      if (i < 0) i += a.L;
      gain *= a.taper[i];
      tile[ty + 8 * k][tx] = cscale(F[(b * N + pc) * Nf + f], gain);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = j0 + ty + 8 * k, c = c0 + tx;
    if (c < N && j < W) A[(b * W + j) * N + c] = tile[tx][ty + 8 * k];
  }
}

// step 6 loader: row r = (b, t0) of B, element j, times e^{2 pi i j t0 / L}
struct WOutLoad {
  static constexpr bool kIsLds = false;
  const float2* in;
  int64_t r0, last;
  int W, N, L;
  __device__ __forceinline__ float2 load(int row, int j) const {
    const int64_t r = min(r0 + row, last);
    const int t0 = (int)(r % N);
    const float2 v = in[r * W + j];
    const int64_t m = ((int64_t)j * t0) % L;
    double s, c;
    sincospi(2.0 * (double)m / (double)L, &s, &c);
    return cmul(v, make_float2((float)c, (float)s));
  }
};

// step 6 store: keep t1 in [t1_lo, t1_hi), spans phase, scale, scatter to the output
struct WOutStore {
  static constexpr bool kIsLds = false;
  float2* out;
  int64_t r0, n_rows, blk0, out_limit;
  int N, t1_lo, t1_hi, Lov, Lkeep, spans;
  float scale;
  __device__ __forceinline__ void store(int row, int t1, float2 v) const {
    const int64_t r = r0 + row;
    if (r >= n_rows || t1 < t1_lo || t1 >= t1_hi) return;
    const int64_t b = r / N;
    const int t0 = (int)(r - b * N);
    const int64_t rel = t0 + (int64_t)N * t1 - Lov;  // kept position (L_ov need not be a multiple of N)
    if (rel < 0 || rel >= Lkeep) return;
    const int64_t idx = (blk0 + b) * Lkeep + rel;
    if (idx >= out_limit) return;
    if (spans) {
      double s, c;
      sincospi(-(double)t0 / (double)N, &s, &c);
      v = cmul(v, make_float2((float)c, (float)s));
      if (t1 & 1) v = make_float2(-v.x, -v.y);
    }
    out[idx] = cscale(v, scale);
  }
};

template <int W>
__global__ __launch_bounds__(NT) void w_out_kernel(WOutLoad ld, WOutStore st, const float2* __restrict__ twW) {
  constexpr int ROWS = RowShape<W>::ROWS;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  WOutLoad l = ld;
  l.r0 = r0;
  WOutStore s = st;
  s.r0 = r0;
  LdsRows rows(smem, RowShape<W>::RS);
  float2* tw = smem + ROWS * RowShape<W>::RS;
  for (int i = threadIdx.x; i < W; i += NT) tw[tw_slot(i)] = twW[i];
  __syncthreads();
  block_fft<W, +1, ROWS, NT>(l, s, rows, tw, threadIdx.x);
}

template <int W>
static hipError_t launch_w_out(const WOutLoad& l, const WOutStore& s, const float2* twW, int64_t rows,
                               hipStream_t st) {
  constexpr int ROWS = RowShape<W>::ROWS;
  const size_t bytes = ((size_t)ROWS * RowShape<W>::RS + tw_slots(W)) * sizeof(float2);
  auto kern = w_out_kernel<W>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((rows + ROWS - 1) / ROWS));
  return launch_kernel(kern, grid, dim3(NT), bytes, st, l, s, twW);
}

static hipError_t dispatch_w_out(int W, const WOutLoad& l, const WOutStore& s, const float2* twW,
                                 int64_t rows, hipStream_t st) {
  switch (W) {
    case 96: return launch_w_out<96>(l, s, twW, rows, st);
    case 112: return launch_w_out<112>(l, s, twW, rows, st);
    case 192: return launch_w_out<192>(l, s, twW, rows, st);
    case 216: return launch_w_out<216>(l, s, twW, rows, st);
    case 224: return launch_w_out<224>(l, s, twW, rows, st);
    case 448: return launch_w_out<448>(l, s, twW, rows, st);
    case 896: return launch_w_out<896>(l, s, twW, rows, st);
    default: return hipErrorInvalidValue;
  }
}

static hipError_t transpose(const float2* in, int64_t ios, int64_t irs, float2* out, int64_t oos,
                            int64_t ors, int64_t n_outer, int rows, int cols, hipStream_t s,
                            const float* gain = nullptr) {
  if (n_outer > 65535) return hipErrorInvalidValue;
  dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32), (unsigned)n_outer);
  hipLaunchKernelGGL(tile_transpose_kernel, grid, dim3(256), 0, s, in, ios, irs, out, oos, ors, rows, cols,
                     gain);
  return hipGetLastError();
}

bool spectral_synth_supported(int Nf, int W, int N) {
  return pow2_supported(Nf) && (pow2_supported(N) || mixed_chan_supported(N)) &&
         (W == 96 || W == 112 || W == 192 || W == 216 || W == 224 || W == 448 || W == 896);
}

hipError_t launch_spectral_synth(const SpectralArgs& a, hipStream_t s) {
  if (a.nb <= 0) return hipSuccess;
  if (a.nb > 65535) return hipErrorInvalidValue;
  const int N = a.N, Nf = a.Nf, W = a.W;
  for (int pol = 0; pol < a.n_pol; ++pol) {
    const float2* in = a.in + pol * a.in_pol_stride + a.b0 * (int64_t)a.keep * N;
    // 1. X[b][c][t] = window[t] chan[b keep + t][c] (buf0)
    hipError_t e = transpose(in, (int64_t)a.keep * N, N, a.buf0, (int64_t)N * Nf, Nf, a.nb, Nf, N, s,
                             a.window);
    if (e != hipSuccess) return e;
    // 2. F[b][c][f] (buf1): forward Nf-point row FFT
    RowFftArgs f{a.buf0, 0, a.buf1, 0, a.nb * N, nullptr, nullptr, a.twNf, 1.0f, 0, 0, 0, a.nb * N};
    e = dispatch_row_fft<-1>(Nf, f, 1, s);
    if (e != hipSuccess) return e;
    // 3. A[b][j][c] (buf0)
    {
      dim3 grid((unsigned)((W + 31) / 32), (unsigned)((N + 31) / 32), (unsigned)a.nb);
      hipLaunchKernelGGL(spec_select_kernel, grid, dim3(256), 0, s, a, (const float2*)a.buf1, a.buf0);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    // 4. A1[b][j][t0] (buf1): inverse N-point row FFT over the channels
    RowFftArgs c{a.buf0, 0, a.buf1, 0, a.nb * W, nullptr, nullptr, a.twN, 1.0f, 0, 0, 0, a.nb * W};
    e = dispatch_row_fft<+1>(N, c, 1, s);
    if (e != hipSuccess) return e;
    // 5. B[b][t0][j] (buf0)
    e = transpose(a.buf1, (int64_t)W * N, N, a.buf0, (int64_t)N * W, W, a.nb, W, N, s);
    if (e != hipSuccess) return e;
    // 6. W-point inverse row FFT with the four-step twiddle -> output samples
    const WOutLoad l{a.buf0, 0, a.nb * N - 1, W, N, a.L};
    const WOutStore o{a.out + pol * a.out_pol_stride, 0, a.nb * N, a.b0, a.out_limit, N, a.t1_lo,
                      a.t1_hi, a.Lov, a.Lkeep, a.spans, a.scale};
    e = dispatch_w_out(W, l, o, a.twW, a.nb * N, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace pfb
