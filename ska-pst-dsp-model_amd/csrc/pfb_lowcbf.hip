// pfb_lowcbf.hip — the SKA-Low CBF PST filterbank (polyphase_analysis_lowcbf.m:1-49
// wrapping PSTFilterbank.m:1-46), the bit-faithful firmware model plugged in as a third
// analysis function (test.config.json "lowpsi").
//
// Per output sample k (0-based) and polarisation:
//   u[n]   = sum_{m<12} h[n + 256 m] x[192 k + n + 256 m - pad]      (PSTFilterbank.m:28-30)
//   F      = FFT_256(u)                                             (:35, forward)
//   y[j]   = F[(j + 128) mod 256] * i^{(k (j - 128)) mod 4}        (fftshift, :35-42)
//   out[c] = y[20 + c] * 2^12,  c < 216                             (:44 and the wrapper's
//            2^9 * 2048 * 256 rescale of the /2^9 and /128 firmware scalings)
// pad = 1536 zeros on the first call only (the wrapper's `persistent do_padding`).
//
// One workgroup = 16 output rows of one polarisation: thread n owns polyphase arm n
// (12 taps in registers), the FIR sums go to LDS rows, the 256-point FFT runs as two
// radix-16 Stockham passes in LDS and the last pass applies fftshift, derotation,
// channel selection and scale on its way to HBM.  HBM-bound: 8 B read per input
// sample, 216 * 8 B written per 192 input samples.
#include "pfb_common.hpp"
#include "pfb_pair.hpp"

#include <cstdlib>

namespace pfb {

namespace {

constexpr int LN = 256, LM = 192, LP = 12, LKEEP = 216, LFIRST = 20, LROWS = 16;

struct LowCbfStore {
  static constexpr bool kIsLds = false;
  float2* out;
  int64_t k0, K;
  float scale;
  __device__ __forceinline__ void store(int row, int c, float2 v) const {
    const int64_t k = k0 + row;
    const int j = (c + LN / 2) & (LN - 1);  // fftshift position of FFT bin c
    if (k < K && j >= LFIRST && j < LFIRST + LKEEP) {
      // mod(k (j - 128), 4); & 3 is the non-negative residue in two's complement
      const int rot = (int)((k & 3) * ((j - LN / 2) & 3)) & 3;
      float2 w = cscale(v, scale);
      if (rot == 1) w = make_float2(-w.y, w.x);
      else if (rot == 2) w = make_float2(-w.x, -w.y);
      else if (rot == 3) w = make_float2(w.y, -w.x);
      out[k * LKEEP + (j - LFIRST)] = w;
    }
  }
};

__global__ __launch_bounds__(NT) void lowcbf_kernel(LowCbfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  constexpr int RS = lds_row(LN);
  const int pol = blockIdx.y;
  const int64_t k0 = (int64_t)blockIdx.x * LROWS;
  const int n = threadIdx.x;  // NT == LN: one polyphase arm per thread
  const float2* __restrict__ x = a.in + pol * a.in_pol_stride;
  float f[LP];
#pragma unroll
  for (int m = 0; m < LP; ++m) f[m] = a.taps[n + LN * m];
  LdsRows rows(smem, RS);
  float2* tw = smem + LROWS * RS;
  tw[tw_slot(n)] = a.tw[n];
  const bool interior = k0 * LM - a.pad >= 0 &&
                        (k0 + LROWS - 1) * LM + LN * LP - a.pad <= a.n_dat && k0 + LROWS <= a.K;
  if (interior) {
    // 4 M = 3 N: row k + 4 reads the samples of row k shifted by 3 taps, so each of the
    // 4 commutator residues keeps a 12-sample register window and loads 3 new samples
    // per row (84 loads per thread instead of 192)
    static_assert(4 * LM == 3 * LN && LROWS % 4 == 0, "commutator period");
    const float2* __restrict__ xb = x + (k0 * LM + n - a.pad);
#pragma unroll 1
    for (int rho = 0; rho < 4; ++rho) {
      v2f w[LP];
#pragma unroll
      for (int m = 0; m < LP; ++m) {
        const float2 v = xb[rho * LM + m * LN];
        w[m] = v2f{v.x, v.y};
      }
#pragma unroll
      for (int jj = 0; jj < LROWS / 4; ++jj) {
        const int r = rho + 4 * jj;
        v2f nw[3];
        if (jj + 1 < LROWS / 4) {
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const float2 v = xb[(r + 4) * LM + (LP - 3 + i) * LN];
            nw[i] = v2f{v.x, v.y};
          }
        }
        v2f acc{0.f, 0.f};
#pragma unroll
        for (int m = 0; m < LP; ++m) acc = __builtin_elementwise_fma(v2f{f[m], f[m]}, w[m], acc);
        rows.store(r, n, make_float2(acc.x, acc.y));
        if (jj + 1 < LROWS / 4) {
#pragma unroll
          for (int m = 0; m < LP - 3; ++m) w[m] = w[m + 3];
#pragma unroll
          for (int i = 0; i < 3; ++i) w[LP - 3 + i] = nw[i];
        }
      }
    }
  } else {
    for (int r = 0; r < LROWS; ++r) {
      float ax = 0.f, ay = 0.f;
      const int64_t k = k0 + r;
      if (k < a.K) {
#pragma unroll
        for (int m = 0; m < LP; ++m) {
          const int64_t g = k * LM + n + m * LN - a.pad;
          if (g >= 0 && g < a.n_dat) {
            const float2 v = x[g];
            ax = fmaf(f[m], v.x, ax);
            ay = fmaf(f[m], v.y, ay);
          }
        }
      }
      rows.store(r, n, make_float2(ax, ay));
    }
  }
  __syncthreads();
  LowCbfStore st{a.out + pol * a.out_pol_stride, k0, a.K, a.scale};
  block_fft<LN, -1, LROWS, NT>(rows, st, rows, tw, n);
}

}  // namespace

hipError_t launch_lowcbf(const LowCbfArgs& a, hipStream_t s) {
  if (a.K <= 0) return hipSuccess;
  // streaming path (analysis_stream_kernel<256, 12, 4, 3, LCBF>): persistent workgroups,
  // each input sample loaded once; PFB_LOWCBF_STREAM=0 keeps the one-shot kernel below
  static const bool one_shot = knob("PFB_LOWCBF_STREAM") && std::atoi(knob("PFB_LOWCBF_STREAM")) == 0;
  if (!one_shot) {
    AnalysisArgs b{};
    b.in = a.in;
    b.in_pol_stride = a.in_pol_stride;
    b.n_dat = a.n_dat;
    b.out = a.out;
    b.out_pol_stride = a.out_pol_stride;
    b.row0 = 0;
    b.K = a.K;
    b.K_total = a.K;
    b.n_pol = a.n_pol;
    b.N = LN;
    b.M = LM;
    b.P = LP;
    b.nu = 4;
    b.variant = kBunton;
    b.taps = a.taps;
    b.twN = a.tw;
    b.pad = a.pad;
    b.lcbf_scale = a.scale;
    return launch_lowcbf_stream(b, s);
  }
  static_assert(NT == LN, "one thread per polyphase arm");
  const size_t bytes = ((size_t)LROWS * lds_row(LN) + tw_slots(LN)) * sizeof(float2);
  hipError_t e = set_lds(lowcbf_kernel, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((a.K + LROWS - 1) / LROWS), (unsigned)a.n_pol);
  return launch_kernel(lowcbf_kernel, grid, dim3(NT), bytes, s, a);
}

}  // namespace pfb
