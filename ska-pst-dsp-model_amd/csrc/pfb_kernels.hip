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
#include "pfb_pair.hpp"

#include <algorithm>
#include <cstdlib>

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
// Synthesis block kernel (polyphase_synthesis.m:163-316, re-ordered).
// Workgroup (tg, b) owns the TG = 2 * PAIRS output phases t0 .. t0+TG-1 of block b of
// one polarisation.  Each thread carries the same element of TWO phases in packed
// FP32 lanes (pfb_pair.hpp), pair rows fastest across lanes, so
//   * the first Nf-point pass reads Z straight from HBM (16-byte loads, PAIRS*16-byte
//     runs per time row) and applies the temporal taper on the way in;
//   * the last Nf-point pass keeps the W bins (fftshift + discard), multiplies by the
//     deripple gain x four-step twiddle and stores the W-point rows;
//   * the last W-point pass writes the kept output samples straight to HBM through a
//     range-checked buffer descriptor (overlap-discard and the output limit cost no
//     VALU: out-of-range stores are dropped by the hardware).
// LDS round trips per block: 2 with a fused plan (below), else 3.
constexpr int NTP = 128;  // threads per synthesis workgroup

template <int NF, int W, int PAIRS>
struct SynthPairShape {
  // pair-row strides (16-byte slots): N + 7 minimises ds_read/write_b128 bank
  // conflicts of the radix-16 passes (scripts/lds_bank_sim.py)
  static constexpr int RSF = NF + 7;
  static constexpr int RSW = W + 7;
  static constexpr int RSMAX = RSF > RSW ? RSF : RSW;
  static constexpr int TWOFF = PAIRS * RSMAX * 2;  // float2 offset of the twiddle tables
  static constexpr size_t lds_bytes = (size_t)(TWOFF + NF + W) * sizeof(float2) + NF * sizeof(float);
};

template <int NF, int W, bool SPANS>
__device__ __forceinline__ int kept_slot(int f) {
  // slot j' of Nf-point FFT bin f, or -1 if the bin is discarded (:188, :240, :265-278)
  if constexpr (SPANS) {
    if (f < W / 2) return f;
    if (f >= NF - W / 2) return f - (NF - W);
    return -1;
  } else {
    if (f >= NF - W / 2) return f - (NF - W / 2);
    if (f < W / 2) return f + W / 2;
    return -1;
  }
}

// first Nf-point pass input: Z[tau][t0 + 2q .. +1] x taper[tau]
template <int NB>
struct PairZIn {
  static constexpr bool kIsLds = false;
  __amdgpu_buffer_rsrc_t z;  // block base + t0
  int N;
  const float* win;
  template <class P, class RR>
  __device__ __forceinline__ cpx2 load(int q, int tau, P, RR) const {
    const int j = tau - RR::value * NB;  // thread part (folds with the caller's j)
    const v4u x = __builtin_amdgcn_raw_buffer_load_b128(z, (j * N + 2 * q) * 8, RR::value * NB * N * 8, 0);
    return cscale(from_interleaved(__builtin_bit_cast(v4f, x)), win[tau]);
  }
};

// first Nf-point pass input from prefetched registers
template <int PER, int R>
struct PairRegsIn {
  static constexpr bool kIsLds = false;
  const cpx2 (&zv)[PER][R];
  const float* win;
  template <class P, class RR>
  __device__ __forceinline__ cpx2 load(int, int tau, P, RR) const {
    return cscale(zv[P::value][RR::value], win[tau]);
  }
};

// last Nf-point pass output: keep W bins, x deripple gain x four-step twiddle (from the
// [j'][t0] table, L2-resident; the loads are unconditional so they issue back to back)
template <int NF, int W, bool SPANS>
struct PairSelect {
  static constexpr bool kIsLds = true;
  LdsPairs rows;
  __amdgpu_buffer_rsrc_t tw4;  // table + t0
  int N;
  template <class P, class RR>
  __device__ __forceinline__ void store(int q, int f, cpx2 v, P p, RR r) const {
    const int jp = kept_slot<NF, W, SPANS>(f);
    const v4u x = __builtin_amdgcn_raw_buffer_load_b128(tw4, (max(jp, 0) * N + 2 * q) * 8, 0, 0);
    if (jp >= 0) rows.store(q, jp, cmul(v, from_interleaved(__builtin_bit_cast(v4f, x))), p, r);
  }
};

struct PairOut {
  static constexpr bool kIsLds = false;
  // o: first kept output sample of the block, records = kept samples in bytes;
  // o1: the same shifted by one sample (the odd phase of each pair).  Separate
  // descriptors keep the two 8-byte stores from being merged into one 16-byte store,
  // so each sample is range-checked on its own (the output limit may split a pair).
  __amdgpu_buffer_rsrc_t o, o1;
  int N, t1_lo, t0;
  float scale;
  template <class P, class RR>
  __device__ __forceinline__ void store(int q, int t1, cpx2 v, P, RR) const {
    // negative offsets (t1 < t1_lo) wrap past 2^31 bytes and are dropped by the range check
    const int off = ((t1 - t1_lo) * N + t0 + 2 * q) * 8;
    const Interleaved y = to_interleaved(cscale(v, scale));
    __builtin_amdgcn_raw_buffer_store_b64(as_u(y.lo), o, off, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(as_u(y.hi), o1, off, 0, 0);
  }
};

// Transform plans of the synthesis block.  When the last Nf-point pass has NBL
// butterflies per row with NBL | W/2, the W bins a thread keeps after that pass are
// exactly j + NBL * r'' (r'' < W / NBL), i.e. the inputs of one radix-(W/NBL) butterfly
// of a W-point transform whose first pass has stride NBL: the kept-bin selection, the
// gain x twiddle AND the first W-point pass then run in registers, saving one LDS round
// trip and one barrier ("fused" plans).  Other sizes use the generic 3-exchange path.
template <int NF, int W>
struct SynthPlan {
  static constexpr bool fused = false;
};
template <int R1_, class Mid_, int RL_, class Wrest_>
struct FusedPlan {
  static constexpr bool fused = true;
  static constexpr int R1 = R1_;  // first Nf pass (loads from HBM)
  using Mid = Mid_;                // Nf passes between the first and the last
  static constexpr int RL = RL_;   // last Nf pass (fused with the selection)
  using Wrest = Wrest_;            // W passes after the fused one
};
template <> struct SynthPlan<256, 224> : FusedPlan<16, Radices<>, 16, Radices<16>> {};
template <> struct SynthPlan<256, 192> : FusedPlan<16, Radices<>, 16, Radices<16>> {};
template <> struct SynthPlan<128, 112> : FusedPlan<8, Radices<>, 16, Radices<8>> {};
template <> struct SynthPlan<128, 96> : FusedPlan<8, Radices<>, 16, Radices<8>> {};
template <> struct SynthPlan<512, 448> : FusedPlan<8, Radices<4>, 16, Radices<8, 4>> {};
template <> struct SynthPlan<1024, 896> : FusedPlan<16, Radices<4>, 16, Radices<8, 8>> {};

template <int NF, int W>
constexpr int synth_first_radix() {
  if constexpr (SynthPlan<NF, W>::fused) return SynthPlan<NF, W>::R1;
  else return FirstPassOf<NF, 1, 1>::R;
}

// Register slot r'' of the fused pass <- output register r of the last Nf pass.
template <int NF, int W, int NBL, bool SPANS>
constexpr int fused_src(int rr) {
  constexpr int H = W / (2 * NBL);  // slots per half band
  if constexpr (SPANS) return rr < H ? rr : rr + (NF - W) / NBL;
  else return rr < H ? rr + (NF - W / 2) / NBL : rr - H;
}

// gain x four-step twiddle of the fused pass inputs: slot r'' of pair row q, butterfly j
// is bin j' = j + NBL r'' ([j'][t0] table, 16-byte loads, all unconditional)
template <int NBL, int RW1, int PAIRS, int NTH>
__device__ __forceinline__ void load_t4(cpx2 (&t4)[(PAIRS * NBL + NTH - 1) / NTH][RW1],
                                        __amdgpu_buffer_rsrc_t tr, int N, int tid) {
  constexpr int TOT = PAIRS * NBL;
  static_for<0, (TOT + NTH - 1) / NTH>([&](auto p) {
    const int b = min(tid + p * NTH, TOT - 1);
    const int q = b % PAIRS, j = b / PAIRS;
    static_for<0, RW1>([&](auto rr) {
      const v4u x = __builtin_amdgcn_raw_buffer_load_b128(tr, ((j + NBL * rr) * N + 2 * q) * 8, 0, 0);
      t4[p][rr] = from_interleaved(__builtin_bit_cast(v4f, x));
    });
  });
}

// Last Nf-point pass (forward, radix RL, NS = NBL) + kept-bin selection + gain x
// twiddle + first W-point pass (inverse, radix RW1, NS = 1), LDS rowsF -> LDS rowsW
// (in place; one barrier between the loads and the stores).
template <int NF, int W, int RL, bool SPANS, int PAIRS, int NTH>
__device__ __forceinline__ void fused_select_pass(const LdsPairs& rowsF, const LdsPairs& rowsW,
                                                  const float2* __restrict__ twF,
                                                  const cpx2 (&t4)[(PAIRS * (NF / RL) + NTH - 1) / NTH]
                                                                  [W / (NF / RL)],
                                                  int tid) {
  constexpr int NBL = NF / RL;
  constexpr int RW1 = W / NBL;
  static_assert(NBL * RW1 == W && (W / 2) % NBL == 0, "plan is not fusable");
  constexpr int TOT = PAIRS * NBL;
  constexpr int PER = (TOT + NTH - 1) / NTH;
  cpx2 v[PER][RL];
  static_for<0, PER>([&](auto p) {
    const int b = tid + p * NTH;
    if (TOT % NTH == 0 || b < TOT) {
      const int q = b % PAIRS, j = b / PAIRS;
      static_for<0, RL>([&](auto r) { v[p][r] = rowsF.load(q, j + r * NBL, p, r); });
    }
  });
  __syncthreads();
  static_for<0, PER>([&](auto p) {
    const int b = tid + p * NTH;
    if (TOT % NTH == 0 || b < TOT) {
      const int q = b % PAIRS, j = b / PAIRS;
      static_for<1, RL>([&](auto r) { v[p][r] = cmul(v[p][r], table_tw<-1>(twF, r * j)); });
      sdft<RL, -1>(v[p]);
      cpx2 u[RW1];
      static_for<0, RW1>([&](auto rr) {
        constexpr int r = fused_src<NF, W, NBL, SPANS>(decltype(rr)::value);
        u[rr] = cmul(v[p][r], t4[p][rr]);
      });
      sdft<RW1, +1>(u);
      static_for<0, RW1>([&](auto rr) { rowsW.store(q, j * RW1 + rr, u[rr], p, rr); });
    }
  });
}

// PERSIST: workgroup (tg, rr) walks a range of blocks and prefetches the next one's
// first-pass inputs into registers while it transforms the current one.
template <int NF, int W, int PAIRS, bool SPANS, bool PERSIST>
__global__ __launch_bounds__(NTP) void synth_block_kernel(SynthBlockArgs a) {
  using SS = SynthPairShape<NF, W, PAIRS>;
  using SP = SynthPlan<NF, W>;
  constexpr int R1 = synth_first_radix<NF, W>();
  constexpr int NB1 = NF / R1;
  constexpr int TG = 2 * PAIRS;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int tid = threadIdx.x;
  const int N = a.N;
  const int groups = N / TG;
  const int tg = blockIdx.x % groups;
  const int rr = blockIdx.x / groups;
  const int Rg = gridDim.x / groups;
  // PERSIST: a contiguous range of blocks per workgroup.  (Strided assignment rr + k Rg
  // keeps the 2 Ov overlap rows in L2, -30 % HBM reads, but measured 10 % slower.)
  const int b_begin = PERSIST ? (int)((int64_t)a.n_blocks * rr / Rg) : rr;
  const int b_end = PERSIST ? (int)((int64_t)a.n_blocks * (rr + 1) / Rg) : rr + 1;
  const int b_step = 1;
  if (b_begin >= b_end) return;
  const int t0 = tg * TG;
  const int pol = blockIdx.y;

  float2* twF = smem + SS::TWOFF;  // Nf twiddles, then W twiddles, then the taper
  float2* twWl = twF + NF;
  float* win = reinterpret_cast<float*>(twWl + W);
  for (int j = tid; j < NF + W; j += NTP) twF[j] = (j < NF) ? a.twNf[j] : a.twW[j - NF];
  for (int j = tid; j < NF; j += NTP) win[j] = a.window[j];

  const float2* zpol = a.Z + pol * a.z_pol_stride + t0;
  const uint32_t zbytes = (a.timing_mask & 1) ? 0u : (uint32_t)((NF - 1) * N + TG) * 8u;
  const uint32_t twbytes = (a.timing_mask & 4) ? 0u : (uint32_t)((W - 1) * N + TG) * 8u;
  const __amdgpu_buffer_rsrc_t tw4r = make_rsrc(a.tw4 + t0, twbytes);
  const LdsPairs rowsF{reinterpret_cast<v4f*>(smem), SS::RSF};
  const LdsPairs rowsW{reinterpret_cast<v4f*>(smem), SS::RSW};
  float2* opol = a.out + pol * a.out_pol_stride;
  auto out_for = [&](int b) {
    // overlap-discard (:302) and 1/L * de/nu (:285) on the store
    const int64_t ob = (a.block0 + b) * (int64_t)a.Lkeep;  // first kept output sample
    const int64_t avail = a.out_limit - ob;
    const int64_t nk =
        (a.timing_mask & 2) ? 0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
    return PairOut{make_rsrc(opol + ob, (uint32_t)nk * 8u),
                   make_rsrc(opol + ob + 1, (uint32_t)max((int64_t)0, nk - 1) * 8u), N, a.t1_lo, t0,
                   a.scale};
  };

  if constexpr (!SP::fused) {
    // generic: Nf FFT (taper in, select + gain x twiddle out), W FFT, 3 LDS exchanges
    static_assert(!PERSIST, "persistent variant needs a fused plan");
    __syncthreads();  // tables
    const int b = b_begin;
    const PairZIn<NB1> in{make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes), N, win};
    const PairSelect<NF, W, SPANS> sel{rowsW, tw4r, N};
    block_fft_pair<NF, -1, PAIRS, NTP>(in, sel, rowsF, twF, tid);
    __syncthreads();
    block_fft_pair<W, +1, PAIRS, NTP>(rowsW, out_for(b), rowsW, twWl, tid);
  } else {
    constexpr int NBL = NF / SP::RL;
    constexpr int RW1 = W / NBL;
    constexpr int PT = (PAIRS * NBL + NTP - 1) / NTP;
    // Nf passes 1 .. last-1 (the first from `in`), then the fused pass, then W passes 2..
    auto run_block = [&](const auto& in, int b, auto after_first) {
      stockham_pass_pair<NF, R1, 1, -1, PAIRS, NTP>(in, rowsF, twF, tid);
      after_first();
      cpx2 t4[PT][RW1];
      load_t4<NBL, RW1, PAIRS, NTP>(t4, tw4r, N, tid);
      __syncthreads();
      if constexpr (!std::is_same_v<typename SP::Mid, Radices<>>) {
        run_fft_mid<NF, -1, PAIRS, NTP, R1>(rowsF, twF, tid, typename SP::Mid{});
        __syncthreads();
      }
      fused_select_pass<NF, W, SP::RL, SPANS, PAIRS, NTP>(rowsF, rowsW, twF, t4, tid);
      __syncthreads();
      run_fft_tail<W, +1, PAIRS, NTP, RW1>(rowsW, out_for(b), twWl, tid, typename SP::Wrest{});
    };
    if constexpr (!PERSIST) {
      __syncthreads();  // tables
      const int b = b_begin;
      const PairZIn<NB1> in{make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes), N, win};
      run_block(in, b, [] {});
    } else {
      constexpr int PF = (PAIRS * NB1 + NTP - 1) / NTP;
      cpx2 zv[PF][R1];
      auto prefetch = [&](int b) {
        const __amdgpu_buffer_rsrc_t z = make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes);
        static_for<0, PF>([&](auto p) {
          const int bb = min(tid + p * NTP, PAIRS * NB1 - 1);
          const int q = bb % PAIRS, j = bb / PAIRS;
          static_for<0, R1>([&](auto r) {
            const v4u x = __builtin_amdgcn_raw_buffer_load_b128(z, (j * N + 2 * q) * 8, r * NB1 * N * 8, 0);
            zv[p][r] = from_interleaved(__builtin_bit_cast(v4f, x));
          });
        });
      };
      prefetch(b_begin);
      const PairRegsIn<PF, R1> in{zv, win};
#pragma unroll 1
      for (int b = b_begin; b < b_end; b += b_step) {
        __syncthreads();  // tables / previous block's W transform done with the rows
        run_block(in, b, [&] {
          if (b + b_step < b_end) prefetch(b + b_step);
        });
      }
    }
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

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
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
  if (a.P == 13) return launch_fused<N, 13, VARIANT, 1, true>(a, s);
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

template <int NF, int W, int PAIRS, bool SPANS>
static hipError_t launch_sb(const SynthBlockArgs& a, hipStream_t s) {
  using SS = SynthPairShape<NF, W, PAIRS>;
  const int groups = a.N / (2 * PAIRS);
  if (a.ranges != 0 && SynthPlan<NF, W>::fused) {
    // persistent: block ranges so that ~LDS-limited workgroups per CU are resident
    auto kern = synth_block_kernel<NF, W, PAIRS, SPANS, SynthPlan<NF, W>::fused>;
    hipError_t e = set_lds(kern, SS::lds_bytes);
    if (e != hipSuccess) return e;
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / SS::lds_bytes));
    int ranges = a.ranges > 0 ? a.ranges : std::max(1, cu_count() * per_cu / (groups * a.n_pol));
    ranges = std::min(ranges, a.n_blocks);
    dim3 grid((unsigned)(groups * ranges), (unsigned)a.n_pol);
    hipLaunchKernelGGL(kern, grid, dim3(NTP), SS::lds_bytes, s, a);
    return hipGetLastError();
  }
  auto kern = synth_block_kernel<NF, W, PAIRS, SPANS, false>;
  hipError_t e = set_lds(kern, SS::lds_bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)(groups * a.n_blocks), (unsigned)a.n_pol);
  hipLaunchKernelGGL(kern, grid, dim3(NTP), SS::lds_bytes, s, a);
  return hipGetLastError();
}

// pair rows per workgroup: enough for every thread to own one first-pass butterfly,
// fewer when the channel count is small (2 * PAIRS must divide N)
template <int NF, int W, bool SPANS>
static hipError_t launch_sb_p(const SynthBlockArgs& a, hipStream_t s) {
  constexpr int POPT = NTP / (NF / synth_first_radix<NF, W>());
  static_assert(POPT >= 1, "first pass wider than the workgroup");
  if (a.N % (2 * POPT) == 0) return launch_sb<NF, W, POPT, SPANS>(a, s);
  if (a.N % 2 == 0) return launch_sb<NF, W, 1, SPANS>(a, s);
  return hipErrorInvalidValue;
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
  if (a.Nf == a_ && a.W == b_)  \
    return a.spans ? launch_sb_p<a_, b_, true>(a, s) : launch_sb_p<a_, b_, false>(a, s);
  PFB_SYNTH_SIZES(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace pfb
