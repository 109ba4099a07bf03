// pfb_analysis.hip — hand-written CDNA4 (gfx950) analysis kernels of the PFB round trip.
//
//   analysis_stream_kernel polyphase_analysis.m:83-121 for the SKA-Low shapes (N = 256):
//                          one thread per output position c streams one column of the
//                          input (rows of N samples) through a register window — the FIR
//                          and the circshift need no LDS staging; T = 16 rows per step
//                          are transformed by an N-point FFT in LDS.
//   analysis_fused_kernel  polyphase_analysis.m:83-121 / polyphase_analysis_padded.m:106-156
//                          for N <= 256: one workgroup = T output rows of one polarisation,
//                          the input span staged in LDS once, the taps of the thread's
//                          polyphase arm in registers, the circular shift applied as the
//                          LDS write address, the N-point FFT in LDS, the last Stockham
//                          pass writing the rows straight to HBM (coalesced).
//   fir_generic_kernel     same maths for N > 256 (SKA-Mid 4096 channels): the FIR writes
//                          the shifted polyphase sums, row_fft_kernel transforms them.
#include "pfb_ana_stream.hpp"

namespace pfb {

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

// Stage x[base, base + S) into LDS (zero outside [0, n_dat)).  Interior tiles issue
// all of their 16-byte loads back to back before the first LDS write.
// pad > 0 (round 6, a padded stream object's carry): series sample g is pre[g] for
// g < pad and x[g - pad] above — the concatenation of FilterBank.m:85-88 without copying it.
template <int CH>
__device__ __forceinline__ void stage_span(float2* smem, const float2* __restrict__ x,
                                           int64_t base, int S, int64_t n_dat, int tid,
                                           const float2* __restrict__ pre = nullptr, int64_t pad = 0) {
  const int S2 = (S + 1) >> 1;
  const int64_t bx = base - pad;  // the span's first sample in x
  const bool interior = bx >= 0 && bx + 2 * (int64_t)S2 <= n_dat &&
                        ((reinterpret_cast<uintptr_t>(x + bx) & 15) == 0);
  if (interior) {
    const float4* __restrict__ src = reinterpret_cast<const float4*>(x + bx);
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
      float2 v = make_float2(0.f, 0.f);
      if (g >= pad) {
        if (g - pad < n_dat) v = x[g - pad];
      } else if (pre != nullptr && g >= 0) {
        v = pre[g];
      }
      smem[s] = v;
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
  const int64_t k0 = a.row0 + (int64_t)xcd_tile(blockIdx.x, gridDim.x) * T;
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
  stage_span<S_::CH>(smem, x, base, S, a.n_dat, tid, a.pre ? a.pre + pol * a.pre_pol_stride : nullptr, a.pad);
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
  if (tid < N) smem[T * S_::RS + tw_slot(tid)] = twv;

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
      // idx = ((nu - (kg mod nu)) (N - M)) mod N = (M kg) mod N, since nu M = de N
      const int idx = (int)((kg * M) & (N - 1));
      pos = (n - idx + N) & (N - 1);
    }
    rows.store(k, pos, u[e]);
  }
  __syncthreads();

  // 5. N-point DFT of every row; Bunton N*fft (forward), padded N^2*ifft (inverse dir.)
  AnalysisStore st{a.out + pol * a.out_pol_stride, a.K, a.K_total, k0, N, a.sds, VARIANT == kPadded,
                   (float)N};
  block_fft<N, (VARIANT == kBunton) ? -1 : +1, T, NT>(rows, st, rows, smem + T * S_::RS, tid);
}

// ----------------------------------------------------------------------- streaming
// (analysis_stream_kernel: pfb_ana_stream.hpp)

template <int VARIANT>
__global__ __launch_bounds__(NT) void fir_generic_kernel(AnalysisArgs a) {
  const int pol = blockIdx.y;
  const int N = a.N, M = a.M, P = a.P;
  const int64_t idx = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (idx >= (a.K - a.row0) * N) return;
  const int64_t kl = idx / N;  // row within the launch
  const int64_t k = a.row0 + kl;
  const int n = (int)(idx - kl * N);
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
  a.scratch[(int64_t)pol * (a.K - a.row0) * N + kl * N + pos] = make_float2(ax, ay);
}

// Generic-N FIR with a per-thread register window (N > 256: SKA-Mid 4096 channels with
// 100 353 taps, polyphase_analysis_padded.m:106-126 / polyphase_analysis.m:83-115).
// With NU M = DE N, output row k + NU reads exactly the input samples of row k shifted
// by DE arms: Bunton x[kM + pN + n] -> p' = p - DE, padded x[kM - 1 - pN - n] -> p' =
// p + DE.  Thread (n, s) walks the rows k = s + NU j of its range with the PW samples of
// arm n in registers and loads only the DE new ones per row (instead of P): the L2 read
// traffic of the FIR drops by P / DE (3.6x on C3).  The circular-shift position of arm
// n depends only on k mod NU (= s), so each thread writes one fixed column.
template <int PW, int DE, int VARIANT, int U = 1>
__global__ __launch_bounds__(NT) void fir_window_kernel(AnalysisArgs a, int ranges, int slice_map) {
  const int N = a.N, M = a.M, NU = a.nu;
  const int chunks = N / NT;
  int bid = blockIdx.x;
  const int d = bid % chunks;
  bid /= chunks;
  const int s = bid % NU;
  const int rg = bid / NU;
  // Residue s reads input columns (s M + n) mod N (Bunton) / (s M - 1 - n) mod N (padded)
  // of every N-sample row: with M a multiple of NT, the NU residues of one column slice d
  // are NU different thread chunks.  The fast block index is the slice d, so all blocks
  // reading slice d share blockIdx mod 8, i.e. one XCD and its L2 (chunk-major order
  // spreads each slice over 4 XCDs: 4.7x the input read from HBM on C3).
  int chunk = d;
  if (slice_map) {
    const int sh = (int)(((int64_t)s * M % N) / NT);
    chunk = VARIANT == kBunton ? (d - sh + chunks) % chunks : ((sh - 1 - d) % chunks + chunks) % chunks;
  }
  const int pol = blockIdx.y;
  const int n = chunk * NT + threadIdx.x;
  // rows of residue s in [row0, K): k = s + NU j, j in [jlo, jhi)
  const int64_t jlo = a.row0 > s ? (a.row0 - s + NU - 1) / NU : 0;
  const int64_t jhi = a.K > s ? (a.K - s + NU - 1) / NU : 0;
  const int64_t nj = jhi - jlo;
  const int64_t j0 = jlo + nj * rg / ranges, j1 = jlo + nj * (rg + 1) / ranges;
  if (j0 >= j1) return;
  float f[PW];
#pragma unroll
  for (int p = 0; p < PW; ++p) f[p] = a.taps[p * N + n];  // zero-padded to 32 N
  const int64_t kfirst = s + (int64_t)NU * j0;
  // descriptor base at the lowest sample the range can touch (offsets stay 32-bit;
  // samples outside [0, n_dat) read as 0 through the range check)
  int64_t b0 = VARIANT == kBunton ? kfirst * M : kfirst * M - 1 - (int64_t)(PW - 1) * N - (N - 1);
  b0 = max(b0, (int64_t)0);
  const float2* xpol = a.in + pol * a.in_pol_stride;
  const int64_t avail = a.n_dat - b0;
  // (launch_fir_window_t sizes the ranges so that one range spans <= kRsrcMaxBytes)
  const __amdgpu_buffer_rsrc_t xr =
      make_rsrc(xpol + b0, (uint32_t)min(max(avail, (int64_t)0) * 8, kRsrcMaxBytes));
  auto ld = [&](int64_t g) {
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(xr, (uint32_t)((g - b0) * 8), 0, 0);
    return __builtin_bit_cast(v2f, v);
  };
  auto gidx = [&](int64_t k, int p) -> int64_t {
    return VARIANT == kBunton ? k * M + (int64_t)p * N + n : k * M - 1 - (int64_t)p * N - n;
  };
  int pos;
  if constexpr (VARIANT == kBunton) {
    pos = (int)((n + ((int64_t)s * M) % N) % N);
  } else {
    const int ix = (s == 0) ? 0 : (int)(((int64_t)(NU - s) * (N - M)) % N);
    pos = (n - ix + N) % N;
  }
  float2* sc = a.scratch + (int64_t)pol * (a.K - a.row0) * N + pos;
  // round trip (a.z): the synthesis stage-1 row of channelised row t is the N-point
  // inverse DFT across channels of row t = the row FFT of these sums, i.e. N^2 times
  // this row (Bunton: same column; padded, whose row FFT is an inverse one: column
  // (-pos) mod N), at the padded variant's circularly shifted row t = (k - sds) mod K
  const int zcol = VARIANT == kBunton ? pos : (N - pos) % N;
  float2* zc = a.z ? a.z + pol * a.z_pol_stride : nullptr;
  const bool zrun = a.zblk == 2;  // Z rows in 2-row runs per column (the SKA-Mid wave synthesis)
  const float zscale = (float)N * (float)N;
  auto emit = [&](int64_t k, v2f acc) {
    if (!zc) sc[(k - a.row0) * N] = make_float2(acc.x, acc.y);
    if (zc) {
      int64_t t = k;
      if constexpr (VARIANT != kBunton) {
        t = k - a.sds;
        while (t < 0) t += a.K_total;
      }
      if (t >= a.z_row0)
        st_nt<kNtFirZ>(zc + z_index(t - a.z_row0, zcol, N, zrun), make_float2(zscale * acc.x, zscale * acc.y));
    }
  };
  if constexpr (U > 1) {
    // U rows per iteration, their U DE new samples loaded together one iteration ahead:
    // a thread waits once per U rows and moves PW + (U-1) DE window registers per U rows
    // instead of PW + DE per row (C3, measured: U = 1 517 us, 2 487 us, 3 540 us — three
    // waves per SIMD at U = 2 and 3 instead of four; a move-free ring window with one or
    // two rows of loads ahead, 491 / 510 us, was no better).  Extended window X[i] = the sample of arm q(i) of row
    // k + (U-1) NU, q = i (padded) / PW-1-i (Bunton); arm p of row k + u NU is
    // X[(U-1-u) DE + q(p)], and the next iteration's window is X shifted by U DE.
    constexpr int XS = PW + (U - 1) * DE;
    v2f X[XS];
#pragma unroll
    for (int i = 0; i < XS; ++i) {
      const int u = i >= (U - 1) * DE ? 0 : U - 1 - i / DE;
      const int q = i - (U - 1 - u) * DE;
      X[i] = ld(gidx(kfirst + (int64_t)u * NU, VARIANT == kBunton ? PW - 1 - q : q));
    }
    vm_drain();  // (no store wait at the loop head)
#pragma unroll 1
    for (int64_t j = j0; j < j1; j += U) {
      const int64_t k = s + (int64_t)NU * j;
      v2f L[U * DE];
#pragma unroll
      for (int i = 0; i < U * DE; ++i) {
        const int u = 2 * U - 1 - i / DE, q = i % DE;
        L[i] = ld(gidx(k + (int64_t)u * NU, VARIANT == kBunton ? PW - 1 - q : q));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // same arm order and pairing as the U = 1 loop (bit-identical sums)
        v2f acc0{0.f, 0.f}, acc1{0.f, 0.f};
#pragma unroll
        for (int p = 0; p < PW; p += 2) {
          const int i0 = (U - 1 - u) * DE + (VARIANT == kBunton ? PW - 1 - p : p);
          acc0 = __builtin_elementwise_fma(v2f{f[p], f[p]}, X[i0], acc0);
          if (p + 1 < PW) {
            const int i1 = (U - 1 - u) * DE + (VARIANT == kBunton ? PW - 2 - p : p + 1);
            acc1 = __builtin_elementwise_fma(v2f{f[p + 1], f[p + 1]}, X[i1], acc1);
          }
        }
        if (j + u < j1) emit(k + (int64_t)u * NU, acc0 + acc1);
      }
#pragma unroll
      for (int i = XS - 1; i >= U * DE; --i) X[i] = X[i - U * DE];
#pragma unroll
      for (int i = 0; i < U * DE; ++i) X[i] = L[i];
    }
    return;
  }
  v2f w[PW];
#pragma unroll
  for (int p = 0; p < PW; ++p) w[p] = ld(gidx(kfirst, p));
  vm_drain();  // (no store wait at the loop head)
#pragma unroll 1
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t k = s + (int64_t)NU * j;
    // next row's DE new samples first, so their latency overlaps this row's MACs
    v2f nw[DE];
#pragma unroll
    for (int i = 0; i < DE; ++i)
      nw[i] = ld(gidx(k + NU, VARIANT == kBunton ? PW - DE + i : i));
    v2f acc0{0.f, 0.f}, acc1{0.f, 0.f};
#pragma unroll
    for (int p = 0; p < PW; p += 2) {
      acc0 = __builtin_elementwise_fma(v2f{f[p], f[p]}, w[p], acc0);
      if (p + 1 < PW) acc1 = __builtin_elementwise_fma(v2f{f[p + 1], f[p + 1]}, w[p + 1], acc1);
    }
    emit(k, acc0 + acc1);
    if constexpr (VARIANT == kBunton) {
#pragma unroll
      for (int p = 0; p < PW - DE; ++p) w[p] = w[p + DE];
#pragma unroll
      for (int i = 0; i < DE; ++i) w[PW - DE + i] = nw[i];
    } else {
#pragma unroll
      for (int p = PW - 1; p >= DE; --p) w[p] = w[p - DE];
#pragma unroll
      for (int i = 0; i < DE; ++i) w[i] = nw[i];
    }
  }
}

// ------------------------------------------------------------- LDS-shared transposed FIR
// Same sums as fir_window_kernel, organised so that the NU residues reading the same
// input columns share one workgroup: thread (cl, s) owns column c = c0 + cl of the input
// viewed as rows of N samples and residue s, i.e. arm n_s(c) (padded (s M - 1 - c) mod N,
// Bunton (c - s M) mod N; both write channel position N - 1 - c / c).  Each input sample
// of the workgroup's CW columns is loaded from HBM ONCE into an LDS ring of x rows and
// read from there by its NU residue threads (fir_window_kernel loads it NU times).
// Row step q (rows k = NU q + s) brings DE new samples per thread; in transposed form
// each new sample is multiplied by every tap it will meet while it slides through the
// window (taps i + j DE, padded; PW - DE + i - j DE, Bunton) into the accumulators of the
// outputs q .. q + NJ - 1, so no sample window is kept or shifted: NJ accumulators, the
// oldest completes every step.  A range starts NJ - 1 steps early (warm-up, no output).
// U steps per barrier, the next U steps' rows loaded into registers one iteration ahead.
template <int NU, int DE>
struct FirLdsShape {
  static constexpr int CW = NT / NU;                       // columns per workgroup
  static constexpr int U = DE >= 7 ? 3 : 4;                // row steps per barrier
  static constexpr int BATCH = U * DE * CW;                // samples staged per iteration
  static constexpr int NPF = (BATCH + NT - 1) / NT;        // prefetch registers per thread
  static constexpr int SPAN = 2 * U * DE + DE + NU + 2;    // live ring rows (bound)
  static constexpr int RR = SPAN <= 32 ? 32 : SPAN <= 64 ? 64 : 128;  // ring rows (pow2)
  static constexpr int MIR = U * DE;                       // mirrored rows past the ring end
  static constexpr int CWP = CW + 1;                       // padded ring row (banks)
};

// PFD: iterations of input rows held in registers ahead of the ring (1; 2 — twice the bytes
// in flight per workgroup — was measured no faster in rounds 1 and 4 and its knob retired)
template <int PW, int DE, int NU, int VARIANT, int PFD = 1>
__global__ __launch_bounds__(NT) void fir_lds_kernel(AnalysisArgs a, int ranges, int cs, int xcd) {
  using SH = FirLdsShape<NU, DE>;
  constexpr int CW = SH::CW, U = SH::U, RR = SH::RR, CWP = SH::CWP, NPF = SH::NPF, MIR = SH::MIR;
  constexpr int NJ = (PW + DE - 1) / DE;  // outputs a sample contributes to
  // ring rows 0 .. MIR - 1 are mirrored at RR .. RR + MIR - 1, so one iteration's U DE
  // consecutive rows are read from a single base with immediate offsets (no wrap masks)
  __shared__ v2f ring[(RR + MIR) * CWP];
  auto ring_put = [&](int64_t rho, int col, v2f v) {
    const int m = (int)(rho & (RR - 1));
    ring[m * CWP + col] = v;
    if (m < MIR) ring[(m + RR) * CWP + col] = v;
  };
  __shared__ int e_ext[2];
  const int N = a.N, M = a.M;
  const int chunks = N / CW;
  // XCD-aware order (xcd != 0): consecutive chunks of a range on one XCD, so the input
  // lines two neighbouring chunks share (the padded round trip's chunks start one column
  // early) are fetched into one L2; else b and b + chunks (same chunk) share an XCD
  const int lt = xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int chunk = lt % chunks, rg = lt / chunks;
  const int pol = blockIdx.y;
  const int tid = threadIdx.x;
  const int cl = tid % CW, s = tid / CW;
  // cs = N - 1 (padded round trip): the chunk's columns start one early, so the Z columns
  // it writes, (c + 1) mod N, are the aligned run c0 .. c0 + CW - 1 (full 128-B lines)
  const int c0 = chunk * CW, c = (c0 + cl + cs) % N;
  const int64_t sM = (int64_t)s * M;
  int n, ar;
  if constexpr (VARIANT == kBunton) {
    n = (int)(((c - sM) % N + N) % N);
    ar = (int)((sM + n - c) / N);
  } else {
    n = (int)(((sM - 1 - c) % N + N) % N);
    ar = (int)((sM - 1 - c - n) / N);
  }
  // newest input row of step q relative to DE q (padded: tap 0; Bunton: tap PW - 1)
  const int e = VARIANT == kBunton ? ar + PW - 1 : ar;
  if (tid == 0) {
    e_ext[0] = INT32_MAX;
    e_ext[1] = INT32_MIN;
  }
  __syncthreads();
  atomicMin(&e_ext[0], e);
  atomicMax(&e_ext[1], e);
  __syncthreads();
  const int e_min = e_ext[0], e_max = e_ext[1];

  // this workgroup's row steps q (rows k = NU q + s in [row0, K)), plus the warm-up
  const int64_t q_lo = a.row0 / NU, q_hi = (a.K + NU - 1) / NU, nq = q_hi - q_lo;
  const int64_t q0 = q_lo + nq * rg / ranges, q1 = q_lo + nq * (rg + 1) / ranges;
  if (q0 >= q1) return;
  const int64_t qw = q0 - (NJ - 1);

  // input descriptor from the lowest row the range touches (samples outside [0, n_dat)
  // read as 0 through the range check; the launcher keeps the extent within a descriptor)
  const float2* xpol = a.in + pol * a.in_pol_stride;
  const int64_t rho_min = (int64_t)DE * qw + e_min - DE;
  const int64_t b0 = max((int64_t)0, rho_min * N);
  const int64_t avail = a.n_dat - b0;
  const __amdgpu_buffer_rsrc_t xr =
      make_rsrc(xpol + b0, (uint32_t)min(max(avail, (int64_t)0) * 8, kRsrcMaxBytes));
  auto ld = [&](int64_t rho, int col) {  // x[rho N + col]
    const int64_t g = rho * N + col;
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(xr, (uint32_t)((g - b0) * 8), 0, kNtlFir ? 2 : 0);
    return __builtin_bit_cast(v2f, v);
  };
  // taps by (new-sample slot i, lag j): padded i + j DE, Bunton PW - DE + i - j DE
  float f[PW];
#pragma unroll
  for (int p = 0; p < PW; ++p) f[p] = a.taps[p * N + n];  // zero-padded to 32 N
  // ring: rows (DE qw + e_min - DE, DE qw + e_max - DE] now; each iteration adds U DE rows
  for (int i = tid; i < (e_max - e_min) * CW; i += NT) {
    const int64_t rho = (int64_t)DE * (qw - 1) + e_min + 1 + i / CW;
    ring_put(rho, i % CW, ld(rho, (c0 + i % CW + cs) % N));
  }
  v2f pf[PFD][NPF];
  auto prefetch = [&](int64_t qi, v2f* d) {  // rows (DE (qi - 1) + e_max, DE (qi - 1) + e_max + U DE]
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int i = min(tid + j * NT, SH::BATCH - 1);
      d[j] = ld((int64_t)DE * (qi - 1) + e_max + 1 + i / CW, (c0 + i % CW + cs) % N);
    }
  };
#pragma unroll
  for (int k = 0; k < PFD; ++k) prefetch(qw + k * U, pf[k]);

  // outputs: Z rows (round trip) or scratch rows at channel position pos
  const int pos = VARIANT == kBunton ? c : N - 1 - c;
  float2* sc = a.scratch + (int64_t)pol * (a.K - a.row0) * N + pos;
  const int zcol = VARIANT == kBunton ? pos : (N - pos) % N;
  float2* zc = a.z ? a.z + pol * a.z_pol_stride : nullptr;
  const bool zrun = a.zblk == 2;  // Z rows in 2-row runs per column (the SKA-Mid wave synthesis)
  const float zscale = (float)N * (float)N;
  auto emit = [&](int64_t k, v2f acc) {
    if (k < a.row0 || k >= a.K) return;
    if (!zc) {
      sc[(k - a.row0) * N] = make_float2(acc.x, acc.y);
    } else {
      int64_t t = k;
      if constexpr (VARIANT != kBunton) {
        t = k - a.sds;
        while (t < 0) t += a.K_total;  // once, unless the series is shorter than sds rows
      }
      if (t >= a.z_row0)
        st_nt<kNtFirZ>(zc + z_index(t - a.z_row0, zcol, N, zrun), make_float2(zscale * acc.x, zscale * acc.y));
    }
  };

  v2f acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = v2f{0.f, 0.f};
  vm_drain();  // (no store wait at the loop head)
#pragma unroll 1
  for (int64_t qi = qw; qi < q1; qi += U) {
    // rows of this iteration -> ring, next iteration's rows -> registers
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      const int i = tid + j * NT;
      if (i < SH::BATCH) {
        const int64_t rho = (int64_t)DE * (qi - 1) + e_max + 1 + i / CW;
        ring_put(rho, i % CW, pf[0][j]);
      }
    }
#pragma unroll
    for (int k = 0; k + 1 < PFD; ++k)
#pragma unroll
      for (int j = 0; j < NPF; ++j) pf[k][j] = pf[k + 1][j];
    prefetch(qi + PFD * U, pf[PFD - 1]);
    __syncthreads();
    // this iteration's rows DE qi + e - DE + 1 + [0, U DE): one base, immediate offsets
    const v2f* rb = ring + (int)(((int64_t)DE * qi + e - DE + 1) & (RR - 1)) * CWP + cl;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = qi + u;
      // the DE new samples of step q: rows DE q + e - DE + 1 + ii (ii = DE - 1 newest)
      v2f xn[DE];
#pragma unroll
      for (int ii = 0; ii < DE; ++ii) xn[ii] = rb[(u * DE + ii) * CWP];
#pragma unroll
      for (int ii = 0; ii < DE; ++ii) {
        // slot i: padded tap p = DE - 1 - ii (row DE q + ar - p), Bunton p = PW - DE + ii
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int p = VARIANT == kBunton ? PW - DE + ii - j * DE : DE - 1 - ii + j * DE;
          if (p >= 0 && p < PW) acc[j] = __builtin_elementwise_fma(v2f{f[p], f[p]}, xn[ii], acc[j]);
        }
      }
      if (q >= q0 && q < q1) emit((int64_t)NU * q + s, acc[0]);
#pragma unroll
      for (int j = 0; j < NJ - 1; ++j) acc[j] = acc[j + 1];
      acc[NJ - 1] = v2f{0.f, 0.f};
    }
  }
}

template <int PW, int DE>
static hipError_t launch_fir_lds_t(const AnalysisArgs& a, hipStream_t s) {
  constexpr int NU = DE == 7 ? 8 : 4;
  using SH = FirLdsShape<NU, DE>;
  const int chunks = a.N / SH::CW;
  const int64_t nq = (a.K + NU - 1) / NU - a.row0 / NU;
  static const int target = [] {
    const char* v = knob("PFB_FIR_LDS_WGS");
    return v ? std::max(1, std::atoi(v)) : 2048;
  }();
  int64_t ranges = std::max<int64_t>(1, std::min<int64_t>(target / chunks, nq / (4 * SH::U)));
  // one range reads rows [DE (q0 - NJ) + e_min - DE, DE q1 + e_max + 2 U DE]: within a descriptor
  const int64_t halo_rows = PW + 3 * DE + 3 * SH::U * DE + 2 * NU + 4;  // (3 U DE: PFD <= 2)
  const int64_t fit_rows = kRsrcMaxBytes / 8 / a.N - halo_rows;
  if (fit_rows <= 0) return hipErrorInvalidValue;
  ranges = std::max(ranges, (nq * DE + fit_rows - 1) / fit_rows);
  if (ranges * chunks > INT32_MAX) return hipErrorInvalidValue;
  dim3 grid((unsigned)(chunks * ranges), (unsigned)a.n_pol);
  // padded round trip: shift the column chunks so the Z stores are line-aligned
  // (PFB_FIR_ZALIGN=0: unshifted, A/B)
  static const bool no_zalign = knob("PFB_FIR_ZALIGN") && std::atoi(knob("PFB_FIR_ZALIGN")) == 0;
  const int cs = (a.variant == kPadded && a.z && !no_zalign) ? a.N - 1 : 0;
  static const int xcd = knob("PFB_FIR_LDS_XCD") ? std::atoi(knob("PFB_FIR_LDS_XCD")) : 1;
  // (launch_kernel: timed by the profiler's armed events like every other single launch)
  if (a.variant == kBunton)
    return launch_kernel(fir_lds_kernel<PW, DE, NU, kBunton>, grid, dim3(NT), 0, s, a, (int)ranges, cs, xcd);
  return launch_kernel(fir_lds_kernel<PW, DE, NU, kPadded>, grid, dim3(NT), 0, s, a, (int)ranges, cs, xcd);
}

template <int PW, int DE>
static hipError_t launch_fir_window_t(const AnalysisArgs& a, hipStream_t s) {
  const int chunks = a.N / NT;
  const int base = chunks * a.nu * a.n_pol;
  static const int target = [] {
    const char* v = knob("PFB_FIR_BLOCKS");
    return v ? std::max(1, std::atoi(v)) : 4 * 1024;
  }();
  static const int rows = [] {
    const char* v = knob("PFB_FIR_ROWS");
    return v ? std::atoi(v) : 2;
  }();
  static const bool no_map = knob("PFB_FIR_NO_SLICE_MAP") != nullptr;
  const int slice_map = !no_map && a.M % NT == 0;
  int ranges = std::max(1, (target + base - 1) / base);
  // one range of residue s reads input samples [k_first M - (PW + 1) N, k_last M + PW N]:
  // keep that within one buffer descriptor (huge single series: more, shorter ranges)
  const int64_t rows_s = (a.K - a.row0 + a.nu - 1) / a.nu + 1;
  const int64_t halo = ((int64_t)PW + 2) * a.N + (int64_t)a.nu * a.M;
  const int64_t fit = kRsrcMaxBytes / 8 - halo;  // samples of row advance one range may span
  if (fit <= 0) return hipErrorInvalidValue;
  const int64_t need = (rows_s * a.nu * a.M + fit - 1) / fit;
  if (need > ranges) {
    if (need * chunks * a.nu > INT32_MAX) return hipErrorInvalidValue;
    ranges = (int)need;
  }
  dim3 grid((unsigned)(chunks * a.nu * ranges), (unsigned)a.n_pol);
  // (launch_kernel already read and cleared the launch error: return its value, a second
  // hipGetLastError() would report a failed launch as hipSuccess)
  auto go = [&](auto u) -> hipError_t {
    // (wide DE: the U DE loads in flight would not fit the register budget)
    constexpr int U = DE * decltype(u)::value <= 21 ? decltype(u)::value : 1;
    if (a.variant == kBunton)
      return launch_kernel(fir_window_kernel<PW, DE, kBunton, U>, grid, dim3(NT), 0, s, a, ranges, slice_map);
    return launch_kernel(fir_window_kernel<PW, DE, kPadded, U>, grid, dim3(NT), 0, s, a, ranges, slice_map);
  };
  if (rows == 1) return go(std::integral_constant<int, 1>{});
  if (rows == 2) return go(std::integral_constant<int, 2>{});
  return go(std::integral_constant<int, 3>{});
}

// register-window FIR if the shape has an instance (window PW >= P, DE | exact M)
template <int DE>
static bool launch_fir_window_de(const AnalysisArgs& a, hipStream_t s, hipError_t* e) {
  if (a.P > 32 || a.P < DE) return false;
  // the LDS-shared form where NU divides the workgroup (8/7, 4/3); PFB_FIR_LDS=0: A/B
  static const bool no_lds = knob("PFB_FIR_LDS") && std::atoi(knob("PFB_FIR_LDS")) == 0;
  if constexpr (DE == 7 || DE == 3) {
    constexpr int NU = DE == 7 ? 8 : 4;
    if (!no_lds && a.nu == NU && a.N % (NT / NU) == 0) {
      if (a.P <= 13) *e = launch_fir_lds_t<13, DE>(a, s);
      else if (a.P <= 16) *e = launch_fir_lds_t<16, DE>(a, s);
      else if (a.P <= 25) *e = launch_fir_lds_t<25, DE>(a, s);
      else *e = launch_fir_lds_t<32, DE>(a, s);
      return true;
    }
  }
  if (a.P <= 13) *e = launch_fir_window_t<13, DE>(a, s);
  else if (a.P <= 16) *e = launch_fir_window_t<16, DE>(a, s);
  else if (a.P <= 25) *e = launch_fir_window_t<25, DE>(a, s);
  else *e = launch_fir_window_t<32, DE>(a, s);
  return true;
}

static bool fir_window_applies(const AnalysisArgs& a) {
  if (a.N % NT != 0 || (int64_t)a.M * a.nu % a.N != 0) return false;
  if (knob("PFB_FIR_NO_WINDOW")) return false;
  const int de = (int)((int64_t)a.M * a.nu / a.N);
  return (de == 7 || de == 3 || de == 27) && a.P <= 32 && a.P >= de;
}

static bool launch_fir_window(const AnalysisArgs& a, hipStream_t s, hipError_t* e) {
  if (!fir_window_applies(a)) return false;
  const int de = (int)((int64_t)a.M * a.nu / a.N);
  if (de == 7) return launch_fir_window_de<7>(a, s, e);
  if (de == 3) return launch_fir_window_de<3>(a, s, e);
  if (de == 27) return launch_fir_window_de<27>(a, s, e);
  return false;
}

template <int N, int PMAX, int VARIANT, int TDIV, bool EXACT = false>
static hipError_t launch_fused(const AnalysisArgs& a, hipStream_t s) {
  using S_ = AnaShape<N, PMAX, TDIV>;
  const size_t span = (size_t)a.M * (S_::T - 1) + (size_t)a.P * N;
  const size_t rows = (size_t)S_::T * S_::RS + tw_slots(N);  // FFT rows + twiddle table
  const size_t bytes = ((span + 1 > rows) ? span + 1 : rows) * sizeof(float2);
  auto kern = analysis_fused_kernel<N, PMAX, VARIANT, TDIV, EXACT>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((a.K - a.row0 + S_::T - 1) / S_::T), (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(NT), bytes, s, a);
}

template <int N, int P, int NU, int DE, bool LCBF = false>
static hipError_t launch_stream(const AnalysisArgs& a, hipStream_t s) {
  using SH = StreamShape<N, P, NU, DE>;
  auto kern = LCBF ? analysis_stream_kernel<N, P, NU, DE, 0, true>
              : a.z ? (a.zblk == 4   ? analysis_stream_kernel<N, P, NU, DE, 4>
                       : a.zblk == 2 ? analysis_stream_kernel<N, P, NU, DE, 2>
                                     : analysis_stream_kernel<N, P, NU, DE, 1>)
              : a.out_rs == 1 && a.sel_n == 0 ? analysis_stream_kernel<N, P, NU, DE, 0, false, 2>
              : a.out_rs > 0                  ? analysis_stream_kernel<N, P, NU, DE, 0, false, 1>
                                              : analysis_stream_kernel<N, P, NU, DE, 0>;
  // channel-major stores go out in row pairs: the launch's rows must start and end even
  if (!LCBF && !a.z && a.out_rs == 1 && a.sel_n == 0 && ((a.row0 & 1) || (a.K & 1))) return hipErrorInvalidValue;
  // the carry (pre) is read only in each workgroup's first WIN-row window prologue: every
  // pad sample must lie inside the first window (the caller checks B <= WIN N)
  if (a.pre && (a.pad < 0 || a.pad > (int64_t)SH::WIN * N)) return hipErrorInvalidValue;
  hipError_t e = set_lds(kern, SH::lds_bytes);
  if (e != hipSuccess) return e;
  const int64_t q_lo = a.row0 / NU;
  const int64_t n_steps = ((a.K + NU - 1) / NU - q_lo + SH::QS - 1) / SH::QS;
  // LDS-limited resident workgroups per CU, each a contiguous range of steps
  // two persistent workgroups per CU (one below the LDS-resident count of 3): longer step
  // ranges amortise each workgroup's start-up window load; measured 4 % faster than 3
  // (PFB_ANA_WG_PER_CU overrides, A/B knob)
  int per_cu = (int)std::max<size_t>(1, std::min<size_t>(2, (160 * 1024) / SH::lds_bytes));
  static const int env_wpc = knob("PFB_ANA_WG_PER_CU") ? std::atoi(knob("PFB_ANA_WG_PER_CU")) : 0;
  if (env_wpc > 0) per_cu = env_wpc;
  const int64_t per_pol = std::max<int64_t>(1, (per_cu * cu_count()) / a.n_pol);
  int64_t wgs = std::min<int64_t>(n_steps, per_pol);
  // a workgroup's rows (its steps' NEW rows each + the WIN-row window) must fit one
  // buffer descriptor: huge single series get more, shorter ranges
  const int64_t fit_steps = (kRsrcMaxBytes / (8 * N) - SH::WIN) / SH::NEW;
  wgs = std::max(wgs, (n_steps + fit_steps - 1) / fit_steps);
  // (PFB_ANA_STEPS=S: S steps per workgroup, ceil(n_steps / S) workgroups instead of the
  // resident count; PFB_ANA_LINEAR=1: linear workgroup order — experiments A/B)
  AnalysisArgs b = a;
  if constexpr (kExperiments) {
    static const int steps = knob("PFB_ANA_STEPS") ? std::atoi(knob("PFB_ANA_STEPS")) : 0;
    static const int lin = knob("PFB_ANA_LINEAR") ? std::atoi(knob("PFB_ANA_LINEAR")) : -1;
    if (steps > 0) wgs = std::max(wgs, (n_steps + steps - 1) / steps);
    if (lin >= 0) b.linear = lin;
  }
  if constexpr (kExperiments && !LCBF) {
    // (PFB_ANA_WPE=3: the round trip's 2-row-run kernel at 3 waves per SIMD, 3 workgroups
    // per CU unless PFB_ANA_WG_PER_CU says otherwise — experiments A/B)
    static const int wpe = knob("PFB_ANA_WPE") ? std::atoi(knob("PFB_ANA_WPE")) : 0;
    // (PFB_ANA_TV=1..7: the timing variants of the round trip's kernel, results invalid; 8: the
    // FFT with workgroup barriers, the pre-round-6 kernel)
    static const int tv = knob("PFB_ANA_TV") ? std::atoi(knob("PFB_ANA_TV")) : 0;
    if (a.z && a.zblk == 2 && (tv == 8 || tv == 16)) {
      kern = tv == 8 ? analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 8>
                     : analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 16>;
      e = set_lds(kern, SH::lds_bytes);
      if (e != hipSuccess) return e;
    }
    if (a.z && a.zblk == 2 && tv > 0 && tv < 8) {
      switch (tv) {
        case 1: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 1>; break;
        case 2: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 2>; break;
        case 3: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 3>; break;
        case 4: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 4>; break;
        case 5: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 5>; break;
        case 6: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 6>; break;
        default: kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 2, 7>; break;
      }
      e = set_lds(kern, SH::lds_bytes);
      if (e != hipSuccess) return e;
    }
    if (wpe == 3 && a.z && a.zblk == 2) {
      kern = analysis_stream_kernel<N, P, NU, DE, 2, false, 0, 3>;
      e = set_lds(kern, SH::lds_bytes);
      if (e != hipSuccess) return e;
      if (env_wpc <= 0) {
        const int64_t pp = std::max<int64_t>(1, (3 * cu_count()) / a.n_pol);
        wgs = std::max(std::min<int64_t>(n_steps, pp), (n_steps + fit_steps - 1) / fit_steps);
      }
    }
  }
  if (wgs > INT32_MAX) return hipErrorInvalidValue;
  dim3 grid((unsigned)wgs, (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(NT), SH::lds_bytes, s, b);
}

// streaming kernel for the SKA-Low shapes (N = 256, Bunton); 0 = not compiled
static bool stream_shape(const AnalysisArgs& a) {
  if (a.variant != kBunton || a.N != 256) return false;
  if (a.nu == 8 && a.M == 224) return a.P == 13 || a.P == 12;
  if (a.nu == 4 && a.M == 192) return a.P == 13 || a.P == 12;
  return false;
}

static hipError_t launch_stream_any(const AnalysisArgs& a, hipStream_t s) {
  if (a.nu == 8) return a.P == 13 ? launch_stream<256, 13, 8, 7>(a, s) : launch_stream<256, 12, 8, 7>(a, s);
  return a.P == 13 ? launch_stream<256, 13, 4, 3>(a, s) : launch_stream<256, 12, 4, 3>(a, s);
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

hipError_t launch_lowcbf_stream(const AnalysisArgs& a, hipStream_t s) {
  if (a.N != 256 || a.M != 192 || a.P != 12 || a.nu != 4) return hipErrorInvalidValue;
  return launch_stream<256, 12, 4, 3, true>(a, s);
}

bool analysis_supported(int N, int P, int variant, bool* fused) {
  (void)variant;
  const bool f = (N >= 8 && N <= 256 && pow2_supported(N) && P <= 32);
  if (fused) *fused = f;
  return pow2_supported(N);
}

bool analysis_can_emit_z(const AnalysisArgs& a) {
  if (stream_shape(a) && knob("PFB_ANALYSIS_NO_STREAM") == nullptr) return true;
  bool fused = false;
  return analysis_supported(a.N, a.P, a.variant, &fused) && !fused && fir_window_applies(a);
}

bool analysis_can_emit_zblk(const AnalysisArgs& a) {
  return stream_shape(a) && knob("PFB_ANALYSIS_NO_STREAM") == nullptr && StreamShape<256, 13, 8, 7>::T == 16;
}

// the fused (one-launch FIR + FFT) kernel handles the shape: it stages its rows' input span
// through stage_span, which reads a stream carry from `pre`
bool analysis_fused_takes_carry(const AnalysisArgs& a) {
  bool fused = false;
  return analysis_supported(a.N, a.P, a.variant, &fused) && fused && !stream_shape(a) && a.variant != kLowCbf &&
         knob("PFB_FUSED_NO_CARRY") == nullptr;
}

bool analysis_takes_offset(const AnalysisArgs& a) {
  return stream_shape(a) && knob("PFB_ANALYSIS_NO_STREAM") == nullptr;
}

hipError_t launch_analysis(const AnalysisArgs& a, hipStream_t s) {
  if (a.K <= a.row0) return hipSuccess;
  // (a read offset: the streaming kernel, or — with the carried samples in `pre` — the fused
  // kernel, whose span staging reads them, analysis_fused_takes_carry)
  if (a.pad != 0 && !analysis_takes_offset(a) && !(a.pre != nullptr && analysis_fused_takes_carry(a)))
    return hipErrorInvalidValue;
  if (a.z && !analysis_can_emit_z(a)) return hipErrorInvalidValue;
  bool fused = false;
  if (!analysis_supported(a.N, a.P, a.variant, &fused)) return hipErrorInvalidValue;
  // stage-1 rows in runs: the streaming kernel's 2/4/16-row runs (N = 256), or the 2-row
  // runs of the generic path's FIR (fir_lds / fir_window) for the SKA-Mid wave synthesis
  if (a.z && a.zblk > 1) {
    const bool stream_ok = analysis_can_emit_zblk(a) && ((a.row0 - a.z_row0) % 16) == 0 &&
                           (a.zblk == 2 || a.zblk == 4);
    const bool generic_ok = !fused && a.zblk == 2 && a.z_row0 == 0 && fir_window_applies(a);
    if (!stream_ok && !generic_ok) return hipErrorInvalidValue;
  }
  static const bool no_stream = knob("PFB_ANALYSIS_NO_STREAM") != nullptr;
  if (fused && stream_shape(a) && !no_stream) {
    static const int mask = knob("PFB_ANA_MASK") ? std::atoi(knob("PFB_ANA_MASK")) : 0;
    AnalysisArgs b = a;
    b.timing_mask = mask;
    return launch_stream_any(b, s);
  }
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
  if (!a.scratch && !a.z) return hipErrorInvalidValue;
  if (a.z_stage != 0 && !a.z) return hipErrorInvalidValue;
  // generic: FIR into scratch, then row FFT (with the padded circular time shift)
  const int64_t rows = a.K - a.row0;
  const int64_t total = rows * a.N;
  hipError_t e = hipSuccess;
  if (a.z_stage == 2) {
    // (the FIR half ran before, into the same Z)
  } else if (!launch_fir_window(a, s, &e)) {
    dim3 grid((unsigned)((total + NT - 1) / NT), (unsigned)a.n_pol);
    if (a.variant == kBunton) hipLaunchKernelGGL(fir_generic_kernel<kBunton>, grid, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL(fir_generic_kernel<kPadded>, grid, dim3(NT), 0, s, a);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  if (a.z && a.z_stage == 1) return hipSuccess;
  if (a.z) {
    // round trip: the channelised rows come from the Z rows (already in output-row order,
    // N^2 x the FIR sums, index-reversed for the padded variant): the same row FFT on
    // the same values scaled by 2^k, so the result is bit-identical to the scratch path
    // (z_stage 2 on rows [row0, K): Z rows are output rows, so both sides start at row0)
    if ((a.row0 != 0 && a.z_stage != 2) || a.z_row0 != 0 || (a.variant == kPadded && !a.zrev))
      return hipErrorInvalidValue;
    // (2-row runs: row0 of the row FFT is even — the round trip runs it from row 0 — so the
    // run of row0 starts at element row0 N)
    if (a.zblk == 2 && (a.row0 & 1)) return hipErrorInvalidValue;
    RowFftArgs rz{a.z + a.row0 * a.N, a.z_pol_stride, a.out + a.row0 * a.N, a.out_pol_stride, rows, a.zrev,
                  nullptr, a.twN, 1.0f / (float)a.N, 0, 0, 0, a.K_total};
    rz.in_run = a.zblk == 2 ? 1 : 0;
    rz.rev = a.zrev != nullptr ? 1 : 0;  // (zrev is always the index reversal, pfb_api.hip)
    if (a.variant == kBunton) return dispatch_row_fft<-1>(a.N, rz, a.n_pol, s);
    return dispatch_row_fft<+1>(a.N, rz, a.n_pol, s);
  }
  RowFftArgs r{a.scratch, rows * a.N, a.out, a.out_pol_stride, rows, nullptr, nullptr, a.twN,
               (float)a.N, a.sds, a.variant == kPadded, a.row0, a.K_total};
  if (a.variant == kBunton) return dispatch_row_fft<-1>(a.N, r, a.n_pol, s);
  return dispatch_row_fft<+1>(a.N, r, a.n_pol, s);
}

}  // namespace pfb
