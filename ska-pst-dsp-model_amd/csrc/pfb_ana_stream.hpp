// pfb_ana_stream.hpp — the streaming Bunton analysis for N = 256 (polyphase_analysis.m:83-121),
// analysis_stream_kernel (instantiated in pfb_analysis.hip).
#pragma once
#include "pfb_common.hpp"

namespace pfb {


// Bunton analysis for N = 256 with the FIR in registers and no LDS staging of the
// input.  View the input as rows of N samples, X[r][c] = x[r N + c].  With M = N DE/NU,
// output row k = NU q + s (s < NU) starts at kM = DE N q + sM, and the circular shift
// of polyphase_analysis.m:102-105 moves arm n to position (n + sM) mod N.  The thread
// that owns position c therefore computes, for every s, arm n_s = (c - a_s) mod N with
// a_s = sM mod N, and its samples are one COLUMN of X:
//     v_k[c] = sum_m f[m N + n_s] X[DE q + m + b_s + e_s][c],
//     b_s = floor(sM / N), e_s = [c < a_s].
// Folding e_s into the taps (g_s[m'] = f[(m' - e_s) N + n_s] = F[(m' + 1) N + c - a_s]
// with F = [N zeros, f, zeros], P + 1 taps) makes the row index DE q + m' + b_s a
// compile-time offset into a register window that slides down the column: each input
// sample is loaded once, coalesced (a wave reads 512 contiguous bytes of one row), and
// the circshift costs nothing — v_k[c] is already at its shifted position.  The taps
// are read from LDS (lane-contiguous, conflict-free; each read feeds QS rows);
// T = 16 rows per step go to LDS for the N-point FFT.
template <int N, int P, int NU, int DE>
struct StreamShape {
  static_assert(N == NT, "one thread per column");
  static_assert(16 % NU == 0, "NU must divide 16");
  static constexpr int M = N * DE / NU;
  static_assert(M * NU == N * DE, "M = N de/nu must be integral");
  static constexpr int PE = P + 1;        // taps per chain after folding e_s
  static constexpr int QS = 16 / NU;      // commutator periods per step
  static constexpr int T = QS * NU;       // output rows per step (16)
  static constexpr int NEW = DE * QS;     // input rows consumed per step
  static constexpr int WIN = NEW + PE - 1;  // register window (rows)
  static constexpr int RS = lds_row(N);
  static constexpr int TW_OFF = T * RS;               // float2 offset of the twiddles
  static constexpr int F_OFF = 2 * (TW_OFF + tw_slots(N));  // float offset of the taps F
  static constexpr int F_LEN = (P + 2) * N;
  static constexpr size_t lds_bytes = (size_t)F_OFF * sizeof(float) + F_LEN * sizeof(float);
};

// ZOUT (round trip): each step's channelised rows are also inverse-transformed across
// channels in LDS and written as synthesis stage-1 rows (AnalysisArgs::z), so the
// synthesis does not re-read them from HBM.
// LCBF: the SKA-Low CBF PST filterbank (polyphase_analysis_lowcbf.m / PSTFilterbank.m,
// N 256, M 192, 12 taps) through the same FIR: its FFT of the UNshifted sums times the
// derotation i^{k (j - 128)} equals the FFT of the Bunton-shifted sums v_k (the shift
// r = 192 k mod 256 is a multiple of 64, e^{-2 pi i f r / 256} = i^{k f}, exact), and
// fftshift + the 216-channel selection is output channel c = (f - 148) mod 256 < 216,
// scaled by 2^12 (LowCbfArgs::scale).  Leading pre-padding zeros via AnalysisArgs::pad.
// The last FFT pass's output staged channel-major in the LDS rows' space (channel c at
// c * (T + 1), odd stride: conflict-light column writes and row-pair reads) for the
// channel-major store of a strided launch (out_rs = 1).
template <int T>
struct ColMajorLds {
  static constexpr bool kIsLds = true;
  float2* b;
  __device__ __forceinline__ void store(int row, int c, float2 v) const { b[c * (T + 1) + row] = v; }
  __device__ __forceinline__ float2 load(int row, int c) const { return b[c * (T + 1) + row]; }
};

// timing variant TV 16: a store functor that only keeps the value live (no instruction)
struct SinkStore {
  static constexpr bool kIsLds = false;
  __device__ __forceinline__ void store(int, int, float2 v) const { asm volatile("" ::"v"(v)); }
};

// ZOUT: 0 no stage-1 rows; 1 rows [row][c] (AnalysisArgs::z); 2 / 4: runs of ZOUT rows per
// column (AnalysisArgs::zblk) for the synthesis wave kernel.
// Streaming analysis of step range w of nw (steps of T rows from row0) for polarisation
// pol.
// TV: compile-time timing variants (experiments build only, results invalid): 1 no FIR (one
// window row per output row instead of the PE-tap sums), 2 no FFT (no channelised rows), 4 no
// window slide (the prefetched rows are not moved into the window), 16 the FFT without its
// channelised-row stores (17 of the kernel's 80 us, r06_v16; written instead as whole 1-KB
// runs from the wave-owned LDS rows they took 2 us MORE, r06_v17 — rejected); 8 (valid, the A/B of
// round 6): workgroup barriers inside the FFT (the pre-round-6 form)
// The step's N-point FFT: thread c's butterfly of both radix-16 passes lies in row c / 16, so
// wave w owns rows 4w .. 4w + 3 for the whole transform (wave_rows_ok) and the two barriers
// inside it are wave barriers (round 6; timing variants r06_v14: the FFT was 30 of the
// kernel's 78 us with four workgroup barriers a step, memory traffic masked or not)
template <int N, int P, int NU, int DE, int ZOUT, bool LCBF, int GS, int TV = 0>
__device__ __forceinline__ void analysis_stream_body(const AnalysisArgs& a, int pol, int w, int nw) {
  using SH = StreamShape<N, P, NU, DE>;
  constexpr int M = SH::M, PE = SH::PE, QS = SH::QS, T = SH::T, NEW = SH::NEW, WIN = SH::WIN;
  constexpr bool kWR = (TV & 8) == 0 && wave_rows_ok<N, T, NT>();
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int c = threadIdx.x;
  if constexpr (ZOUT == 0 && !LCBF) {  // (stream objects only: no round-trip / LowCBF kernel)
  if (a.carry_out) {
    // the next call's carry, grid-stride over this polarisation's workgroups (its few
    // thousand samples are a fraction of one row of work per workgroup); before any early
    // return, so every workgroup takes its share
    // (a uniform loop with a per-lane guard — no lane-dependent trip count)
    const float2* src = a.in + pol * a.in_pol_stride + a.carry_src;
    float2* dst = a.carry_out + pol * a.carry_pol_stride;
    for (int64_t i0 = (int64_t)w * NT; i0 < a.carry_n; i0 += (int64_t)nw * NT) {
      const int64_t i = i0 + c;
      if (i < a.carry_n) dst[i] = src[i];
    }
  }
  }
  // this workgroup's steps (XCD-aware order: neighbouring ranges share halo rows in L2)
  const int64_t q_lo = a.row0 / NU;
  const int64_t n_steps = ((a.K + NU - 1) / NU - q_lo + QS - 1) / QS;
  const int64_t st0 = n_steps * w / nw, st1 = n_steps * (w + 1) / nw;
  if (st0 >= st1) return;

  // input column c from row DE q_first on; range-checked buffer loads return 0 past n_dat
  const int64_t row_first = (int64_t)DE * (q_lo + st0 * QS);
  const float2* xpol = a.in + pol * a.in_pol_stride;
  // window row r, column c is x[(row_first + r) N + c - pad]: the descriptor starts at the
  // first real sample the range reads; pre-padding rows give negative offsets, which wrap
  // past the range check and read as zeros
  const int64_t g0 = row_first * N - a.pad;
  const int64_t gb = max(g0, (int64_t)0);
  const int shift = (int)(g0 - gb);
  const int64_t avail = a.n_dat - gb;
  // the launcher sizes the ranges so that a workgroup's rows span <= kRsrcMaxBytes
  // (launch_stream); the min() only bounds the series tail beyond the range
  uint32_t nbytes = (uint32_t)min(max(avail, (int64_t)0) * 8, kRsrcMaxBytes);
  if (tmask(a.timing_mask) & 1) nbytes = 0;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xpol + gb, nbytes);
  // rows past the last window of the range (the unconditional last prefetch) re-read the
  // last row instead: an L2 hit rather than HBM traffic nobody uses
  const int r_last = (int)(st1 - st0 - 1) * NEW + WIN - 1;
  auto ld = [&](int r) {  // window row r (relative to row_first)
    const v2u v = __builtin_amdgcn_raw_buffer_load_b64(xr, (uint32_t)((min(r, r_last) * N + c + shift) * 8), 0, kAuxIn);
    return __builtin_bit_cast(v2f, v);
  };
  // (re, im) as a packed pair: one v_pk_fma_f32 per complex x real tap MAC
  v2f win[WIN];
  if (a.pre != nullptr && g0 < 0) {
    // a stream object's carried samples in front of the input: window sample (row i, column
    // c) is sample (row_first + i) N + c of the carry-then-input series; below pad it is
    // pre[pol][...], at or above it the input (each range-checked load returns 0 outside
    // its part, so the sum is the one sample)
    const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.pre + pol * a.pre_pol_stride, (uint32_t)(a.pad * 8));
#pragma unroll
    for (int i = 0; i < WIN; ++i) {
      const v2u pv = __builtin_amdgcn_raw_buffer_load_b64(pr, (uint32_t)(((row_first + i) * N + c) * 8), 0, 0);
      win[i] = ld(i) + __builtin_bit_cast(v2f, pv);
    }
  } else {
#pragma unroll
    for (int i = 0; i < WIN; ++i) win[i] = ld(i);
  }

  // LDS: twiddles behind the FFT rows, then F = [N zeros, taps, zeros]
  float* F = reinterpret_cast<float*>(smem) + SH::F_OFF;
  smem[SH::TW_OFF + tw_slot(c)] = a.twN[c];
#pragma unroll
  for (int m = 0; m < P + 2; ++m) F[m * N + c] = (m >= 1 && m <= P) ? a.taps[(m - 1) * N + c] : 0.f;

  float2* opol = a.out + pol * a.out_pol_stride;
  float2* zpol = ZOUT ? a.z + pol * a.z_pol_stride - a.z_row0 * N : nullptr;  // Z row k - z_row0
  LdsRows rows(smem, SH::RS);
  const float2* tw = smem + SH::TW_OFF;
  vm_drain();
#pragma unroll 1
  for (int64_t stp = st0; stp < st1; ++stp) {
    const int rel = (int)(stp - st0) * NEW;  // window row 0 of this step
    // prefetch the next step's new rows (consumed when the window slides)
    // (unconditional: past the range it reads rows nobody uses, or zeros past n_dat —
    // a conditional prefetch makes vmcnt path-dependent and the next step waits for
    // every store as well)
    v2f pf[NEW];
#pragma unroll
    for (int i = 0; i < NEW; ++i) pf[i] = ld(rel + WIN + i);
    __syncthreads();  // previous step's FFT has read its rows (first step: F staged)
    // all NU x QS rows accumulate together (tap-outer order): consecutive FMAs are
    // independent, so the 4-cycle FMA latency never stalls issue
    v2f acc[NU][QS];
    static_for<0, NU>([&](auto sv) {
#pragma unroll
      for (int qq = 0; qq < QS; ++qq) acc[decltype(sv)::value][qq] = v2f{0.f, 0.f};
    });
    if constexpr ((TV & 1) != 0) {
      static_for<0, NU>([&](auto sv) {
        static_for<0, QS>([&](auto qv) {
          acc[decltype(sv)::value][decltype(qv)::value] = win[DE * decltype(qv)::value + decltype(sv)::value];
        });
      });
    } else
    static_for<0, PE>([&](auto mv) {
      constexpr int m = decltype(mv)::value;
      float gm[NU];
      static_for<0, NU>([&](auto sv) {
        constexpr int s = decltype(sv)::value;
        gm[s] = F[(m + 1) * N + c - (s * M) % N];
      });
      static_for<0, NU>([&](auto sv) {
        constexpr int s = decltype(sv)::value;
        constexpr int bs = (s * M) / N;
        static_for<0, QS>([&](auto qv) {
          constexpr int qq = decltype(qv)::value;
          acc[s][qq] = __builtin_elementwise_fma(v2f{gm[s], gm[s]}, win[DE * qq + m + bs], acc[s][qq]);
        });
      });
    });
    const int64_t k0 = (q_lo + stp * QS) * NU;
    // ZOUT: the synthesis stage-1 row of output row k is the N-point inverse DFT across
    // channels of out[k] = N FFT_N(v_k), i.e. N^2 v_k exactly — the FIR output this
    // thread already holds at position c (v_k[c]).  It goes to HBM straight from the
    // registers (no inverse FFT; N^2 is a power of two, so the scaling is exact).
    const BufRowStore zs = BufRowStore::rows(ZOUT ? zpol : opol, k0, T, max(a.row0, a.z_row0), a.K,
                                             N, (float)N * (float)N);
    // ZOUT >= 2: the step's T = 16 rows of column c are 16 / ZOUT runs of this column, row
    // k - z_row0 = ZB g + gi at z[pol][(g N + c) ZB + gi]; rows (2m, 2m+1) go out as one 16-B
    // store once both are summed (the launcher guarantees that k0 - z_row0 is a multiple
    // of 16; rows past K land in the buffer's padding)
    const int64_t kz = k0 - a.z_row0;
    const __amdgpu_buffer_rsrc_t zb =
        make_rsrc(ZOUT >= 2 ? a.z + pol * a.z_pol_stride + max(kz, (int64_t)0) * N : opol,
                  (ZOUT >= 2 && kz >= 0 && !(tmask(a.timing_mask) & 4)) ? (uint32_t)(N * T * 8) : 0u);
    static_for<0, NU>([&](auto sv) {
      constexpr int s = decltype(sv)::value;
      static_for<0, QS>([&](auto qv) {
        constexpr int qq = decltype(qv)::value;
        const float2 v = make_float2(acc[s][qq].x, acc[s][qq].y);
        rows.store(qq * NU + s, c, v);
        if constexpr (ZOUT == 1) zs.store(qq * NU + s, c, v);
        if constexpr (ZOUT >= 2 && (s & 1)) {
          constexpr int r1 = qq * NU + s, r0 = r1 - 1;
          constexpr float n2 = (float)N * (float)N;
          const v2f a0 = acc[s - 1][qq] * n2, a1 = acc[s][qq] * n2;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{a0.x, a0.y, a1.x, a1.y}), zb,
                                                 (uint32_t)((((r0 / ZOUT) * N + c) * ZOUT + r0 % ZOUT) * 8), 0,
                                                 kAuxZst);
        }
      });
    });
    __syncthreads();
    if constexpr ((TV & 2) != 0) {
    } else if constexpr (LCBF) {
      const LcbfRowStore st = LcbfRowStore::rows(opol, k0, T, a.row0, a.K, a.lcbf_scale);
      block_fft<N, -1, T, NT, kWR>(rows, st, rows, tw, c);
    } else if constexpr (GS == 2) {
      // channel-major (a cascade's stage-2 series, out_rs = 1, no chomp): the last pass
      // lands in LDS by channel, then each 8-lane group writes one channel's T = 16
      // consecutive samples as 8 x 16 B (one 128-B run) instead of 16 scattered 8-B stores.
      // The launch's first and last rows are even (launch_stream checks), so a row pair is
      // valid or not as a whole: one store per pair, always issued, invalid pairs sent out
      // of the descriptor's range.  (Stores under a branch made the count path-dependent,
      // and the loop-end wait for the next step's rows then waited for the stores as well;
      // the strided store (GS 1) is a kernel of its own for the same reason: a different
      // store count per step.)
      static_assert(N * (T + 1) <= T * SH::RS, "channel-major staging exceeds the LDS rows");
      const ColMajorLds<T> cm{smem};
      block_fft<N, -1, T, NT, kWR>(rows, cm, rows, tw, c);
      __syncthreads();
      const int hi = (int)min(max(a.K - k0, (int64_t)0), (int64_t)T);
      const int lo = (int)min(max(a.row0 - k0, (int64_t)0), (int64_t)T);
      const __amdgpu_buffer_rsrc_t r =
          make_rsrc_u(opol + k0, hi > 0 ? (uint32_t)(((int64_t)(N - 1) * a.out_cs + hi) * 8) : 0u);
      static_for<0, (T / 2) * N / NT>([&](auto iv) {
        const int idx = c + decltype(iv)::value * NT;
        const int ch = idx / (T / 2), r0 = 2 * (idx % (T / 2));
        const float2 v0 = cscale(cm.load(r0, ch), (float)N), v1 = cscale(cm.load(r0 + 1, ch), (float)N);
        const uint32_t off = (r0 >= lo && r0 + 1 < hi) ? (uint32_t)((ch * a.out_cs + r0) * 8) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{v0.x, v0.y, v1.x, v1.y}), r, off, 0,
                                               kAuxColMajor);
      });
    } else if constexpr (GS == 1) {
      const StridedRowStore st = StridedRowStore::rows(opol, k0, T, a.row0, a.K, a.out_rs, a.out_cs,
                                                       a.sel_split, a.sel_shift, a.sel_n, N, (float)N);
      block_fft<N, -1, T, NT, kWR>(rows, st, rows, tw, c);
    } else if constexpr ((TV & 16) != 0) {
      // (timing variant: the FFT computed, its channelised rows not stored — kept live only)
      block_fft<N, -1, T, NT, kWR>(rows, SinkStore{}, rows, tw, c);
    } else {
      // (timing mask bit 1, experiments build: no channelised stores)
      const BufRowStore st = BufRowStore::rows(opol, k0, T, a.row0, (tmask(a.timing_mask) & 2) ? k0 : a.K, N, (float)N);
      block_fft<N, -1, T, NT, kWR>(rows, st, rows, tw, c);
    }
    if constexpr ((TV & 4) != 0) {
      // (keep the prefetched rows live: an empty use)
#pragma unroll
      for (int i = 0; i < NEW; ++i) asm volatile("" ::"v"(pf[i]));
    } else {
#pragma unroll
    for (int i = 0; i < PE - 1; ++i) win[i] = win[i + NEW];
#pragma unroll
    for (int i = 0; i < NEW; ++i) win[PE - 1 + i] = pf[i];
    }
  }
}

// WPE: waves per SIMD the register allocation targets (2: 184 VGPRs for the C2 round trip;
// 3: <= 168, three 51-KB workgroups per CU)
template <int N, int P, int NU, int DE, int ZOUT, bool LCBF = false, int GS = 0, int WPE = 2, int TV = 0>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE))) void analysis_stream_kernel(AnalysisArgs a) {
  const int w = a.linear ? (int)blockIdx.x : xcd_tile(blockIdx.x, gridDim.x);
  analysis_stream_body<N, P, NU, DE, ZOUT, LCBF, GS, TV>(a, blockIdx.y, w, gridDim.x);
}

}  // namespace pfb
