// pfb_rowfft.hip — N-point row FFT launchers (row_fft_kernel, pfb_common.hpp): the
// analysis FFT for N > 256 and synthesis stage 1 (the N-point inverse DFT across channels
// of every channelised row, polyphase_synthesis.m:282-285 factored).
#include "pfb_common.hpp"

#include <algorithm>
#include <cstdlib>

namespace pfb {

// ----------------------------------------------------------------- 4096-point row FFT
// The SKA-Mid row FFT (the analysis FFT of polyphase_analysis_padded.m:147 for C3, and the
// synthesis stage 1 of 4096-channel rows) as three explicit radix-16 Stockham passes per
// row, persistent over a contiguous row range (XCD-aware), next row prefetched into
// registers.  Round 5: the twiddles come from per-pass power tables instead of strided
// reads of one 4096-entry table — pass 3 read table entries r k at lane stride r = 2, 4, 8
// (2-, 4- and 8-way LDS bank conflicts, 24 % of the kernel's LDS cycles) — each lane now
// reads w^{2^p}(k) from T3[p][k], contiguous in k (conflict-free).  The entries are the
// same table values (e^{-2 pi i m / 4096}, rounded once from double on the host) and the
// other powers are the same products, so the output is bit-identical to the generic
// passes.  The tables take 8.7 KB instead of 32 KB of LDS: 3 workgroups per CU.
// The row takes two layouts instead of the 1-in-16 pad (whose pass-2 / pass-3 loads wrapped
// one lane of every 32-lane ds_read_b64 group onto bank 0: 2-way, 22 % of the LDS cycles,
// r05_v4 PMC): pass 1 -> pass 2, element 16 j + r at slot kR4kA r + j (rows of kR4kA slots: the
// 16-lane store groups and the load groups, kR4kA (tid mod 16) + tid / 16, on distinct
// banks); pass 2 -> pass 3 unpadded (element e at slot e).  Every access is one lane base
// plus an immediate offset.
// (257: the pass-2 loads compile to ds_read2_b64 — 16-lane groups on 32 banks — whose
// 16 lanes k2 then sit at dword 2 (257 k2 + j) = 2 k2 + 2 j mod 32, all distinct; 258 gave
// 4 k2 mod 32, 2-way, the 18 % of LDS cycles PMC kept counting)
constexpr int kR4kA = 257;         // layout-A row of 16 j + r: slot kR4kA r + j
constexpr int kR4kRow = 15 * kR4kA + 256 + 2;  // slots of the row buffer (layout A; B needs 4096)
constexpr int kR4kTw2 = 4 * 16;    // T2[p][k] = tw[(2^p 16 k) mod N], k < 16
constexpr int kR4kTw3 = 4 * 256;   // T3[p][k] = tw[2^p k], k < 256
constexpr size_t kR4kLds = ((size_t)kR4kRow + kR4kTw2 + kR4kTw3) * sizeof(float2);

template <int DIR>
__device__ __forceinline__ void r4k_twiddles(const float2* t, int k, int stride, float2 (&w)[16]) {
  static_for<0, 4>([&](auto pv) {
    constexpr int p = decltype(pv)::value;
    float2 v = t[p * stride + k];
    if constexpr (DIR > 0) v.y = -v.y;
    w[1 << p] = v;
  });
  static_for<1, 16>([&](auto rv) {
    constexpr int r = decltype(rv)::value;
    constexpr int h = high_bit(r);
    if constexpr (h != r) w[r] = cmul(w[h], w[r - h]);
  });
}

// One row held as v[r] = element tid + 256 r (pass-1 input order): the three radix-16 passes
// through the LDS row; on return v[r] = output element tid + 256 r.  Opens with the barrier
// that orders it after the previous row's pass 3 (and the tables' staging).
template <int DIR>
__device__ __forceinline__ void r4k_fft(float2 (&v)[16], float2* row, const float2* t2, const float2* t3, int tid) {
  const int k2 = tid & 15;
  const int st2 = (tid >> 4) * 256 + k2;     // pass-2 output base (j / 16) 256 + k
  __syncthreads();  // tables staged / the previous row's pass 3 is done with the LDS row
  // pass 1 (NS 1): no twiddles, outputs tid 16 + r
  sdft<16, DIR>(v);
#pragma unroll
  for (int r = 0; r < 16; ++r) row[kR4kA * r + tid] = v[r];  // layout A
  __syncthreads();
  // pass 2 (NS 16): k = tid mod 16, twiddles w^r, r = 1..15, of m = 16 k
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = row[kR4kA * k2 + (tid >> 4) + 16 * r];  // element tid + 256 r
  {
    float2 w[16];
    r4k_twiddles<DIR>(t2, k2, 16, w);
    static_for<1, 16>([&](auto r) { v[r] = cmul(v[r], w[r]); });
  }
  sdft<16, DIR>(v);
  __syncthreads();  // every pass-2 load done before the in-place stores
#pragma unroll
  for (int r = 0; r < 16; ++r) row[st2 + 16 * r] = v[r];  // layout B
  __syncthreads();
  // pass 3 (NS 256): k = tid, twiddles of m = k; outputs tid + 256 r
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = row[tid + 256 * r];
  {
    float2 w[16];
    r4k_twiddles<DIR>(t3, tid, 256, w);
    static_for<1, 16>([&](auto r) { v[r] = cmul(v[r], w[r]); });
  }
  sdft<16, DIR>(v);
}

// Output row rw (row_base + rw, circularly shifted by -sds mod n_total when remap: the padded
// variant's time shift, RowStore's rule) of a [row][N] product -> HBM.
__device__ __forceinline__ void r4k_store_row(const float2 (&v)[16], int tid, const RowFftArgs& a, float2* out,
                                              int64_t rw) {
  int64_t t = a.row_base + rw;
  if (a.remap) {
    t -= a.sds;
    while (t < 0) t += a.n_total;
  }
  // (t is uniform, but the uniformity analysis loses it through the wrap loop: without the
  // read-first-lane every store became a one-trip waterfall loop over the descriptor)
  t = (int64_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)t >> 32)) << 32) |
                __builtin_amdgcn_readfirstlane((uint32_t)t));
  const __amdgpu_buffer_rsrc_t os = make_rsrc(out + t * 4096, (uint32_t)(4096 * 8));
  const uint32_t lane_off = (uint32_t)tid * 8u;
  static_for<0, 16>([&](auto rv) {
    constexpr int r = decltype(rv)::value;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, cscale(v[r], a.scale)), os, lane_off,
                                          r * 2048, kNtRow ? 2 : 0);
  });
}

template <int DIR>
__device__ __forceinline__ void r4k_row(float2 (&v)[16], float2* row, const float2* t2, const float2* t3,
                                        int tid, const RowFftArgs& a, float2* out, int64_t rw) {
  r4k_fft<DIR>(v, row, t2, t3, tid);
  r4k_store_row(v, tid, a, out, rw);
}

// (buffer loads / stores: one descriptor per row, the lane's byte offset tid * 8 and the
// register's r * 2048 as a scalar offset — no 64-bit address per register: <= 168 VGPRs,
// 3 workgroups per CU)
template <int DIR, bool PERM, bool GAIN>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3))) void row_fft4096_kernel(RowFftArgs a) {
  constexpr int N = 4096;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int pol = blockIdx.y;
  const int wg = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t q0 = a.n_rows * wg / gridDim.x, q1 = a.n_rows * (wg + 1) / gridDim.x;
  if (q0 >= q1) return;  // uniform per workgroup
  const int tid = threadIdx.x;
  float2* row = smem;                        // layouts A / B, kR4kRow slots
  float2* t2 = smem + kR4kRow;               // [p][16]
  float2* t3 = t2 + kR4kTw2;                 // [p][256]
  for (int e = tid; e < kR4kTw3; e += NT) {
    const int pp = e >> 8, k = e & 255;
    t3[e] = a.tw[(k << pp) & (N - 1)];
    if (e < kR4kTw2) t2[e] = a.tw[((e & 15) << ((e >> 4) + 4)) & (N - 1)];
  }
  const float2* in = a.in + pol * a.in_pol_stride;
  float2* out = a.out + pol * a.out_pol_stride;
  [[maybe_unused]] uint32_t col[PERM ? 16 : 1];
  [[maybe_unused]] float g[GAIN ? 16 : 1];
  if constexpr (PERM || GAIN) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = tid + r * 256;
      const int c = PERM ? a.perm[i] : i;
      if constexpr (PERM) col[PERM ? r : 0] = (uint32_t)c * 8u;
      if constexpr (GAIN) g[GAIN ? r : 0] = a.cgain[c];
    }
  }
  const uint32_t lane_off = (uint32_t)tid * 8u;
  // input in 2-row runs (a.in_run, z_index): element e of row rr at ((rr / 2) N + e) 2 + rr % 2
  // — the lane and register strides double; the pair's other row is fetched with the same
  // 128-B lines one row later (L2 / Infinity-Cache hits)
  const int ish = __builtin_amdgcn_readfirstlane(a.in_run ? 1 : 0);  // (scalar: the soffsets use it)
  const uint32_t lane_in = lane_off << ish;
  [[maybe_unused]] uint32_t col_in[PERM ? 16 : 1];
  if constexpr (PERM) {
#pragma unroll
    for (int r = 0; r < 16; ++r) col_in[PERM ? r : 0] = col[PERM ? r : 0] << ish;
  }
  float2 pf[16];
  auto load_row = [&](int64_t rr) {
    const int64_t base = a.in_run ? (((rr >> 1) * N) << 1) + (rr & 1) : rr * N;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_u(in + base, (uint32_t)((N * 8) << ish));
    static_for<0, 16>([&](auto rv) {
      constexpr int r = decltype(rv)::value;
      const v2u x = PERM ? __builtin_amdgcn_raw_buffer_load_b64(rs, col_in[PERM ? r : 0], 0, kNtlRow ? 2 : 0)
                         : __builtin_amdgcn_raw_buffer_load_b64(rs, lane_in, (r * 2048) << ish, kNtlRow ? 2 : 0);
      pf[r] = __builtin_bit_cast(float2, x);
    });
  };
  load_row(q0);
  vm_drain();
#pragma unroll 1
  for (int64_t rw = q0; rw < q1; ++rw) {
    float2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = GAIN ? cscale(pf[r], g[GAIN ? r : 0]) : pf[r];
    load_row(min(rw + 1, q1 - 1));  // unconditional: past the end re-reads the last row
    r4k_row<DIR>(v, row, t2, t3, tid, a, out, rw);
  }
}

// Round 6: rows in PAIRS, one pair per workgroup.  RUN (in_run: the SKA-Mid round trip's
// stage-1 rows as the FIR writes them, 2-row runs per column): each lane loads element i of
// both rows with one 16-B buffer load, so the run's 128-B lines cross the memory side once
// (the one-row kernel loaded 8 B of every 16 and re-fetched the partner's lines one row
// later: 913 MB read for 613 MB of rows; 625 MB now, r06 PMC).  !RUN: rows
// [row][N], two 8-B loads per element.  Row 2p is transformed from the first halves while
// row 2p + 1 waits in registers.  REV: the padded variant's index reversal (column (N - i)
// mod N for element i) computed from the lane (element i = tid + 256 r: r >= 1 reads column
// 4096 - 256 r - tid, one lane base (255 - tid) and a scalar offset; r = 0 its own lane
// offset) — 2 registers instead of the 16 column offsets of the generic permutation.  OZS:
// the output in 2-row runs (RowStore::zs = 1, the Nf 512 synthesis' stage-1 layout; row A's
// results held until row B's, one 16-B store per element).  Same passes and tables as the
// one-row kernel: bit-identical.
// SCHED (which pairs a workgroup takes): 0 a contiguous range (XCD-aware order), 1 grid-stride
// from blockIdx.x, 2 one pair per workgroup (grid = pairs) — the default: the dispatcher hands
// out pairs in row order, so the chip's loads in flight stay in one narrow window of the
// rows; 224 vs 262 us per C3 launch (persistent ranges), 243 grid-stride
// (profiles/r06_v3_rowfft_sched_ab.log).  The same holds for a plain float4 copy: one 16-B
// load + store per thread, one-shot grid, 6.6 TB/s; persistent grid-stride or range loops
// 4.7-5.5 TB/s (scripts/copy_probe.hip, profiles/r06_copy_probe.jsonl).
template <int DIR, bool REV, int SCHED, bool RUN = true, bool OZS = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3))) void row_fft4096_pair_kernel(RowFftArgs a) {
  constexpr int N = 4096;
  constexpr uint32_t ES = RUN ? 16u : 8u;  // bytes between elements i and i + 1 of a row
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int pol = blockIdx.y;
  const int64_t np = (a.n_rows + 1) >> 1;
  int64_t p0, p1, pstep = 1;
  if constexpr (SCHED == 0) {
    const int wg = xcd_tile(blockIdx.x, gridDim.x);
    p0 = np * wg / gridDim.x;
    p1 = np * (wg + 1) / gridDim.x;
  } else if constexpr (SCHED == 1) {
    p0 = blockIdx.x;
    p1 = np;
    pstep = gridDim.x;
  } else {
    p0 = blockIdx.x;
    p1 = min(p0 + 1, np);
  }
  if (p0 >= p1) return;  // uniform per workgroup
  const int tid = threadIdx.x;
  float2* row = smem;
  float2* t2 = smem + kR4kRow;
  float2* t3 = t2 + kR4kTw2;
  for (int e = tid; e < kR4kTw3; e += NT) {
    const int pp = e >> 8, k = e & 255;
    t3[e] = a.tw[(k << pp) & (N - 1)];
    if (e < kR4kTw2) t2[e] = a.tw[((e & 15) << ((e >> 4) + 4)) & (N - 1)];
  }
  const float2* in = a.in + pol * a.in_pol_stride;
  float2* out = a.out + pol * a.out_pol_stride;
  const uint32_t lane_a = REV ? (uint32_t)(255 - tid) * ES : (uint32_t)tid * ES;
  const uint32_t lane_0 = REV ? (tid ? (uint32_t)(N - tid) * ES : 0u) : lane_a;
  v4u pf[16];
  auto load_pair = [&](int64_t pp) {
    // (!RUN: the last pair of an odd row count has no row B — its loads leave the range)
    const uint32_t nrec = RUN ? (uint32_t)(N * 16) : (2 * pp + 1 < a.n_rows ? 2u : 1u) * (uint32_t)(N * 8);
    const __amdgpu_buffer_rsrc_t rs = make_rsrc_u(in + pp * 2 * N, nrec);
    static_for<0, 16>([&](auto rv) {
      constexpr int r = decltype(rv)::value;
      constexpr int soff = r == 0 ? 0 : REV ? (3841 - 256 * r) * (int)ES : r * 256 * (int)ES;
      const uint32_t lo = r == 0 ? lane_0 : lane_a;
      if constexpr (RUN) {
        pf[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, lo, soff, kNtlRow ? 2 : 0);
      } else {
        const v2u x0 = __builtin_amdgcn_raw_buffer_load_b64(rs, lo, soff, kNtlRow ? 2 : 0);
        const v2u x1 = __builtin_amdgcn_raw_buffer_load_b64(rs, lo, soff + N * 8, kNtlRow ? 2 : 0);
        pf[r] = v4u{x0.x, x0.y, x1.x, x1.y};
      }
    });
  };
  load_pair(p0);
  vm_drain();
#pragma unroll 1
  for (int64_t pp = p0; pp < p1; pp += pstep) {
    float2 v[16], h[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const v4f x = __builtin_bit_cast(v4f, pf[r]);
      v[r] = make_float2(x.x, x.y);
      h[r] = make_float2(x.z, x.w);
    }
    if constexpr (OZS) {
      // both rows transformed, then element i of rows (2p, 2p + 1) as one 16-B store into
      // run p (row_base even, no remap: launch_row_fft_t checks)
      r4k_fft<DIR>(v, row, t2, t3, tid);
      if constexpr (SCHED != 2) load_pair(pp + pstep < p1 ? pp + pstep : pp);
      r4k_fft<DIR>(h, row, t2, t3, tid);
      const int64_t run = (a.row_base >> 1) + pp;
      const __amdgpu_buffer_rsrc_t os = make_rsrc_u(out + run * 2 * N, (uint32_t)(N * 16));
      auto st = [&](auto aux) {
        static_for<0, 16>([&](auto rv) {
          constexpr int r = decltype(rv)::value;
          const float2 x0 = cscale(v[r], a.scale), x1 = cscale(h[r], a.scale);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{x0.x, x0.y, x1.x, x1.y}), os,
                                                 (uint32_t)tid * 16u, r * 4096, decltype(aux)::value);
        });
      };
      // (RowStore::nt: the default policy for rows the synthesis reads right after from the
      // Infinity Cache; uniform)
      if (a.nt && kNtRow) st(std::integral_constant<int, 2>{});
      else st(std::integral_constant<int, 0>{});
    } else {
      r4k_row<DIR>(v, row, t2, t3, tid, a, out, 2 * pp);
      if constexpr (SCHED != 2)
        load_pair(pp + pstep < p1 ? pp + pstep : pp);  // unconditional: past the end re-reads this pair
      if (2 * pp + 1 < a.n_rows) r4k_row<DIR>(h, row, t2, t3, tid, a, out, 2 * pp + 1);  // (uniform)
    }
  }
}

template <int DIR, bool PERM, bool GAIN>
static hipError_t launch_row_fft4096(const RowFftArgs& r, int n_pol, hipStream_t s, int per_cu) {
  auto kern = row_fft4096_kernel<DIR, PERM, GAIN>;
  hipError_t e = set_lds(kern, kR4kLds);
  if (e != hipSuccess) return e;
  const int64_t wgs = (int64_t)cu_count() * per_cu;
  dim3 grid((unsigned)std::max<int64_t>(1, wgs / n_pol), (unsigned)n_pol);
  return launch_kernel(kern, grid, dim3(NT), kR4kLds, s, r);
}

template <int DIR, bool REV, int SCHED, bool RUN, bool OZS>
static hipError_t launch_r4k_pair(const RowFftArgs& r, int n_pol, hipStream_t s, int per_cu) {
  auto kern = row_fft4096_pair_kernel<DIR, REV, SCHED, RUN, OZS>;
  hipError_t e = set_lds(kern, kR4kLds);
  if (e != hipSuccess) return e;
  const int64_t wgs = SCHED == 2 ? (r.n_rows + 1) / 2 : (int64_t)cu_count() * per_cu / n_pol;
  if (wgs > INT32_MAX) return hipErrorInvalidValue;
  dim3 grid((unsigned)std::max<int64_t>(1, wgs), (unsigned)n_pol);
  return launch_kernel(kern, grid, dim3(NT), kR4kLds, s, r);
}
template <int DIR, bool REV, bool RUN, bool OZS>
static hipError_t launch_row_fft4096_pair(const RowFftArgs& r, int n_pol, hipStream_t s, int per_cu) {
  // (PFB_ROWFFT_SCHED: 0 ranges, 1 grid-stride, 2 one pair per workgroup — experiments A/B)
  static const int sched = knob("PFB_ROWFFT_SCHED") ? std::atoi(knob("PFB_ROWFFT_SCHED")) : 2;
  if constexpr (kExperiments) {
    if (sched == 0) return launch_r4k_pair<DIR, REV, 0, RUN, OZS>(r, n_pol, s, per_cu);
    if (sched == 1) return launch_r4k_pair<DIR, REV, 1, RUN, OZS>(r, n_pol, s, per_cu);
  }
  return launch_r4k_pair<DIR, REV, 2, RUN, OZS>(r, n_pol, s, per_cu);
}

template <int N, int DIR, bool PERM, bool GAIN>
static hipError_t launch_row_fft_t(const RowFftArgs& r, int n_pol, hipStream_t s) {
  constexpr int ROWS = RowShape<N>::ROWS;
  if constexpr (N == 4096) {
    // persistent workgroups (row_fft_persist_kernel) once there are several rows per
    // resident workgroup; PFB_ROWFFT_PERSIST=0: one workgroup per row (A/B)
    static const bool off = knob("PFB_ROWFFT_PERSIST") && std::atoi(knob("PFB_ROWFFT_PERSIST")) == 0;
    const size_t bytes = row_fft_persist_lds<N>();
    const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / bytes);
    const int64_t wgs = (int64_t)cu_count() * per_cu;
    // the explicit-pass kernel with per-pass twiddle tables (PFB_ROWFFT_4K=0: the generic
    // persistent kernel; PFB_ROWFFT_WPC: its workgroups per CU, default the 3 LDS allows —
    // experiments A/B)
    static const bool k4 = !(knob("PFB_ROWFFT_4K") && std::atoi(knob("PFB_ROWFFT_4K")) == 0);
    static const int wpc = knob("PFB_ROWFFT_WPC") ? std::atoi(knob("PFB_ROWFFT_WPC")) : 0;
    const int per_cu4 = wpc > 0 ? wpc : (int)std::max<size_t>(1, std::min<size_t>(3, (160 * 1024) / kR4kLds));
    // the pair kernel (no per-channel gain, no permutation but the padded index reversal;
    // output rows [row][N], or 2-row runs from an even first row without the time shift);
    // PFB_ROWFFT_PAIR=0: the one-row kernel (A/B)
    static const bool no_pair = knob("PFB_ROWFFT_PAIR") && std::atoi(knob("PFB_ROWFFT_PAIR")) == 0;
    if constexpr (!GAIN) {
      const bool ozs = r.zs == 1 && !r.remap && (r.row_base & 1) == 0 && (r.n_rows & 1) == 0;
      if (!off && k4 && !no_pair && (!PERM || r.rev) && (r.zs == 0 || ozs) && r.n_rows >= 2) {
        if (r.in_run) return ozs ? launch_row_fft4096_pair<DIR, PERM, true, true>(r, n_pol, s, per_cu4)
                                 : launch_row_fft4096_pair<DIR, PERM, true, false>(r, n_pol, s, per_cu4);
        return ozs ? launch_row_fft4096_pair<DIR, PERM, false, true>(r, n_pol, s, per_cu4)
                   : launch_row_fft4096_pair<DIR, PERM, false, false>(r, n_pol, s, per_cu4);
      }
    }
    if (!off && k4 && r.zs == 0 && r.n_rows >= 4 * (int64_t)cu_count() * per_cu4)
      return launch_row_fft4096<DIR, PERM, GAIN>(r, n_pol, s, per_cu4);
    if (!off && r.n_rows >= 4 * wgs) {
      auto kern = row_fft_persist_kernel<N, DIR, PERM, GAIN>;
      hipError_t e = set_lds(kern, bytes);
      if (e != hipSuccess) return e;
      dim3 grid((unsigned)std::max<int64_t>(1, wgs / n_pol), (unsigned)n_pol);
      return launch_kernel(kern, grid, dim3(NT), bytes, s, r);
    }
  }
  const size_t bytes = ((size_t)ROWS * RowShape<N>::RS + tw_slots(N)) * sizeof(float2);
  auto kern = row_fft_kernel<N, DIR, PERM, GAIN>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((r.n_rows + ROWS - 1) / ROWS), (unsigned)n_pol);
  return launch_kernel(kern, grid, dim3(NT), bytes, s, r);
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
hipError_t dispatch_row_fft(int N, const RowFftArgs& r, int n_pol, hipStream_t s) {
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
    default: break;
  }
  if constexpr (DIR > 0) {
    switch (N) {
      case 14: return launch_row_fft<14, DIR>(r, n_pol, s);
      case 28: return launch_row_fft<28, DIR>(r, n_pol, s);
      case 56: return launch_row_fft<56, DIR>(r, n_pol, s);
      case 112: return launch_row_fft<112, DIR>(r, n_pol, s);
      case 216: return launch_row_fft<216, DIR>(r, n_pol, s);
      case 224: return launch_row_fft<224, DIR>(r, n_pol, s);
      case 432: return launch_row_fft<432, DIR>(r, n_pol, s);
      case 448: return launch_row_fft<448, DIR>(r, n_pol, s);
      case 864: return launch_row_fft<864, DIR>(r, n_pol, s);
      case 192: return launch_row_fft<192, DIR>(r, n_pol, s);
      case 384: return launch_row_fft<384, DIR>(r, n_pol, s);
      case 768: return launch_row_fft<768, DIR>(r, n_pol, s);
      case 896: return launch_row_fft<896, DIR>(r, n_pol, s);
      case 1536: return launch_row_fft<1536, DIR>(r, n_pol, s);
      case 1792: return launch_row_fft<1792, DIR>(r, n_pol, s);
      case 3072: return launch_row_fft<3072, DIR>(r, n_pol, s);
      case 3584: return launch_row_fft<3584, DIR>(r, n_pol, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

template hipError_t dispatch_row_fft<-1>(int, const RowFftArgs&, int, hipStream_t);
template hipError_t dispatch_row_fft<+1>(int, const RowFftArgs&, int, hipStream_t);

bool chan_ifft_supported(int N) { return pow2_supported(N) || mixed_chan_supported(N); }

hipError_t launch_chan_ifft(const ChanIfftArgs& c, hipStream_t s) {
  if (c.n_rows <= 0) return hipSuccess;
  // (the stage-1 rows are read by the synthesis right after: default store policy while they
  // fit the 256 MB Infinity Cache with room to spare — the nontemporal rows of the generic
  // policy made the synthesis-only C2 path's block kernel read them from HBM)
  bool fits = (double)c.n_pol * c.n_rows * c.N * 8.0 <= 160.0 * (1 << 20);
  if constexpr (kExperiments) {  // (PFB_CHAN_IFFT_NT=1: nontemporal as before, A/B)
    static const bool force_nt = knob("PFB_CHAN_IFFT_NT") && std::atoi(knob("PFB_CHAN_IFFT_NT")) == 1;
    if (force_nt) fits = false;
  }
  RowFftArgs r{c.in, c.in_pol_stride, c.out, c.out_pol_stride, c.n_rows, c.perm, c.cgain, c.twN,
               1.0f, 0, 0, 0, c.n_rows, c.zblk == 4 ? 2 : c.zblk == 2 ? 1 : 0, fits ? 0 : 1};
  if (c.zblk != 1 && c.zblk != 2 && c.zblk != 4) return hipErrorInvalidValue;
  return dispatch_row_fft<+1>(c.N, r, c.n_pol, s);
}

}  // namespace pfb
