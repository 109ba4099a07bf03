// pfb_synth_wave.hpp — synthesis stage 2 for Nf = 256 with one output phase per 16 lanes
// (the algorithm: pfb_synth_wave.hip), instantiated by synth_wave_kernel.
#pragma once
#include "pfb_common.hpp"

namespace pfb {

namespace {

constexpr int kWgThreads = 256;
constexpr int kCols = 16;        // output phases per workgroup
// LDS: one 16 x 16 tile per phase, rows of 144 B (16 values + 16 B).  In-wave (non-XW)
// kernels: the tile of phase col = 4 w + cc at col * 2560 + 16 (w + 4 cc) bytes, lane =
// 4 l + cc in passes 1-2 and 16 slot + col in pass 3: every ds_read_b128 of either swap is
// conflict-free, the swap ds_write_b64 at most 2-way.  XW kernels: col_base_xw and the
// lane roles below, every swap access conflict-free.  Every address is a lane constant
// plus an immediate.
constexpr int kRowB = 144;
constexpr int kColStride = 2560;
constexpr int kTilesB = kCols * kColStride;
constexpr int kTw2RowB = 112;    // tw2 row: 14 values (RW <= 14)
constexpr int kWinRowB = 80;     // window row: 16 floats + 16 B pad
constexpr int kTw1Off = kTilesB;
constexpr int kTw2Off = kTw1Off + 16 * kRowB;
constexpr int kWinOff = kTw2Off + 16 * kTw2RowB;
constexpr int kLdsB = kWinOff + 16 * kWinRowB;

__device__ __forceinline__ int col_base(int col) { return col * kColStride + 16 * ((col >> 2) + 4 * (col & 3)); }
// XW kernels (round 5, scripts/lds_bank_model.py): the tile of phase c at c * 2560 + 16 (c >> 1)
// with the lane roles below make all four swap accesses bank-conflict-free (the layout
// above left the swap-1 and swap-2 ds_write_b64 2-way: 32 % of the LDS cycles):
//   pass 1 (l1, p1):  16-lane write groups = the 8 even or odd phases x 2 FFT lanes
//   passes 2 / A (l, phase): 16-lane groups = one phase x its 16 FFT lanes
//   pass 3 (phase, t1a): each ds_read_b128 lane group = 8 phases of one parity x 2 t1a
__device__ __forceinline__ int col_base_xw(int col) { return col * kColStride + 16 * (col >> 1); }
// pass-3 role of lane `lane` (XW): its ds_read_b128 group g (MI355X_MICROARCH.md §LDS:
// {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32) and position q in it -> phase
// 2 (q mod 8) + (g mod 2), t1a index j = 2 (q / 8) + g / 2
__device__ __forceinline__ void pass3_role_xw(int lane, int& phase, int& j) {
  const int x = lane & 31;
  int g, q;
  if (x < 4) { g = 0; q = x; }
  else if (x < 12) { g = 1; q = x - 4; }
  else if (x < 16) { g = 0; q = x - 8; }
  else if (x < 20) { g = 1; q = x - 8; }
  else if (x < 28) { g = 0; q = x - 12; }
  else { g = 1; q = x - 16; }
  phase = 2 * (q & 7) + g;
  j = 2 * (q >> 3) + (lane >> 5);
}

// 2 consecutive float2 of an LDS row (one ds_read_b128)
__device__ __forceinline__ void lds_pair(const char* p, float2& a, float2& b) {
  const v4f q = *reinterpret_cast<const v4f*>(p);
  a = make_float2(q.x, q.y);
  b = make_float2(q.z, q.w);
}

// kept slot r'' of pass-2 bin f2 (f = f1 + 16 f2), -1 if discarded; H = RW / 2
template <int RW, bool SPANS>
constexpr int kept_r(int f2) {
  constexpr int H = RW / 2;
  if (f2 < H) return SPANS ? f2 : f2 + H;
  if (f2 >= 16 - H) return SPANS ? f2 - (16 - RW) : f2 - (16 - H);
  return -1;
}
// pass-2 bin of kept slot r''
template <int RW, bool SPANS>
constexpr int bin_of(int rr) {
  for (int f2 = 0; f2 < 16; ++f2)
    if (kept_r<RW, SPANS>(f2) == rr) return f2;
  return -1;
}

}  // namespace

// Stage-1 rows read from Z (the streaming analysis wrote them)
struct NoFir {
  static constexpr bool kOn = false;
  static constexpr int NU = 1, DE = 1, PE = 1, S = 1, RS = 0;
  static constexpr int rows(int) { return 0; }
  static constexpr int loads(int) { return 1; }
};
// Stage-1 rows recomputed from the input series (SynthBlockArgs::fir_x): lane (l, col) of
// pass 1 needs Z rows k = NU q0 + keep b + l + 16 r of phase c = t0g + col, i.e. residue
// s = l mod NU and commutator step q = q0 + (keep / NU) b + l / NU + (16 / NU) r, whose FIR
// sum (pfb_ana_stream.hpp) is sum_m g_s[m][c] X[DE q + b_s + m][c] over PE taps, X the
// input as rows of N.  So row r of the lane reads input rows T0(b) + o_l + S r + m with
// T0(b) = DE (q0 + (keep / NU) b), o_l = DE (l / NU) + b_s, S = 16 DE / NU: the workgroup's
// 16 columns of those rows go through an LDS tile (rows of RS bytes; the reads of one
// 32-lane group hit 8 distinct rows x 4 columns, spread over the banks by the 32-B pad).
template <int NU_, int DE_, int PE_>
struct FirShape {
  static constexpr bool kOn = true;
  static constexpr int NU = NU_, DE = DE_, PE = PE_;
  static constexpr int S = DE * 16 / NU;
  static constexpr int OMAX = DE * (16 / NU - 1) + ((NU - 1) * DE) / NU;  // largest o_l
  static constexpr int RS = 160;
  static constexpr int rows(int r_lo) { return OMAX + (15 - r_lo) * S + PE; }  // tile rows for r >= r_lo
  static constexpr int loads(int r_lo) { return (rows(r_lo) + 31) / 32; }      // 16-B loads per thread
};

// The workgroup's blocks: a contiguous range, each block's first 16 - DK register rows
// taken from the previous block.  (A schedule class, so that a producer-consumer launch can
// supply blocks in the order their rows are ready and wait for each — the one-launch
// round trip measured and rejected in round 3)
struct RangeSched {
  static constexpr bool kReuse = true;
  static constexpr int kLoadAux = kAuxZld;
  int b_begin, n;
  __device__ int count() const { return n; }
  __device__ int block(int i) const { return b_begin + i; }
  __device__ void wait(int) const {}
};

// DK: overlap reuse, keep = 16 DK (the next block's rows l + 16 r, r < 16 - DK, are this
// block's registers r + DK).  tg: the workgroup's phase group (16 output phases).
// XW: pass-1 lanes (phase p, FFT lane l) spread over the workgroup (lane = 16 (l mod 4) + p
// in wave l / 4): one Z load instruction reads 2 row pairs x the 16 phases (256-B runs)
// instead of 8 row pairs x 4 phases (64-B runs), and swap 1 crosses waves (one more
// workgroup barrier per block)
// WFLAT: the temporal window is exactly 1 on rows [48, 208) of the block (tukey with Ov <= 48,
// SynthBlockArgs::win_flat): registers r = 3 .. 12 (rows l + 16 r) skip the multiply — the
// product by 1 is exact, so the output is bit-identical
// PRIO (bit mask): raise the wave's issue priority (s_setprio 2) between the loop-top
// barrier and the swap-1 barrier (1), from the swap-2 barrier to the block's stores (2),
// from the swap-1 barrier to the swap-2 barrier (4); 8 / 16: as 1 with priority 3 / 1;
// 32: the loop-top barrier moved below pass 1
// V (bit mask, round 6):
//   1  KEPT: with keep = 160 = 16 DK and Ov = 48 the kept outputs are t1 in [3 RW, 13 RW)
//      (L_ov = 3 RW N), i.e. exactly pass-3 registers t1b in [3, 13) of every lane: only
//      those 10 are formed (the other 6 of the 16-point IDFT are dead code) and stored, and a
//      whole block stores them through scalar row offsets from ONE lane offset register that
//      stays fixed for the kernel.  (Before: 16 stores a block, 6 of them always out of
//      range, each with its own hoisted address register — 16 VGPRs.)
//   2  PP: the block loop unrolled by two over two register sets, so block b + 1's rows load
//      straight into the registers block b + 1 reads.  (Before: one set; pass 1 still held
//      its registers when the prefetch was issued, so the loads went to temporaries and the
//      compiler's copies into the loop-carried set, scheduled into pass 2, each waited for its
//      load — the prefetch's HBM latency exposed half a block after issue.)
//   8, 16  timing variants (experiments build, results invalid): 8 wave barriers instead of
//      the block loop's workgroup barriers, 16 a uniform twiddle instead of the LDS tables
//   4  DEFER (with KEPT, as synth_wave512_kernel): block b's stores are issued at the top of
//      block b + 1, right after its first barrier, from registers reserved until block b + 1's
//      pass 3; stores at the end of their own block made the loop latch's copies of the
//      prefetched rows wait for them (vmcnt counts the stores issued after the loads).
template <int RW, bool SPANS, int DK, class SCHED, bool XW = false, class FIRV = NoFir, bool WFLAT = false,
          int PRIO = 0, int V = 0>
__device__ __forceinline__ void synth_wave_body(const SynthBlockArgs& a, int pol, int tg, const SCHED& sch) {
  constexpr int W = 16 * RW;
  constexpr bool KEPT = (V & 1) != 0, PP = (V & 2) != 0, DEFER = (V & 4) != 0;
  static_assert(RW <= 14 && RW % 2 == 0, "W = 16 RW with RW even and <= 14");
  static_assert(DK >= 1 && DK <= 16, "keep = 16 DK");
  static_assert(!KEPT || DK == 10, "KEPT: keep = 160, pass-3 registers [3, 13)");
  static_assert(!PP || !FIRV::kOn, "PP: stored stage-1 rows only");
  static_assert(!DEFER || (KEPT && !FIRV::kOn), "DEFER: KEPT stores of stored stage-1 rows");
  static_assert(!FIRV::kOn || !XW, "the FIR synthesis uses the in-wave pass-1 mapping");
  static_assert(!FIRV::kOn || FIRV::rows(0) <= kTilesB / 160, "FIR tile exceeds the phase tiles");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int l = XW ? (lane & 15) : lane >> 2;  // FFT lane within the phase (passes 1-2)
  const int cc = XW ? (lane >> 4) : lane & 3;  // phase within the wave (passes 1-2)
  const int col = wave * 4 + cc;               // phase within the workgroup (passes 1-2)
  auto cbase = [](int c) { return XW ? col_base_xw(c) : col_base(c); };
  const int N = a.N;
  const int nb = sch.count();
  if (nb <= 0) return;           // uniform per workgroup: no barrier is skipped by part of it
  const int t0g = tg * kCols;    // the workgroup's first output phase

  // ---- tables (once per launch): tw1[i][f1] = e^{-2 pi i i f1 / 256}, tw2[f1][t1a] =
  // e^{+2 pi i f1 t1a / W}, window transposed winT[i][r] = win[i + 16 r]
  for (int e = tid; e < 256; e += kWgThreads) {
    const int i = e >> 4, f = e & 15;
    *reinterpret_cast<float2*>(lds + kTw1Off + i * kRowB + f * 8) = a.twNf[(i * f) & 255];
    if (f < RW) {
      float2 w = a.twW[(i * f) % W];  // e^{-2 pi i m / W}: conjugate for the inverse
      w.y = -w.y;
      *reinterpret_cast<float2*>(lds + kTw2Off + i * kTw2RowB + f * 8) = w;
    }
    *reinterpret_cast<float*>(lds + kWinOff + i * kWinRowB + f * 4) = a.window[i + 16 * f];
  }
  // ---- lane constants: gain x four-step twiddle x output scale of the kept bins
  // j' = l + 16 r'' at phase t0g + col (table [j'][t0], scale folded on the host)
  float2 t4[RW];
  {
    const __amdgpu_buffer_rsrc_t tr = make_rsrc(a.tw4s + t0g, (uint32_t)((W - 1) * N + kCols) * 8u);
    static_for<0, RW>([&](auto r) {
      const v2u x = __builtin_amdgcn_raw_buffer_load_b64(tr, (uint32_t)(((l + 16 * r) * N + col) * 8), 0, 0);
      t4[r] = __builtin_bit_cast(float2, x);
    });
  }
  // (fused round trip: one wave waits for the first block's rows; the barrier releases the rest)
  if (wave == 0) sch.wait(sch.block(0));
  __syncthreads();  // tables staged

  // swap addresses (lane constants; the row / register offsets are immediates)
  const int wr = cbase(col) + 8 * l;                  // swap writes: slot l of rows 0..15
  // pass 1 (XW: its own lane mapping): FFT lane l1 of phase p1
  const int l1 = XW ? 4 * wave + ((lane >> 3) & 1) + 2 * (lane >> 5) : l;
  const int p1 = XW ? 2 * (lane & 7) + ((lane >> 4) & 1) : col;
  const int wr1 = cbase(p1) + 8 * l1;                 // swap-1 writes
  const int rd1 = cbase(col) + l * kRowB;             // swap 1 reads: row l
  int col2, j3;                                       // pass 3: phase, t1a = wave + 4 j3
  if constexpr (XW) pass3_role_xw(lane, col2, j3);
  else {
    col2 = lane & 15;
    j3 = lane >> 4;
  }
  const int t1a = wave + 4 * j3;                      // pass 3: t1a (valid below RW)
  const int rd2 = cbase(col2) + min(t1a, 15) * kRowB;
  const char* tw1row = lds + kTw1Off + l1 * kRowB;
  const char* tw2row = lds + kTw2Off + l * kTw2RowB;
  const char* winrow = lds + kWinOff + l1 * kWinRowB;

  // stage-1 rows in runs of ZB rows per phase (AnalysisArgs::zblk): row ZB g + gi of phase
  // t at Z[(g N + t) ZB + gi]; ZB = 1 is the plain [row][t0] layout.  Row 16 r + l of the
  // block: lane constant + r 16 N (the register's immediate)
  const int ZB = max(a.zblk, 1);
  const float2* zpol = a.Z + pol * a.z_pol_stride + (int64_t)(t0g + (XW ? 0 : wave * 4)) * ZB;
  const uint32_t zbytes = (tmask(a.timing_mask) & 1) ? 0u : (uint32_t)((16 * 16 * N) * 8);
  const uint32_t zlane = XW ? (uint32_t)((((l1 / ZB) * N) * ZB + p1 * ZB + l1 % ZB) * 8)
                            : (uint32_t)((((l / ZB) * N) * ZB + cc * ZB + l % ZB) * 8);
  float2* opol = a.out + pol * a.out_pol_stride;

  float2 x[16];  // raw Z values of the next block, rows l + 16 r

  // ---- FIR synthesis (FIRV::kOn): the lane's folded taps, its tile row offset, the input
  constexpr int NU = FIRV::NU, DE = FIRV::DE, PE = FIRV::PE, S = FIRV::kOn ? FIRV::S : 1;
  constexpr int RL = 16 - DK;  // first register row a later block computes (the others are reused)
  // (the taps are re-read from the L1/L2-resident table for every block: kept in registers
  // across the FFT passes they would push the kernel past the 168-VGPR budget of 3 waves
  // per SIMD)
  [[maybe_unused]] float g[PE];
  [[maybe_unused]] int fir_o = 0;
  [[maybe_unused]] const float* gl = nullptr;
  [[maybe_unused]] const __amdgpu_buffer_rsrc_t xr =
      FIRV::kOn ? make_rsrc(a.fir_x + pol * a.fir_x_pol_stride, (uint32_t)min(a.fir_n_dat * 8, (int64_t)kRsrcMaxBytes))
                : make_rsrc(a.Z, 0u);
  if constexpr (FIRV::kOn) {
    const int sr = l % NU;
    fir_o = DE * (l / NU) + (sr * DE) / NU;
    gl = a.fir_g + ((int64_t)sr * N + t0g + col) * 16;
  }
  auto load_taps = [&]() {  // the lane's PE taps: 16 contiguous floats, 4 x 16-B loads
    static_for<0, 4>([&](auto k) {
      const v4f q = *reinterpret_cast<const v4f*>(gl + 4 * decltype(k)::value);
      static_for<0, 4>([&](auto e) {
        constexpr int m = 4 * decltype(k)::value + decltype(e)::value;
        if constexpr (m < PE) g[m] = q[decltype(e)::value];
      });
    });
  };
  // input rows T0(b) + S r_lo + j (j = tid / 8 + 32 i), 16 B of the workgroup's 16 columns each
  auto tile_load = [&](int b, auto r_lo, v4u* pf) {
    constexpr int NL = FIRV::loads(decltype(r_lo)::value);
    const int64_t row0 = (int64_t)DE * (a.fir_q0 + (int64_t)(a.keep / NU) * b) + S * decltype(r_lo)::value;
    uint32_t o = (uint32_t)(((row0 + (tid >> 3)) * N + t0g + 2 * (tid & 7)) * 8);
    asm volatile("" : "+v"(o));  // (no per-load offsets hoisted out of the block loop)
    static_for<0, NL>([&](auto i) {
      pf[decltype(i)::value] =
          __builtin_amdgcn_raw_buffer_load_b128(xr, o + (uint32_t)(decltype(i)::value * 32 * N * 8), 0, 0);
    });
  };
  auto tile_store = [&](auto r_lo, const v4u* pf) {
    constexpr int NL = FIRV::loads(decltype(r_lo)::value);
    static_for<0, NL>([&](auto i) {
      const int j = (tid >> 3) + 32 * decltype(i)::value;
      *reinterpret_cast<v4u*>(lds + j * FIRV::RS + 16 * (tid & 7)) = pf[decltype(i)::value];
    });
  };
  // x[r], r >= r_lo, from the tile (tile row 0 = input row T0(b) + S r_lo); the FMA order of
  // the streaming analysis (m ascending from 0) with N^2-scaled taps: N^2 x its sums exactly
  auto fir_rows = [&](auto r_lo) {
    constexpr int R_LO = decltype(r_lo)::value;
    const char* tb = lds + fir_o * FIRV::RS + col * 8;
    v2f acc[16 - R_LO];
    static_for<0, 16 - R_LO>([&](auto rv) { acc[decltype(rv)::value] = v2f{0.f, 0.f}; });
    static_for<0, PE>([&](auto mv) {
      constexpr int m = decltype(mv)::value;
      static_for<0, 16 - R_LO>([&](auto rv) {
        constexpr int rr = decltype(rv)::value;
        const v2f xv = *reinterpret_cast<const v2f*>(tb + (rr * S + m) * FIRV::RS);
        acc[rr] = __builtin_elementwise_fma(v2f{g[m], g[m]}, xv, acc[rr]);
      });
    });
    static_for<0, 16 - R_LO>([&](auto rv) {
      constexpr int rr = decltype(rv)::value;
      x[R_LO + rr] = make_float2(acc[rr].x, acc[rr].y);
    });
  };

  // block b's rows into xd (xd[r] = xs[r + DK] for the reused rows, the others loaded)
  auto prefetch_into = [&](int b, auto reuse, float2 (&xs)[16], float2 (&xd)[16]) {
    constexpr int R0 = decltype(reuse)::value ? 16 - DK : 0;
    static_for<0, R0>([&](auto r) { xd[r] = xs[r + DK]; });
    const __amdgpu_buffer_rsrc_t z = make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes);
    static_for<R0, 16>([&](auto r) {
      const v2u v = __builtin_amdgcn_raw_buffer_load_b64(z, zlane, r * N * 16 * 8, SCHED::kLoadAux);
      xd[r] = __builtin_bit_cast(float2, v);
    });
  };
  auto prefetch = [&](int b, auto reuse) { prefetch_into(b, reuse, x, x); };
  [[maybe_unused]] v4u pf[FIRV::kOn ? FIRV::loads(RL) : 1];
  if constexpr (FIRV::kOn) {
    // first block: all 16 register rows from one tile (the phase tiles are not in use yet)
    v4u pf0[FIRV::loads(0)];
    tile_load(sch.block(0), std::integral_constant<int, 0>{}, pf0);
    load_taps();
    tile_store(std::integral_constant<int, 0>{}, pf0);
    __syncthreads();
    fir_rows(std::integral_constant<int, 0>{});
  } else {
    prefetch(sch.block(0), std::false_type{});
  }
  vm_drain();  // (no store wait at the loop head)

  // [[maybe_unused]]: the KEPT full-block store offset of the lane (fixed for the kernel)
  [[maybe_unused]] const int kept_lane = (t1a < RW) ? (t1a * N + t0g + col2) * 8 : (int)0x80000000;
  constexpr int TL = KEPT ? 3 : 0, TH = KEPT ? 13 : 16;  // pass-3 registers stored
  // block b's outputs: y[t - TL] = pass-3 register t of the lane
  auto store_block = [&](int b, const float2* y) {
    const int64_t ob = (a.block0 + b) * (int64_t)a.Lkeep;  // first kept output sample
    const int64_t avail = a.out_limit - ob;
    const int64_t nk = (tmask(a.timing_mask) & 2)
                           ? 0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
    const __amdgpu_buffer_rsrc_t o = make_rsrc(opol + ob, (uint32_t)nk * 8u);
    if (KEPT && nk == a.Lkeep) {  // uniform: a whole block, every kept output in range
      // output (t1a + RW t1b) N + t0 - L_ov = lane offset + (t1b - 3) RW N (scalar, >= 0)
      static_for<TL, TH>([&](auto t) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, y[t - TL]), o, (uint32_t)kept_lane,
                                              (decltype(t)::value - TL) * RW * N * 8, kAuxOut);
      });
    } else {
      // lanes t1a >= RW hold no output: their offsets leave the descriptor's range (as do
      // the discarded t1 < t1_lo, whose negative offsets wrap past 2^31)
      int base = (t1a < RW) ? (t1a * N - a.Lov + t0g + col2) * 8 : (int)0x80000000;
      // (FIR variant: recomputed every block — 16 hoisted store offsets would spill; KEPT: the
      // ragged last block only)
      if constexpr (FIRV::kOn || KEPT) asm volatile("" : "+v"(base));
      // (the whole offset in the lane register: the buffer range check covers the lane
      // offset, not a scalar offset, and discards the negative t1 < t1_lo offsets)
      static_for<TL, TH>([&](auto t) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, y[t - TL]), o,
                                              (uint32_t)(base + t * RW * N * 8), 0, kAuxOut);
      });
    }
  };
  [[maybe_unused]] float2 yprev[TH - TL];  // DEFER: the previous block's outputs
  // WFLAT: the lane's window values that are not exactly 1 (rows l + 16 r, r < 3 and r > 12),
  // held in registers for the whole launch (round 6: 2 LDS reads a block fewer)
  [[maybe_unused]] v4f wq0{}, wq3{};
  if constexpr (WFLAT) {
    wq0 = *reinterpret_cast<const v4f*>(winrow);
    wq3 = *reinterpret_cast<const v4f*>(winrow + 48);
  }
  // one block: pass 1 reads xc, block i + 1's rows go to xn (xn == xc without PP)
  auto run_block = [&](int i, float2 (&xc)[16], float2 (&xn)[16]) {
    const int b = sch.block(i);
    // every wave has read the previous block's swap-2 data (from all tiles), and the
    // four waves move through the Z and output lines together
    // (fused round trip: one wave waits for the next block's rows before the barrier, so
    // every wave may load them after it)
    if (wave == 0 && i + 1 < nb) sch.wait(sch.block(i + 1));
    // (PRIO & 32: this barrier moves down to just before the swap-1 writes — pass 1 touches
    // only the constant tables in LDS, so it may overlap other waves' pass 3)
    if constexpr (!(PRIO & 32)) wave_wg_sync<V>();
    if constexpr (DEFER) {
      if (i > 0) store_block(sch.block(i - 1), yprev);  // uniform per workgroup
    }
    if constexpr (PRIO & 1) __builtin_amdgcn_s_setprio(2);
    if constexpr (PRIO & 8) __builtin_amdgcn_s_setprio(3);
    if constexpr (PRIO & 16) __builtin_amdgcn_s_setprio(1);
    // ---- pass 1: taper, 16-point DFT over r, twiddle
    float2 v[16];
    if constexpr (WFLAT) {
      static_for<0, 16>([&](auto rv) {
        constexpr int r = decltype(rv)::value;
        if constexpr (r < 3) v[r] = cscale(xc[r], wq0[r]);
        else if constexpr (r > 12) v[r] = cscale(xc[r], wq3[r - 12]);
        else v[r] = xc[r];
      });
    } else {
      float wv[16];
      static_for<0, 4>([&](auto k) {
        const v4f q = *reinterpret_cast<const v4f*>(winrow + 16 * k);
        wv[4 * k] = q.x;
        wv[4 * k + 1] = q.y;
        wv[4 * k + 2] = q.z;
        wv[4 * k + 3] = q.w;
      });
      static_for<0, 16>([&](auto r) { v[r] = cscale(xc[r], wv[r]); });
    }
    // the next block's rows (the last block re-reads itself: the wait count stays fixed)
    if constexpr (FIRV::kOn)
      tile_load(sch.block(min(i + 1, nb - 1)), std::integral_constant<int, RL>{}, pf);
    else
      prefetch_into(sch.block(min(i + 1, nb - 1)), std::integral_constant<bool, (SCHED::kReuse && DK < 16)>{}, xc, xn);
    sdft<16, -1>(v);
    {
      float2 w[16];
      if constexpr ((V & 16) != 0) {  // (timing variant: a uniform twiddle, no table reads)
        static_for<0, 16>([&](auto k) { w[k] = make_float2(a.scale, a.scale); });
      } else {
        static_for<0, 8>([&](auto k) { lds_pair(tw1row + 16 * k, w[2 * k], w[2 * k + 1]); });
      }
      static_for<1, 16>([&](auto f) { v[f] = cmul(v[f], w[f]); });
    }
    if constexpr ((PRIO & 32) != 0) __syncthreads();
    // ---- swap 1 (inside the wave): element (row f1, slot l) of this phase's tile
    static_for<0, 16>([&](auto f) {
      constexpr int fr = decltype(f)::value;
      *reinterpret_cast<float2*>(lds + wr1 + fr * kRowB) = v[fr];
    });
    if constexpr (PRIO & 25) __builtin_amdgcn_s_setprio(0);
    if constexpr (XW) wave_wg_sync<V>();  // the phase tiles were written by every wave
    else __builtin_amdgcn_wave_barrier();
    if constexpr (PRIO & 4) __builtin_amdgcn_s_setprio(2);
    static_for<0, 8>([&](auto k) {
      lds_pair(lds + rd1 + 16 * k, v[2 * k], v[2 * k + 1]);
    });
    // ---- pass 2: 16-point DFT over i; kept bins x t4; RW-point IDFT; W-pass twiddle
    sdft<16, -1>(v);
    float2 u[RW];
    static_for<0, RW>([&](auto r) {
      constexpr int f2 = bin_of<RW, SPANS>(decltype(r)::value);
      u[r] = cmul(v[f2], t4[r]);
    });
    sdft<RW, +1>(u);
    {
      float2 w[RW];
      if constexpr ((V & 16) != 0) {
        static_for<0, RW>([&](auto k) { w[k] = make_float2(a.scale, a.scale); });
      } else {
        static_for<0, RW / 2>([&](auto k) { lds_pair(tw2row + 16 * k, w[2 * k], w[2 * k + 1]); });
      }
      static_for<1, RW>([&](auto t) { u[t] = cmul(u[t], w[t]); });
    }
    // ---- swap 2 (across the workgroup): element (row t1a, slot f1 = l) of this phase's
    // tile (the wave's own swap-1 reads of the tile are issued before these writes)
    __builtin_amdgcn_wave_barrier();
    static_for<0, RW>([&](auto t) {
      constexpr int tr = decltype(t)::value;
      *reinterpret_cast<float2*>(lds + wr + tr * kRowB) = u[tr];
    });
    if constexpr (PRIO & 4) __builtin_amdgcn_s_setprio(0);
    wave_wg_sync<V>();
    if constexpr (PRIO & 2) __builtin_amdgcn_s_setprio(2);
    static_for<0, 8>([&](auto k) {
      lds_pair(lds + rd2 + 16 * k, v[2 * k], v[2 * k + 1]);
    });
    // ---- pass 3: 16-point IDFT over f1 -> t1 = t1a + RW t1b; overlap-discard on the store
    // (KEPT: registers t1b outside [3, 13) are never read, so their outputs are not formed)
    if constexpr (DEFER) {
      // (the stored registers stay reserved until here — an empty use — so nothing else is
      // allocated into them while their stores are in flight)
#pragma unroll
      for (int t = 0; t < TH - TL; ++t) asm volatile("" ::"v"(yprev[t]));
    }
    sdft<16, +1>(v);
    if constexpr (DEFER) {
      static_for<TL, TH>([&](auto t) { yprev[t - TL] = v[t]; });
    } else {
      store_block(b, v + TL);
    }
    if constexpr (PRIO & 2) __builtin_amdgcn_s_setprio(0);
    if constexpr (FIRV::kOn) {
      if (i + 1 < nb) {  // uniform per workgroup
        // the next block: its first RL register rows are this block's last, the others come
        // from the input rows loaded above, staged in the phase tiles once every wave has
        // read its swap-2 data (the next iteration's first barrier orders the FIR reads
        // before that block's swap 1)
        static_for<0, RL>([&](auto r) { x[decltype(r)::value] = x[decltype(r)::value + DK]; });
        __syncthreads();
        load_taps();
        tile_store(std::integral_constant<int, RL>{}, pf);
        __syncthreads();
        fir_rows(std::integral_constant<int, RL>{});
      }
    }
  };
  if constexpr (PP) {
    float2 x2[16];
    int i = 0;
#pragma unroll 1
    for (; i + 1 < nb; i += 2) {
      run_block(i, x, x2);
      run_block(i + 1, x2, x);
    }
    if (i < nb) run_block(i, x, x2);  // uniform per workgroup
  } else {
#pragma unroll 1
    for (int i = 0; i < nb; ++i) run_block(i, x, x);
  }
  if constexpr (DEFER) store_block(sch.block(nb - 1), yprev);  // the range's last block
}

template <int RW, bool SPANS, int DK, bool XW = false, class FIRV = NoFir, bool WFLAT = false, int PRIO = 0,
          int V = 0>
__global__ __launch_bounds__(kWgThreads) __attribute__((amdgpu_waves_per_eu(3)))
void synth_wave_kernel(SynthBlockArgs a) {
  const int groups = a.N / kCols;
  const int lt = a.linear ? (int)blockIdx.x : xcd_tile(blockIdx.x, gridDim.x);
  const int rr = lt / groups;
  const int Rg = gridDim.x / groups;
  const int b_begin = (int)((int64_t)a.n_blocks * rr / Rg);
  const int b_end = (int)((int64_t)a.n_blocks * (rr + 1) / Rg);
  synth_wave_body<RW, SPANS, DK, RangeSched, XW, FIRV, WFLAT, PRIO, V>(a, blockIdx.y, lt % groups,
                                                                 RangeSched{b_begin, b_end - b_begin});
}

}  // namespace pfb
