// pfb_synth_wave512.hip — synthesis stage 2 for Nf = 512, W = 448 (SKA-Mid at OS 8/7, keep
// 256: Ov 128) with one output phase per 32 lanes (polyphase_synthesis.m:163-316,
// re-ordered as DESIGN.md §5 derives; the Nf = 256 counterpart is pfb_synth_wave.hip).
//
// Per block b and output phase t0 (one column of the stage-1 rows Z[row][t0]):
//   Nf-point FFT over time (taper on the way in), keep W bins, x gain x four-step twiddle
//   (x the output scale), W-point IFFT, overlap-discard.
// Lane m (< 32) of a phase holds 16 values at every stage:
//   pass 1   x[m + 32 r] (r < 16)          -> 16-point DFT over r, x w_512^{m f1}
//   swap 1   lane (f1, h) <- A_{l' + 16 h}[f1], l' < 16  (transpose through the wave's LDS)
//   pass 2   32-point DFT over m = l' + 16 h by decimation in frequency: one radix-2
//            butterfly across the lane pair h = 0/1 (DPP quad_perm: lane 2k <-> 2k+1), lane
//            g = h keeping the bins f2 = 2 f2'' + g, x w_32^{g l'}, 16-point DFT over l'
//            -> lane g holds the bins f = f1 + 16 (2 f2'' + g), f2'' < 16
//   select   registers f2'' in [0, 7) and [9, 16) of BOTH lanes are the kept bins; in W-bin
//            order they are j' = f1 + 16 r'' with r'' = g + 2 k, k < 14 (the W-point IFFT
//            is 16 x 28 and the lane holds the odd or even half of its 28-point group),
//            x t4[j'] (lane constants)
//   pass A   28-point IDFT over r'' by decimation in time: 14-point IDFT over k in
//            registers, x w_28^{+g t'}, radix-2 across the lane pair -> lane e holds
//            t1a = t' + 14 e; x e^{+2 pi i f1 t1a / W}
//   swap 2   (t1a, phase) <- Y_f1[t1a], f1 < 16, across the workgroup
//   pass B   16-point IDFT over f1          -> y[t1a + 28 t1b]; the kept outputs t1 in
//            [L_ov / N, W - L_ov / N) = [112, 336) are exactly t1b in [4, 12), so only those
//            8 of the 16 outputs are formed and stored.
// Both lane-pair butterflies compute self + sigma * partner in one fma per float (sigma = -1
// on the second lane of the pair); the sign that leaves on that lane's result is folded
// into its next twiddle table row, so no lane needs a select.
// A wave holds 2 phases (64 lanes), a 256-thread workgroup 8 adjacent phases; the
// workgroups of neighbouring phase groups run on the same XCD (64-B halves of every Z
// and output line).  Every twiddle is a table entry rounded once from double; the gain x
// twiddle x scale constants come from the plan's tw4s table, once per launch.
// Register budget: 3 waves per SIMD (<= 168 VGPRs); LDS 47 KB per workgroup (3 per CU).
// LDS layout (scripts/lds_bank_model.py; round 5): every swap access is bank-conflict-free —
// phase tiles 4624 B apart (1156 dwords: the 8 tiles of a swap-1 ds_write_b64 group on
// distinct 16-B bank quads), swap-1 rows [f1][h] 288 / 144 B apart, swap-2 row t1a at slot
// kSw2Row[t1a] (rows of 144 B): a ds_write_b64 group's two lane halves (e = 0 / 1) 576 B
// apart and each pass-B ds_read_b128 group's 4 rows x 4 phases on 16 distinct 16-B units
// (round 4: 37.6 % of the LDS cycles were bank conflicts, the model gives the same figure).
#include "pfb_common.hpp"

#include <cstdlib>

namespace pfb {

namespace {

constexpr int kW5Threads = 256;
constexpr int kW5Cols = 8;       // output phases per workgroup
constexpr int kRowB = 144;       // 16 values + 16 B
constexpr int kTileB = 2 * 16 * kRowB + 16;  // one phase: swap 1 [f1][h][l'] (f1 stride 288 B),
                                             // swap 2 row slots of 144 B (32 slots, 28 used)
// swap-2 row slot of t1a = t' + 14 e: sw2_slot(t') + 4 e (slots s with 9 s mod 16 in the
// pattern the pass-B read groups need, lds_bank_model.py)
constexpr int sw2_slot(int t) {
  constexpr int s[14] = {0, 16, 8, 24, 9, 25, 1, 2, 18, 10, 26, 11, 27, 3};
  return s[t];
}
// the same for a run-time t (< 28), from two packed constants (5 bits per slot)
constexpr uint64_t sw2_pack(int t0) {
  uint64_t v = 0;
  for (int i = 0; i < 7; ++i) v |= (uint64_t)sw2_slot(t0 + i) << (5 * i);
  return v;
}
__device__ __forceinline__ int sw2_slot_rt(int t1a) {
  const int tp = t1a % 14;
  const uint64_t pk = tp < 7 ? sw2_pack(0) : sw2_pack(7);
  return (int)((pk >> (5 * (tp % 7))) & 31u) + 4 * (t1a / 14);
}
constexpr int kTw1Off = kW5Cols * kTileB;          // [m][f1], 32 rows
constexpr int kTw32Off = kTw1Off + 32 * kRowB;     // [h][f2'], 2 rows
constexpr int kRow14B = 112;                       // 14 values
constexpr int kW28Off = kTw32Off + 2 * kRowB;      // [hi][r_a], 2 rows
constexpr int kTw2Off = kW28Off + 2 * kRow14B;     // [f1][e][t'], 32 rows
constexpr int kWinRowB = 80;                       // 16 floats + 16 B
constexpr int kWinOff = kTw2Off + 32 * kRow14B;    // [m][r], 32 rows
constexpr int kW5LdsB = kWinOff + 32 * kWinRowB;

__device__ __forceinline__ void lds_pair2(const char* p, float2& a, float2& b) {
  const v4f q = *reinterpret_cast<const v4f*>(p);
  a = make_float2(q.x, q.y);
  b = make_float2(q.z, q.w);
}

// a + sg * (the value of the other lane of the pair, lane ^ 1): ONE v_fmac_f32 with the DPP
// swizzle quad_perm:[1,0,3,2] on its first source (the compiler does not fuse a separate
// v_mov_b32_dpp into the fma: 30 VALU instructions a block saved; its hazard recognizer
// places the wait states the DPP read needs)
__device__ __forceinline__ float pair_fma(float a, float sg) {
  float r;
  asm("v_fmac_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(a), "v"(sg), "0"(a));
  return r;
}
// self + sg * partner
__device__ __forceinline__ float2 pair_bfly(float2 a, float sg) {
  return make_float2(pair_fma(a.x, sg), pair_fma(a.y, sg));
}

// v[i] *= row[i], i < 2 NP (one ds_read_b128 per pair, multiplied as it arrives; TM bit 4,
// a compile-time timing variant of the experiments build: a uniform value u instead)
template <int NP, int TM = 0>
__device__ __forceinline__ void twiddle_rows(float2* v, const char* row, float u = 0.f) {
  static_for<0, NP>([&](auto k) {
    float2 w0, w1;
    if constexpr ((TM & 16) != 0) {
      w0 = w1 = make_float2(u, u);
    } else {
      lds_pair2(row + 16 * k, w0, w1);
    }
    v[2 * k] = cmul(v[2 * k], w0);
    v[2 * k + 1] = cmul(v[2 * k + 1], w1);
  });
}

// y[j] = sum_f v[f] e^{+2 pi i f (4 + j) / 16}, j < 8: outputs 4 .. 11 of the 16-point
// inverse DFT — sdft<16, +1>'s 4 x 4 split (output k1 + 4 k2) with only k2 = 1, 2 formed
__device__ __forceinline__ void idft16_mid8(const float2* v, float2* y) {
  float2 t[4][4];
  static_for<0, 4>([&](auto n1) {
    constexpr int a1 = decltype(n1)::value;
    static_for<0, 4>([&](auto n2) { t[a1][decltype(n2)::value] = v[4 * decltype(n2)::value + a1]; });
    sdft<4, +1>(t[a1]);
    static_for<1, 4>([&](auto k1) {
      t[a1][decltype(k1)::value] = ctw<a1 * decltype(k1)::value, 16, +1>(t[a1][decltype(k1)::value]);
    });
  });
  static_for<0, 4>([&](auto k1) {
    constexpr int c1 = decltype(k1)::value;
    // X[1] = (z0 - z2) + i (z1 - z3), X[2] = (z0 + z2) - (z1 + z3) of z[n1] = t[n1][k1]
    const float2 d02 = csub(t[0][c1], t[2][c1]), s02 = cadd(t[0][c1], t[2][c1]);
    const float2 d13 = crot90<+1>(csub(t[1][c1], t[3][c1])), s13 = cadd(t[1][c1], t[3][c1]);
    y[c1] = cadd(d02, d13);       // t1b = 4 + k1
    y[4 + c1] = csub(s02, s13);   // t1b = 8 + k1
  });
}

}  // namespace

// XW: pass-1 lanes (phase p, FFT lane m) spread over the workgroup (lane = 8 (m mod 8) + p in
// wave m / 8): one Z load instruction reads 8 rows x the 8 phases (64-B runs) instead of 32
// rows x 2 phases, and swap 1 crosses waves (one more workgroup barrier per block)
// WFLAT: the temporal window is exactly 1 on rows [128, 384) (tukey with Ov <= 128,
// SynthBlockArgs::win_flat): registers r = 4 .. 11 (rows m + 32 r) skip the multiply (exact)
// PRIO: as synth_wave_kernel (1: issue priority 2 from the loop-top barrier to the swap-1
// barrier)
// DEFER (round 5): block b's 8 output stores are issued at the top of block b + 1 (right
// after its first barrier), from registers that stay live until block b + 1's pass B.  The
// compiler makes any write to a register that is still the data source of an outstanding
// buffer store wait for that store (vmcnt); with the stores at the end of their own block,
// the next block's first register writes waited at the loop top for the stores it had just
// issued (s_waitcnt vmcnt(0) there) — a store round trip per block, exposed.
// TM: compile-time timing variants (experiments build only, results invalid): 8 wave
// barriers instead of the block loop's workgroup barriers, 16 a uniform twiddle instead of
// the four LDS twiddle tables
// CT (round 6): the two lane-pair twiddles (pass 2's -w_32^{l'} and pass A's w_28^{+t'}) are
// 1 on lane h = 0 and a compile-time constant per register on lane h = 1, so lane h = 1
// multiplies by compile-time constants (ctw: quarter turns exact, the others rounded once
// from double) under an exec mask and lane h = 0 skips them — 15 of the block's 30 twiddle
// ds_read_b128 gone, no VALU added.  (Before: rows [h][l'] of two LDS tables.)
template <bool SPANS, bool XW, bool WFLAT = false, int PRIO = 0, bool DEFER = true, int TM = 0, bool CT = true>
__global__ __launch_bounds__(kW5Threads) __attribute__((amdgpu_waves_per_eu(3)))
void synth_wave512_kernel(SynthBlockArgs a) {
  constexpr int W = 448, DK = 8;  // keep = 256 rows = 8 register rows of 32
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int N = a.N;
  const int groups = N / kW5Cols;
  const int lt = a.linear ? (int)blockIdx.x : xcd_tile(blockIdx.x, gridDim.x);
  const int rr = lt / groups;
  const int Rg = gridDim.x / groups;
  const int b_begin = (int)((int64_t)a.n_blocks * rr / Rg);
  const int b_end = (int)((int64_t)a.n_blocks * (rr + 1) / Rg);
  const int nb = b_end - b_begin;
  if (nb <= 0) return;  // uniform per workgroup
  const int t0g = (lt % groups) * kW5Cols;
  const int pol = blockIdx.y;

  // ---- tables (once per launch)
  for (int e = tid; e < 512; e += kW5Threads) {
    const int i = e >> 4, f = e & 15;  // i < 32
    *reinterpret_cast<float2*>(lds + kTw1Off + i * kRowB + f * 8) = a.twNf[(i * f) & 511];
    *reinterpret_cast<float*>(lds + kWinOff + i * kWinRowB + f * 4) = a.window[i + 32 * f];
    if (i < 2) {
      // pass-2 pair butterfly: lane 1 holds A_hi - A_lo, x -w_32^{l'} = (A_lo - A_hi) w_32^{l'}
      const float2 w = a.twNf[16 * f];
      *reinterpret_cast<float2*>(lds + kTw32Off + i * kRowB + f * 8) =
          i ? make_float2(-w.x, -w.y) : make_float2(1.f, 0.f);
      if (f < 14) {
        const float2 v = a.twW[16 * f];  // e^{-2 pi i f / 28}; the inverse takes its conjugate
        *reinterpret_cast<float2*>(lds + kW28Off + i * kRow14B + f * 8) =
            i ? make_float2(v.x, -v.y) : make_float2(1.f, 0.f);
      }
    }
  }
  // W-pass twiddle e^{+2 pi i f1 t1a / W}, t1a = t + 14 e; x -1 on e = 1 (the pass-A pair
  // butterfly leaves -Y there)
  for (int e = tid; e < 16 * 2 * 14; e += kW5Threads) {
    const int f1 = e / 28, q = e % 28, ee = q / 14, t = q % 14;
    const float2 w = a.twW[(f1 * (t + 14 * ee)) % W];
    *reinterpret_cast<float2*>(lds + kTw2Off + (2 * f1 + ee) * kRow14B + t * 8) =
        ee ? make_float2(-w.x, w.y) : make_float2(w.x, -w.y);
  }

  // lane roles.  Pass 1 / swap-1 writes: phase c1, FFT lane m.  Pass 2 to swap-2 writes:
  // (ph, f1, h) with lane = 32 ph + 2 f1 + h, phase col = 2 wave + ph.  Pass B: (col2, t1a).
  const int ph = lane >> 5;
  const int m = XW ? 8 * wave + (lane >> 3) : lane & 31;
  const int c1 = XW ? (lane & 7) : 2 * wave + ph;
  const int col = 2 * wave + ph;
  const int h = lane & 1;
  const int f1 = (lane >> 1) & 15;
  const float sg = h ? -1.f : 1.f;     // pair butterflies: self + sg * partner
  const int tile = col * kTileB;

  // ---- lane constants: gain x four-step twiddle x output scale of the lane's kept bins
  // j' = f1 + 16 (h + 2 k), k < 14
  float2 t4[14];
  {
    const __amdgpu_buffer_rsrc_t tr = make_rsrc(a.tw4s + t0g, (uint32_t)((W - 1) * N + kW5Cols) * 8u);
    static_for<0, 14>([&](auto k) {
      const int jp = f1 + 16 * (h + 2 * decltype(k)::value);
      const v2u x = __builtin_amdgcn_raw_buffer_load_b64(tr, (uint32_t)((jp * N + col) * 8), 0, 0);
      t4[decltype(k)::value] = __builtin_bit_cast(float2, x);
    });
  }
  __syncthreads();  // tables staged

  const int wr1 = c1 * kTileB + (m >> 4) * kRowB + (m & 15) * 8;  // swap-1 writes (+ f1 * 288)
  const int rd1 = tile + f1 * (2 * kRowB) + h * kRowB;     // swap-1 reads (+ 16 k)
  const int wr2 = tile + h * (4 * kRowB) + f1 * 8;         // swap-2 writes (+ sw2_slot(t') * 144)
  const int col2 = lane & 7;
  const int t1a = (lane >> 3) < 7 ? 7 * wave + (lane >> 3) : 28;  // 28: no output (8 lanes a wave)
  // (the idle lanes read the row of t1a = 7 wave + 6: a slot their read groups leave free)
  const int rd2 = col2 * kTileB + sw2_slot_rt(t1a < 28 ? t1a : 7 * wave + 6) * kRowB;  // (+ 16 k)
  const char* tw1row = lds + kTw1Off + m * kRowB;
  const char* tw32row = lds + kTw32Off + h * kRowB;
  const char* w28row = lds + kW28Off + h * kRow14B;
  const char* tw2row = lds + kTw2Off + (2 * f1 + h) * kRow14B;
  const char* winrow = lds + kWinOff + m * kWinRowB;

  const float2* zpol = a.Z + pol * a.z_pol_stride + (a.zblk == 2 ? 2 * t0g : t0g);
  const uint32_t zbytes = (tmask(a.timing_mask) & 1) ? 0u : (uint32_t)((511 * N + kW5Cols) * 8);
  // (zblk 2: Z rows in 2-row runs per column, z_index — lanes m and m + 1 read one 16-B pair,
  // a load instruction 4 whole 128-B lines of 2 rows x 8 phases instead of 8 half lines; the
  // row offsets 32 r N are pair-aligned, the same bytes either way)
  const uint32_t zlane = a.zblk == 2 ? (uint32_t)(((((m >> 1) * N + c1) << 1) + (m & 1)) * 8)
                                     : (uint32_t)((m * N + c1) * 8);
  float2* opol = a.out + pol * a.out_pol_stride;

  float2 x[16];  // raw Z values of the next block, rows m + 32 r
  auto prefetch = [&](int b, auto reuse) {
    constexpr int R0 = decltype(reuse)::value ? 16 - DK : 0;
    static_for<0, R0>([&](auto r) { x[r] = x[r + DK]; });
    const __amdgpu_buffer_rsrc_t z = make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes);
    static_for<R0, 16>([&](auto r) {
      const v2u v = __builtin_amdgcn_raw_buffer_load_b64(z, zlane, r * 32 * N * 8, kNtlW5 ? 2 : 0);
      x[r] = __builtin_bit_cast(float2, v);
    });
  };
  prefetch(b_begin, std::false_type{});
  // (the first block's rows are complete before the loop: no wait for the previous block's
  // stores at the loop head — vm_drain)
  vm_drain();

  // output stores of one block: y[t] = y[t1a + 28 (t1b - 4)] of phase t0g + col2, t1b in [4, 12)
  // (lanes t1a >= 28 hold no output: their offsets leave the descriptor's range; the whole
  // offset is in the lane register — the buffer range check covers the lane offset, not a
  // scalar offset, so a ragged last block drops its tail stores)
  const int obase = (t1a < 28) ? (t1a * N + t0g + col2) * 8 : (int)0x80000000;
  // a block's kept outputs end exactly at L_keep (t1a + 28 (t1b - 4) <= 223): for a whole
  // block the row offsets t 28 N 8 can be scalar offsets and the lane offset register stays
  // the same for the whole kernel (a store's address register rewritten while the store is
  // in flight makes the compiler wait for it too); a ragged last block (nk < L_keep) keeps
  // the whole offset in the range-checked lane register
  auto out_nk = [&](int b) {
    const int64_t ob = (a.block0 + b) * (int64_t)a.Lkeep;  // first kept output sample
    const int64_t avail = a.out_limit - ob;
    return (tmask(a.timing_mask) & 2) ? (int64_t)0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
  };
  auto store_block = [&](int b, const float2* yv) {
    const int64_t nk = out_nk(b);
    const __amdgpu_buffer_rsrc_t o = make_rsrc(opol + (a.block0 + b) * (int64_t)a.Lkeep, (uint32_t)nk * 8u);
    if (nk == a.Lkeep) {  // uniform
      static_for<0, 8>([&](auto t) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, yv[t]), o, (uint32_t)obase,
                                              t * 28 * N * 8, kNtW5 ? 2 : 0);
      });
    } else {
      int base = obase;
      asm volatile("" : "+v"(base));
      static_for<0, 8>([&](auto t) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, yv[t]), o,
                                              (uint32_t)(base + t * 28 * N * 8), 0, kNtW5 ? 2 : 0);
      });
    }
  };
  [[maybe_unused]] float2 yprev[8];
  // WFLAT: the lane's 8 window values that are not exactly 1 (rows m + 32 r, r < 4 and
  // r >= 12), held in registers for the whole launch (round 6: 2 LDS reads a block fewer)
  [[maybe_unused]] v4f wq0{}, wq3{};
  if constexpr (WFLAT) {
    wq0 = *reinterpret_cast<const v4f*>(winrow);
    wq3 = *reinterpret_cast<const v4f*>(winrow + 48);
  }

#pragma unroll 1
  for (int i = 0; i < nb; ++i) {
    const int b = b_begin + i;
    // every wave has read the previous block's swap-2 data (from all tiles)
    wave_wg_sync<TM>();
    if constexpr (DEFER) {
      if (i > 0) store_block(b - 1, yprev);  // uniform per workgroup
    }
    if constexpr (PRIO & 1) __builtin_amdgcn_s_setprio(2);
    // ---- pass 1: taper, 16-point DFT over r, x w_512^{m f1}
    float2 v[16];
    if constexpr (WFLAT) {
      static_for<0, 16>([&](auto rv) {
        constexpr int r = decltype(rv)::value;
        if constexpr (r < 4) v[r] = cscale(x[r], wq0[r]);            // r < 4
        else if constexpr (r >= 12) v[r] = cscale(x[r], wq3[r - 12]);  // r >= 12
        else v[r] = x[r];
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
      static_for<0, 16>([&](auto r) { v[r] = cscale(x[r], wv[r]); });
    }
    // the next block's rows (the last block re-reads itself: the wait count stays fixed)
    prefetch(min(b + 1, b_end - 1), std::true_type{});
    sdft<16, -1>(v);
    twiddle_rows<8, TM>(v, tw1row, a.scale);
    // ---- swap 1 (inside the wave): A_m[f1] -> tile[f1][m >> 4][m & 15]
    static_for<0, 16>([&](auto f) {
      *reinterpret_cast<float2*>(lds + wr1 + decltype(f)::value * (2 * kRowB)) = v[decltype(f)::value];
    });
    if constexpr (PRIO & 1) __builtin_amdgcn_s_setprio(0);
    if constexpr (XW) wave_wg_sync<TM>();  // the phase tiles were written by every wave
    else __builtin_amdgcn_wave_barrier();
    static_for<0, 8>([&](auto k) { lds_pair2(lds + rd1 + 16 * k, v[2 * k], v[2 * k + 1]); });
    // ---- pass 2: radix-2 across the lane pair (m = l' + 16 h), x (-)w_32^{g l'},
    // 16-point DFT over l'
    static_for<0, 16>([&](auto l) { v[l] = pair_bfly(v[l], sg); });
    if constexpr (CT && !(TM & 16)) {
      // lane h = 1: x -w_32^{l'} = e^{-2 pi i (l' + 16) / 32}
      if (h) static_for<0, 16>([&](auto l) { v[l] = ctw<decltype(l)::value + 16, 32, -1>(v[l]); });
    } else {
      twiddle_rows<8, TM>(v, tw32row, a.scale);
    }
    sdft<16, -1>(v);
    // ---- kept bins (registers f2'' < 7 and >= 9) x t4, 14-point IDFT over k,
    // x w_28^{g t'}, radix-2 across the pair, x e^{+2 pi i f1 t1a / W}
    float2 u[14];
    static_for<0, 14>([&](auto k) {
      constexpr int kk = decltype(k)::value;
      // spans: k < 7 <-> f2'' = k (f < 224), k >= 7 <-> f2'' = k + 2 (f >= 288);
      // critical: the halves swap (j' = f + 224 / f - 288)
      constexpr int reg = SPANS ? (kk < 7 ? kk : kk + 2) : (kk < 7 ? kk + 9 : kk - 7);
      u[kk] = cmul(v[reg], t4[kk]);
    });
    sdft<14, +1>(u);
    if constexpr (CT && !(TM & 16)) {
      // lane h = 1: x e^{+2 pi i t' / 28}
      if (h) static_for<0, 14>([&](auto t) { u[t] = ctw<decltype(t)::value, 28, +1>(u[t]); });
    } else {
      twiddle_rows<7, TM>(u, w28row, a.scale);
    }
    static_for<0, 14>([&](auto t) { u[t] = pair_bfly(u[t], sg); });
    twiddle_rows<7, TM>(u, tw2row, a.scale);
    // ---- swap 2 (across the workgroup): Y_f1[t1a = t' + 14 e] -> tile[t1a][f1] (the wave's
    // own swap-1 reads of the tile are issued before these writes)
    __builtin_amdgcn_wave_barrier();
    static_for<0, 14>([&](auto t) {
      *reinterpret_cast<float2*>(lds + wr2 + sw2_slot(decltype(t)::value) * kRowB) = u[decltype(t)::value];
    });
    wave_wg_sync<TM>();
    static_for<0, 8>([&](auto k) { lds_pair2(lds + rd2 + 16 * k, v[2 * k], v[2 * k + 1]); });
    // ---- pass B: 16-point IDFT over f1 -> t1 = t1a + 28 t1b, only t1b in [4, 12) (the kept
    // outputs: L_ov = 112 N); stored as output sample (t1a + 28 (t1b - 4)) N + t0
    if constexpr (DEFER) {
      // (the stored registers stay reserved until here — an empty use — so nothing else is
      // allocated into them while their stores are in flight: no store wait in this block)
#pragma unroll
      for (int t = 0; t < 8; ++t) asm volatile("" ::"v"(yprev[t]));
      idft16_mid8(v, yprev);
    } else {
      float2 y[8];
      idft16_mid8(v, y);
      store_block(b, y);
    }
  }
  if constexpr (DEFER) store_block(b_end - 1, yprev);  // the range's last block
}

bool synth_wave512_supported(const SynthBlockArgs& a) {
  // (PFB_SYNTH_WAVE512=0: the block kernel, experiments build — checked here so the round
  // trip's 2-row Z layout, which only this kernel reads, is turned off with it)
  static const bool no_w5 = knob("PFB_SYNTH_WAVE512") && std::atoi(knob("PFB_SYNTH_WAVE512")) == 0;
  if (no_w5) return false;
  // (32-bit byte offsets: 512 rows x N phases x 8 B per block stay below 2^31)
  // (L_ov = 112 N: pass B forms and stores only t1b in [4, 12))
  return a.Nf == 512 && a.W == 448 && a.keep == 256 && (a.zblk <= 2) && a.N % kW5Cols == 0 &&
         a.N <= 65536 && a.tw4s != nullptr && a.Lov == 112 * a.N;
}

template <bool SPANS, bool XW, bool WFLAT = false>
static hipError_t launch_w5(const SynthBlockArgs& a, hipStream_t s) {
  auto kern = synth_wave512_kernel<SPANS, XW, WFLAT>;
  if constexpr (kExperiments && XW && WFLAT) {
    // (PFB_W5_CT=0: the lane-pair twiddles from the LDS tables — experiments build only)
    static const bool noct = knob("PFB_W5_CT") && std::atoi(knob("PFB_W5_CT")) == 0;
    if (noct) kern = synth_wave512_kernel<SPANS, XW, WFLAT, 0, true, 0, false>;
    // (PFB_W5_DEFER=0: stores at the end of their own block — experiments build only)
    static const bool nodefer = knob("PFB_W5_DEFER") && std::atoi(knob("PFB_W5_DEFER")) == 0;
    if (nodefer) kern = synth_wave512_kernel<SPANS, XW, WFLAT, 0, false>;
    // (PFB_W5_TM=8/16/24: the timing variants, results invalid)
    static const int tm = knob("PFB_W5_TM") ? std::atoi(knob("PFB_W5_TM")) : 0;
    if (tm == 8) kern = synth_wave512_kernel<SPANS, XW, WFLAT, 0, true, 8>;
    if (tm == 16) kern = synth_wave512_kernel<SPANS, XW, WFLAT, 0, true, 16>;
    if (tm == 24) kern = synth_wave512_kernel<SPANS, XW, WFLAT, 0, true, 24>;
  }
  // (PFB_W5_LDS_PAD: extra LDS per workgroup, so fewer workgroups fit a CU — the occupancy
  // slope, experiments build only)
  size_t lds = kW5LdsB;
  if constexpr (kExperiments) {
    static const int pad = knob("PFB_W5_LDS_PAD") ? std::atoi(knob("PFB_W5_LDS_PAD")) : 0;
    if (pad > 0) lds += (size_t)pad;
  }
  hipError_t e = set_lds(kern, lds);
  if (e != hipSuccess) return e;
  const int groups = a.N / kW5Cols;
  // resident workgroups: 3 per CU; ranges so that the grid is about two rounds of them
  const int slots = cu_count() * 3;
  int ranges = std::max(1, (2 * slots + groups * a.n_pol - 1) / (groups * a.n_pol));
  static const int env_r = knob("PFB_W5_RANGES") ? std::atoi(knob("PFB_W5_RANGES")) : 0;  // A/B
  if (env_r > 0) ranges = env_r;
  ranges = std::min(ranges, a.n_blocks);
  SynthBlockArgs b = a;
  if constexpr (kExperiments) {  // (PFB_W5_LINEAR=1: linear workgroup order, A/B)
    static const int lin = knob("PFB_W5_LINEAR") ? std::atoi(knob("PFB_W5_LINEAR")) : -1;
    if (lin >= 0) b.linear = lin;
  }
  dim3 grid((unsigned)(groups * ranges), (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(kW5Threads), lds, s, b);
}

hipError_t launch_synth_wave512(const SynthBlockArgs& a, hipStream_t s) {
  if (a.n_blocks <= 0) return hipSuccess;
  if (!synth_wave512_supported(a)) return hipErrorInvalidValue;
  // (PFB_W5_XW=0: pass-1 lanes inside one wave per phase pair, experiments build A/B)
  static const bool xw = !(knob("PFB_W5_XW") && std::atoi(knob("PFB_W5_XW")) == 0);
  // (PFB_WAVE_WFLAT=0: the general taper, experiments A/B)
  static const bool wf_off = knob("PFB_WAVE_WFLAT") && std::atoi(knob("PFB_WAVE_WFLAT")) == 0;
  if (a.win_flat && !wf_off)
    return a.spans ? launch_w5<true, true, true>(a, s) : launch_w5<false, true, true>(a, s);
  if (!kExperiments || xw) return a.spans ? launch_w5<true, true>(a, s) : launch_w5<false, true>(a, s);
  return a.spans ? launch_w5<true, false>(a, s) : launch_w5<false, false>(a, s);
}

}  // namespace pfb
