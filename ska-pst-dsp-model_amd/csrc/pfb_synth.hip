// pfb_synth.hip — synthesis stage 2 (polyphase_synthesis.m:163-316, re-ordered; see
// DESIGN.md §5): per block x group of output phases t0, Nf-point FFT over time, kept-bin
// selection with deripple and the four-step twiddle, W-point inverse FFT,
// overlap-discard and the 1/L * de/nu scale.
#include "pfb_common.hpp"

namespace pfb {

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
  // pair-row strides (16-byte slots): N + 7 minimises ds_read/write_b128 bank conflicts
  // of the radix-16 passes of the SKA-Low shapes; the SKA-Mid plan (Nf 512 = 8 x 4 x 16,
  // W 448 = 14 x 8 x 4, 4 pair rows) is conflict-free except its fused reads with
  // Nf + 2 / W + 4 (LDS bank model over every pass's lane groups)
  static constexpr int RSF = NF + (NF == 512 ? 2 : 7);
  static constexpr int RSW = W + (W == 448 ? 4 : 7);
  static constexpr int RSMAX = RSF > RSW ? RSF : RSW;
  static constexpr int TWOFF = PAIRS * RSMAX * 2;  // float2 offset of the twiddle tables
  static constexpr size_t lds_bytes =
      (size_t)(TWOFF + tw_slots(NF) + tw_slots(W)) * sizeof(float2) + NF * sizeof(float);
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

// first Nf-point pass input from prefetched registers, kept in memory order until used:
// from_interleaved's v_swap_b32 is inline asm, so converting at load time would make
// the wave wait for the HBM prefetch right after issuing it
template <int PER, int R>
struct PairRegsIn {
  static constexpr bool kIsLds = false;
  const v4f (&zv)[PER][R];
  const float* win;
  template <class P, class RR>
  __device__ __forceinline__ cpx2 load(int, int tau, P, RR) const {
    return cscale(from_interleaved(zv[P::value][RR::value]), win[tau]);
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

// P16: the kept range of every block ends on a pair boundary (even output limit), so
// one 16-byte store per sample pair is dropped or kept as a whole exactly when its two
// samples are (t0 + 2q and Lkeep are even); otherwise two range-checked 8-byte stores.
template <bool P16>
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
    // negative offsets (t1 < t1_lo, q = kDropPair) wrap past 2^31 bytes and are dropped
    // by the range check
    const int off = ((t1 - t1_lo) * N + t0 + 2 * q) * 8;
    const Interleaved y = to_interleaved(cscale(v, scale));
    if constexpr (P16) {
      // (t0 + 2q even, nk even): a pair never straddles the range end, so the 16-byte
      // store is dropped or kept as a whole exactly when its two samples are
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(v4u, v4f{y.lo.x, y.lo.y, y.hi.x, y.hi.y}), o, off, 0, 0);
    } else {
      __builtin_amdgcn_raw_buffer_store_b64(as_u(y.lo), o, off, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b64(as_u(y.hi), o1, off, 0, 0);
    }
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

// Overlap-reuse instance per transform size: DK = keep / (NF / R1) for the configured
// overlap (SKA-Low Nf 256 / Ov 48: keep 160; 'test' Nf 128 / Ov 16: keep 96; SKA-Mid
// Nf 512 / Ov 128: keep 256).  Other overlaps run the plain persistent instance.
template <int NF, int W>
constexpr int synth_reuse_dk() {
  if constexpr (NF == 256) return 10;
  else if constexpr (NF == 128) return 6;
  else if constexpr (NF == 512) return 4;
  else return 0;
}

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
// (memory order; converted where the fused pass uses them, see PairRegsIn)
template <int NBL, int RW1, int PAIRS, int NTH>
__device__ __forceinline__ void load_t4(v4f (&t4)[(PAIRS * NBL + NTH - 1) / NTH][RW1],
                                        __amdgpu_buffer_rsrc_t tr, int N, int tid) {
  constexpr int TOT = PAIRS * NBL;
  static_for<0, (TOT + NTH - 1) / NTH>([&](auto p) {
    const int b = min(tid + p * NTH, TOT - 1);
    const int q = b % PAIRS, j = b / PAIRS;
    static_for<0, RW1>([&](auto rr) {
      const v4u x = __builtin_amdgcn_raw_buffer_load_b128(tr, ((j + NBL * rr) * N + 2 * q) * 8, 0, 0);
      t4[p][rr] = __builtin_bit_cast(v4f, x);
    });
  });
}

// the same from the workgroup's LDS copy of its TG columns of the table ([j'][pair q])
template <int NBL, int RW1, int PAIRS, int NTH>
__device__ __forceinline__ void load_t4_lds(v4f (&t4)[(PAIRS * NBL + NTH - 1) / NTH][RW1],
                                            const v4f* t4l, int tid) {
  constexpr int TOT = PAIRS * NBL;
  static_for<0, (TOT + NTH - 1) / NTH>([&](auto p) {
    const int b = min(tid + p * NTH, TOT - 1);
    const int q = b % PAIRS, j = b / PAIRS;
    static_for<0, RW1>([&](auto rr) { t4[p][rr] = t4l[(j + NBL * rr) * PAIRS + q]; });
  });
}

// Last Nf-point pass (forward, radix RL, NS = NBL) + kept-bin selection + gain x
// twiddle + first W-point pass (inverse, radix RW1, NS = 1), LDS rowsF -> LDS rowsW
// (in place; one barrier between the loads and the stores).
template <int NF, int W, int RL, bool SPANS, int PAIRS, int NTH>
__device__ __forceinline__ void fused_select_pass(const LdsPairs& rowsF, const LdsPairs& rowsW,
                                                  const float2* __restrict__ twF,
                                                  const v4f (&t4)[(PAIRS * (NF / RL) + NTH - 1) / NTH]
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
      float2 w[RL];
      twiddle_powers<RL, -1>(twF, j, w);
      static_for<1, RL>([&](auto r) { v[p][r] = cmul(v[p][r], w[r]); });
      sdft<RL, -1>(v[p]);
      cpx2 u[RW1];
      static_for<0, RW1>([&](auto rr) {
        constexpr int r = fused_src<NF, W, NBL, SPANS>(decltype(rr)::value);
        u[rr] = cmul(v[p][r], from_interleaved(t4[p][rr]));
      });
      sdft<RW1, +1>(u);
      static_for<0, RW1>([&](auto rr) { rowsW.store(q, j * RW1 + rr, u[rr], p, rr); });
    }
  });
}

// PERSIST: workgroup (tg, rr) walks a range of blocks and prefetches the next one's
// first-pass inputs into registers while it transforms the current one.
// DK > 0 (keep = DK * NF / R1): consecutive blocks overlap by 2 Ov = NF - keep rows, and
// first-pass register r of a thread holds row j + r NF/R1 — so the next block's
// registers 0 .. R1-DK-1 are this block's registers DK .. R1-1: they move in registers
// and only DK of the R1 rows are read from HBM (the 2 Ov overlap re-read disappears).
// T4L: the workgroup's TG columns of the gain x twiddle table are copied to LDS once
// and read from there every block (SKA-Mid: the 14.7 MB table was re-read from L2/MALL
// for each of a workgroup's blocks; only where the copy keeps 4 workgroups per CU).
template <int NF, int W, int PAIRS, bool SPANS, bool PERSIST, int DK = 0, bool P16 = false,
          bool T4L = false, int NTPW = NTP>
__global__ __launch_bounds__(NTPW) __attribute__((amdgpu_waves_per_eu(2))) void synth_block_kernel(SynthBlockArgs a) {
  using SS = SynthPairShape<NF, W, PAIRS>;
  using SP = SynthPlan<NF, W>;
  constexpr int R1 = synth_first_radix<NF, W>();
  constexpr int NB1 = NF / R1;
  constexpr int TG = 2 * PAIRS;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int tid = threadIdx.x;
  const int N = a.N;
  const int groups = N / TG;
  // XCD-aware: consecutive phase groups (which share Z and output cache lines when
  // TG * 8 B < 128 B, e.g. SKA-Mid's TG = 4) land on the same XCD and its L2
  const int lt = a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tg = lt % groups;
  const int rr = lt / groups;
  const int Rg = gridDim.x / groups;
  // PERSIST: a contiguous range of blocks per workgroup.  (Strided assignment rr + k Rg
  // keeps the 2 Ov overlap rows in L2, -30 % HBM reads, but measured 10 % slower.)
  const int b_begin = PERSIST ? (int)((int64_t)a.n_blocks * rr / Rg) : rr;
  const int b_end = PERSIST ? (int)((int64_t)a.n_blocks * (rr + 1) / Rg) : rr + 1;
  const int b_step = 1;
  if (b_begin >= b_end) return;
  const int t0 = tg * TG;
  const int pol = blockIdx.y;

  float2* twF = smem + SS::TWOFF;  // Nf twiddles, then W twiddles (padded), then the taper
  float2* twWl = twF + tw_slots(NF);
  float* win = reinterpret_cast<float*>(twWl + tw_slots(W));
  for (int j = tid; j < NF + W; j += NTPW) {
    if (j < NF) twF[tw_slot(j)] = a.twNf[j];
    else twWl[tw_slot(j - NF)] = a.twW[j - NF];
  }
  for (int j = tid; j < NF; j += NTPW) win[j] = a.window[j];

  const float2* zpol = a.Z + pol * a.z_pol_stride + t0;
  const uint32_t zbytes = (a.timing_mask & 1) ? 0u : (uint32_t)((NF - 1) * N + TG) * 8u;
  const uint32_t twbytes = (a.timing_mask & 4) ? 0u : (uint32_t)((W - 1) * N + TG) * 8u;
  const __amdgpu_buffer_rsrc_t tw4r = make_rsrc(a.tw4 + t0, twbytes);
  v4f* t4l = reinterpret_cast<v4f*>(reinterpret_cast<char*>(smem) + SS::lds_bytes);
  if constexpr (T4L) {
    for (int i = tid; i < W * PAIRS; i += NTPW) {
      const int jr = i / PAIRS, q = i % PAIRS;
      t4l[i] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(tw4r, (jr * N + 2 * q) * 8, 0, 0));
    }
  }
  const LdsPairs rowsF{reinterpret_cast<v4f*>(smem), SS::RSF};
  const LdsPairs rowsW{reinterpret_cast<v4f*>(smem), SS::RSW};
  float2* opol = a.out + pol * a.out_pol_stride;
  auto out_for = [&](int b) {
    // overlap-discard (:302) and 1/L * de/nu (:285) on the store
    const int64_t ob = (a.block0 + b) * (int64_t)a.Lkeep;  // first kept output sample
    const int64_t avail = a.out_limit - ob;
    const int64_t nk =
        (a.timing_mask & 2) ? 0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
    return PairOut<P16>{make_rsrc(opol + ob, (uint32_t)nk * 8u),
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
    block_fft_pair<NF, -1, PAIRS, NTPW>(in, sel, rowsF, twF, tid);
    __syncthreads();
    block_fft_pair<W, +1, PAIRS, NTPW>(rowsW, out_for(b), rowsW, twWl, tid);
  } else {
    constexpr int NBL = NF / SP::RL;
    constexpr int RW1 = W / NBL;
    constexpr int PT = (PAIRS * NBL + NTPW - 1) / NTPW;
    // Nf passes 1 .. last-1 (the first from `in`), then the fused pass, then W passes 2..
    auto run_block = [&](const auto& in, int b, auto after_first) {
      stockham_pass_pair<NF, R1, 1, -1, PAIRS, NTPW>(in, rowsF, twF, tid);
      // the gain x twiddle loads go out BEFORE the next block's prefetch: vmcnt retires
      // in order, so waiting for them must not mean waiting for the HBM prefetch too
      v4f t4[PT][RW1];
      if constexpr (T4L) load_t4_lds<NBL, RW1, PAIRS, NTPW>(t4, t4l, tid);
      else load_t4<NBL, RW1, PAIRS, NTPW>(t4, tw4r, N, tid);
      after_first();
      __syncthreads();
      if constexpr (!std::is_same_v<typename SP::Mid, Radices<>>) {
        run_fft_mid<NF, -1, PAIRS, NTPW, R1>(rowsF, twF, tid, typename SP::Mid{});
        __syncthreads();
      }
      fused_select_pass<NF, W, SP::RL, SPANS, PAIRS, NTPW>(rowsF, rowsW, twF, t4, tid);
      __syncthreads();
      run_fft_tail<W, +1, PAIRS, NTPW, RW1>(rowsW, out_for(b), twWl, tid, typename SP::Wrest{});
    };
    if constexpr (!PERSIST) {
      __syncthreads();  // tables
      const int b = b_begin;
      const PairZIn<NB1> in{make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes), N, win};
      run_block(in, b, [] {});
    } else {
      constexpr int PF = (PAIRS * NB1 + NTPW - 1) / NTPW;
      v4f zv[PF][R1];
      static_assert(DK >= 0 && DK <= R1, "overlap reuse needs keep = DK * NF / R1");
      auto prefetch = [&](int b, auto reuse) {
        constexpr int R0 = decltype(reuse)::value ? R1 - DK : 0;  // registers kept
        const __amdgpu_buffer_rsrc_t z = make_rsrc(zpol + (int64_t)b * a.keep * N, zbytes);
        static_for<0, PF>([&](auto p) {
          const int bb = min(tid + p * NTPW, PAIRS * NB1 - 1);
          const int q = bb % PAIRS, j = bb / PAIRS;
          static_for<0, R0>([&](auto r) { zv[p][r] = zv[p][r + DK]; });
          static_for<R0, R1>([&](auto r) {
            const v4u x = __builtin_amdgcn_raw_buffer_load_b128(z, (j * N + 2 * q) * 8, r * NB1 * N * 8, 0);
            zv[p][r] = __builtin_bit_cast(v4f, x);
          });
        });
      };
      prefetch(b_begin, std::false_type{});
      const PairRegsIn<PF, R1> in{zv, win};
#pragma unroll 1
      for (int b = b_begin; b < b_end; b += b_step) {
        __syncthreads();  // tables / previous block's W transform done with the rows
        run_block(in, b, [&] {
          // unconditional (the last block re-reads itself): a conditional prefetch
          // leaves the vmcnt count path-dependent, and the compiler then waits for the
          // prefetch together with the gain x twiddle loads in the fused pass
          prefetch(min(b + b_step, b_end - 1), std::integral_constant<bool, (DK > 0)>{});
        });
      }
    }
  }
}

template <int NF, int W, int PAIRS, bool SPANS, int NTPW = NTP>
static hipError_t launch_sb(const SynthBlockArgs& a, hipStream_t s) {
  using SS = SynthPairShape<NF, W, PAIRS>;
  const int groups = a.N / (2 * PAIRS);
  // workgroups per CU the registers allow at the kernel's 2 waves per SIMD
  constexpr int vgpr_wgs = 8 * 64 / NTPW;
  if (a.ranges != 0 && SynthPlan<NF, W>::fused) {
    // persistent: block ranges so that ~LDS-limited workgroups per CU are resident;
    // the overlap-reuse instance when keep matches the compiled DK
    constexpr int NB1 = NF / synth_first_radix<NF, W>();
    constexpr int DK = synth_reuse_dk<NF, W>();
    constexpr bool FU = SynthPlan<NF, W>::fused;
    const bool reuse = DK > 0 && a.keep == DK * NB1 && !a.no_reuse;
    const bool p16 = (a.out_limit % 2 == 0) && (a.Lkeep % 2 == 0);
    // table copy in LDS where it still leaves 4 two-wave workgroups per CU (the VGPR
    // limit): SKA-Mid 25.7 + 14 KB; not SKA-Low (38.5 + 28 KB)
    constexpr size_t t4_bytes = (size_t)W * PAIRS * 16;
    constexpr bool T4 = SS::lds_bytes + t4_bytes <= (160 * 1024) / vgpr_wgs;
    static const bool no_t4l = std::getenv("PFB_SYNTH_NO_T4LDS") != nullptr;
    const bool t4l = T4 && !no_t4l && reuse && p16;
    const size_t lds = SS::lds_bytes + (t4l ? t4_bytes : 0);
    auto kern = t4l ? synth_block_kernel<NF, W, PAIRS, SPANS, FU, DK, true, T4, NTPW>
              : reuse ? (p16 ? synth_block_kernel<NF, W, PAIRS, SPANS, FU, DK, true, false, NTPW>
                             : synth_block_kernel<NF, W, PAIRS, SPANS, FU, DK, false, false, NTPW>)
                      : (p16 ? synth_block_kernel<NF, W, PAIRS, SPANS, FU, 0, true, false, NTPW>
                             : synth_block_kernel<NF, W, PAIRS, SPANS, FU, 0, false, false, NTPW>);
    hipError_t e = set_lds(kern, lds);
    if (e != hipSuccess) return e;
    const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(vgpr_wgs, (160 * 1024) / lds));
    // resident-capacity ranges; when that leaves more than 16 blocks per range (many
    // phase groups per block row: SKA-Mid N / TG = 1024 gives one range of 72 blocks),
    // ranges of 6 blocks instead (oversubscribed, evenly split): C3 1.59 -> 1.51 ms.
    // C2 (64 ranges of ~7 blocks) keeps the capacity rule.
    int ranges = a.ranges;
    if (ranges <= 0) {
      ranges = std::max(1, cu_count() * per_cu / (groups * a.n_pol));
      if (ranges * 16 < a.n_blocks) ranges = (a.n_blocks + 5) / 6;
    }
    ranges = std::min(ranges, a.n_blocks);
    dim3 grid((unsigned)(groups * ranges), (unsigned)a.n_pol);
    return launch_kernel(kern, grid, dim3(NTPW), lds, s, a);
  }
  auto kern = synth_block_kernel<NF, W, PAIRS, SPANS, false, 0, false, false, NTPW>;
  hipError_t e = set_lds(kern, SS::lds_bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)(groups * a.n_blocks), (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(NTPW), SS::lds_bytes, s, a);
}

// pair rows per workgroup: enough for every thread to own one first-pass butterfly,
// fewer when the channel count is small (2 * PAIRS must divide N)
template <int NF, int W, bool SPANS>
static hipError_t launch_sb_p(const SynthBlockArgs& a, hipStream_t s) {
  // Nf >= 512 (SKA-Mid): 256-thread workgroups, so one workgroup reads 8 output phases
  // (64 B of every stage-1 row instead of 32) and the per-workgroup tables are shared
  // by twice the threads (PFB_SYNTH_NTP=128 restores the 128-thread shape)
  static const int ntp_env = std::getenv("PFB_SYNTH_NTP") ? std::atoi(std::getenv("PFB_SYNTH_NTP")) : 0;
  if constexpr (NF >= 512) {
    constexpr int P2 = 256 / (NF / synth_first_radix<NF, W>());
    if (ntp_env != 128 && a.N % (2 * P2) == 0) return launch_sb<NF, W, P2, SPANS, 256>(a, s);
  }
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
