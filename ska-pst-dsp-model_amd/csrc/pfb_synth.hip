// pfb_synth.hip — synthesis stage 2 (polyphase_synthesis.m:163-316, re-ordered; see
// DESIGN.md §5): per block x group of output phases t0, Nf-point FFT over time, kept-bin
// selection with deripple and the four-step twiddle, W-point inverse FFT,
// overlap-discard and the 1/L * de/nu scale.
#include "pfb_synth.hpp"

namespace pfb {

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
  const uint32_t zbytes = (tmask(a.timing_mask) & 1) ? 0u : (uint32_t)((NF - 1) * N + TG) * 8u;
  const uint32_t twbytes = (tmask(a.timing_mask) & 4) ? 0u : (uint32_t)((W - 1) * N + TG) * 8u;
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
        (tmask(a.timing_mask) & 2) ? 0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
    return PairOut<P16>{make_rsrc(opol + ob, (uint32_t)nk * 8u), N, a.Lov, t0, a.scale};
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
      vm_drain();
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
    const bool p16 = (a.out_limit % 2 == 0) && (a.Lkeep % 2 == 0) && (a.Lov % 2 == 0);
    // table copy in LDS where it still leaves 4 two-wave workgroups per CU (the VGPR
    // limit): SKA-Mid 25.7 + 14 KB; not SKA-Low (38.5 + 28 KB)
    constexpr size_t t4_bytes = (size_t)W * PAIRS * 16;
    constexpr bool T4 = SS::lds_bytes + t4_bytes <= (160 * 1024) / vgpr_wgs;
    static const bool no_t4l = knob("PFB_SYNTH_NO_T4LDS") != nullptr;
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
    // phase groups per block row: SKA-Mid N / TG = 512 gives one range of 72 blocks),
    // ranges of ~18 blocks instead (oversubscribed, evenly split: 4 rounds of resident
    // workgroups).  Round 1 (no LDS table copy) chose 6 blocks: 1.59 -> 1.51 ms; with
    // the per-workgroup table copy (T4L) longer ranges copy it less often — r02_v13 sweep
    // of the C3 synthesis: 1 / 2 / 4 / 12 / 24 ranges = 515 / 496 / 492 / 526-537 / 593 us
    // (profiles/r02_v13_c3_ranges_ab.txt).  C2 (64 ranges of ~7 blocks) keeps the
    // capacity rule.
    int ranges = a.ranges;
    if (ranges <= 0) {
      ranges = std::max(1, cu_count() * per_cu / (groups * a.n_pol));
      if (ranges * 16 < a.n_blocks) ranges = (a.n_blocks + 17) / 18;
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
  static const int ntp_env = knob("PFB_SYNTH_NTP") ? std::atoi(knob("PFB_SYNTH_NTP")) : 0;
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
  // SKA-Mid shape (Nf 512, W 448, Ov 128): the wave kernel, on rows or 2-row runs (zblk 2)
  // (PFB_SYNTH_WAVE512=0: the block kernel, experiments build — synth_wave512_supported)
  if (a.Nf == 512 && synth_wave512_supported(a)) return launch_synth_wave512(a, s);
  // stage-1 rows for the Nf = 256 wave kernel (the fused round trip: zblk = run length)
  if (a.zblk || a.fir_x) return launch_synth_wave(a, s);
#define X(a_, b_) \
  if (a.Nf == a_ && a.W == b_)  \
    return a.spans ? launch_sb_p<a_, b_, true>(a, s) : launch_sb_p<a_, b_, false>(a, s);
  PFB_SYNTH_SIZES(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace pfb
