// pfb_synth_wave.hip — synthesis stage 2 for Nf = 256 (SKA-Low: W = 224 at OS 8/7, 192 at
// 4/3) with one output phase per 16 lanes and no workgroup barrier in the block loop
// (polyphase_synthesis.m:163-316, re-ordered as DESIGN.md §5 derives).
//
// Per block b and output phase t0 (one column of the stage-1 rows Z[row][t0]):
//   Nf-point FFT over time (taper on the way in), keep W bins, x gain x four-step twiddle
//   (x the output scale), W-point IFFT, overlap-discard.
// Lane l of a 16-lane group holds 16 values of the column at every stage:
//   pass 1   x[l + 16 r] (r < 16)       -> 16-point DFT over r, x w_256^{l f1}
//   swap 1   lane f1 <- B_i[f1], i < 16  (16 x 16 transpose through the wave's LDS tile)
//   pass 2   16-point DFT over i         -> bins f = f1 + 16 f2; the RW = W/16 kept bins of
//            the lane are j' = f1 + 16 r'', the inputs of one RW-point butterfly of the W-point
//            IFFT (W = 16 RW): x t4[j'] (lane constants, loaded once), RW-point IDFT over r'',
//            x e^{+2 pi i f1 t1a / W}
//   swap 2   (t1a, phase) <- C_f1[t1a], f1 < 16, across the workgroup (below)
//   pass 3   16-point IDFT over f1       -> y[t1a + RW t1b], stored when t1 is kept.
// A wave holds 4 output phases in passes 1-2 (64 lanes), a 256-thread workgroup 16
// adjacent phases (one 128-B line of every Z row and output row).
// Memory access in wide segments: the stage-1 rows come in the run layout the streaming
// analysis writes for this kernel (AnalysisArgs::zblk = ZB: ZB consecutive rows of one
// phase are adjacent), so one load instruction reads ZB rows x the wave's 4 phases as one
// contiguous 32 ZB-byte segment per row group (ZB = 2, the default: 8 segments of 64 B
// instead of 16 of 32 B); swap 2 is the one exchange that crosses waves: pass 3 lane (phase,
// t1a) of wave w takes t1a = w + 4 slot for all 16 phases, so one store instruction writes
// 4 whole 128-B output rows.  Swap 1 stays inside the wave (LDS instructions of one wave
// execute in order); two workgroup barriers per block order swap 2 (before its reads, and
// before the next block's swap 1 rewrites the tiles other waves read).  Every twiddle is a
// table entry rounded once from double; the per-lane gain x twiddle values (t4, 14 complex)
// are constant for the workgroup's whole block range and loaded once per launch.
#include "pfb_synth_wave.hpp"

namespace pfb {

bool synth_wave_supported(const SynthBlockArgs& a) {
  if (a.Nf != 256 || (a.W != 224 && a.W != 192)) return false;
  if (a.N % kCols != 0) return false;
  if (a.fir_x) return synth_wave_fir_supported(a);
  return (a.zblk == 1 || a.zblk == 2 || a.zblk == 4) && a.keep == 160;
}

// recomputed stage-1 rows: the streaming analysis shapes (N 256; 8/7 with W 224, 4/3 with
// W 192; P 12 or 13 -> PE 13 or 14 folded taps) and input offsets within one descriptor
bool synth_wave_fir_supported(const SynthBlockArgs& a) {
  if (a.Nf != 256 || a.keep != 160 || a.N != 256 || !a.fir_x || !a.fir_g) return false;
  const bool s87 = a.W == 224 && a.fir_nu == 8 && a.fir_de == 7;
  const bool s43 = a.W == 192 && a.fir_nu == 4 && a.fir_de == 3;
  if (!(s87 || s43) || (a.fir_pe != 13 && a.fir_pe != 14) || a.fir_q0 < 0) return false;
  // tile offsets of the last block stay below 2^31 bytes
  return (a.fir_n_dat + 512 * (int64_t)a.N) * 8 < kRsrcMaxBytes;
}

template <int RW, bool SPANS, bool XW, class FIRV = NoFir, bool WFLAT = false>
static hipError_t launch_wave_t(const SynthBlockArgs& a, hipStream_t s) {
  // the XW kernels raise their issue priority from the loop-top barrier to the swap-1
  // barrier (PRIO 1): a workgroup's waves reach the cross-wave exchange together instead of
  // trailing the other two resident workgroups' waves (C2 synthesis 63.6-65.6 -> 61.9-62.8
  // us, profiles/r04_v11_wave_prio_ab.jsonl)
  auto kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, XW ? 1 : 0>;
  if constexpr (kExperiments && RW == 14 && SPANS && XW && WFLAT) {
    // (PFB_WAVE_PRIO=0/2/3: other priority schedules, experiments build only)
    static const int prio = knob("PFB_WAVE_PRIO") ? std::atoi(knob("PFB_WAVE_PRIO")) : 1;
    if (prio == 0) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 0>;
    if (prio == 2) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 2>;
    if (prio == 3) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 3>;
    if (prio == 4) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 4>;
    if (prio == 5) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 5>;
    if (prio == 8) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 8>;
    if (prio == 16) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 16>;
    if (prio == 32) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 32>;
    if (prio == 33) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, 33>;
  }
  if constexpr (!FIRV::kOn && RW <= 14) {
    // stored stage-1 rows with L_ov = 3 RW N (keep 160, Ov 48): the kept-register stores
    // (V 1, round 6, pfb_synth_wave.hpp): 134 instead of 164 VGPRs, 10 stores a block instead
    // of 16, no load or store wait inside the block.  Measured equal to the old kernel
    // (63.2-64.8 vs 64.0-65.6 us on C2, interleaved); the ping-pong (2) and deferred-store (4)
    // forms gain nothing on top (profiles/r06_v5_c2_wave_v_ab.jsonl).  PFB_WAVE_V=0/1/3/5/7:
    // the variants (experiments build A/B)
    int v = 1;
    if constexpr (kExperiments) {
      static const int ev = knob("PFB_WAVE_V") ? std::atoi(knob("PFB_WAVE_V")) : -1;
      if (ev >= 0) v = ev;
    }
    if (a.Lov != 3 * RW * a.N) v = 0;
    constexpr int P = XW ? 1 : 0;
    if (v == 1) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 1>;
    if (v == 3) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 3>;
    if (v == 5) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 5>;
    if (v == 7) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 7>;
    if constexpr (kExperiments && RW == 14 && SPANS && XW && WFLAT) {
      // timing variants of V 1 (results invalid): 8 no workgroup barriers, 16 no twiddle tables
      if (v == 9) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 9>;
      if (v == 17) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 17>;
      if (v == 25) kern = synth_wave_kernel<RW, SPANS, 10, XW, FIRV, WFLAT, P, 25>;
    }
  }
  hipError_t e = set_lds(kern, kLdsB);
  if (e != hipSuccess) return e;
  const int groups = a.N / kCols;
  // resident workgroups: 3 per CU (3 waves per SIMD at <= 168 VGPRs; LDS would allow 4)
  int per_cu = std::max(1, std::min(3, (160 * 1024) / kLdsB));
  static const int env_wpc = knob("PFB_WAVE_PER_CU") ? std::atoi(knob("PFB_WAVE_PER_CU")) : 0;  // A/B
  if (env_wpc > 0) per_cu = env_wpc;
  int ranges = std::max(1, cu_count() * per_cu / (groups * a.n_pol));
  // (PFB_WAVE_RANGES=R: R block ranges; PFB_WAVE_LINEAR=1: linear order — experiments A/B)
  SynthBlockArgs b = a;
  if constexpr (kExperiments) {
    static const int env_r = knob("PFB_WAVE_RANGES") ? std::atoi(knob("PFB_WAVE_RANGES")) : 0;
    static const int lin = knob("PFB_WAVE_LINEAR") ? std::atoi(knob("PFB_WAVE_LINEAR")) : -1;
    if (env_r > 0) ranges = env_r;
    if (lin >= 0) b.linear = lin;
  }
  ranges = std::min(ranges, a.n_blocks);
  dim3 grid((unsigned)(groups * ranges), (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(kWgThreads), kLdsB, s, b);
}

// the flat-window choice of the stored-rows kernel (PFB_WAVE_WFLAT=0: off, experiments A/B)
static bool use_wflat(const SynthBlockArgs& a) {
  static const bool wf_off = knob("PFB_WAVE_WFLAT") && std::atoi(knob("PFB_WAVE_WFLAT")) == 0;
  return a.win_flat && !wf_off;
}

template <int RW, int NU, int DE, bool WFLAT>
static hipError_t launch_wave_fir_w(const SynthBlockArgs& a, hipStream_t s) {
  if (a.fir_pe == 14)
    return a.spans ? launch_wave_t<RW, true, false, FirShape<NU, DE, 14>, WFLAT>(a, s)
                   : launch_wave_t<RW, false, false, FirShape<NU, DE, 14>, WFLAT>(a, s);
  return a.spans ? launch_wave_t<RW, true, false, FirShape<NU, DE, 13>, WFLAT>(a, s)
                 : launch_wave_t<RW, false, false, FirShape<NU, DE, 13>, WFLAT>(a, s);
}
// (the same taper form as the stored-rows kernel: with a flat window the products by 1 are
// dropped in both, so the compiler fuses the same multiplies into the same FMAs and the
// outputs stay bit-identical)
template <int RW, int NU, int DE>
static hipError_t launch_wave_fir(const SynthBlockArgs& a, hipStream_t s) {
  return use_wflat(a) ? launch_wave_fir_w<RW, NU, DE, true>(a, s) : launch_wave_fir_w<RW, NU, DE, false>(a, s);
}

hipError_t launch_synth_wave(const SynthBlockArgs& a, hipStream_t s) {
  if (a.n_blocks <= 0) return hipSuccess;
  if (!synth_wave_supported(a)) return hipErrorInvalidValue;
  if (a.fir_x) return a.W == 224 ? launch_wave_fir<14, 8, 7>(a, s) : launch_wave_fir<12, 4, 3>(a, s);
  // pass-1 lanes spread over the workgroup (synthesis 78.5-80.2 -> 74.2-75.1 us on C2,
  // profiles/r03_v8_c2_wave_xw_ab.jsonl); PFB_WAVE_XW=0: within the wave (experiments A/B)
  static const bool xw = !(knob("PFB_WAVE_XW") && std::atoi(knob("PFB_WAVE_XW")) == 0);
  if (!kExperiments || xw) {
    // a window flat over rows [48, 208) (tukey, Ov <= 48: C2) skips 10 of the 16 taper
    // multiplies per lane and block (PFB_WAVE_WFLAT=0: the general kernel, experiments A/B)
    if (use_wflat(a)) {
      if (a.W == 224)
        return a.spans ? launch_wave_t<14, true, true, NoFir, true>(a, s) : launch_wave_t<14, false, true, NoFir, true>(a, s);
      return a.spans ? launch_wave_t<12, true, true, NoFir, true>(a, s) : launch_wave_t<12, false, true, NoFir, true>(a, s);
    }
    if (a.W == 224) return a.spans ? launch_wave_t<14, true, true>(a, s) : launch_wave_t<14, false, true>(a, s);
    return a.spans ? launch_wave_t<12, true, true>(a, s) : launch_wave_t<12, false, true>(a, s);
  }
  if (a.W == 224) return a.spans ? launch_wave_t<14, true, false>(a, s) : launch_wave_t<14, false, false>(a, s);
  return a.spans ? launch_wave_t<12, true, false>(a, s) : launch_wave_t<12, false, false>(a, s);
}

}  // namespace pfb
