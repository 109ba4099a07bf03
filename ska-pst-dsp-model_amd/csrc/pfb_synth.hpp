// pfb_synth.hpp — shared pieces of the synthesis stage-2 kernels (pfb_synth.hip: block
// kernel; pfb_synth_fir.hip: the round trip's block kernel that recomputes its stage-1
// rows): pair-row LDS shapes, transform plans, the fused selection pass, I/O functors.
#pragma once
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
  // o: first kept output sample of the block, records = kept samples in bytes.  Without
  // P16 each sample of a pair is range-checked on its own (the output limit or an odd L_ov
  // may split a pair): the odd sample's offset is hidden from the optimiser so the two
  // 8-byte stores are never merged into one 16-byte store.  (It must be off + 8 on o, not
  // off on a descriptor based one sample later: at kept position 0 that offset is -8,
  // which the range check drops.)
  __amdgpu_buffer_rsrc_t o;
  int N, lov, t0;  // lov = L_ov: the block's first kept sample is t0 + N t1 = L_ov
  float scale;
  template <class P, class RR>
  __device__ __forceinline__ void store(int q, int t1, cpx2 v, P, RR) const {
    // sample t0 + 2q + N t1 of the block goes to kept position t0 + 2q + N t1 - L_ov:
    // negative offsets (the discarded head, q = kDropPair) wrap past 2^31 bytes and are
    // dropped by the range check, as is the discarded tail past L_keep (L_ov need not be a
    // multiple of N: normalize(os, Ov) may be fractional, e.g. 48 x 27/32 for 'sps')
    const int off = (t1 * N - lov + t0 + 2 * q) * 8;
    const Interleaved y = to_interleaved(cscale(v, scale));
    if constexpr (P16) {
      // (t0 + 2q even, nk even): a pair never straddles the range end, so the 16-byte
      // store is dropped or kept as a whole exactly when its two samples are
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(v4u, v4f{y.lo.x, y.lo.y, y.hi.x, y.hi.y}), o, off, 0, kAuxOut);
    } else {
      int off1 = off + 8;
      asm volatile("" : "+v"(off1));
      __builtin_amdgcn_raw_buffer_store_b64(as_u(y.lo), o, off, 0, kAuxOut);
      __builtin_amdgcn_raw_buffer_store_b64(as_u(y.hi), o, off1, 0, kAuxOut);
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

}  // namespace pfb
