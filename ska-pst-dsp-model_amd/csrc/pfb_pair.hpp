// pfb_pair.hpp — two transforms per thread in packed-FP32 lanes (gfx950).
//
// CDNA4 executes v_pk_{add,mul,fma}_f32 on register pairs.  A single complex
// transform held as interleaved (re, im) pairs packs the additions well but every
// complex multiply and every multiply-by-i needs lane swizzles (v_mov / v_pk_mov),
// and the compiler falls back to scalar ops around them.  Holding the SAME element
// of TWO independent transforms (two rows of a batch) as
//     re = (re_a, re_b), im = (im_a, im_b)
// makes every butterfly op, twiddle multiply (the twiddle is common to both rows)
// and multiply-by-i a plain packed op with no swizzles: two rows for the VALU
// cost of one.  Used by the synthesis block kernel, whose rows are the output
// phases t0 of one block ("Synthesis block kernel").
#pragma once

#include "pfb_device.hpp"

namespace pfb {

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

struct cpx2 {
  v2f re, im;
};

__device__ __forceinline__ cpx2 cadd(cpx2 a, cpx2 b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cpx2 csub(cpx2 a, cpx2 b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cpx2 cscale(cpx2 a, float s) { return {a.re * s, a.im * s}; }
__device__ __forceinline__ cpx2 czero(cpx2) { return {v2f{0.f, 0.f}, v2f{0.f, 0.f}}; }
__device__ __forceinline__ cpx2 cneg(cpx2 a) { return {-a.re, -a.im}; }
__device__ __forceinline__ cpx2 cfmar(float c, cpx2 a, cpx2 b) { return {c * a.re + b.re, c * a.im + b.im}; }
__device__ __forceinline__ cpx2 ctwc(cpx2 a, float c, float s) {
  return {a.re * c - a.im * s, a.re * s + a.im * c};
}
template <int DIR>
__device__ __forceinline__ cpx2 crot90(cpx2 a) {
  if constexpr (DIR < 0) return {a.im, -a.re};
  else return {-a.im, a.re};
}
// same twiddle for both rows
__device__ __forceinline__ cpx2 cmul(cpx2 a, float2 w) { return ctwc(a, w.x, w.y); }
// per-row factors
__device__ __forceinline__ cpx2 cmul(cpx2 a, cpx2 w) {
  return {a.re * w.re - a.im * w.im, a.re * w.im + a.im * w.re};
}

// (re_a, im_a, re_b, im_b) in memory order  <->  cpx2.  The middle two lanes trade
// places with one v_swap_b32 (the compiler otherwise spends three v_mov per value).
__device__ __forceinline__ cpx2 from_interleaved(v4f x) {
  float a = x.y, b = x.z;
  asm("v_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return {v2f{x.x, a}, v2f{b, x.w}};
}
// the two samples of a pair as (re, im) each: lo = row a, hi = row b
struct Interleaved {
  v2f lo, hi;
};
__device__ __forceinline__ Interleaved to_interleaved(cpx2 v) {
  float a = v.re.y, b = v.im.x;
  asm("v_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return {v2f{v.re.x, a}, v2f{b, v.im.y}};  // after the swap: a = im_a, b = re_b
}
// NB: never __builtin_bit_cast an ext-vector swizzle (x.zw): clang lowers it as a
// cast of the leading elements.  Cast whole vectors only.
__device__ __forceinline__ v2u as_u(v2f x) { return __builtin_bit_cast(v2u, x); }

// ------------------------------------------------------------------ buffer resources
// Raw buffer descriptors (32-bit byte offsets, hardware range check: loads past
// num_records return 0, stores past it are dropped).  Built from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// The same from values that ARE wave-uniform but that the uniformity analysis may not prove
// so (computed after divergent control flow, through loops): read from the first lane, so
// the descriptor lives in scalar registers.  Otherwise every buffer access through it
// becomes a one-trip waterfall loop (measured: the strided-store cascade kernel had 33 of
// them per step, the LowCBF kernel 17 after an unrelated divergent loop was added).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u(const void* base, uint32_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint64_t bu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  return make_rsrc(reinterpret_cast<const void*>(bu), (uint32_t)__builtin_amdgcn_readfirstlane(bytes));
}

// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt / lgkmcnt left at their maxima).  A software-
// pipelined loop whose prologue issues the first loads should drain them before the loop:
// the wait-count pass merges the loop head's entry path (those loads last in flight) with
// the back edge (the prefetch loads, then the previous iteration's stores), and the merged
// count makes the first use of the prefetched registers wait for the stores as well.
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// ------------------------------------------------------------------ LDS pair rows
// Pair row q (rows 2q, 2q+1 of the batch) at base + q * rs, element i is one 16-byte
// cpx2 slot {re_a, re_b, im_a, im_b}: ds_read_b128 / ds_write_b128, and the address is
// affine in i (no padding function), so the per-register offsets fold into the
// instruction's immediate.
struct LdsPairs {
  static constexpr bool kIsLds = true;
  v4f* base;
  int rs;
  template <class P, class RR>
  __device__ __forceinline__ cpx2 load(int q, int i, P, RR) const {
    const v4f x = base[q * rs + i];
    return {x.xy, x.zw};
  }
  template <class P, class RR>
  __device__ __forceinline__ void store(int q, int i, cpx2 v, P, RR) const {
    base[q * rs + i] = v4f{v.re.x, v.re.y, v.im.x, v.im.y};
  }
};

// Pair-row index that sends an HBM store out of its buffer descriptor's range (dropped).
constexpr int kDropPair = -(1 << 24);

// One Stockham pass of radix R over PAIRS pair-rows (2 * PAIRS transforms of length N).
// Thread b owns butterfly j = b / PAIRS of pair row q = b % PAIRS (pair rows fastest).
template <int N, int R, int NS, int DIR, int PAIRS, int NTH, class In, class Out>
__device__ __forceinline__ void stockham_pass_pair(const In& in, const Out& out,
                                                   const float2* __restrict__ tw, int tid) {
  constexpr int NB = N / R;
  constexpr int TOT = PAIRS * NB;
  constexpr int PER = (TOT + NTH - 1) / NTH;
  // A pass that stores to HBM with idle threads (TOT not a multiple of NTH) runs them on a
  // clamped butterfly with their stores pointed out of range instead of branching around
  // them: the wave then issues the same number of stores on every path, so the vmcnt
  // bookkeeping stays exact and a later wait for a load never waits for these stores.
  constexpr bool CLAMP = !Out::kIsLds && (TOT % NTH != 0);
  cpx2 v[PER][R];
  static_for<0, PER>([&](auto p) {
    const int b = CLAMP ? min(tid + p * NTH, TOT - 1) : tid + p * NTH;
    if (CLAMP || TOT % NTH == 0 || b < TOT) {
      const int q = b % PAIRS, j = b / PAIRS;
      static_for<0, R>([&](auto r) { v[p][r] = in.load(q, j + r * NB, p, r); });
    }
  });
  if constexpr (In::kIsLds && Out::kIsLds) __syncthreads();
  static_for<0, PER>([&](auto p) {
    const int b0 = tid + p * NTH;
    const int b = CLAMP ? min(b0, TOT - 1) : b0;
    if (CLAMP || TOT % NTH == 0 || b < TOT) {
      const int q = b % PAIRS, j = b / PAIRS;
      const int k = j % NS;
      if constexpr (NS > 1) {
        float2 w[R];
        twiddle_powers<R, DIR>(tw, k * (N / (NS * R)), w);
        static_for<1, R>([&](auto r) { v[p][r] = cmul(v[p][r], w[r]); });
      }
      sdft<R, DIR>(v[p]);
      const int idxD = (j / NS) * NS * R + k;
      const int qs = (CLAMP && b0 >= TOT) ? kDropPair : q;
      static_for<0, R>([&](auto r) { out.store(qs, idxD + r * NS, v[p][r], p, r); });
    }
  });
}

template <int N, int DIR, int PAIRS, int NTH, int NS, int R, int... Rest, class First, class Last>
__device__ __forceinline__ void run_passes_pair_impl(const First& first, const Last& last,
                                                     const LdsPairs& lds, const float2* tw, int tid) {
  if constexpr (sizeof...(Rest) == 0) {
    stockham_pass_pair<N, R, NS, DIR, PAIRS, NTH>(first, last, tw, tid);
  } else {
    stockham_pass_pair<N, R, NS, DIR, PAIRS, NTH>(first, lds, tw, tid);
    __syncthreads();
    run_passes_pair_impl<N, DIR, PAIRS, NTH, NS * R, Rest...>(lds, last, lds, tw, tid);
  }
}

template <int N, int DIR, int PAIRS, int NTH, class First, class Last, int... Rs>
__device__ __forceinline__ void run_fft_pair(const First& first, const Last& last, const LdsPairs& lds,
                                             const float2* tw, int tid, Radices<Rs...>) {
  run_passes_pair_impl<N, DIR, PAIRS, NTH, 1, Rs...>(first, last, lds, tw, tid);
}

// The first pass alone / all passes after it (lets a caller slot work in between,
// e.g. re-issuing a register prefetch once the first pass has consumed it).
template <int N, int DIR, int PAIRS, int NTH, class First, int R0, int... Rest>
__device__ __forceinline__ void first_pass_pair(const First& first, const LdsPairs& lds,
                                                const float2* tw, int tid, Radices<R0, Rest...>) {
  stockham_pass_pair<N, R0, 1, DIR, PAIRS, NTH>(first, lds, tw, tid);
}
template <int N, int DIR, int PAIRS, int NTH, class Last, int R0, int... Rest>
__device__ __forceinline__ void rest_passes_pair(const Last& last, const LdsPairs& lds, const float2* tw,
                                                 int tid, Radices<R0, Rest...>) {
  static_assert(sizeof...(Rest) > 0, "transform has a single pass");
  run_passes_pair_impl<N, DIR, PAIRS, NTH, R0, Rest...>(lds, last, lds, tw, tid);
}

// Middle passes LDS -> LDS, starting at stride NS0 (barriers between passes, none after).
template <int N, int DIR, int PAIRS, int NTH, int NS0, int... Rs>
__device__ __forceinline__ void run_fft_mid(const LdsPairs& lds, const float2* tw, int tid, Radices<Rs...>) {
  run_passes_pair_impl<N, DIR, PAIRS, NTH, NS0, Rs...>(lds, lds, lds, tw, tid);
}
// Remaining passes from LDS, starting at stride NS0; the last stores through `last`.
template <int N, int DIR, int PAIRS, int NTH, int NS0, class Last, int... Rs>
__device__ __forceinline__ void run_fft_tail(const LdsPairs& lds, const Last& last, const float2* tw, int tid,
                                             Radices<Rs...>) {
  run_passes_pair_impl<N, DIR, PAIRS, NTH, NS0, Rs...>(lds, last, lds, tw, tid);
}

// Whole transform over the pair rows: first pass loads through `first`, last pass
// stores through `last`, the passes in between exchange through `lds`.
template <int N, int DIR, int PAIRS, int NTH, class First, class Last>
__device__ __forceinline__ void block_fft_pair(const First& first, const Last& last, const LdsPairs& lds,
                                               const float2* tw, int tid) {
  run_fft_pair<N, DIR, PAIRS, NTH>(first, last, lds, tw, tid, typename FFTPlan<N>::type{});
}

}  // namespace pfb
