// pfb_synth_fir.hip — the round trip's synthesis block kernel that evaluates its own
// stage-1 rows from the analysis input (launch_synth_fir).  Built with
// the SI load/store merger off (Makefile): it would fuse the FIR's ds_read_b64 pairs into
// ds_read2_b64, which moves half the bytes per LDS cycle (MI355X_MICROARCH.md §LDS).
#include "pfb_synth.hpp"

#ifndef PFB_SF_WPE
#define PFB_SF_WPE 2  // waves per SIMD the register budget is set for
#endif

namespace pfb {

// ======================================================================= round trip, Z recomputed
// Synthesis block kernel of the round trip that evaluates its stage-1 rows from the
// analysis INPUT instead of reading them from HBM.  Stage-2 work for the phases
// t0 .. t0 + TG - 1 needs only column t0 .. of the stage-1 rows Z = N^2 v_k, and the
// Bunton FIR sum v_k[c] of the streaming analysis (analysis_stream_kernel) depends only
// on input column c (rows of N samples, X[r][c] = x[r N + c]):
//     v_{NU p + s}[c] = sum_{m < PE} F[(m + 1) N + c - a_s] X[DE p + m + b_s][c],
//     a_s = (s M) mod N, b_s = floor(s M / N), F = [N zeros, taps, N zeros].
// So the workgroup of phase group t0 reads the TG input columns of its blocks (128-B
// rows, each input row once per block plus a PE-row halo) and computes the FIR itself:
// the analysis no longer writes Z and the synthesis no longer reads it (2 x 8 nu/de B
// per input sample less HBM traffic; the analysis input is read twice instead).
// Thread (q, j) of the first Nf pass owns block rows j + NB1 r, i.e. (with k0 + keep b
// a multiple of NU) residue s = j mod NU and period p = .. + j / NU + (NB1 / NU) r: it
// computes exactly the rows its first pass consumes, with the taps of its two columns
// for residue s, from an LDS tile of the block's input rows.  The FMA order (m = 0 ..
// PE - 1 from 0) and the N^2 scaling are those of analysis_stream_kernel, so the rows —
// and the output — are bit-identical to the Z path.
// LDS tile: row rho of the phase at byte rho * 8 TG, column c at 8 (c ^ ((rho >> 1) & 1))
// (the row-pair swap makes the ds_read_b64 of the NU residues conflict-free).
template <int NF, int W, int PAIRS, bool SPANS, int DK, bool P16, int NU, int DE, int PE, bool B128>
__global__ __launch_bounds__(NTP) __attribute__((amdgpu_waves_per_eu(PFB_SF_WPE))) void synth_fir_kernel(SynthBlockArgs a) {
  using SS = SynthPairShape<NF, W, PAIRS>;
  using SP = SynthPlan<NF, W>;
  static_assert(SP::fused, "needs a fused plan");
  constexpr int R1 = synth_first_radix<NF, W>();
  constexpr int NB1 = NF / R1;
  constexpr int TG = 2 * PAIRS;
  static_assert(PAIRS * NB1 == NTP, "one first-pass butterfly per thread");
  static_assert(NB1 % NU == 0, "residue fixed per thread");
  constexpr int R0 = R1 - DK;           // rows carried over from the previous block
  constexpr int SPR = NB1 / NU;         // periods per first-pass register step
  constexpr int BMAX = ((NU - 1) * DE) / NU;
  constexpr int ROWB = TG * 8;          // tile row bytes
  // input rows of the registers [0, R0) / [R0, R1) of one block
  constexpr int NRA = DE * (SPR * R0 - 1) + BMAX + PE, NRB = DE * (SPR * DK - 1) + BMAX + PE;
  static_assert((size_t)NRA * ROWB <= (size_t)SS::TWOFF * 8 && (size_t)NRB * ROWB <= (size_t)SS::TWOFF * 8,
                "input tile exceeds the row area");
  constexpr int NPA = (NRA * PAIRS + NTP - 1) / NTP, NPB = (NRB * PAIRS + NTP - 1) / NTP;
  extern __shared__ __attribute__((aligned(16))) float2 smem[];
  const int tid = threadIdx.x;
  const int N = a.N;
  const int groups = N / TG;
  const int lt = a.xcd ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int tg = lt % groups;
  const int rr = lt / groups;
  const int Rg = gridDim.x / groups;
  const int b_begin = (int)((int64_t)a.n_blocks * rr / Rg);
  const int b_end = (int)((int64_t)a.n_blocks * (rr + 1) / Rg);
  if (b_begin >= b_end) return;
  const int t0 = tg * TG;
  const int pol = blockIdx.y;

  float2* twF = smem + SS::TWOFF;
  float2* twWl = twF + tw_slots(NF);
  float* win = reinterpret_cast<float*>(twWl + tw_slots(W));
  for (int j = tid; j < NF + W; j += NTP) {
    if (j < NF) twF[tw_slot(j)] = a.twNf[j];
    else twWl[tw_slot(j - NF)] = a.twW[j - NF];
  }
  for (int j = tid; j < NF; j += NTP) win[j] = a.window[j];
  const uint32_t twbytes = (a.timing_mask & 4) ? 0u : (uint32_t)((W - 1) * N + TG) * 8u;
  const __amdgpu_buffer_rsrc_t tw4r = make_rsrc(a.tw4 + t0, twbytes);
  const LdsPairs rowsF{reinterpret_cast<v4f*>(smem), SS::RSF};
  const LdsPairs rowsW{reinterpret_cast<v4f*>(smem), SS::RSW};
  char* tile = reinterpret_cast<char*>(smem);
  float2* opol = a.out + pol * a.out_pol_stride;
  auto out_for = [&](int b) {
    const int64_t ob = (a.block0 + b) * (int64_t)a.Lkeep;
    const int64_t avail = a.out_limit - ob;
    const int64_t nk =
        (a.timing_mask & 2) ? 0 : max((int64_t)0, avail < a.Lkeep ? avail : (int64_t)a.Lkeep);
    return PairOut<P16>{make_rsrc(opol + ob, (uint32_t)nk * 8u),
                        make_rsrc(opol + ob + 1, (uint32_t)max((int64_t)0, nk - 1) * 8u), N, a.t1_lo, t0,
                        a.scale};
  };

  // this thread's first-pass butterfly, residue and tile read addresses
  const int q = tid % PAIRS, j = tid / PAIRS;
  const int s = j % NU, jh = j / NU;
  const int bs = (s * DE) / NU;                     // b_s (M = N DE / NU)
  const int as = (int)(((int64_t)s * a.fir_M) % N);  // a_s
  const int base_t = DE * jh + bs;                  // tile row of (r = RLO, m = 0)
  // even column of tile row base_t + k: byte base_t ROWB + 16 q + 8 sw(base_t + k)
  const int e_t = base_t * ROWB + 16 * q;

  // input column slice: descriptor from the workgroup's first input row
  const int64_t pblk = a.fir_k0 / NU;  // period of Z row 0
  const int64_t rho_first = (int64_t)DE * (pblk + (int64_t)b_begin * (a.keep / NU));
  const float2* xpol = a.x + pol * a.x_pol_stride;
  const int64_t xavail = a.n_dat - rho_first * N;
  uint32_t xbytes = (uint32_t)min(max(xavail, (int64_t)0) * 8, kRsrcMaxBytes);
  if (a.timing_mask & 1) xbytes = 0;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xpol + rho_first * N + t0, xbytes);
  // first tile row of registers [rlo, ..) of block b, relative to rho_first
  auto rho_lo = [&](int b, int rlo) { return (int)(DE * ((int64_t)(b - b_begin) * (a.keep / NU) + SPR * rlo)); };
  auto load_x = [&](auto& xv, int rho0, auto nr) {  // tile rows [rho0, rho0 + NR) -> registers
    constexpr int NR = decltype(nr)::value;
    constexpr int NP = (NR * PAIRS + NTP - 1) / NTP;
    static_for<0, NP>([&](auto k) {
      const int i = min(tid + (int)k * NTP, NR * PAIRS - 1);
      const int row = i / PAIRS, qq = i % PAIRS;
      const v4u v = __builtin_amdgcn_raw_buffer_load_b128(xr, ((rho0 + row) * N + 2 * qq) * 8, 0, 0);
      xv[k] = __builtin_bit_cast(v4f, v);
    });
  };
  auto store_tile = [&](const auto& xv, auto nr) {
    constexpr int NR = decltype(nr)::value;
    constexpr int NP = (NR * PAIRS + NTP - 1) / NTP;
    static_for<0, NP>([&](auto k) {
      const int i = tid + (int)k * NTP;
      if (NR * PAIRS % NTP == 0 || i < NR * PAIRS) {
        const int row = i / PAIRS, qq = i % PAIRS;
        const v4f v = xv[k];
        if constexpr (B128) {
          *reinterpret_cast<v4f*>(tile + row * ROWB + 16 * qq) = v;
        } else {
          const bool sw = (row >> 1) & 1;
          *reinterpret_cast<v4f*>(tile + row * ROWB + 16 * qq) = sw ? v4f{v.z, v.w, v.x, v.y} : v;
        }
      }
    });
  };
  v4f zv[1][R1];
  // FIR of registers [RLO, RHI) from the tile (rows relative to the phase's first row)
  const __amdgpu_buffer_rsrc_t fr = make_rsrc(a.fir_f, (uint32_t)((a.fir_P + 2) * N * 4));
  const int fbase = (t0 + 2 * q - as) * 4;  // F[(m + 1) N + c - a_s] = fbase + (m + 1) N, bytes
  // the thread's taps, loaded ahead of the tile barrier so their latency overlaps it
  // (opaque copy: keeps the compiler from hoisting the loads out of the block loop, where
  // they would hold 2 PE registers through the transforms)
  auto load_taps = [&](v2f (&g)[PE]) {
    int fb = fbase;
    asm volatile("" : "+v"(fb));
#pragma unroll
    for (int m = 0; m < PE; ++m)
      g[m] = __builtin_bit_cast(v2f, __builtin_amdgcn_raw_buffer_load_b64(fr, fb + (m + 1) * N * 4, 0, 0));
  };
  auto fir = [&](auto rlo, auto rhi, const v2f (&g)[PE]) {
    constexpr int RLO = decltype(rlo)::value, RHI = decltype(rhi)::value;
    int et = e_t;
    asm volatile("" : "+v"(et));
    const int e0 = et + 8 * ((base_t >> 1) & 1), e1 = et + 8 * (((base_t + 1) >> 1) & 1);
    const int e2 = e0 ^ 8, e3 = e1 ^ 8;
    if (a.timing_mask & 8) {  // timing experiment: no FIR arithmetic (results invalid)
      static_for<RLO, RHI>([&](auto rv) { zv[0][decltype(rv)::value] = v4f{g[0].x, g[0].y, 0.f, 0.f}; });
      return;
    }
    // tap-outer order: the RHI - RLO registers' sums are independent chains, so one tap's
    // tile reads for all of them are in flight together (register-outer order leaves ~2
    // reads in flight and the FIR waits on LDS latency); each sum still runs m = 0 ..
    // PE - 1 from 0, as in the analysis kernel
    constexpr int NRG = RHI - RLO;
    v2f ae[NRG], ao[NRG];
    static_for<0, PE>([&](auto mv) {
      constexpr int m = decltype(mv)::value;
      static_for<0, NRG>([&](auto iv) {
        constexpr int i = decltype(iv)::value;
        constexpr int off = DE * SPR * i + m;
        v2f xe, xo;
        if constexpr (B128) {  // one ds_read_b128 per row (both columns; 1.5-way conflicts)
          const v4f x = *reinterpret_cast<const v4f*>(tile + et + off * ROWB);
          xe = v2f{x.x, x.y};
          xo = v2f{x.z, x.w};
        } else {
          const int ea = (off & 3) == 0 ? e0 : (off & 3) == 1 ? e1 : (off & 3) == 2 ? e2 : e3;
          const int eo = (off & 3) == 0 ? e2 : (off & 3) == 1 ? e3 : (off & 3) == 2 ? e0 : e1;
          xe = *reinterpret_cast<const v2f*>(tile + ea + off * ROWB);
          xo = *reinterpret_cast<const v2f*>(tile + eo + off * ROWB);
        }
        const v2f ze = m == 0 ? v2f{0.f, 0.f} : ae[i], zo = m == 0 ? v2f{0.f, 0.f} : ao[i];
        ae[i] = __builtin_elementwise_fma(v2f{g[m].x, g[m].x}, xe, ze);
        ao[i] = __builtin_elementwise_fma(v2f{g[m].y, g[m].y}, xo, zo);
      });
      // one tap: all its tile reads first, then its FMAs (left alone, the scheduler keeps
      // a single read in flight and each FMA waits out the LDS latency)
      __builtin_amdgcn_sched_group_barrier(0x100, B128 ? NRG : 2 * NRG, 0);  // DS reads
      __builtin_amdgcn_sched_group_barrier(0x002, 2 * NRG, 0);               // VALU
    });
    const float zs = (float)N * (float)N;
    static_for<0, NRG>([&](auto iv) {
      constexpr int i = decltype(iv)::value;
      zv[0][RLO + i] = v4f{zs * ae[i].x, zs * ae[i].y, zs * ao[i].x, zs * ao[i].y};
    });
  };

  constexpr int NBL = NF / SP::RL;
  constexpr int RW1 = W / NBL;
  constexpr int PT = (PAIRS * NBL + NTP - 1) / NTP;
  const PairRegsIn<1, R1> in{zv, win};
  v4f xb[NPB];
  {
    // first block of the range: registers [0, R0) from their own tile, then [R0, R1)
    v4f xa[NPA];
    load_x(xa, rho_lo(b_begin, 0), std::integral_constant<int, NRA>{});
    load_x(xb, rho_lo(b_begin, R0), std::integral_constant<int, NRB>{});
    v2f g[PE];
    load_taps(g);
    __syncthreads();  // tables
    store_tile(xa, std::integral_constant<int, NRA>{});
    __syncthreads();
    fir(std::integral_constant<int, 0>{}, std::integral_constant<int, R0>{}, g);
  }
#pragma unroll 1
  for (int b = b_begin; b < b_end; ++b) {
    if (b != b_begin) static_for<0, R0>([&](auto r) { zv[0][r] = zv[0][r + DK]; });
    v2f g[PE];
    load_taps(g);
    __syncthreads();  // the previous block's W transform / the first FIR done with the tile
    if (!(a.timing_mask & 16)) store_tile(xb, std::integral_constant<int, NRB>{});
    __syncthreads();
    fir(std::integral_constant<int, R0>{}, std::integral_constant<int, R1>{}, g);
    {
      const int tidl = tid;
      __syncthreads();  // tile reads done before the first pass writes the rows
      stockham_pass_pair<NF, R1, 1, -1, PAIRS, NTP>(in, rowsF, twF, tidl);
      v4f t4[PT][RW1];
      load_t4<NBL, RW1, PAIRS, NTP>(t4, tw4r, N, tidl);
      __syncthreads();
      if constexpr (!std::is_same_v<typename SP::Mid, Radices<>>) {
        run_fft_mid<NF, -1, PAIRS, NTP, R1>(rowsF, twF, tid, typename SP::Mid{});
        __syncthreads();
      }
      fused_select_pass<NF, W, SP::RL, SPANS, PAIRS, NTP>(rowsF, rowsW, twF, t4, tidl);
      // next block's input rows (unconditional: the last block re-reads its own); issued
      // once the gain x twiddle registers are dead (register budget)
      load_x(xb, rho_lo(min(b + 1, b_end - 1), R0), std::integral_constant<int, NRB>{});
      __syncthreads();
      run_fft_tail<W, +1, PAIRS, NTP, RW1>(rowsW, out_for(b), twWl, tid, typename SP::Wrest{});
    }
  }
}

template <int NF, int W, int NU, int DE, int PE>
static hipError_t launch_sf(const SynthBlockArgs& a, hipStream_t s) {
  constexpr int PAIRS = NTP / (NF / synth_first_radix<NF, W>());
  constexpr int DK = synth_reuse_dk<NF, W>();
  using SS = SynthPairShape<NF, W, PAIRS>;
  const int groups = a.N / (2 * PAIRS);
  const bool p16 = (a.out_limit % 2 == 0) && (a.Lkeep % 2 == 0);
  // PFB_SYNTH_FIR_RD=64: the swizzled ds_read_b64 tile (A/B)
  static const bool rd64 = std::getenv("PFB_SYNTH_FIR_RD") && std::atoi(std::getenv("PFB_SYNTH_FIR_RD")) == 64;
  auto pick = [&](auto b128) {
    constexpr bool B = decltype(b128)::value;
    return a.spans ? (p16 ? synth_fir_kernel<NF, W, PAIRS, true, DK, true, NU, DE, PE, B>
                          : synth_fir_kernel<NF, W, PAIRS, true, DK, false, NU, DE, PE, B>)
                   : (p16 ? synth_fir_kernel<NF, W, PAIRS, false, DK, true, NU, DE, PE, B>
                          : synth_fir_kernel<NF, W, PAIRS, false, DK, false, NU, DE, PE, B>);
  };
  auto kern = rd64 ? pick(std::false_type{}) : pick(std::true_type{});
  const size_t lds = SS::lds_bytes;
  hipError_t e = set_lds(kern, lds);
  if (e != hipSuccess) return e;
  constexpr int vgpr_wgs = 4 * PFB_SF_WPE * 64 / NTP;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(vgpr_wgs, (160 * 1024) / lds));
  int ranges = a.ranges > 0 ? a.ranges : std::max(1, cu_count() * per_cu / (groups * a.n_pol));
  if (a.ranges <= 0 && ranges * 16 < a.n_blocks) ranges = (a.n_blocks + 5) / 6;
  // a range's input rows (keep DE / NU per block + one block's halo) within a descriptor
  const int64_t rows_per_block = (int64_t)a.keep / NU * DE;
  const int64_t fit_blocks = (kRsrcMaxBytes / ((int64_t)8 * a.N) - 2 * (int64_t)NF) / rows_per_block;
  if (fit_blocks <= 0) return hipErrorInvalidValue;
  ranges = (int)std::max<int64_t>(ranges, (a.n_blocks + fit_blocks - 1) / fit_blocks);
  ranges = std::min(ranges, a.n_blocks);
  if ((int64_t)groups * ranges > INT32_MAX) return hipErrorInvalidValue;
  dim3 grid((unsigned)(groups * ranges), (unsigned)a.n_pol);
  return launch_kernel(kern, grid, dim3(NTP), lds, s, a);
}

bool synth_fir_supported(const SynthBlockArgs& a) {
  if (a.Nf != 256 || (a.W != 224 && a.W != 192) || a.keep != 160 || a.N % 16 != 0) return false;
  if (a.no_reuse) return false;
  if (!((a.fir_nu == 8 && a.fir_de == 7) || (a.fir_nu == 4 && a.fir_de == 3))) return false;
  if ((int64_t)a.fir_M * a.fir_nu != (int64_t)a.N * a.fir_de) return false;
  if (a.fir_P != 12 && a.fir_P != 13) return false;
  return a.fir_k0 % a.fir_nu == 0 && a.fir_k0 >= 0 && a.x && a.fir_f;
}

hipError_t launch_synth_fir(const SynthBlockArgs& a, hipStream_t s) {
  if (!synth_fir_supported(a)) return hipErrorInvalidValue;
  if (a.n_blocks <= 0) return hipSuccess;
#define SF(W_, NU_, DE_)                                                                   \
  if (a.W == W_ && a.fir_nu == NU_)                                                        \
    return a.fir_P == 13 ? launch_sf<256, W_, NU_, DE_, 14>(a, s) : launch_sf<256, W_, NU_, DE_, 13>(a, s);
  SF(224, 8, 7)
  SF(192, 4, 3)
#undef SF
  return hipErrorInvalidValue;
}

}  // namespace pfb
