// pfb_roundtrip.hip — the SKA-Low round trip (polyphase_analysis.m:83-121 followed by
// polyphase_synthesis.m:163-316, the sequence of test_data_pipeline.m:114,132) as ONE
// launch: analysis and synthesis workgroups side by side on every CU.
//
// The two-kernel round trip runs the HBM-bound analysis (input + channelised product +
// stage-1 rows) and the latency-bound wave synthesis one after the other.  Here blockIdx.x
// < nA are analysis workgroups — analysis_stream_body over contiguous step ranges, exactly
// as analysis_stream_kernel — and the rest are synthesis workgroups running
// synth_wave_body over a block schedule.  Every analysis range publishes how many of its
// steps have their stage-1 rows in memory (a progress word per range, relaxed agent-scope
// store after the rows' write-through stores have drained: cdna_hip_programming.md
// Guideline 16, R1); a synthesis workgroup waits for the ranges that hold a block's rows
// before loading them (sc1 loads).  All ranges advance together, so blocks become ready
// spread over the whole launch; the schedule (host, round_trip_schedule) hands every XCD's
// synthesis workgroups the blocks of the analysis ranges on that XCD in the order they
// become ready, so a block's rows are read shortly after they are written (from the XCD's
// L2 or the Infinity Cache instead of HBM) and the synthesis runs beside the analysis.
//
// Results are the same as the two-kernel round trip bit for bit (same bodies, same
// arithmetic; only the order of blocks and the load cache policy differ).  Progress words
// are zeroed by a memset node before every launch; waits are bounded: a wait that gives up
// (workgroups not co-resident) sets the plan's error word, which the next call reports.
#include "pfb_ana_stream.hpp"
#include "pfb_synth_wave.hpp"

namespace pfb {

namespace {

// analysis side: publish "n steps of this range have their stage-1 rows in memory"
struct StepPublisher {
  static constexpr bool kOn = true;
  unsigned* word;
  __device__ void step_done(int64_t n) const {
    if (threadIdx.x == 0 && n > 0) __hip_atomic_store(word, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ void range_done(int64_t n) const {
    if (threadIdx.x == 0) __hip_atomic_store(word, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// synthesis side: blocks list[0], list[stride], ... ; block b waits for the analysis ranges
// holding its rows [z_row0 + b keep, z_row0 + b keep + Nf)
struct FusedSched {
  static constexpr bool kReuse = false;
  static constexpr int kLoadAux = kSc1;
  const int* list;
  int n, stride;
  const unsigned* prog;  // this polarisation's progress words
  unsigned* err;
  int nA;
  int64_t n_steps, z_row0;
  int keep, Nf;
  unsigned spin_max;
  mutable bool gave_up = false;  // after one timed-out wait this workgroup waits no more

  __device__ int count() const { return n; }
  __device__ int block(int i) const { return list[(int64_t)i * stride]; }
  __device__ void wait(int b) const {
    if (gave_up) return;
    const int64_t r0 = z_row0 + (int64_t)b * keep;
    const int64_t s_lo = r0 / 16, s_hi = min((r0 + Nf - 1) / 16, n_steps - 1);
    int w = (int)(((s_lo + 1) * nA + n_steps - 1) / n_steps) - 1;  // range holding step s_lo
    for (;;) {
      const int64_t st0 = n_steps * w / nA, st1 = n_steps * (w + 1) / nA;
      const unsigned need = (unsigned)(min(s_hi + 1, st1) - st0);
      unsigned v = __hip_atomic_load(prog + w * kProgStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (unsigned spins = 0; v < need; ++spins) {
        if (spins >= spin_max) {
          __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-visible
          gave_up = true;
          return;
        }
        __builtin_amdgcn_s_sleep(8);
        v = __hip_atomic_load(prog + w * kProgStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (st1 > s_hi) break;
      ++w;
    }
    // the rows are loaded with sc1 loads: no acquire, only keep them below the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

}  // namespace

// Workgroup roles: x % 3 == 0 analysis, else synthesis, so that whichever way the
// dispatcher fills the CUs (one workgroup per CU per pass, or a CU at a time) every CU holds
// one analysis and two synthesis workgroups.  XCD = x % 8 (gridDim.x % 8 == 0); within
// a period of 24 = lcm(3, 8) workgroups each XCD gets one analysis and two synthesis
// workgroups, so XCD xc holds analysis ranges xc nA/8 + t and synthesis workgroups 2 t + j
// (t = x / 24).
template <int P, int NU, int DE, int RW, bool SPANS>
__global__ __launch_bounds__(kWgThreads) __attribute__((amdgpu_waves_per_eu(3)))
void roundtrip_fused_kernel(AnalysisArgs aa, SynthBlockArgs sa, RtFusedArgs f) {
  const int pol = blockIdx.y;
  const int bx = blockIdx.x;
  const int xc = bx & 7, t = bx / 24, r = bx % 24;
  if (bx % 3 == 0) {
    // the producer's waves issue first: the synthesis fills the cycles the analysis leaves
    if (f.prio) __builtin_amdgcn_s_setprio(3);
    const int w = xc * (f.nA / 8) + t;
    analysis_stream_body<256, P, NU, DE, 2, false, false>(aa, pol, w, f.nA,
                                                           StepPublisher{f.prog + (pol * f.nA + w) * kProgStride});
    return;
  }
  // r is one of xc, xc + 8, xc + 16; the two that are not multiples of 3, in order
  const int j = (r - xc) / 8 - ((xc % 3 == 0) ? 1 : ((xc + 8) % 3 == 0 && r == xc + 16) ? 1 : 0);
  const int local = 2 * t + j;
  const int groups = sa.N / kCols;
  const int g = local % groups, k = local / groups;
  const int s0 = f.seg[xc], len = f.seg[xc + 1] - s0;
  const int n = len > k ? (len - k + f.lanes - 1) / f.lanes : 0;
  const FusedSched sch{f.order + s0 + k, n, f.lanes, f.prog + pol * f.nA * kProgStride, f.err, f.nA,
                       f.n_steps, f.z_row0, sa.keep, sa.Nf, tmask(f.nowait) ? 0u : f.spin_max, tmask(f.nowait) != 0};
  synth_wave_body<RW, SPANS, 10>(sa, pol, g, sch);
}

template <int P, int NU, int DE, int RW, bool SPANS>
static size_t fused_lds() {
  return std::max<size_t>(StreamShape<256, P, NU, DE>::lds_bytes, (size_t)kLdsB);
}

template <int P, int NU, int DE, int RW, bool SPANS>
static hipError_t launch_t(const AnalysisArgs& aa, const SynthBlockArgs& sa, const RtFusedArgs& f,
                           hipStream_t s, bool query, int* per_cu) {
  auto kern = roundtrip_fused_kernel<P, NU, DE, RW, SPANS>;
  const size_t lds = fused_lds<P, NU, DE, RW, SPANS>();
  hipError_t e = set_lds(kern, lds);
  if (e != hipSuccess) return e;
  if (query) {
    int nb = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kWgThreads, lds);
    *per_cu = nb;
    return e;
  }
  dim3 grid((unsigned)(f.nA + f.nS), (unsigned)aa.n_pol);
  return launch_kernel(kern, grid, dim3(kWgThreads), lds, s, aa, sa, f);
}

// the compiled shapes: 256 channels, 13 tap phases, OS 8/7 (W 224) or 4/3 (W 192)
static int fused_shape(const AnalysisArgs& aa, const SynthBlockArgs& sa) {
  if (aa.variant != kBunton || aa.N != 256 || aa.P != 13 || sa.N != 256 || sa.Nf != 256 || sa.keep != 160)
    return -1;
  if (aa.nu == 8 && aa.M == 224 && sa.W == 224) return 0;
  if (aa.nu == 4 && aa.M == 192 && sa.W == 192) return 1;
  return -1;
}

static hipError_t dispatch(const AnalysisArgs& aa, const SynthBlockArgs& sa, const RtFusedArgs& f, hipStream_t s,
                           bool query, int* per_cu) {
  const int shape = fused_shape(aa, sa);
  if (shape == 0)
    return sa.spans ? launch_t<13, 8, 7, 14, true>(aa, sa, f, s, query, per_cu)
                    : launch_t<13, 8, 7, 14, false>(aa, sa, f, s, query, per_cu);
  if (shape == 1)
    return sa.spans ? launch_t<13, 4, 3, 12, true>(aa, sa, f, s, query, per_cu)
                    : launch_t<13, 4, 3, 12, false>(aa, sa, f, s, query, per_cu);
  return hipErrorInvalidValue;
}

bool roundtrip_fused_supported(const AnalysisArgs& aa, const SynthBlockArgs& sa, int* per_cu) {
  if (fused_shape(aa, sa) < 0 || aa.zblk != 2 || sa.zblk != 2) return false;
  return dispatch(aa, sa, RtFusedArgs{}, nullptr, true, per_cu) == hipSuccess;
}

hipError_t launch_roundtrip_fused(const AnalysisArgs& aa, const SynthBlockArgs& sa, const RtFusedArgs& f,
                                  hipStream_t s) {
  // roles by x % 3 over periods of 24 (see roundtrip_fused_kernel): nS = 2 nA, nA % 8 == 0
  if (f.nA <= 0 || f.nA % 8 != 0 || f.nS != 2 * f.nA || f.nS % (8 * (sa.N / kCols)) != 0) return hipErrorInvalidValue;
  return dispatch(aa, sa, f, s, false, nullptr);
}

int roundtrip_cu_count() { return cu_count(); }

}  // namespace pfb
