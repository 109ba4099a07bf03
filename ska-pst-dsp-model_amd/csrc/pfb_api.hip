// pfb_api.hip — C ABI of the MI355X PFB engine (declared in include/pfb_api.h).
//
// Host-side plan management: tap padding, twiddle / deripple / window tables computed
// in double and rounded once to float, device scratch, the FilterBank /
// InverseFilterBank streaming state (carry-over buffers) and kernel dispatch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cxxabi.h>
#include <string>
#include <vector>

#include "pfb_api.h"
#include "pfb_kernels.hpp"

namespace {

thread_local std::string g_err;

pfb_status fail(pfb_status s, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(e_ == hipErrorOutOfMemory ? PFB_ERR_OOM : PFB_ERR_HIP, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(e_), __FILE__, __LINE__);                  \
  } while (0)

// ------------------------------------------------------------------ device buffer
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 256));
    if (e == hipSuccess) bytes = std::max<size_t>(n, 256);
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

template <class T>
hipError_t upload(DevBuf& b, const std::vector<T>& v) {
  hipError_t e = b.ensure(v.size() * sizeof(T));
  if (e != hipSuccess) return e;
  return hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
}

// e^{sign 2 pi i m / n}, accurate reduction in double
std::vector<float2> twiddles(int64_t n, int sign) {
  std::vector<float2> t((size_t)n);
  for (int64_t m = 0; m < n; ++m) {
    int64_t mm = m;
    if (2 * mm > n) mm -= n;
    const double a = 2.0 * M_PI * (double)mm / (double)n;
    t[(size_t)m] = make_float2((float)std::cos(a), (float)(sign * std::sin(a)));
  }
  return t;
}

// ------------------------------------------------------------------ profiling
struct ProfRec {
  int which;
  hipEvent_t a, b;
  double bytes;
};
struct Profiler {
  bool enabled = false;
  std::vector<ProfRec> pending;
  std::vector<hipEvent_t> pool;
  // 0 analysis, 1 chan IFFT, 2 block, 3 analysis + chan IFFT, 4 / 5 the FIR / row FFT of
  // the generic (N > 256) round trip (launched one by one so each is timed alone)
  static constexpr int kClasses = 6;
  double total_ms[kClasses] = {};
  int64_t launches[kClasses] = {};
  double bytes[kClasses] = {};
  std::string names[kClasses];  // kernel of each class's last single-kernel launch (demangled)
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
  }
  void drain() {
    for (auto& r : pending) {
      float ms = 0.f;
      if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
        total_ms[r.which] += ms;
        launches[r.which] += 1;
        bytes[r.which] += r.bytes;
      }
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    pending.clear();
  }
};
Profiler g_prof;
thread_local pfb::LaunchEvents g_armed;
thread_local const char* g_launched = nullptr;

static std::string demangle(const char* name) {
  if (!name) return std::string();
  int st = 0;
  char* d = abi::__cxa_demangle(name, nullptr, nullptr, &st);
  std::string out = (st == 0 && d) ? std::string(d) : std::string(name);
  std::free(d);
  return out;
}

// Times the launch(es) issued while in scope.  single = true: exactly one kernel launch
// goes through pfb::launch_kernel, which records the two events inside its own dispatch
// (hipExtLaunchKernelGGL) — the kernel's own duration, as a kernel trace measures it.
// single = false (multi-kernel paths): events recorded on the stream around the scope.
struct ProfScope {
  hipEvent_t a = nullptr, b = nullptr;
  int which;
  double bytes;
  hipStream_t s;
  bool single;
  ProfScope(int w, double by, hipStream_t st, bool one = true) : which(w), bytes(by), s(st), single(one) {
    if (g_prof.enabled) {
      a = g_prof.get();
      b = g_prof.get();
      if (a && b) {
        if (single) {
          pfb::armed_launch_events() = pfb::LaunchEvents{a, b};
          pfb::launched_kernel_name() = nullptr;
        }
        else (void)hipEventRecord(a, s);
      }
    }
  }
  ~ProfScope() {
    if (g_prof.enabled && a && b) {
      if (single) {
        pfb::LaunchEvents& ev = pfb::armed_launch_events();
        if (ev.start) {  // not consumed (no kernel launched): drop the record
          ev = pfb::LaunchEvents{};
          g_prof.pool.push_back(a);
          g_prof.pool.push_back(b);
          return;
        }
        if (pfb::launched_kernel_name()) g_prof.names[which] = demangle(pfb::launched_kernel_name());
      } else {
        (void)hipEventRecord(b, s);
      }
      g_prof.pending.push_back({which, a, b, bytes});
    }
  }
};

int64_t floordiv(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

// n_pol rows of n complex samples at (dst + q*dps) <- (src + q*sps): one 2-D copy, not
// n_pol calls (the two-stage cascades run thousands of series through one plan)
hipError_t copy_pols(float2* dst, int64_t dps, const float2* src, int64_t sps, int64_t n, int n_pol,
                     hipMemcpyKind kind, hipStream_t s) {
  if (n <= 0 || n_pol <= 0) return hipSuccess;
  if (n_pol == 1) return hipMemcpyAsync(dst, src, n * sizeof(float2), kind, s);
  if (kind == hipMemcpyDeviceToDevice) return pfb::launch_copy_rows(dst, dps, src, sps, n, n_pol, s);
  hipError_t e = hipMemcpy2DAsync(dst, dps * sizeof(float2), src, sps * sizeof(float2), n * sizeof(float2),
                                  n_pol, kind, s);
  if (e == hipSuccess) return e;
  (void)hipGetLastError();  // large row pitches: one copy per row instead
  for (int q = 0; q < n_pol; ++q) {
    e = hipMemcpyAsync(dst + q * dps, src + q * sps, n * sizeof(float2), kind, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

pfb::LaunchEvents& pfb::armed_launch_events() { return g_armed; }
const char*& pfb::launched_kernel_name() { return g_launched; }

// error channel shared with the other C-ABI translation units (pfb_layout.hip)
pfb_status pfb_set_error(pfb_status s, const char* msg) { return fail(s, "%s", msg); }

// ====================================================================== analysis plan
// LowCBF: every call consumes the one-time pre-padding (polyphase_analysis_lowcbf.m:27-34)
struct PadConsume {
  bool* flag;
  ~PadConsume() { *flag = false; }
};

struct pfb_analysis_plan {
  uint64_t serial = 0;  // unique per plan (the split round trip's key: pointers get reused)
  int device = 0;
  int variant = 0, N = 0, nu = 1, de = 1, M = 0, P = 0, n_pol = 1, sds = 0;
  int C = 0;                  // output channels per row (N; 216 for the LowCBF filterbank)
  bool lowcbf_pad = false;    // LowCBF: the next call pre-pads 1536 zeros (persistent do_padding)
  int64_t n_taps = 0;
  bool fused = false;
  DevBuf taps, twN, scratch;
  // streaming shapes: the folded taps x N^2 [s][c][16] of analysis_stream_kernel, for the
  // synthesis that recomputes the stage-1 rows (SynthBlockArgs::fir_g); empty otherwise
  DevBuf gtab;
  DevBuf zrev;  // padded generic round trip: index reversal (N - i) mod N of the row FFT input
  // streaming (FilterBank.m:13-14 input_buffer / buffered_samples)
  DevBuf carry, work, stage_in, stage_out;
  DevBuf carry_next;  // device streams: the streaming kernel writes the next carry here, then swap
  int64_t buffered = 0;
  // round trip (pfb_roundtrip_execute): the analysis runs on this stream, ahead of the
  // synthesis on the caller's stream; one event per chunk orders them
  hipStream_t aux = nullptr;
  std::vector<hipEvent_t> events;
};

// Rows [row0, K_end) of a call whose output has K_total rows per pol (the padded
// variant's circular shift is modulo K_total).  `in`/`out` are the call's bases.
// z (round trip only): also emit the synthesis stage-1 rows of rows >= z_row0 into
// z[pol][k - z_row0][t0] (AnalysisArgs::z).
// Strided channelised output of the streaming analysis kernel (AnalysisArgs::out_rs):
// pfb_filterbank_execute_strided
struct OutLayout {
  int64_t rs, cs;
  int32_t split, shift, nsel;
};

static pfb::AnalysisArgs analysis_args(const pfb_analysis_plan* p, const float2* in, int64_t in_ps, int64_t n_dat,
                                       float2* out, int64_t out_ps, int64_t row0, int64_t K_end,
                                       int64_t K_total, float2* z, int64_t z_ps, int64_t z_row0, int64_t pad,
                                       const OutLayout* lay, int zblk, const float2* pre = nullptr);

// the next call's carry copied by the streaming kernel itself (AnalysisArgs::carry_out)
struct CarryOut {
  float2* dst;
  int64_t src, n, dst_ps;
};

static pfb_status analysis_run(pfb_analysis_plan* p, const float2* in, int64_t in_ps, int64_t n_dat,
                               float2* out, int64_t out_ps, int64_t row0, int64_t K_end,
                               int64_t K_total, hipStream_t s, float2* z = nullptr,
                               int64_t z_ps = 0, int64_t z_row0 = 0, int64_t pad = 0,
                               const OutLayout* lay = nullptr, int zblk = 0, const float2* pre = nullptr,
                               int z_stage = 0, const CarryOut* co = nullptr) {
  if (K_end <= row0) return PFB_OK;
  if (p->variant == pfb::kLowCbf) {
    pfb::LowCbfArgs l{};
    l.in = in;
    l.in_pol_stride = in_ps;
    l.n_dat = n_dat;
    l.pad = p->lowcbf_pad ? 1536 : 0;
    l.out = out;
    l.out_pol_stride = out_ps;
    l.K = K_end;
    l.n_pol = p->n_pol;
    l.taps = p->taps.as<float>();
    l.tw = p->twN.as<float2>();
    l.scale = 4096.0f;  // 2^9 * 2048 * 256 / 2^9 / 128
    ProfScope ps(0, (double)p->n_pol * (8.0 * n_dat + 8.0 * K_end * p->C), s);
    HIPCHK(pfb::launch_lowcbf(l, s));
    return PFB_OK;
  }
  pfb::AnalysisArgs a = analysis_args(p, in, in_ps, n_dat, out, out_ps, row0, K_end, K_total, z, z_ps, z_row0,
                                      pad, lay, zblk, pre);
  a.z_stage = z_stage;
  if (co) {
    a.carry_out = co->dst;
    a.carry_src = co->src;
    a.carry_n = co->n;
    a.carry_pol_stride = co->dst_ps;
  }
  a.scratch = nullptr;
  if (!p->fused && !z) {
    HIPCHK(p->scratch.ensure((size_t)p->n_pol * (K_end - row0) * p->N * sizeof(float2)));
    a.scratch = p->scratch.as<float2>();
  }
  // algorithmic bytes: each input sample read once (the rows' new samples, the tail of
  // the series with the last rows), each output sample written once
  const int64_t in_samples = (K_end == K_total && row0 == 0)
                                 ? n_dat
                                 : (K_end - row0) * p->M + (K_end == K_total ? n_dat - K_total * p->M : 0);
  // (with z: the stage-1 rows are a synthesis intermediate, not algorithmic bytes —
  // the synthesis' algorithmic read of its input is counted by the block kernel)
  const double bytes = (double)p->n_pol * (8.0 * in_samples + 8.0 * (K_end - row0) * p->N);
  // generic path = FIR + row FFT launches (z_stage 1 / 2: one of them, timed as its own
  // class; their bytes: the FIR reads the input and writes the stage-1 rows, the row FFT
  // reads them and writes the channelised product)
  const double zrow_bytes = (double)p->n_pol * 8.0 * (K_end - row0) * p->N;
  const int cls = !z ? 0 : z_stage == 1 ? 4 : z_stage == 2 ? 5 : 3;
  const double cls_bytes = z_stage == 1 ? (double)p->n_pol * 8.0 * in_samples + zrow_bytes
                           : z_stage == 2 ? 2.0 * zrow_bytes : bytes;
  ProfScope ps(cls, cls_bytes, s, p->fused || z_stage != 0);
  HIPCHK(pfb::launch_analysis(a, s));
  return PFB_OK;
}

static pfb::AnalysisArgs analysis_args(const pfb_analysis_plan* p, const float2* in, int64_t in_ps, int64_t n_dat,
                                       float2* out, int64_t out_ps, int64_t row0, int64_t K_end,
                                       int64_t K_total, float2* z, int64_t z_ps, int64_t z_row0, int64_t pad,
                                       const OutLayout* lay, int zblk, const float2* pre) {
  pfb::AnalysisArgs a{};
  a.pre = pre;        // the pad samples in front of `in` (stream carry); null: zeros
  a.pre_pol_stride = pad;
  a.z = z;
  a.z_pol_stride = z_ps;
  a.z_row0 = z_row0;
  a.zblk = zblk;
  a.in = in;
  a.in_pol_stride = in_ps;
  a.n_dat = n_dat;
  a.out = out;
  a.out_pol_stride = out_ps;
  a.row0 = row0;
  a.K = K_end;
  a.K_total = K_total;
  a.n_pol = p->n_pol;
  a.N = p->N;
  a.M = p->M;
  a.P = p->P;
  a.nu = p->nu;
  a.sds = p->sds;
  a.variant = p->variant;
  a.taps = p->taps.as<float>();
  a.twN = p->twN.as<float2>();
  a.zrev = p->zrev.p ? p->zrev.as<int>() : nullptr;
  a.pad = pad;  // `in` starts `pad` samples into the series (streaming kernel only)
  if (lay) {
    a.out_rs = (int)lay->rs;
    a.out_cs = (int)lay->cs;
    a.sel_split = lay->split;
    a.sel_shift = lay->shift;
    a.sel_n = lay->nsel;
  }
  return a;
}

// the plan's analysis runs on the streaming kernel, which takes a read offset (pad)
static bool analysis_offset_ok(const pfb_analysis_plan* p) {
  pfb::AnalysisArgs a{};
  a.variant = p->variant;
  a.N = p->N;
  a.M = p->M;
  a.P = p->P;
  a.nu = p->nu;
  return pfb::analysis_takes_offset(a);
}

static bool analysis_fused_carry_ok(const pfb_analysis_plan* p) {
  pfb::AnalysisArgs a{};
  a.variant = p->variant;
  a.N = p->N;
  a.M = p->M;
  a.P = p->P;
  a.nu = p->nu;
  return pfb::analysis_fused_takes_carry(a);
}

static bool analysis_emits_z(const pfb_analysis_plan* p) {
  pfb::AnalysisArgs a{};
  a.variant = p->variant;
  a.N = p->N;
  a.M = p->M;
  a.P = p->P;
  a.nu = p->nu;
  return pfb::analysis_can_emit_z(a);  // streaming kernel (N = 256) or register-window FIR
}

static bool analysis_emits_zblk(const pfb_analysis_plan* p) {
  pfb::AnalysisArgs a{};
  a.variant = p->variant;
  a.N = p->N;
  a.M = p->M;
  a.P = p->P;
  a.nu = p->nu;
  return pfb::analysis_can_emit_zblk(a);  // streaming kernel (N = 256)
}

static int64_t analysis_K(const pfb_analysis_plan* p, int64_t n_dat) {
  if (p->variant == pfb::kLowCbf) {  // PSTFilterbank.m:14-15
    const int64_t k = floordiv(n_dat + (p->lowcbf_pad ? 1536 : 0) - 3072, 192);
    return std::max<int64_t>(k, 0);
  }
  if (p->variant == pfb::kBunton) {
    const int64_t k = floordiv(n_dat - (int64_t)p->P * p->N, p->M);
    return std::max<int64_t>(k, 0);
  }
  return std::max<int64_t>(n_dat / p->M, 0);
}

extern "C" {

const char* pfb_last_error(void) { return g_err.c_str(); }
int32_t pfb_api_version(void) { return PFB_API_VERSION; }

int32_t pfb_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// Descriptor checks of pfb_analysis_plan_create (no device needed); fills the plan's
// scalar parameters into `p`
static pfb_status analysis_validate(const pfb_analysis_desc* d, pfb_analysis_plan* p) {
  if (!d) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (d->variant == PFB_ANALYSIS_LOWCBF &&
      (d->n_chan != 256 || d->os_nu != 4 || d->os_de != 3 || d->n_taps != 3072))
    return fail(PFB_ERR_INVALID_ARG,
                "polyphase_analysis_lowcbf is the fixed 256-channel 4/3 PST filterbank with "
                "3072 taps (PSTFilterbank.m:7-15); got n_chan=%d os=%d/%d taps=%lld",
                d->n_chan, d->os_nu, d->os_de, (long long)d->n_taps);
  if (d->variant != PFB_ANALYSIS_BUNTON && d->variant != PFB_ANALYSIS_PADDED &&
      d->variant != PFB_ANALYSIS_LOWCBF)
    return fail(PFB_ERR_INVALID_ARG, "unknown analysis variant %d", d->variant);
  if (d->n_chan <= 0 || d->os_nu <= 0 || d->os_de <= 0 || d->os_de > d->os_nu)
    return fail(PFB_ERR_INVALID_ARG, "invalid n_chan/os_factor (%d, %d/%d)", d->n_chan, d->os_nu,
                d->os_de);
  if (!d->taps || d->n_taps <= 0) return fail(PFB_ERR_INVALID_ARG, "no filter taps");
  if (d->n_pol <= 0) return fail(PFB_ERR_INVALID_ARG, "n_pol must be positive");
  if (d->n_pol > 65535)  // polarisations map to grid.y of every launch
    return fail(PFB_ERR_INVALID_ARG, "n_pol = %d exceeds 65535 series per plan", d->n_pol);
  // (sizes whose products the tables and kernels form in 32-bit ints: far beyond any
  // configuration, rejected before any arithmetic on them)
  if (d->n_chan > (1 << 24) || d->os_nu > (1 << 16) || d->n_taps > ((int64_t)1 << 30))
    return fail(PFB_ERR_UNSUPPORTED, "analysis parameters out of range (n_chan %d, os_nu %d, %lld taps)",
                d->n_chan, d->os_nu, (long long)d->n_taps);
  p->variant = d->variant;
  p->N = d->n_chan;
  p->nu = d->os_nu;
  p->de = d->os_de;
  p->M = (int)(((int64_t)d->n_chan * d->os_de) / d->os_nu);  // floor, polyphase_analysis.m:56
  p->n_taps = d->n_taps;
  p->P = (int)((d->n_taps + d->n_chan - 1) / d->n_chan);    // pad_filter.m:10
  p->n_pol = d->n_pol;
  if (p->M <= 0) return fail(PFB_ERR_INVALID_ARG, "commutator step M = floor(N de/nu) is zero");
  p->sds = (int)std::ceil((double)(d->n_taps - 1) / 2.0 / (double)p->M);  // padded.m:89
  p->C = p->N;
  if (p->variant == pfb::kLowCbf) {
    p->C = 216;
    p->lowcbf_pad = true;
    p->fused = true;
  } else if (!pfb::analysis_supported(p->N, p->P, p->variant, &p->fused)) {
    return fail(PFB_ERR_UNSUPPORTED, "no analysis kernel for n_chan=%d", d->n_chan);
  }
  return PFB_OK;
}

// Host-side tables of an analysis plan
struct AnaHost {
  std::vector<float> taps, g;
  std::vector<int> rev;
};

static void analysis_host_tables(const pfb_analysis_desc* d, const pfb_analysis_plan* p, AnaHost& h) {
  // zero rows up to the fused kernel's PMAX (32) so its tap loads are unconditional
  h.taps.assign((size_t)std::max(p->P, 32) * p->N, 0.f);
  for (int64_t i = 0; i < d->n_taps; ++i) h.taps[(size_t)i] = (float)d->taps[i];  // cast(filt, 'single')
  if (analysis_emits_zblk(p) && p->N == 256) {
    // g_s[m][c] = N^2 F[(m + 1) N + c - (s M mod N)], F = [N zeros, taps, zeros] — the
    // streaming kernel's folded taps (pfb_ana_stream.hpp), scaled by the power of two N^2
    // (exact), lags m < P + 1, zero-padded to 16 per (s, c)
    const int N = p->N, PE = p->P + 1;
    const float n2 = (float)N * (float)N;
    h.g.assign((size_t)p->nu * N * 16, 0.f);
    for (int sr = 0; sr < p->nu; ++sr) {
      const int as = (int)(((int64_t)sr * p->M) % N);
      for (int c = 0; c < N; ++c)
        for (int m = 0; m < PE; ++m) {
          const int j = (m + 1) * N + c - as;
          const float f = (j >= N && j < (p->P + 1) * N) ? h.taps[(size_t)(j - N)] : 0.f;
          h.g[((size_t)sr * N + c) * 16 + m] = n2 * f;
        }
    }
  }
  if (!p->fused && p->variant == pfb::kPadded) {
    h.rev.resize((size_t)p->N);
    for (int i = 0; i < p->N; ++i) h.rev[(size_t)i] = (p->N - i) % p->N;
  }
}

static void analysis_release(pfb_analysis_plan* p) {
  for (DevBuf* b : {&p->taps, &p->twN, &p->zrev, &p->gtab, &p->scratch, &p->carry, &p->carry_next, &p->work, &p->stage_in,
                    &p->stage_out})
    b->release();
}

pfb_status pfb_analysis_plan_validate(const pfb_analysis_desc* d) {
  pfb_analysis_plan p;
  const pfb_status st = analysis_validate(d, &p);
  if (st != PFB_OK) return st;
  AnaHost h;
  analysis_host_tables(d, &p, h);
  return PFB_OK;
}

pfb_status pfb_analysis_plan_create(const pfb_analysis_desc* d, pfb_analysis_plan** out) {
  if (!d || !out) return fail(PFB_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  pfb_analysis_plan tmp;
  const pfb_status vst = analysis_validate(d, &tmp);
  if (vst != PFB_OK) return vst;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(PFB_ERR_NO_DEVICE, "no HIP device available");
  if (d->device < 0 || d->device >= ndev)
    return fail(PFB_ERR_INVALID_ARG, "device %d out of range (%d devices)", d->device, ndev);
  if (hipSetDevice(d->device) != hipSuccess) return fail(PFB_ERR_HIP, "hipSetDevice(%d) failed", d->device);
  AnaHost h;
  analysis_host_tables(d, &tmp, h);
  static std::atomic<uint64_t> next_serial{1};
  auto* p = new pfb_analysis_plan(tmp);
  p->serial = next_serial++;
  p->device = d->device;
  hipError_t e = upload(p->taps, h.taps);
  if (e == hipSuccess) e = upload(p->twN, twiddles(p->N, -1));
  if (e == hipSuccess && !h.g.empty()) e = upload(p->gtab, h.g);
  if (e == hipSuccess && !h.rev.empty()) e = upload(p->zrev, h.rev);
  if (e != hipSuccess) {
    analysis_release(p);
    delete p;
    return fail(PFB_ERR_HIP, "analysis plan upload: %s", hipGetErrorString(e));
  }
  *out = p;
  return PFB_OK;
}

pfb_status pfb_analysis_plan_destroy(pfb_analysis_plan* p) {
  if (!p) return PFB_OK;
  (void)hipSetDevice(p->device);
  analysis_release(p);
  for (hipEvent_t e : p->events) (void)hipEventDestroy(e);
  if (p->aux) (void)hipStreamDestroy(p->aux);
  delete p;
  return PFB_OK;
}

int32_t pfb_analysis_output_channels(const pfb_analysis_plan* p) { return p ? p->C : -1; }

int64_t pfb_analysis_output_length(const pfb_analysis_plan* p, int64_t n_dat) {
  if (!p) return -1;
  return analysis_K(p, n_dat);
}

pfb_status pfb_analysis_execute(pfb_analysis_plan* p, const pfb_cf32* in, int64_t in_ps,
                                int64_t n_dat, pfb_cf32* out, int64_t out_ps, int64_t cap,
                                int64_t* n_out, int32_t mem, void* stream) {
  if (!p || (!in && n_dat > 0)) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (n_dat < 0) return fail(PFB_ERR_INVALID_ARG, "negative n_dat");
  HIPCHK(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t K = analysis_K(p, n_dat);
  PadConsume pad_once{&p->lowcbf_pad};
  if (n_out) *n_out = K;
  if (K == 0) return PFB_OK;
  if (!out) return fail(PFB_ERR_INVALID_ARG, "null output");
  if (cap < K) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld rows",
                           (long long)cap, (long long)K);
  if (mem == PFB_MEM_DEVICE) {
    if (in_ps < n_dat || out_ps < K * p->C)
      return fail(PFB_ERR_INVALID_ARG, "polarisation stride smaller than the data");
    return analysis_run(p, (const float2*)in, in_ps, n_dat, (float2*)out, out_ps, 0, K, K, s);
  }
  // host staging (synchronous)
  HIPCHK(p->stage_in.ensure((size_t)p->n_pol * n_dat * sizeof(float2)));
  HIPCHK(p->stage_out.ensure((size_t)p->n_pol * K * p->C * sizeof(float2)));
  HIPCHK(copy_pols(p->stage_in.as<float2>(), n_dat, (const float2*)in, in_ps, n_dat, p->n_pol,
                   hipMemcpyHostToDevice, s));
  pfb_status st = analysis_run(p, p->stage_in.as<float2>(), n_dat, n_dat,
                               p->stage_out.as<float2>(), K * p->C, 0, K, K, s);
  if (st != PFB_OK) return st;
  HIPCHK(copy_pols((float2*)out, out_ps, p->stage_out.as<float2>(), K * p->C, K * p->C, p->n_pol,
                   hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return PFB_OK;
}

static pfb_status filterbank_exec(pfb_analysis_plan* p, const pfb_cf32* in, int64_t in_ps, int64_t n_in,
                                  pfb_cf32* out, int64_t out_ps, int64_t cap, int64_t* n_out, int32_t mem,
                                  void* stream, const OutLayout* lay);

pfb_status pfb_filterbank_execute(pfb_analysis_plan* p, const pfb_cf32* in, int64_t in_ps,
                                  int64_t n_in, pfb_cf32* out, int64_t out_ps, int64_t cap,
                                  int64_t* n_out, int32_t mem, void* stream) {
  return filterbank_exec(p, in, in_ps, n_in, out, out_ps, cap, n_out, mem, stream, nullptr);
}

int64_t pfb_filterbank_output_rows(const pfb_analysis_plan* p, int64_t n_in) {
  if (!p || n_in < 0) return -1;
  const int64_t K = analysis_K(p, p->buffered + n_in);
  return K - (K % p->nu);
}

pfb_status pfb_filterbank_execute_strided(pfb_analysis_plan* p, const pfb_cf32* in, int64_t in_ps,
                                          int64_t n_in, pfb_cf32* out, int64_t out_ps,
                                          int64_t row_stride, int64_t chan_stride, int32_t sel_split,
                                          int32_t sel_shift, int32_t sel_n, int64_t cap,
                                          int64_t* n_out, void* stream) {
  if (!p || (!in && n_in > 0) || !out) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (p->variant != pfb::kBunton || !analysis_offset_ok(p) || p->lowcbf_pad)
    return fail(PFB_ERR_UNSUPPORTED, "strided output needs the streaming Bunton analysis kernel");
  if (row_stride <= 0 || chan_stride <= 0 || sel_n < 0 || sel_split < 0 || sel_shift < 0 ||
      (sel_n > 0 && sel_split + sel_shift > p->C) || sel_n > p->C)
    return fail(PFB_ERR_INVALID_ARG, "bad strided output layout");
  // one 16-row step's extent must fit a 32-bit buffer descriptor (StridedRowStore)
  const int64_t jn = sel_n > 0 ? sel_n : p->C;
  if ((64 * row_stride + jn * chan_stride + 1) * 8 > pfb::kRsrcMaxBytes)
    return fail(PFB_ERR_UNSUPPORTED, "strided output extent exceeds a buffer descriptor");
  // out_capacity counts pfb_cf32 elements from `out`: the furthest element this call writes
  // must lie inside it (a wrong stride is rejected, not written past the buffer)
  const int64_t Kt = pfb_filterbank_output_rows(p, n_in);
  if (n_out) *n_out = Kt;
  if (Kt > 0) {
    const int64_t last = (int64_t)(p->n_pol - 1) * out_ps + (Kt - 1) * row_stride + (jn - 1) * chan_stride;
    if (last >= cap)
      return fail(PFB_ERR_BUFFER_TOO_SMALL,
                  "strided output: element %lld is written but out_capacity is %lld elements",
                  (long long)last, (long long)cap);
  }
  const OutLayout lay{row_stride, chan_stride, sel_split, sel_shift, sel_n};
  return filterbank_exec(p, in, in_ps, n_in, out, out_ps, std::max<int64_t>(Kt, 0), n_out, PFB_MEM_DEVICE,
                         stream, &lay);
}

}  // extern "C"

static pfb_status filterbank_exec(pfb_analysis_plan* p, const pfb_cf32* in, int64_t in_ps, int64_t n_in,
                                  pfb_cf32* out, int64_t out_ps, int64_t cap, int64_t* n_out, int32_t mem,
                                  void* stream, const OutLayout* lay) {
  if (!p || (!in && n_in > 0)) return fail(PFB_ERR_INVALID_ARG, "null argument");
  HIPCHK(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t total = p->buffered + n_in;
  const hipMemcpyKind kin = mem == PFB_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  {
    // Carry without the concatenation copy (streaming analysis kernel, device input):
    // rows k >= ceil(B / M) read only the new input, so they run on it in place with the
    // carried B samples as a read offset (AnalysisArgs::pad); the few rows before that run
    // on a small stitched buffer of the carry and the head of the input.  The result is the
    // same per row as the concatenated run (same kernel, same samples).
    const int64_t B = p->buffered;
    const int64_t K = analysis_K(p, total);
    const int64_t Kt = K - (K % p->nu);
    const int64_t input_idat = (Kt * p->N * p->de) / p->nu;
    static const bool no_split = pfb::knob("PFB_FB_NO_SPLIT") != nullptr;  // A/B
    if (!no_split && mem == PFB_MEM_DEVICE && B > 0 && p->variant == pfb::kBunton && analysis_offset_ok(p) &&
        input_idat >= B && p->lowcbf_pad == false) {
      if (n_out) *n_out = Kt;
      if (Kt > cap) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld rows",
                                (long long)cap, (long long)Kt);
      const int64_t M = p->M, PN = (int64_t)p->P * p->N;
      // the streaming kernel's register window: DE (16 / NU) new rows per step + P (its first
      // window holds every carried sample a workgroup's rows read when B fits in it —
      // launch_stream checks the same bound)
      const int64_t win = ((int64_t)p->de * (16 / p->nu) + p->P) * p->N;
      if (B <= win) {
        // ONE launch: the streaming kernel reads the carried samples through a second
        // descriptor in its first window (AnalysisArgs::pre) — no stitched rows, no copies
        // before it; then the new carry (stream order: after the kernel read the old one).
        // (Round 5: the bound was P N; a cascade's stage-2 carry of up to P N + NU M samples
        // per series then took the stitched path — two copies and a small launch per call.)
        // (round 5) the kernel also copies the next carry into the second carry buffer —
        // no copy launch after it — and the two buffers swap
        const int64_t nb = total - input_idat;
        CarryOut co{nullptr, input_idat - B, nb, nb};
        if (nb > 0) {
          HIPCHK(p->carry_next.ensure((size_t)p->n_pol * nb * sizeof(float2)));
          co.dst = p->carry_next.as<float2>();
        }
        pfb_status st = analysis_run(p, (const float2*)in, in_ps, n_in, (float2*)out, out_ps, 0, Kt, K, s,
                                     nullptr, 0, 0, B, lay, 0, p->carry.as<float2>(), 0, nb > 0 ? &co : nullptr);
        if (st != PFB_OK) return st;
        if (nb > 0) std::swap(p->carry, p->carry_next);
        p->buffered = std::max<int64_t>(nb, 0);
        return PFB_OK;
      }
      // (even: a channel-major strided launch stores row pairs; Kt is a multiple of nu)
      const int64_t k_split = std::min(Kt, (((B + M - 1) / M) + 1) & ~(int64_t)1);
      if (k_split > 0) {
        const int64_t L = std::min(total, (k_split - 1) * M + PN);
        HIPCHK(p->work.ensure((size_t)p->n_pol * L * sizeof(float2)));
        float2* wk = p->work.as<float2>();
        HIPCHK(copy_pols(wk, L, p->carry.as<float2>(), B, std::min(B, L), p->n_pol, hipMemcpyDeviceToDevice, s));
        if (L > B) HIPCHK(copy_pols(wk + B, L, (const float2*)in, in_ps, L - B, p->n_pol, hipMemcpyDeviceToDevice, s));
        pfb_status st = analysis_run(p, wk, L, L, (float2*)out, out_ps, 0, k_split, K, s, nullptr, 0, 0, 0, lay);
        if (st != PFB_OK) return st;
      }
      if (Kt > k_split) {
        pfb_status st = analysis_run(p, (const float2*)in, in_ps, n_in, (float2*)out, out_ps, k_split, Kt, K, s,
                                     nullptr, 0, 0, B, lay);
        if (st != PFB_OK) return st;
      }
      // carry = input(:, :, input_idat + 1 : end): all of it lies in the new input
      const int64_t nb = total - input_idat;
      if (nb > 0) {
        HIPCHK(p->carry.ensure((size_t)p->n_pol * nb * sizeof(float2)));
        HIPCHK(copy_pols(p->carry.as<float2>(), nb, (const float2*)in + (input_idat - B), in_ps, nb, p->n_pol,
                         hipMemcpyDeviceToDevice, s));
      }
      p->buffered = std::max<int64_t>(nb, 0);
      return PFB_OK;
    }
  }
  {
    // Carry without the concatenation copy (fused one-launch kernels: N <= 256 shapes the
    // streaming kernel does not take, e.g. a padded cascade's stage 2): the kernel stages each
    // row's input span from the carry (`pre`, the first B samples of the series) and the input
    // in place (round 6; the SKA-Mid padded cascade copied its 613 MB of stage-2 series here).
    const int64_t B = p->buffered;
    const int64_t K = analysis_K(p, total);
    const int64_t Kt = K - (K % p->nu);
    const int64_t input_idat = (Kt * p->N * p->de) / p->nu;
    if (mem == PFB_MEM_DEVICE && B > 0 && !lay && !p->lowcbf_pad && p->fused && analysis_fused_carry_ok(p) &&
        input_idat >= B && Kt > 0) {
      if (n_out) *n_out = Kt;
      if (Kt > cap) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld rows",
                                (long long)cap, (long long)Kt);
      const int64_t Krun = p->variant == pfb::kPadded ? K : Kt;
      float2* dst = (float2*)out;
      int64_t dps = out_ps;
      if (Krun > cap) {
        HIPCHK(p->stage_out.ensure((size_t)p->n_pol * Krun * p->C * sizeof(float2)));
        dst = p->stage_out.as<float2>();
        dps = Krun * p->C;
      }
      pfb_status st = analysis_run(p, (const float2*)in, in_ps, n_in, dst, dps, 0, Krun, K, s, nullptr, 0, 0, B,
                                   nullptr, 0, p->carry.as<float2>());
      if (st != PFB_OK) return st;
      if (dst != (float2*)out)
        HIPCHK(copy_pols((float2*)out, out_ps, dst, dps, Kt * p->C, p->n_pol, hipMemcpyDeviceToDevice, s));
      // carry = series[input_idat, total): all of it in the new input; into the second carry
      // buffer (the kernel just enqueued still reads the first), then swap
      const int64_t nb = total - input_idat;
      if (nb > 0) {
        HIPCHK(p->carry_next.ensure((size_t)p->n_pol * nb * sizeof(float2)));
        HIPCHK(copy_pols(p->carry_next.as<float2>(), nb, (const float2*)in + (input_idat - B), in_ps, nb, p->n_pol,
                         hipMemcpyDeviceToDevice, s));
        std::swap(p->carry, p->carry_next);
      }
      p->buffered = std::max<int64_t>(nb, 0);
      return PFB_OK;
    }
  }
  // input = cat(3, input_buffer, input)   (FilterBank.m:85-88); with nothing buffered and
  // the input already on the device the kernels read it in place (no copy)
  const float2* w;
  int64_t wps;
  if (p->buffered == 0 && mem == PFB_MEM_DEVICE) {
    w = (const float2*)in;
    wps = in_ps;
  } else {
    HIPCHK(p->work.ensure((size_t)p->n_pol * std::max<int64_t>(total, 1) * sizeof(float2)));
    float2* wk = p->work.as<float2>();
    HIPCHK(copy_pols(wk, total, p->carry.as<float2>(), p->buffered, p->buffered, p->n_pol,
                     hipMemcpyDeviceToDevice, s));
    HIPCHK(copy_pols(wk + p->buffered, total, (const float2*)in, in_ps, n_in, p->n_pol, kin, s));
    w = wk;
    wps = total;
  }
  const int64_t K = analysis_K(p, total);
  PadConsume pad_once{&p->lowcbf_pad};
  const int64_t Kt = K - (K % p->nu);  // trim to a multiple of nu (FilterBank.m:93-104)
  if (n_out) *n_out = Kt;
  if (Kt > cap) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld rows",
                            (long long)cap, (long long)Kt);
  if (Kt > 0) {
    // rows are independent except for the padded variant's circular shift over all K
    // rows: the others compute just the Kt kept rows, straight into the caller's buffer
    const int64_t Krun = p->variant == pfb::kPadded ? K : Kt;
    float2* dst;
    int64_t dps;
    if (mem == PFB_MEM_HOST) {
      HIPCHK(p->stage_out.ensure((size_t)p->n_pol * Krun * p->C * sizeof(float2)));
      dst = p->stage_out.as<float2>();
      dps = Krun * p->C;
    } else {
      dst = (float2*)out;
      dps = out_ps;
      // padded: K rows computed (the circular shift spans all of them), Kt returned; they go
      // straight into the caller's buffer when it has room for K rows (rows [Kt, K) are then
      // scratch, pfb_filterbank_execute's contract), else through a staging buffer and a copy
      // (round 6: the SKA-Mid cascade's stage 2 lost a 244-us copy per call)
      if (Krun > cap) {
        HIPCHK(p->stage_out.ensure((size_t)p->n_pol * Krun * p->C * sizeof(float2)));
        dst = p->stage_out.as<float2>();
        dps = Krun * p->C;
      }
    }
    if (lay && dst != (float2*)out) return fail(PFB_ERR_UNSUPPORTED, "strided output through a staging buffer");
    pfb_status st = analysis_run(p, w, wps, total, dst, dps, 0, Krun, K, s, nullptr, 0, 0, 0, lay);
    if (st != PFB_OK) return st;
    if (dst != (float2*)out) {
      const hipMemcpyKind ko = mem == PFB_MEM_HOST ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
      HIPCHK(copy_pols((float2*)out, out_ps, dst, dps, Kt * p->C, p->n_pol, ko, s));
    }
  }
  // carry = input(:,:,input_idat+1:end), input_idat = T_out N de / nu   (FilterBank.m:119-126)
  const int64_t input_idat = (Kt * p->N * p->de) / p->nu;
  const int64_t nb = total - input_idat;
  if (nb > 0) {
    HIPCHK(p->carry.ensure((size_t)p->n_pol * nb * sizeof(float2)));
    // carry may alias nothing in `work` (separate buffer); copy per pol
    HIPCHK(copy_pols(p->carry.as<float2>(), nb, w + input_idat, wps, nb, p->n_pol,
                     hipMemcpyDeviceToDevice, s));
  }
  p->buffered = std::max<int64_t>(nb, 0);
  if (mem == PFB_MEM_HOST) HIPCHK(hipStreamSynchronize(s));
  return PFB_OK;
}

extern "C" {

int64_t pfb_filterbank_buffered(const pfb_analysis_plan* p) { return p ? p->buffered : -1; }

pfb_status pfb_filterbank_reset(pfb_analysis_plan* p) {
  if (!p) return fail(PFB_ERR_INVALID_ARG, "null plan");
  p->buffered = 0;
  p->lowcbf_pad = p->variant == pfb::kLowCbf;
  return PFB_OK;
}

}  // extern "C"

// ====================================================================== synthesis plan
struct pfb_synthesis_plan {
  int device = 0;
  int N = 0, nu = 1, de = 1, Nf = 0, Ov = 0, spans = 1, combine = 1, n_pol = 1;
  int W = 0, keep = 0, L = 0, Lov = 0, Lkeep = 0, t1_lo = 0, t1_hi = 0;
  bool deripple = false;
  int chunk_blocks = 0;
  int stage1 = PFB_STAGE1_AUTO;  // pfb_synthesis_set_stage1_rows
  int last_stage1 = 0;           // pfb_synthesis_last_stage1_rows: where the last launch got its rows
  int rt_chunk_blocks = 64;  // round-trip pipeline chunk (PFB_RT_CHUNK_BLOCKS)
  int timing_mask = 0;  // PFB_TIMING_MASK (timing experiments; results invalid when set)
  int ranges = -1;  // PFB_SYNTH_RANGES: 0 one workgroup per block, -1 persistent auto, >0 persistent
  int no_reuse = 0;  // PFB_SYNTH_NO_REUSE: re-read the overlap rows (A/B measurement only)
  int xcd = 1;       // PFB_SYNTH_XCD=0: plain workgroup order (A/B measurement only)
  bool identity_perm = true;
  bool win_flat = false;  // SynthBlockArgs::win_flat
  bool has_cgain = false;
  bool has_spectral = false;  // non-identity spectral taper: pfb_spectral.hip path
  DevBuf window, tw4, tw4s, twN, twNf, twW, perm, cgain;
  DevBuf taper, gainj, sbuf0, sbuf1;  // spectral taper (L), deripple gains (W), scratch
  DevBuf Z, carry, work, stage_in, stage_out;
  int64_t buffered = 0;
  int64_t ifb_offset = 0;  // InverseFilterBank.sample_offset (0-based; InverseFilterBank.m:12)
  // split round trip: what the analysis half left in Z (analysis plan, n_dat, sample
  // offset, row layout, rows) — the synthesis half must match it; cleared whenever Z is
  // written by anything else
  uint64_t zkey_plan = 0;
  int64_t zkey[5] = {-1, -1, -1, -1, -1};
  // (recomputed rows: the analysis half left no rows, only the input the synthesis reads)
  const void* zkey_x = nullptr;
  int64_t zkey_xps = -1;
};

// PFB_STAGE1_AUTO: recomputed stage-1 rows in the Nf = 256 round trip
constexpr bool kSynthFirDefault = false;

static void zkey_clear(pfb_synthesis_plan* p) {
  p->zkey_plan = 0;
  std::fill(p->zkey, p->zkey + 5, (int64_t)-1);
  p->zkey_x = nullptr;
  p->zkey_xps = -1;
}

// the input series a synthesis recomputes its stage-1 rows from (SynthBlockArgs::fir_*)
struct FirSrc {
  const float2* x;
  int64_t x_ps, n_dat, q0;
  const float* g;
  int nu, de, pe;
};

static void hann_sym(int L, std::vector<double>& h) {
  h.resize((size_t)L);
  if (L == 1) {
    h[0] = 1.0;
    return;
  }
  for (int n = 0; n < L; ++n) h[(size_t)n] = 0.5 * (1.0 - std::cos(2.0 * M_PI * n / (L - 1)));
}

static int64_t synth_blocks(const pfb_synthesis_plan* p, int64_t n_dat) {
  const int64_t b = floordiv(n_dat - 2 * (int64_t)p->Ov, p->keep);
  return std::max<int64_t>(b, 0);
}

static pfb_status synthesis_blocks(pfb_synthesis_plan* p, const float2* Z, int64_t z_ps, int64_t b0,
                                   int64_t nb, float2* out, int64_t out_ps, int64_t out_limit,
                                   hipStream_t s, int zblk = 0, const FirSrc* fir = nullptr);
static pfb::SynthBlockArgs synth_args(const pfb_synthesis_plan* p, const float2* Z, int64_t z_ps,
                                      int64_t b0, int64_t nb, float2* out, int64_t out_ps,
                                      int64_t out_limit, int zblk = 0, const FirSrc* fir = nullptr);

// Blocks [b0, b0 + nb) with a spectral taper (pfb_spectral.hip): Matlab's order — per
// channel FFT, stitch x taper, then the L-point IFFT as row FFTs — in sub-chunks whose
// scratch stays within 2^26 values per buffer.
static pfb_status synthesis_spectral(pfb_synthesis_plan* p, const float2* in, int64_t in_ps, int64_t b0,
                                     int64_t nb, float2* out, int64_t out_ps, int64_t out_limit,
                                     hipStream_t s) {
  p->last_stage1 = PFB_STAGE1_STORED;  // (the spectral passes read the channelised rows)
  const int64_t per_block = (int64_t)p->N * std::max(p->Nf, p->W);
  const int64_t sub = std::max<int64_t>(1, std::min<int64_t>(65535, ((int64_t)1 << 26) / per_block));
  const int64_t nsub = std::min(sub, nb);
  HIPCHK(p->sbuf0.ensure((size_t)nsub * per_block * sizeof(float2)));
  HIPCHK(p->sbuf1.ensure((size_t)nsub * per_block * sizeof(float2)));
  for (int64_t c0 = b0; c0 < b0 + nb; c0 += nsub) {
    pfb::SpectralArgs a{};
    a.in = in;
    a.in_pol_stride = in_ps;
    a.out = out;
    a.out_pol_stride = out_ps;
    a.out_limit = out_limit;
    a.b0 = c0;
    a.nb = std::min(nsub, b0 + nb - c0);
    a.n_pol = p->n_pol;
    a.N = p->N;
    a.Nf = p->Nf;
    a.W = p->W;
    a.keep = p->keep;
    a.L = p->L;
    a.Lov = p->Lov;
    a.Lkeep = p->Lkeep;
    a.t1_lo = p->t1_lo;
    a.t1_hi = p->t1_hi;
    a.spans = p->spans;
    a.scale = (float)((double)p->de / (double)p->nu / (double)p->L);
    a.window = p->window.as<float>();
    a.cgain = p->has_cgain ? p->cgain.as<float>() : nullptr;
    a.perm = p->identity_perm ? nullptr : p->perm.as<int>();
    a.gainj = p->gainj.as<float>();
    a.taper = p->taper.as<float>();
    a.twNf = p->twNf.as<float2>();
    a.twN = p->twN.as<float2>();
    a.twW = p->twW.as<float2>();
    a.buf0 = p->sbuf0.as<float2>();
    a.buf1 = p->sbuf1.as<float2>();
    ProfScope ps(2, (double)p->n_pol * a.nb * ((double)p->keep * p->N * 8.0 + p->Lkeep * 8.0), s, false);
    HIPCHK(pfb::launch_spectral_synth(a, s));
  }
  return PFB_OK;
}

// Blocks [b0, b0 + nb) of a call: channel IFFT of their rows into Z, then the block
// kernel.  `in` is the call's first channelised row (sample_offset applied).
// (row_shift: `in` holds the call's channelised rows from row row_shift on — a streaming
// call whose carried rows are not in front of it; blocks b0.. must not read before it.  A
// negative row_shift: block 0 starts -row_shift rows into `in` (InverseFilterBank's
// sample_offset applied to the concatenated rows))
static pfb_status synthesis_chunk(pfb_synthesis_plan* p, const float2* in, int64_t in_ps, int64_t b0,
                                  int64_t nb, float2* out, int64_t out_ps, int64_t out_limit,
                                  hipStream_t s, int64_t row_shift = 0) {
  if (p->has_spectral) {
    // (a negative row shift: the blocks start -row_shift rows into `in` — a sample offset)
    if (row_shift > 0) return fail(PFB_ERR_UNSUPPORTED, "row shift with a spectral taper");
    return synthesis_spectral(p, in + (-row_shift) * p->N, in_ps, b0, nb, out, out_ps, out_limit, s);
  }
  const int64_t rows = nb * p->keep + 2 * (int64_t)p->Ov;
  zkey_clear(p);
  HIPCHK(p->Z.ensure((size_t)p->n_pol * rows * p->N * sizeof(float2)));
  float2* Z = p->Z.as<float2>();
  pfb::ChanIfftArgs c{};
  c.in = in + (b0 * p->keep - row_shift) * p->N;
  c.in_pol_stride = in_ps;
  c.out = Z;
  c.out_pol_stride = rows * p->N;
  c.n_rows = rows;
  c.n_pol = p->n_pol;
  c.N = p->N;
  c.perm = p->identity_perm ? nullptr : p->perm.as<int>();
  c.cgain = p->has_cgain ? p->cgain.as<float>() : nullptr;
  c.twN = p->twN.as<float2>();
  // the Nf = 256 shapes: Z in the 2-row run layout the wave kernel reads (256-B runs per
  // load instruction, as the fused round trip's analysis writes it); every other shape
  // [row][t0] for the block kernel
  const int zb = pfb::synth_wave_supported(synth_args(p, Z, rows * p->N, b0, nb, out, out_ps, out_limit, 2)) ? 2 : 0;
  c.zblk = zb ? zb : 1;
  {
    ProfScope ps(1, (double)p->n_pol * rows * p->N * 16.0, s);
    HIPCHK(pfb::launch_chan_ifft(c, s));
  }
  return synthesis_blocks(p, Z, rows * p->N, b0, nb, out, out_ps, out_limit, s, zb);
}

// Block kernel over blocks [b0, b0 + nb); Z row 0 is channelised row b0 * keep.
static pfb::SynthBlockArgs synth_args(const pfb_synthesis_plan* p, const float2* Z, int64_t z_ps,
                                      int64_t b0, int64_t nb, float2* out, int64_t out_ps,
                                      int64_t out_limit, int zblk, const FirSrc* fir) {
  pfb::SynthBlockArgs a{};
  if (fir) {
    a.fir_x = fir->x;
    a.fir_x_pol_stride = fir->x_ps;
    a.fir_n_dat = fir->n_dat;
    a.fir_g = fir->g;
    a.fir_q0 = fir->q0;
    a.fir_nu = fir->nu;
    a.fir_de = fir->de;
    a.fir_pe = fir->pe;
  }
  a.Z = Z;
  a.z_pol_stride = z_ps;
  a.out = out;
  a.out_pol_stride = out_ps;
  a.block0 = b0;
  a.n_blocks = (int)nb;
  a.n_pol = p->n_pol;
  a.N = p->N;
  a.Nf = p->Nf;
  a.W = p->W;
  a.keep = p->keep;
  a.L = p->L;
  a.Lov = p->Lov;
  a.Lkeep = p->Lkeep;
  a.t1_lo = p->t1_lo;
  a.t1_hi = p->t1_hi;
  a.scale = (float)((double)p->de / (double)p->nu / (double)p->L);
  a.window = p->window.as<float>();
  a.win_flat = p->win_flat ? 1 : 0;
  a.spans = p->spans;
  a.tw4 = p->tw4.as<float2>();
  a.tw4s = p->tw4s.as<float2>();
  a.twNf = p->twNf.as<float2>();
  a.twW = p->twW.as<float2>();
  a.out_limit = out_limit;
  a.ranges = p->ranges;
  a.no_reuse = p->no_reuse;
  a.xcd = p->xcd;
  a.timing_mask = p->timing_mask;
  a.zblk = zblk;
  return a;
}

static pfb_status synthesis_blocks(pfb_synthesis_plan* p, const float2* Z, int64_t z_ps, int64_t b0,
                                   int64_t nb, float2* out, int64_t out_ps, int64_t out_limit,
                                   hipStream_t s, int zblk, const FirSrc* fir) {
  const pfb::SynthBlockArgs a = synth_args(p, Z, z_ps, b0, nb, out, out_ps, out_limit, zblk, fir);
  p->last_stage1 = fir ? PFB_STAGE1_RECOMPUTED : PFB_STAGE1_STORED;
  {
    ProfScope ps(2, (double)p->n_pol * (nb * p->keep * p->N * 8.0 + nb * p->Lkeep * 8.0), s);
    HIPCHK(pfb::launch_synth_block(a, s));
  }
  return PFB_OK;
}

static int64_t synthesis_chunk_blocks(const pfb_synthesis_plan* p, int64_t B) {
  int64_t CB = p->chunk_blocks;
  if (CB <= 0) {
    // one chunk up to 2^26 channel-rows x channels (512 MB of Z); fewer, larger
    // launches measured faster than MALL-sized chunks (profiles/r01 sweep)
    const int64_t target = (int64_t)1 << 26;
    CB = std::max<int64_t>(1, target / ((int64_t)p->keep * p->N * p->n_pol));
  }
  return std::min<int64_t>(CB, B);
}

// blocks [b_lo, b_hi) in chunks (see synthesis_chunk for row_shift)
static pfb_status synthesis_range(pfb_synthesis_plan* p, const float2* in, int64_t in_ps, int64_t b_lo,
                                  int64_t b_hi, float2* out, int64_t out_ps, int64_t out_limit,
                                  hipStream_t s, int64_t row_shift = 0) {
  if (b_hi <= b_lo) return PFB_OK;
  const int64_t CB = synthesis_chunk_blocks(p, b_hi - b_lo);
  for (int64_t b0 = b_lo; b0 < b_hi; b0 += CB) {
    pfb_status st = synthesis_chunk(p, in, in_ps, b0, std::min<int64_t>(CB, b_hi - b0), out, out_ps,
                                    out_limit, s, row_shift);
    if (st != PFB_OK) return st;
  }
  return PFB_OK;
}

static pfb_status synthesis_run(pfb_synthesis_plan* p, const float2* in, int64_t in_ps, int64_t n_dat,
                                float2* out, int64_t out_ps, int64_t out_limit, hipStream_t s) {
  return synthesis_range(p, in, in_ps, 0, synth_blocks(p, n_dat), out, out_ps, out_limit, s);
}

extern "C" {

// Descriptor checks of pfb_synthesis_plan_create (no device needed)
static pfb_status synthesis_validate(const pfb_synthesis_desc* d) {
  if (!d) return fail(PFB_ERR_INVALID_ARG, "null argument");
  const int N = d->n_chan, nu = d->os_nu, de = d->os_de, Nf = d->input_fft_length,
            Ov = d->input_overlap;
  if (N <= 0 || nu <= 0 || de <= 0 || Nf <= 0 || Ov < 0 || d->n_pol <= 0)
    return fail(PFB_ERR_INVALID_ARG, "invalid synthesis parameters");
  // (sizes whose products the tables and kernels form in 32-bit ints: far beyond any
  // configuration, rejected before any arithmetic on them)
  if (N > (1 << 24) || Nf > (1 << 24) || de > (1 << 16) || nu > (1 << 16))
    return fail(PFB_ERR_UNSUPPORTED, "synthesis parameters out of range (n_chan %d, Nf %d, Ov %d, os %d/%d)",
                N, Nf, Ov, nu, de);
  if (d->n_pol > 65535)  // polarisations map to grid.y of every launch
    return fail(PFB_ERR_INVALID_ARG, "n_pol = %d exceeds 65535 series per plan", d->n_pol);
  if (((int64_t)Nf * de) % nu != 0)
    return fail(PFB_ERR_INVALID_ARG, "input_fft_length*de/nu = %d*%d/%d is not integral", Nf, de, nu);
  if (((int64_t)Ov * de * N) % nu != 0)
    return fail(PFB_ERR_INVALID_ARG, "output_overlap = Ov*de/nu*n_chan is not integral");
  if ((int64_t)Nf - 2 * (int64_t)Ov <= 0)
    return fail(PFB_ERR_INVALID_ARG, "input_keep = Nf - 2 Ov must be positive");
  const int W = (int)(((int64_t)Nf * de) / nu);
  if (W % 2 != 0) return fail(PFB_ERR_INVALID_ARG, "FN_width %d must be even", W);
  if (d->combine < 1 || N % d->combine != 0)
    return fail(PFB_ERR_INVALID_ARG, "combine=%d must divide n_chan=%d", d->combine, N);
  // spectral tapers act on the stitched L-vector (polyphase_synthesis.m:282): 'hann'
  // (PFBWindow.m:70-100, circshift(hann(L), L/2) on an L-row column) or explicit L
  // coefficients; tukey / top_hat index columns 1..Ov of that L x 1 column and have no
  // defined meaning there
  if (d->spectral_taper != PFB_WINDOW_NONE && d->spectral_taper != PFB_WINDOW_HANN &&
      d->spectral_taper != PFB_WINDOW_CUSTOM)
    return fail(PFB_ERR_INVALID_ARG,
                "spectral taper %d: only identity, hann or custom (L coefficients) act on the "
                "stitched spectrum", d->spectral_taper);
  if (d->spectral_taper == PFB_WINDOW_CUSTOM && !d->spectral_coeffs)
    return fail(PFB_ERR_INVALID_ARG, "CUSTOM spectral taper without coefficients");
  if (d->spectral_taper != PFB_WINDOW_NONE &&
      !pfb::spectral_synth_supported(Nf, (int)(((int64_t)Nf * de) / nu), N))
    return fail(PFB_ERR_UNSUPPORTED, "no spectral-taper synthesis kernels for Nf=%d n_chan=%d", Nf, N);
  if (!pfb::chan_ifft_supported(N))
    return fail(PFB_ERR_UNSUPPORTED, "no channel-IFFT kernel for n_chan=%d", N);
  if (!pfb::synth_block_supported(Nf, W))
    return fail(PFB_ERR_UNSUPPORTED, "no synthesis kernel for Nf=%d W=%d", Nf, W);
  // the block kernel's buffer descriptors span one block's output (L_keep samples), the
  // gain x twiddle table (L values) and one block's stage-1 rows (Nf x N): each must fit
  // one 32-bit descriptor extent (pfb::kRsrcMaxBytes) — rejected here, never clamped
  if ((int64_t)W * N * 8 > pfb::kRsrcMaxBytes || (int64_t)Nf * N * 8 > pfb::kRsrcMaxBytes)
    return fail(PFB_ERR_UNSUPPORTED,
                "output_fft_length %lld or Nf x n_chan %lld exceeds a buffer descriptor "
                "(%lld bytes)", (long long)W * N, (long long)Nf * N, (long long)pfb::kRsrcMaxBytes);
  if (d->temporal_taper == PFB_WINDOW_CUSTOM && !d->temporal_coeffs)
    return fail(PFB_ERR_INVALID_ARG, "CUSTOM temporal taper without coefficients");
  if (d->temporal_taper < PFB_WINDOW_NONE || d->temporal_taper > PFB_WINDOW_CUSTOM)
    return fail(PFB_ERR_INVALID_ARG, "unknown temporal taper %d", d->temporal_taper);
  if (d->apply_deripple && (!d->taps || d->n_taps <= 0))
    return fail(PFB_ERR_INVALID_ARG, "deripple requested without filter taps");
  return PFB_OK;
}

// Host-side tables of a synthesis plan (double maths, rounded once to float)
struct SynthHost {
  int N = 0, nu = 1, de = 1, Nf = 0, Ov = 0, W = 0, keep = 0, L = 0, Lov = 0, Lkeep = 0;
  int t1_lo = 0, t1_hi = 0, spans = 1, combine = 1;
  bool deripple = false, identity_perm = true, win_flat = false;
  std::vector<float> window, cgain, taper, gj;
  std::vector<int> perm;
  std::vector<float2> tw4, tw4s;
};

static void synthesis_host_tables(const pfb_synthesis_desc* d, SynthHost& p) {
  const int N = d->n_chan, nu = d->os_nu, de = d->os_de, Nf = d->input_fft_length, Ov = d->input_overlap;
  const int W = (int)(((int64_t)Nf * de) / nu);
  p.N = N;
  p.nu = nu;
  p.de = de;
  p.Nf = Nf;
  p.Ov = Ov;
  p.spans = d->spans_nyquist ? 1 : 0;
  p.combine = d->combine;
  p.W = W;
  p.keep = Nf - 2 * Ov;
  p.L = W * N;
  p.Lov = (int)(((int64_t)Ov * de * N) / nu);
  p.Lkeep = p.L - 2 * p.Lov;
  // the kernels keep y[t0 + N t1] when L_ov <= t0 + N t1 < L - L_ov (sample-exact: L_ov =
  // Ov de/nu N need not be a multiple of N — normalize(os, Ov) = 40.5 for the reference's
  // 'sps' config); [t1_lo, t1_hi) bounds the t1 that hold any kept sample
  p.t1_lo = p.Lov / N;
  p.t1_hi = W - p.t1_lo;
  p.deripple = d->apply_deripple != 0;

  // temporal taper (PFBWindow.m) -> per-time window + per-channel gain (hann quirk)
  std::vector<float>& window = p.window;
  window.assign((size_t)Nf, 1.f);
  switch (d->temporal_taper) {
    case PFB_WINDOW_NONE: break;
    case PFB_WINDOW_TUKEY: {
      std::vector<double> h;
      hann_sym(2 * Ov, h);
      for (int t = 0; t < Ov; ++t) window[(size_t)t] = (float)h[(size_t)t];
      for (int t = 0; t < Ov; ++t) window[(size_t)(Nf - Ov + t)] = (float)h[(size_t)(Ov + t)];
      break;
    }
    case PFB_WINDOW_TOP_HAT:
      for (int t = 0; t < Ov; ++t) {
        window[(size_t)t] = 0.f;
        window[(size_t)(Nf - 1 - t)] = 0.f;
      }
      break;
    case PFB_WINDOW_HANN: {
      // PFBWindow.m:72-99: hann along dim 1 = channels; circshift when n_chan != Nf
      std::vector<double> h;
      hann_sym(N, h);
      p.cgain.resize((size_t)N);
      for (int c = 0; c < N; ++c) {
        const int src = (N != Nf) ? ((c - N / 2) % N + N) % N : c;
        p.cgain[(size_t)c] = (float)h[(size_t)src];
      }
      break;
    }
    case PFB_WINDOW_CUSTOM:
      for (int t = 0; t < Nf; ++t) window[(size_t)t] = (float)d->temporal_coeffs[t];
      break;
    default: break;  // rejected by synthesis_validate
  }

  // combine permutation (polyphase_synthesis.m:198-239): slot chan <- input jchan
  std::vector<int>& perm = p.perm;
  perm.resize((size_t)N);
  for (int c = 0; c < N; ++c) perm[(size_t)c] = c;
  if (p.combine > 1) {
    const int fcc = N / p.combine, fco = N;
    for (int chan = 0; chan < N; ++chan) {
      int fine = (chan + fcc / 2) % fco;
      int coarse = fine / fcc;
      fine -= coarse * fcc;
      coarse = (coarse + p.combine / 2) % p.combine;
      fine = (fine + fcc / 2) % fcc;
      perm[(size_t)chan] = coarse * fcc + fine;
    }
  }
  for (int c = 0; c < N; ++c)
    if (perm[(size_t)c] != c) p.identity_perm = false;

  // kept-bin tables (see oracle.synthesis_tables and DESIGN.md)
  const int W2 = W / 2, d2 = (Nf - W) / 2;
  std::vector<double> g(W2 + 1, 1.0);
  if (p.deripple) {
    // H0 = freqz(h, 1, n), n = N*W/2; filter_response = 1/|H0(0..W/2)|  (:138-150)
    const int64_t nfz = (int64_t)N * W2;
    const int64_t two_n = 2 * nfz;
    for (int k = 0; k <= W2; ++k) {
      double re = 0.0, im = 0.0;
      for (int64_t i = 0; i < d->n_taps; ++i) {
        const int64_t m = ((int64_t)k * i) % two_n;  // angle = pi k i / n = 2 pi m / (2n)
        const double a = 2.0 * M_PI * (double)m / (double)two_n;
        re += d->taps[i] * std::cos(a);
        im -= d->taps[i] * std::sin(a);
      }
      g[(size_t)k] = 1.0 / std::sqrt(re * re + im * im);
    }
  }
  std::vector<int> src((size_t)W), expo((size_t)W);
  std::vector<double> gain((size_t)W);
  for (int jp = 0; jp < W; ++jp) {
    int j, e;
    if (p.spans) {
      j = (jp + W2) % W;
      e = (jp < W2) ? jp : jp - W;
    } else {
      j = jp;
      e = jp;
    }
    src[(size_t)jp] = (d2 + j + Nf / 2) % Nf;
    expo[(size_t)jp] = e;
    gain[(size_t)jp] = (j < W2) ? g[(size_t)(W2 - j)] : g[(size_t)(j - W2)];
  }
  // the rows the wave synthesis kernels treat as flat: [48, 208) at Nf 256, [128, 384) at 512
  p.win_flat = (Nf == 256 || Nf == 512) &&
               std::all_of(window.begin() + (Nf == 256 ? 48 : 128), window.begin() + (Nf == 256 ? 208 : 384),
                           [](float w) { return w == 1.f; });
  // four-step twiddle x deripple gain, laid out [j'][t0] (coalesced in the block kernel)
  p.tw4.resize((size_t)N * W);
  p.tw4s.resize((size_t)N * W);
  const double oscale = (double)p.de / (double)p.nu / (double)p.L;
  for (int t0 = 0; t0 < N; ++t0) {
    for (int jp = 0; jp < W; ++jp) {
      int64_t m = ((int64_t)t0 * expo[(size_t)jp]) % p.L;
      if (m < 0) m += p.L;
      if (2 * m > p.L) m -= p.L;
      const double ang = 2.0 * M_PI * (double)m / (double)p.L;
      const double gj = gain[(size_t)jp];
      p.tw4[(size_t)jp * N + t0] = make_float2((float)(gj * std::cos(ang)), (float)(gj * std::sin(ang)));
      p.tw4s[(size_t)jp * N + t0] =
          make_float2((float)(oscale * gj * std::cos(ang)), (float)(oscale * gj * std::sin(ang)));
    }
  }
  if (d->spectral_taper != PFB_WINDOW_NONE) {
    p.taper.resize((size_t)p.L);
    if (d->spectral_taper == PFB_WINDOW_HANN) {
      // hann(L) circularly shifted by L/2 (PFBWindow.m:83-95: ndat = L != Nf)
      std::vector<double> h;
      hann_sym(p.L, h);
      for (int i = 0; i < p.L; ++i) p.taper[(size_t)i] = (float)h[(size_t)((i - p.L / 2 + p.L) % p.L)];
    } else {
      for (int i = 0; i < p.L; ++i) p.taper[(size_t)i] = (float)d->spectral_coeffs[i];
    }
    // deripple gains in Matlab's FN row order j (polyphase_synthesis.m:244-250)
    p.gj.resize((size_t)W);
    for (int j = 0; j < W; ++j) p.gj[(size_t)j] = (float)((j < W2) ? g[(size_t)(W2 - j)] : g[(size_t)(j - W2)]);
  }
}

static void synthesis_release(pfb_synthesis_plan* p) {
  for (DevBuf* b : {&p->window, &p->tw4, &p->tw4s, &p->twN, &p->twNf, &p->twW, &p->perm, &p->cgain,
                    &p->taper, &p->gainj, &p->sbuf0, &p->sbuf1, &p->Z, &p->carry, &p->work,
                    &p->stage_in, &p->stage_out})
    b->release();
}

pfb_status pfb_synthesis_plan_validate(const pfb_synthesis_desc* d) {
  const pfb_status st = synthesis_validate(d);
  if (st != PFB_OK) return st;
  SynthHost h;
  synthesis_host_tables(d, h);
  return PFB_OK;
}

pfb_status pfb_synthesis_plan_create(const pfb_synthesis_desc* d, pfb_synthesis_plan** out) {
  if (!d || !out) return fail(PFB_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  const pfb_status vst = synthesis_validate(d);
  if (vst != PFB_OK) return vst;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(PFB_ERR_NO_DEVICE, "no HIP device available");
  if (d->device < 0 || d->device >= ndev)
    return fail(PFB_ERR_INVALID_ARG, "device %d out of range", d->device);
  HIPCHK(hipSetDevice(d->device));

  SynthHost h;
  synthesis_host_tables(d, h);
  auto* p = new pfb_synthesis_plan();
  p->device = d->device;
  if (const char* v = pfb::knob("PFB_SYNTH_RANGES")) p->ranges = std::max(-1, std::atoi(v));
  if (const char* v = pfb::knob("PFB_TIMING_MASK")) p->timing_mask = std::atoi(v);
  if (const char* v = pfb::knob("PFB_SYNTH_NO_REUSE")) p->no_reuse = std::atoi(v) != 0;
  if (const char* v = pfb::knob("PFB_SYNTH_XCD")) p->xcd = std::atoi(v) != 0;
  if (const char* v = pfb::knob("PFB_RT_CHUNK_BLOCKS")) p->rt_chunk_blocks = std::max(1, std::atoi(v));
  p->N = h.N;
  p->nu = h.nu;
  p->de = h.de;
  p->Nf = h.Nf;
  p->Ov = h.Ov;
  p->spans = h.spans;
  p->combine = h.combine;
  p->n_pol = d->n_pol;
  p->W = h.W;
  p->keep = h.keep;
  p->L = h.L;
  p->Lov = h.Lov;
  p->Lkeep = h.Lkeep;
  p->t1_lo = h.t1_lo;
  p->t1_hi = h.t1_hi;
  p->deripple = h.deripple;
  p->identity_perm = h.identity_perm;
  p->win_flat = h.win_flat;
  hipError_t e = upload(p->window, h.window);
  if (e == hipSuccess) e = upload(p->tw4, h.tw4);
  if (e == hipSuccess) e = upload(p->tw4s, h.tw4s);
  if (e == hipSuccess) e = upload(p->perm, h.perm);
  if (e == hipSuccess && !h.cgain.empty()) {
    e = upload(p->cgain, h.cgain);
    p->has_cgain = true;
  }
  if (e == hipSuccess) e = upload(p->twN, twiddles(h.N, -1));
  if (e == hipSuccess) e = upload(p->twNf, twiddles(h.Nf, -1));
  if (e == hipSuccess) e = upload(p->twW, twiddles(h.W, -1));
  if (e == hipSuccess && d->spectral_taper != PFB_WINDOW_NONE) {
    p->has_spectral = true;
    e = upload(p->taper, h.taper);
    if (e == hipSuccess) e = upload(p->gainj, h.gj);
  }
  if (e != hipSuccess) {
    synthesis_release(p);
    delete p;
    return fail(PFB_ERR_HIP, "synthesis plan upload: %s", hipGetErrorString(e));
  }
  *out = p;
  return PFB_OK;
}

pfb_status pfb_synthesis_plan_destroy(pfb_synthesis_plan* p) {
  if (!p) return PFB_OK;
  (void)hipSetDevice(p->device);
  synthesis_release(p);
  delete p;
  return PFB_OK;
}

int64_t pfb_synthesis_output_length(const pfb_synthesis_plan* p, int64_t n_dat) {
  if (!p) return -1;
  return synth_blocks(p, n_dat) * p->Lkeep;
}

pfb_status pfb_synthesis_set_stage1_rows(pfb_synthesis_plan* p, int32_t mode) {
  if (!p) return fail(PFB_ERR_INVALID_ARG, "null plan");
  if (mode != PFB_STAGE1_AUTO && mode != PFB_STAGE1_STORED && mode != PFB_STAGE1_RECOMPUTED)
    return fail(PFB_ERR_INVALID_ARG, "unknown stage-1 row mode %d", mode);
  p->stage1 = mode;
  zkey_clear(p);  // a split round trip in flight is not continued under another mode
  return PFB_OK;
}

int32_t pfb_synthesis_last_stage1_rows(const pfb_synthesis_plan* p) { return p ? p->last_stage1 : -1; }

pfb_status pfb_synthesis_set_chunk_blocks(pfb_synthesis_plan* p, int32_t blocks) {
  if (!p) return fail(PFB_ERR_INVALID_ARG, "null plan");
  p->chunk_blocks = std::max(0, blocks);
  return PFB_OK;
}

pfb_status pfb_synthesis_execute(pfb_synthesis_plan* p, const pfb_cf32* in, int64_t in_ps,
                                 int64_t n_dat, int64_t sample_offset, pfb_cf32* out,
                                 int64_t out_ps, int64_t cap, int64_t* n_out, int32_t mem,
                                 void* stream) {
  if (!p || (!in && n_dat > 0)) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (sample_offset < 1) return fail(PFB_ERR_INVALID_ARG, "sample_offset is 1-based (>= 1)");
  HIPCHK(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t off = std::min<int64_t>(sample_offset - 1, std::max<int64_t>(n_dat, 0));
  const int64_t n = n_dat - off;  // in = in(:, :, sample_offset:end)  (:99)
  const int64_t olen = synth_blocks(p, n) * p->Lkeep;
  if (n_out) *n_out = olen;
  if (olen == 0) return PFB_OK;
  if (!out) return fail(PFB_ERR_INVALID_ARG, "null output");
  if (cap < olen) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld",
                              (long long)cap, (long long)olen);
  if (mem == PFB_MEM_DEVICE) {
    if (in_ps < n_dat * p->N || out_ps < olen)
      return fail(PFB_ERR_INVALID_ARG, "polarisation stride smaller than the data");
    return synthesis_run(p, (const float2*)in + off * p->N, in_ps, n, (float2*)out, out_ps, olen, s);
  }
  HIPCHK(p->stage_in.ensure((size_t)p->n_pol * n * p->N * sizeof(float2)));
  HIPCHK(p->stage_out.ensure((size_t)p->n_pol * olen * sizeof(float2)));
  HIPCHK(copy_pols(p->stage_in.as<float2>(), n * p->N, (const float2*)in + off * p->N, in_ps,
                   n * p->N, p->n_pol, hipMemcpyHostToDevice, s));
  pfb_status st = synthesis_run(p, p->stage_in.as<float2>(), n * p->N, n, p->stage_out.as<float2>(),
                                olen, olen, s);
  if (st != PFB_OK) return st;
  HIPCHK(copy_pols((float2*)out, out_ps, p->stage_out.as<float2>(), olen, olen, p->n_pol,
                   hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return PFB_OK;
}

pfb_status pfb_inverse_filterbank_set_sample_offset(pfb_synthesis_plan* p, int64_t sample_offset) {
  if (!p) return fail(PFB_ERR_INVALID_ARG, "null plan");
  if (sample_offset < 0) return fail(PFB_ERR_INVALID_ARG, "sample_offset is 0-based (>= 0)");
  p->ifb_offset = sample_offset;
  return PFB_OK;
}

// InverseFilterBank.m:73-135.  Every call runs polyphase_synthesis on the concatenated
// rows (carry + input) from row `so` = sample_offset on (:92-96, `sample_offset+1`), and the
// carry starts at input_idat = (output length) nu / (n_chan de) = B keep of the
// concatenation — not offset by `so`: the next call skips `so` rows of it again, so
// consecutive calls see the blocks of one continuous run.
pfb_status pfb_inverse_filterbank_execute(pfb_synthesis_plan* p, const pfb_cf32* in, int64_t in_ps,
                                          int64_t n_in, pfb_cf32* out, int64_t out_ps, int64_t cap,
                                          int64_t* n_out, int32_t mem, void* stream) {
  if (!p || (!in && n_in > 0)) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (n_in < 0) return fail(PFB_ERR_INVALID_ARG, "negative n_in");
  HIPCHK(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  const int N = p->N;
  const int64_t total = p->buffered + n_in;
  const hipMemcpyKind kin = mem == PFB_MEM_HOST ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
  const int64_t so = std::min(p->ifb_offset, total);  // in(:, :, sample_offset:end)
  // output length and carry-over rounded up to a multiple of nu (InverseFilterBank.m:104-135)
  const int64_t B = synth_blocks(p, total - so);
  const int64_t full = B * p->Lkeep;
  int64_t input_idat = B * p->keep;
  int64_t buffered = total - input_idat;
  int64_t olen = full;
  const int64_t rem = ((buffered % p->nu) + p->nu) % p->nu;
  if (rem != 0) {
    buffered += p->nu - rem;
    input_idat = total - buffered;
    // output_ndat = input_idat * (n_chan de)/nu, used as a Matlab colon end (floor)
    olen = std::min(std::max<int64_t>(0, floordiv(input_idat * N * p->de, p->nu)), full);
  }
  if (input_idat < 0)
    // no complete block and a carry rounded up past the data: InverseFilterBank.m:104-122
    // would index input(:, :, input_idat + 1 : end) before the first sample (its rounding
    // loop never settles); the call is rejected and the object state is left unchanged
    return fail(PFB_ERR_INVALID_ARG,
                "InverseFilterBank: %lld buffered + %lld new rows hold no complete block and "
                "round the carry past the data (InverseFilterBank.m:104-122); pass more rows",
                (long long)p->buffered, (long long)n_in);
  if (n_out) *n_out = olen;
  if (olen > cap) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld",
                              (long long)cap, (long long)olen);
  {
    // Carry without the concatenation copy: blocks whose rows start at or after the
    // carried Bc rows read the new input in place (row shift Bc - so), the first ones a
    // small stitched buffer; same blocks, same kernels as the concatenated run.
    const int64_t Bc = p->buffered;
    static const bool no_split = pfb::knob("PFB_FB_NO_SPLIT") != nullptr;  // A/B
    if (!no_split && mem == PFB_MEM_DEVICE && Bc > 0 && !p->has_spectral && input_idat >= Bc) {
      if (olen > 0) {
        // first block starting at or after row Bc of the concatenation: so + b keep >= Bc
        const int64_t b_s = std::min(B, std::max<int64_t>(0, (Bc - so + p->keep - 1) / p->keep));
        if (b_s > 0) {
          const int64_t L = std::min(total, so + (b_s - 1) * p->keep + p->Nf);
          HIPCHK(p->work.ensure((size_t)p->n_pol * L * N * sizeof(float2)));
          float2* wk = p->work.as<float2>();
          HIPCHK(copy_pols(wk, L * N, p->carry.as<float2>(), Bc * N, std::min(Bc, L) * N, p->n_pol,
                           hipMemcpyDeviceToDevice, s));
          if (L > Bc)
            HIPCHK(copy_pols(wk + Bc * N, L * N, (const float2*)in, in_ps, (L - Bc) * N, p->n_pol,
                             hipMemcpyDeviceToDevice, s));
          pfb_status st = synthesis_range(p, wk, L * N, 0, b_s, (float2*)out, out_ps, olen, s, -so);
          if (st != PFB_OK) return st;
        }
        pfb_status st =
            synthesis_range(p, (const float2*)in, in_ps, b_s, B, (float2*)out, out_ps, olen, s, Bc - so);
        if (st != PFB_OK) return st;
      }
      if (buffered > 0) {
        HIPCHK(p->carry.ensure((size_t)p->n_pol * buffered * N * sizeof(float2)));
        HIPCHK(copy_pols(p->carry.as<float2>(), buffered * N, (const float2*)in + (input_idat - Bc) * N, in_ps,
                         buffered * N, p->n_pol, hipMemcpyDeviceToDevice, s));
      }
      p->buffered = std::max<int64_t>(buffered, 0);
      return PFB_OK;
    }
  }
  // input = cat(3, input_buffer, input); read in place when nothing is buffered
  const float2* w;
  int64_t wps;
  if (p->buffered == 0 && mem == PFB_MEM_DEVICE) {
    w = (const float2*)in;
    wps = in_ps;
  } else {
    HIPCHK(p->work.ensure((size_t)p->n_pol * std::max<int64_t>(total, 1) * N * sizeof(float2)));
    float2* wk = p->work.as<float2>();
    HIPCHK(copy_pols(wk, total * N, p->carry.as<float2>(), p->buffered * N, p->buffered * N, p->n_pol,
                     hipMemcpyDeviceToDevice, s));
    HIPCHK(copy_pols(wk + p->buffered * N, total * N, (const float2*)in, in_ps, n_in * N, p->n_pol,
                     kin, s));
    w = wk;
    wps = total * N;
  }
  if (olen > 0) {
    if (mem == PFB_MEM_HOST) {
      HIPCHK(p->stage_out.ensure((size_t)p->n_pol * olen * sizeof(float2)));
      pfb_status st = synthesis_range(p, w, wps, 0, B, p->stage_out.as<float2>(), olen, olen, s, -so);
      if (st != PFB_OK) return st;
      HIPCHK(copy_pols((float2*)out, out_ps, p->stage_out.as<float2>(), olen, olen, p->n_pol,
                       hipMemcpyDeviceToHost, s));
    } else {
      pfb_status st = synthesis_range(p, w, wps, 0, B, (float2*)out, out_ps, olen, s, -so);
      if (st != PFB_OK) return st;
    }
  }
  if (buffered > 0) {
    HIPCHK(p->carry.ensure((size_t)p->n_pol * buffered * N * sizeof(float2)));
    HIPCHK(copy_pols(p->carry.as<float2>(), buffered * N, w + input_idat * N, wps, buffered * N,
                     p->n_pol, hipMemcpyDeviceToDevice, s));
  }
  p->buffered = std::max<int64_t>(buffered, 0);
  if (mem == PFB_MEM_HOST) HIPCHK(hipStreamSynchronize(s));
  return PFB_OK;
}

int64_t pfb_inverse_filterbank_buffered(const pfb_synthesis_plan* p) { return p ? p->buffered : -1; }

pfb_status pfb_inverse_filterbank_reset(pfb_synthesis_plan* p) {
  if (!p) return fail(PFB_ERR_INVALID_ARG, "null plan");
  p->buffered = 0;
  return PFB_OK;
}

// ------------------------------------------------------------------ round trip
// Analysis -> synthesis of one call, pipelined in chunks of synthesis blocks (the
// reference's test_data_pipeline.m:114,132 runs the two back to back).  Chunk c's
// analysis rows run on the analysis plan's own stream while chunk c-1 is synthesised
// on the caller's stream, so the two kernels share the chip (each alone leaves HBM and
// VALU partly idle), and the synthesis reads each channelised row shortly after it was
// written (Infinity-Cache resident).  The full channelised product is still written to
// `chan`.  On this chunked path every row and block is computed by the same kernels with
// the same inputs as pfb_analysis_execute + pfb_synthesis_execute, so both results are
// bit-identical to the separate calls (the fused path below: see its comment).

// phase 0: the whole round trip; 1 / 2: only the analysis / only the synthesis half of the
// fused path (pfb_roundtrip_analysis_execute / pfb_roundtrip_synthesis_execute), which hand
// the stage-1 rows over in the synthesis plan's scratch
static pfb_status roundtrip_run(pfb_analysis_plan* pa, pfb_synthesis_plan* ps, const pfb_cf32* in,
                                int64_t in_ps, int64_t n_dat, pfb_cf32* chan, int64_t chan_ps,
                                int64_t chan_cap, int64_t* n_chan_rows, int64_t sample_offset,
                                pfb_cf32* out, int64_t out_ps, int64_t out_cap, int64_t* n_out,
                                void* stream, int phase) {
  if (!pa || !ps || (!in && n_dat > 0 && phase != 2)) return fail(PFB_ERR_INVALID_ARG, "null argument");
  if (pa->device != ps->device) return fail(PFB_ERR_INVALID_ARG, "plans on different devices");
  if (pa->variant == pfb::kLowCbf)
    return fail(PFB_ERR_UNSUPPORTED, "round trip of the LowCBF filterbank: use the separate calls");
  if (pa->N != ps->N || pa->n_pol != ps->n_pol)
    return fail(PFB_ERR_INVALID_ARG, "analysis (%d ch, %d pol) and synthesis (%d ch, %d pol) differ",
                pa->N, pa->n_pol, ps->N, ps->n_pol);
  if (sample_offset < 1) return fail(PFB_ERR_INVALID_ARG, "sample_offset is 1-based (>= 1)");
  if (n_dat < 0) return fail(PFB_ERR_INVALID_ARG, "negative n_dat");
  HIPCHK(hipSetDevice(pa->device));
  hipStream_t s = (hipStream_t)stream;
  const int64_t K = analysis_K(pa, n_dat);
  const int64_t off = std::min<int64_t>(sample_offset - 1, K);
  const int64_t B = synth_blocks(ps, K - off);
  const int64_t olen = B * ps->Lkeep;
  if (n_chan_rows) *n_chan_rows = K;
  if (n_out) *n_out = olen;
  if (K == 0) return PFB_OK;
  if (phase != 2) {
    if (!chan) return fail(PFB_ERR_INVALID_ARG, "null output");
    if (chan_cap < K) return fail(PFB_ERR_BUFFER_TOO_SMALL, "channelised capacity %lld < %lld rows",
                                  (long long)chan_cap, (long long)K);
    if (in_ps < n_dat || chan_ps < K * pa->N)
      return fail(PFB_ERR_INVALID_ARG, "polarisation stride smaller than the data");
  }
  if (phase != 1) {
    if (olen > 0 && !out) return fail(PFB_ERR_INVALID_ARG, "null output");
    if (out_cap < olen) return fail(PFB_ERR_BUFFER_TOO_SMALL, "output capacity %lld < %lld",
                                    (long long)out_cap, (long long)olen);
    if (olen > 0 && out_ps < olen) return fail(PFB_ERR_INVALID_ARG, "polarisation stride smaller than the data");
  }
  const float2* x = (const float2*)in;
  float2* y = (float2*)chan;
  if (B == 0) return phase == 2 ? PFB_OK : analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s);

  // Fused: the analysis kernel also writes the synthesis stage-1 rows (the channel IFFT
  // of every row it produces, taken as N^2 x its FIR sums before the FFT rather than from
  // the rounded channelised row — equal in exact arithmetic, so the output agrees with
  // the separate calls to ~1e-7, not bit for bit) and the block kernel reads them; the
  // channelised product is still written in full (and IS bit-identical).  Needs an
  // analysis kernel that can emit the rows, no combine permutation / per-channel gain,
  // and device memory for the rows (bounded at 16 GiB; an explicit chunk size, or a
  // larger call, takes the chunked pipeline below).
  static const bool no_fuse = pfb::knob("PFB_RT_NO_FUSE") != nullptr;
  // (generic N > 256 path: Z holds all K rows — the row FFT makes the channelised product
  // from them — and the synthesis starts at row `off`; streaming kernel: K - off rows)
  const int64_t z0 = pa->fused ? off : 0;
  const int64_t zr = K - z0;
  // Nf = 256 synthesis through the wave kernel: the streaming analysis writes the rows in
  // the blocked layout it reads (16-row runs per phase; the series' rows from `off` on,
  // which must start a run; rows rounded up to whole runs)
  // (PFB_SYNTH_WAVE=0: the block kernel on rows; PFB_ZBLK: the run length, experiments build)
  static const bool no_wave = pfb::knob("PFB_SYNTH_WAVE") && std::atoi(pfb::knob("PFB_SYNTH_WAVE")) == 0;
  static const int zb_knob = pfb::knob("PFB_ZBLK") ? std::atoi(pfb::knob("PFB_ZBLK")) : 2;
  int zblk = (!no_wave && analysis_emits_zblk(pa) && z0 == off && off % 16 == 0) ? zb_knob : 0;
  if (zblk && !pfb::synth_wave_supported(synth_args(ps, nullptr, 0, 0, B, nullptr, 0, 0, zblk))) zblk = 0;
  // generic path (N > 256, the SKA-Mid round trip): the FIR writes the rows in 2-row runs
  // per column, so the Nf = 512 wave synthesis loads whole 128-B lines (2 rows x 8 phases)
  // — bit-identical; measured (profiles/r05_v17_c3_zrun_kernel_ab/) synthesis -17 us, FIR
  // +8 us, row FFT +4 us (it reads each row's pair partner from the lines fetched one row
  // earlier): net -5 us per unit (PFB_C3_ZRUN=0: rows, experiments build)
  static const bool zrun_on = !(pfb::knob("PFB_C3_ZRUN") && std::atoi(pfb::knob("PFB_C3_ZRUN")) == 0);
  const bool zrun = zrun_on && !zblk && !pa->fused && analysis_emits_z(pa) && off % 2 == 0 &&
                    pfb::synth_wave512_supported(synth_args(ps, nullptr, 0, 0, B, nullptr, 0, 0, 2));
  if (zrun) zblk = 2;
  const int64_t zrows = zrun ? (zr + 1) / 2 * 2 : zblk ? (zr + 15) / 16 * 16 : zr;
  const size_t zbytes = (size_t)pa->n_pol * zrows * pa->N * sizeof(float2);
  bool fuse = !no_fuse && analysis_emits_z(pa) && ps->identity_perm && !ps->has_cgain &&
              !ps->has_spectral && ps->chunk_blocks <= 0 && zbytes <= ((size_t)16 << 30);
  // Recomputed stage-1 rows (SynthBlockArgs::fir_x): the analysis writes only the
  // channelised product and the synthesis evaluates the rows it needs from the input
  // series — the same FIR sums, bit for bit (555 instead of 727 MB of HBM traffic per C2
  // step).  Where the wave kernel takes the run layout (zblk) and has a FIR variant
  // (pfb_synthesis_set_stage1_rows).
  const bool synth_fir_on = ps->stage1 == PFB_STAGE1_RECOMPUTED || (ps->stage1 == PFB_STAGE1_AUTO && kSynthFirDefault);
  FirSrc fsrc{(const float2*)in, in_ps, n_dat, off / std::max(pa->nu, 1), pa->gtab.as<float>(), pa->nu, pa->de,
              pa->P + 1};
  bool fir = false;
  if (synth_fir_on && zblk && pa->gtab.p && off % pa->nu == 0 && phase != 2) {
    fir = pfb::synth_wave_fir_supported(synth_args(ps, nullptr, 0, 0, B, nullptr, 0, 0, 0, &fsrc));
  }
  if (phase == 2 && ps->zkey_x != nullptr) {
    // the analysis half chose recomputed rows: the synthesis reads the input it recorded
    fir = true;
    fsrc.x = (const float2*)ps->zkey_x;
    fsrc.x_ps = ps->zkey_xps;
  }
  const int64_t zkey[5] = {n_dat, off, fir ? -1 : zblk, K, zrows};
  if (fir && fuse) {
    if (phase == 2) {
      if (ps->zkey_plan != pa->serial || !std::equal(zkey, zkey + 5, ps->zkey))
        return fail(PFB_ERR_INVALID_ARG,
                    "split round trip: the synthesis plan holds no analysis half of this analysis plan, "
                    "n_dat %lld and sample_offset %lld (run pfb_roundtrip_analysis_execute with the same "
                    "arguments first)",
                    (long long)n_dat, (long long)sample_offset);
      return synthesis_blocks(ps, nullptr, 0, 0, B, (float2*)out, out_ps, olen, s, 0, &fsrc);
    }
    zkey_clear(ps);
    pfb_status st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s);
    if (st != PFB_OK) return st;
    if (phase == 1) {
      // the synthesis half re-reads this input: the caller keeps it unchanged until then
      ps->zkey_plan = pa->serial;
      std::copy(zkey, zkey + 5, ps->zkey);
      ps->zkey_x = in;
      ps->zkey_xps = in_ps;
      return PFB_OK;
    }
    return synthesis_blocks(ps, nullptr, 0, 0, B, (float2*)out, out_ps, olen, s, 0, &fsrc);
  }
  if (fuse && phase == 2) {
    // the synthesis half reads the rows the analysis half left in the plan's scratch: they
    // must come from this analysis plan with the same n_dat, offset and row layout
    if (!ps->Z.p || ps->Z.bytes < zbytes || ps->zkey_plan != pa->serial ||
        !std::equal(zkey, zkey + 5, ps->zkey))
      return fail(PFB_ERR_INVALID_ARG,
                  "split round trip: the synthesis plan holds no stage-1 rows of this analysis plan, "
                  "n_dat %lld and sample_offset %lld (run pfb_roundtrip_analysis_execute with the same "
                  "arguments first)",
                  (long long)n_dat, (long long)sample_offset);
  } else if (fuse) {
    // the rows of the whole call stay resident; a device without room for them takes the
    // chunked pipeline below (its scratch is one chunk's rows) instead of failing
    const hipError_t ze = ps->Z.ensure(zbytes);
    if (ze == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      fuse = false;
    } else if (ze != hipSuccess) {
      return fail(PFB_ERR_HIP, "round trip stage-1 rows (%zu bytes): %s", zbytes, hipGetErrorString(ze));
    }
  }
  if (phase != 0) {
    // the split round trip exists for the fused path only (one scratch of rows handed over)
    if (!fuse) return fail(PFB_ERR_UNSUPPORTED, "split round trip: these plans take the chunked pipeline "
                                                "(use pfb_roundtrip_execute)");
    float2* Z = ps->Z.as<float2>();
    if (phase == 1) {
      zkey_clear(ps);
      pfb_status st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s, Z, zrows * pa->N, z0, 0, nullptr,
                                   zblk);
      if (st != PFB_OK) return st;
      ps->zkey_plan = pa->serial;
      std::copy(zkey, zkey + 5, ps->zkey);
      return PFB_OK;
    }
    return synthesis_blocks(ps, Z + (off - z0) * pa->N, zrows * pa->N, 0, B, (float2*)out, out_ps, olen, s, zblk);
  }
  zkey_clear(ps);  // phase 0 reuses Z
  if (fuse) {
    float2* Z = ps->Z.as<float2>();
    // (retired round 5, measured slower twice: the row FFT on a second stream beside the
    // synthesis, Infinity-Cache chunking of the generic path and chunked analysis/synthesis
    // concurrency — profiles/HISTORY.md)
    // (generic N > 256 path: the FIR and the row FFT as two calls on the stream — the same
    // two launches as one call, each then timed alone by the profiler)
    pfb_status st = PFB_OK;
    if (!pa->fused) {
      st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s, Z, zrows * pa->N, z0, 0, nullptr, zblk,
                        nullptr, 1);
      if (st == PFB_OK)
        st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s, Z, zrows * pa->N, z0, 0, nullptr, zblk,
                          nullptr, 2);
    } else {
      st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, 0, K, K, s, Z, zrows * pa->N, z0, 0, nullptr, zblk);
    }
    if (st != PFB_OK) return st;
    return synthesis_blocks(ps, Z + (off - z0) * pa->N, zrows * pa->N, 0, B, (float2*)out, out_ps,
                            olen, s, zblk);
  }

  if (!pa->aux) HIPCHK(hipStreamCreateWithFlags(&pa->aux, hipStreamNonBlocking));
  int64_t CB = ps->chunk_blocks > 0 ? ps->chunk_blocks : ps->rt_chunk_blocks;
  CB = std::max<int64_t>(1, std::min<int64_t>(CB, B));
  const int64_t n_chunks = (B + CB - 1) / CB;
  while ((int64_t)pa->events.size() < n_chunks + 2) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    pa->events.push_back(e);
  }
  // fork: the analysis stream starts after everything already queued on the caller's
  HIPCHK(hipEventRecord(pa->events[0], s));
  HIPCHK(hipStreamWaitEvent(pa->aux, pa->events[0], 0));
  const float2* sin_ = y + off * pa->N;  // synthesis input = chan(:, :, sample_offset:end)
  int64_t ra = 0;                        // analysis rows done
  for (int64_t c = 0; c < n_chunks; ++c) {
    const int64_t b0 = c * CB, nb = std::min<int64_t>(CB, B - b0);
    // channelised rows the chunk reads: [off + b0 keep, off + (b0+nb) keep + 2 Ov); the
    // padded variant's output row t comes from analysis row (t + sds) mod K (rows that
    // wrap come from the first rows, produced by chunk 0)
    int64_t need = (c == n_chunks - 1) ? K : off + (b0 + nb) * ps->keep + 2 * (int64_t)ps->Ov;
    if (pa->variant == pfb::kPadded) need += pa->sds;
    const int64_t rb = std::max(ra, std::min(K, need));
    pfb_status st = analysis_run(pa, x, in_ps, n_dat, y, chan_ps, ra, rb, K, pa->aux);
    if (st != PFB_OK) return st;
    ra = rb;
    HIPCHK(hipEventRecord(pa->events[1 + c], pa->aux));
    HIPCHK(hipStreamWaitEvent(s, pa->events[1 + c], 0));
    st = synthesis_chunk(ps, sin_, chan_ps, b0, nb, (float2*)out, out_ps, olen, s);
    if (st != PFB_OK) return st;
  }
  // join (the last chunk already ran the analysis to K)
  HIPCHK(hipEventRecord(pa->events[1 + n_chunks], pa->aux));
  HIPCHK(hipStreamWaitEvent(s, pa->events[1 + n_chunks], 0));
  return PFB_OK;
}

pfb_status pfb_roundtrip_execute(pfb_analysis_plan* pa, pfb_synthesis_plan* ps, const pfb_cf32* in,
                                 int64_t in_ps, int64_t n_dat, pfb_cf32* chan, int64_t chan_ps,
                                 int64_t chan_cap, int64_t* n_chan_rows, int64_t sample_offset,
                                 pfb_cf32* out, int64_t out_ps, int64_t out_cap, int64_t* n_out,
                                 void* stream) {
  return roundtrip_run(pa, ps, in, in_ps, n_dat, chan, chan_ps, chan_cap, n_chan_rows, sample_offset,
                       out, out_ps, out_cap, n_out, stream, 0);
}

pfb_status pfb_roundtrip_analysis_execute(pfb_analysis_plan* pa, pfb_synthesis_plan* ps, const pfb_cf32* in,
                                          int64_t in_ps, int64_t n_dat, pfb_cf32* chan, int64_t chan_ps,
                                          int64_t chan_cap, int64_t* n_chan_rows, int64_t sample_offset,
                                          void* stream) {
  return roundtrip_run(pa, ps, in, in_ps, n_dat, chan, chan_ps, chan_cap, n_chan_rows, sample_offset,
                       nullptr, 0, 0, nullptr, stream, 1);
}

pfb_status pfb_roundtrip_synthesis_execute(pfb_analysis_plan* pa, pfb_synthesis_plan* ps, int64_t n_dat,
                                           int64_t sample_offset, pfb_cf32* out, int64_t out_ps,
                                           int64_t out_cap, int64_t* n_out, void* stream) {
  return roundtrip_run(pa, ps, nullptr, n_dat, n_dat, nullptr, 0, 0, nullptr, sample_offset, out, out_ps,
                       out_cap, n_out, stream, 2);
}

// ------------------------------------------------------------------ utilities
double pfb_calc_output_nbins(int64_t nbins, int32_t channels, int32_t os_nu, int32_t os_de,
                             int64_t filter_taps, int32_t input_fft_length, int32_t input_overlap) {
  // calc_output_nbins.m:17-27, in Matlab's double arithmetic
  const double nu = os_nu, de = os_de, ch = channels;
  const double step = std::floor(ch * de / nu);
  const double nblocks_pfb = std::floor(((double)nbins - (double)filter_taps) / step);
  const double output_pfb = std::floor(step * nblocks_pfb / ch);
  const double input_keep = (double)input_fft_length - 2.0 * input_overlap;
  const double nblocks_ipfb = std::floor((output_pfb - 2.0 * input_overlap) / input_keep);
  const double output_fft_length = (double)input_fft_length * de / nu * ch;  // normalize.m:17
  const double output_overlap = (double)input_overlap * de / nu * ch;
  return (output_fft_length - 2.0 * output_overlap) * nblocks_ipfb;
}

pfb_status pfb_device_malloc(int32_t device, int64_t bytes, void** ptr) {
  if (!ptr || bytes < 0) return fail(PFB_ERR_INVALID_ARG, "bad arguments");
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(ptr, (size_t)std::max<int64_t>(bytes, 1)));
  return PFB_OK;
}
pfb_status pfb_device_free(void* ptr) {
  if (ptr) HIPCHK(hipFree(ptr));
  return PFB_OK;
}
pfb_status pfb_memcpy_h2d(void* dst, const void* src, int64_t bytes, void* stream) {
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return PFB_OK;
}
pfb_status pfb_memcpy_d2h(void* dst, const void* src, int64_t bytes, void* stream) {
  HIPCHK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return PFB_OK;
}
pfb_status pfb_stream_synchronize(void* stream) {
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return PFB_OK;
}

pfb_status pfb_profile_enable(int32_t enable) {
  g_prof.drain();
  g_prof.enabled = enable != 0;
  return PFB_OK;
}
pfb_status pfb_profile_read(int32_t which, double* total_ms, int64_t* launches, double* bytes) {
  if (which < 0 || which >= Profiler::kClasses) return fail(PFB_ERR_INVALID_ARG, "which must be 0..5");
  g_prof.drain();
  if (total_ms) *total_ms = g_prof.total_ms[which];
  if (launches) *launches = g_prof.launches[which];
  if (bytes) *bytes = g_prof.bytes[which];
  return PFB_OK;
}
pfb_status pfb_profile_reset(void) {
  g_prof.drain();
  for (int i = 0; i < Profiler::kClasses; ++i) {
    g_prof.total_ms[i] = 0;
    g_prof.launches[i] = 0;
    g_prof.bytes[i] = 0;
    g_prof.names[i].clear();
  }
  return PFB_OK;
}
pfb_status pfb_profile_kernel_name(int32_t which, char* buf, int64_t len) {
  if (which < 0 || which >= Profiler::kClasses) return fail(PFB_ERR_INVALID_ARG, "which must be 0..5");
  if (!buf || len <= 0) return fail(PFB_ERR_INVALID_ARG, "null or empty buffer");
  const std::string& n = g_prof.names[which];
  const size_t k = std::min<size_t>(n.size(), (size_t)len - 1);
  std::memcpy(buf, n.data(), k);
  buf[k] = 0;
  return PFB_OK;
}
int32_t pfb_build_flags(void) { return pfb::kExperiments ? 1 : 0; }

}  // extern "C"
