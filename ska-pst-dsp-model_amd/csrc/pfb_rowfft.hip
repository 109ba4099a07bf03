// pfb_rowfft.hip — N-point row FFT launchers (row_fft_kernel, pfb_common.hpp): the
// analysis FFT for N > 256 and synthesis stage 1 (the N-point inverse DFT across channels
// of every channelised row, polyphase_synthesis.m:282-285 factored).
#include "pfb_common.hpp"

#include <algorithm>
#include <cstdlib>

namespace pfb {

template <int N, int DIR, bool PERM, bool GAIN>
static hipError_t launch_row_fft_t(const RowFftArgs& r, int n_pol, hipStream_t s) {
  constexpr int ROWS = RowShape<N>::ROWS;
  if constexpr (N == 4096) {
    // persistent workgroups (row_fft_persist_kernel) once there are several rows per
    // resident workgroup; PFB_ROWFFT_PERSIST=0: one workgroup per row (A/B)
    static const bool off = knob("PFB_ROWFFT_PERSIST") && std::atoi(knob("PFB_ROWFFT_PERSIST")) == 0;
    // (PFB_ROWFFT_HT=1: half twiddle table, experiments A/B)
    static const bool ht = kExperiments && knob("PFB_ROWFFT_HT") && std::atoi(knob("PFB_ROWFFT_HT")) == 1;
    const size_t bytes = row_fft_persist_lds<N>(ht);
    const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / bytes);
    int64_t wgs = (int64_t)cu_count() * per_cu;
    // (PFB_ROWFFT_WGS: fewer persistent workgroups, so the row FFT can share the chip with
    // a concurrent synthesis — experiments A/B)
    static const int env_wgs = knob("PFB_ROWFFT_WGS") ? std::atoi(knob("PFB_ROWFFT_WGS")) : 0;
    if (env_wgs > 0) wgs = env_wgs;
    if (!off && r.n_rows >= 4 * wgs) {
      // (PFB_ROWFFT_PF=2: two rows prefetched ahead, experiments A/B)
      auto kern = row_fft_persist_kernel<N, DIR, PERM, GAIN, 1>;
      if constexpr (kExperiments) {
        static const bool pf2 = knob("PFB_ROWFFT_PF") && std::atoi(knob("PFB_ROWFFT_PF")) == 2;
        if (pf2) kern = row_fft_persist_kernel<N, DIR, PERM, GAIN, 2>;
        if (ht) kern = row_fft_persist_kernel<N, DIR, PERM, GAIN, 1, true>;
      }
      hipError_t e = set_lds(kern, bytes);
      if (e != hipSuccess) return e;
      dim3 grid((unsigned)std::max<int64_t>(1, wgs / n_pol), (unsigned)n_pol);
      return launch_kernel(kern, grid, dim3(NT), bytes, s, r);
    }
  }
  const size_t bytes = ((size_t)ROWS * RowShape<N>::RS + tw_slots(N)) * sizeof(float2);
  auto kern = row_fft_kernel<N, DIR, PERM, GAIN>;
  hipError_t e = set_lds(kern, bytes);
  if (e != hipSuccess) return e;
  dim3 grid((unsigned)((r.n_rows + ROWS - 1) / ROWS), (unsigned)n_pol);
  return launch_kernel(kern, grid, dim3(NT), bytes, s, r);
}

template <int N, int DIR>
static hipError_t launch_row_fft(const RowFftArgs& r, int n_pol, hipStream_t s) {
  if constexpr (DIR > 0) {
    if (r.perm && r.cgain) return launch_row_fft_t<N, DIR, true, true>(r, n_pol, s);
    if (r.perm) return launch_row_fft_t<N, DIR, true, false>(r, n_pol, s);
    if (r.cgain) return launch_row_fft_t<N, DIR, false, true>(r, n_pol, s);
  }
  return launch_row_fft_t<N, DIR, false, false>(r, n_pol, s);
}

template <int DIR>
hipError_t dispatch_row_fft(int N, const RowFftArgs& r, int n_pol, hipStream_t s) {
  switch (N) {
    case 8: return launch_row_fft<8, DIR>(r, n_pol, s);
    case 16: return launch_row_fft<16, DIR>(r, n_pol, s);
    case 32: return launch_row_fft<32, DIR>(r, n_pol, s);
    case 64: return launch_row_fft<64, DIR>(r, n_pol, s);
    case 128: return launch_row_fft<128, DIR>(r, n_pol, s);
    case 256: return launch_row_fft<256, DIR>(r, n_pol, s);
    case 512: return launch_row_fft<512, DIR>(r, n_pol, s);
    case 1024: return launch_row_fft<1024, DIR>(r, n_pol, s);
    case 2048: return launch_row_fft<2048, DIR>(r, n_pol, s);
    case 4096: return launch_row_fft<4096, DIR>(r, n_pol, s);
    default: break;
  }
  if constexpr (DIR > 0) {
    switch (N) {
      case 14: return launch_row_fft<14, DIR>(r, n_pol, s);
      case 28: return launch_row_fft<28, DIR>(r, n_pol, s);
      case 56: return launch_row_fft<56, DIR>(r, n_pol, s);
      case 112: return launch_row_fft<112, DIR>(r, n_pol, s);
      case 216: return launch_row_fft<216, DIR>(r, n_pol, s);
      case 224: return launch_row_fft<224, DIR>(r, n_pol, s);
      case 432: return launch_row_fft<432, DIR>(r, n_pol, s);
      case 448: return launch_row_fft<448, DIR>(r, n_pol, s);
      case 864: return launch_row_fft<864, DIR>(r, n_pol, s);
      case 192: return launch_row_fft<192, DIR>(r, n_pol, s);
      case 384: return launch_row_fft<384, DIR>(r, n_pol, s);
      case 768: return launch_row_fft<768, DIR>(r, n_pol, s);
      case 896: return launch_row_fft<896, DIR>(r, n_pol, s);
      case 1536: return launch_row_fft<1536, DIR>(r, n_pol, s);
      case 1792: return launch_row_fft<1792, DIR>(r, n_pol, s);
      case 3072: return launch_row_fft<3072, DIR>(r, n_pol, s);
      case 3584: return launch_row_fft<3584, DIR>(r, n_pol, s);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

template hipError_t dispatch_row_fft<-1>(int, const RowFftArgs&, int, hipStream_t);
template hipError_t dispatch_row_fft<+1>(int, const RowFftArgs&, int, hipStream_t);

bool chan_ifft_supported(int N) { return pow2_supported(N) || mixed_chan_supported(N); }

hipError_t launch_chan_ifft(const ChanIfftArgs& c, hipStream_t s) {
  if (c.n_rows <= 0) return hipSuccess;
  RowFftArgs r{c.in, c.in_pol_stride, c.out, c.out_pol_stride, c.n_rows, c.perm, c.cgain, c.twN,
               1.0f, 0, 0, 0, c.n_rows};
  return dispatch_row_fft<+1>(c.N, r, c.n_pol, s);
}

}  // namespace pfb
