// pfb_kernels.hpp — internal (C++) launcher interface between the C ABI and the
// HIP kernels.  Not part of the public boundary (see include/pfb_api.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

namespace pfb {

// Release builds carry no tuning or timing switches: the A/B knobs (PFB_* environment
// variables read through knob()) and the timing masks that drop a kernel's loads or
// stores exist only in the experiments build (make EXPERIMENTS=1 ->
// lib/libpfb_hip_exp.so, compiled with -DPFB_EXPERIMENTS).  In a release build knob()
// returns null and tmask() 0 at compile time, so no environment variable reaches a
// code path that skips work.
#ifdef PFB_EXPERIMENTS
constexpr bool kExperiments = true;
#else
constexpr bool kExperiments = false;
#endif
inline const char* knob(const char* name) { return kExperiments ? std::getenv(name) : nullptr; }
__host__ __device__ constexpr int tmask(int m) { return kExperiments ? m : 0; }

enum Variant { kBunton = 0, kPadded = 1, kLowCbf = 2 };

// Largest byte extent one raw buffer descriptor may cover: the kernels form 32-bit
// signed byte offsets from it.  Launchers size their per-workgroup ranges (and plans
// reject shapes) so that no descriptor needs more; nothing is clamped silently.
constexpr int64_t kRsrcMaxBytes = 0x7ffffff0;

// Polyphase analysis (polyphase_analysis.m / polyphase_analysis_padded.m).
struct AnalysisArgs {
  const float2* in;        // [pol][t]
  int64_t in_pol_stride;
  int64_t n_dat;
  float2* out;             // [pol][k][c]
  int64_t out_pol_stride;
  int64_t row0;            // first output row of this launch (global row index)
  int64_t K;               // end of this launch's rows (exclusive, global)
  int64_t K_total;         // output rows per pol of the whole call (padded circular shift)
  int n_pol;
  int N, M, P, nu, sds;    // channels, step, phases, os numerator, padded delay shift
  int variant;
  const float* taps;       // P*N padded taps (device)
  const float2* twN;       // e^{-2 pi i m / N}, m < N (device)
  float2* scratch;         // generic path: [pol][K - row0][N] (device) or null
  int timing_mask;         // timing experiments only (PFB_ANA_MASK, results invalid): bit0 no
                           // input loads, bit1 no channelised stores, bit2 no Z stores
                           // (streaming kernel)
  // Round trip only (pfb_roundtrip_execute): when z is set, every output row k >= z_row0
  // is also transformed by the synthesis stage-1 channel IFFT (the exact computation
  // row_fft_kernel<N, +1> performs on the stored row) into z[pol][k - z_row0][t0].
  float2* z;
  int64_t z_pol_stride;
  int64_t z_row0;
  // generic path (N > 256) with z: the FIR writes only the Z rows (all K of them,
  // z_row0 = 0) and the row FFT makes the channelised rows from them through this
  // index reversal (padded variant; null for Bunton) — see fir_window_kernel
  const int* zrev;
  // leading zeros in front of `in` (the LowCBF wrapper's one-time pre-padding) — the
  // streaming kernel reads x[r N + c - pad] (zero for negative indices); 0 otherwise
  int64_t pad;
  // with pad > 0: the pad samples in front of `in` are pre[pol][0, pad) (a stream object's
  // carried samples; null: zeros, the LowCBF pre-padding).  Streaming kernel only, read by the
  // first window of every workgroup whose window starts before `in` (launch_stream rejects
  // pad > WIN N)
  const float2* pre;
  int64_t pre_pol_stride;
  float lcbf_scale;  // LowCBF streaming path: output scale (2^12)
  // Strided channelised output (streaming kernel only, out_rs > 0): bin c of row k goes to
  // out[pol][k * out_rs + j * out_cs] with j = c (sel_n = 0) or the two-stage chomp
  // j = c < sel_split ? c : c - sel_shift, kept when c < sel_split or c >= sel_split +
  // sel_shift, and j < sel_n (TwoStageFilterBank.m:102-105); out_rs = 0: [pol][k][c]
  int out_rs, out_cs;
  int sel_split, sel_shift, sel_n;
  // z in a grouped layout (streaming kernel, round trip into synth_wave_kernel): zblk = ZB
  // in {2, 4, 16} puts row k - z_row0 = ZB g + gi of column c at z[pol][g][c][gi] — ZB
  // consecutive rows of one column are one run; needs (row0 - z_row0) % 16 == 0
  // (launch_analysis checks); 0 or 1: rows [row][c]
  int zblk;
  // generic path (N > 256) with z: 0 both launches; 1 only the FIR (Z rows); 2 only the
  // row FFT (channelised rows from Z) — so the row FFT can run beside the synthesis, which
  // reads the same Z rows
  int z_stage;
  // stream objects (streaming kernel only): also copy in[pol][carry_src, carry_src + carry_n)
  // — the next call's carry, FilterBank.m:119-126 — to carry_out[pol][0, carry_n) (a buffer
  // other than `pre`), spread over the grid before the main loop: no separate copy launch
  float2* carry_out;
  int64_t carry_src, carry_n, carry_pol_stride;
  // workgroup -> step range order: 0 XCD-aware (xcd_tile), 1 linear (blockIdx.x: the
  // dispatcher's order is the rows' order, so the chip's loads in flight stay in one window)
  int linear = 0;
};
// SKA-Low CBF PST filterbank through the streaming analysis kernel (pfb_analysis.hip)
hipError_t launch_lowcbf_stream(const AnalysisArgs& a, hipStream_t s);
// analysis kernels that can also emit the synthesis stage-1 rows (see AnalysisArgs::z)
bool analysis_can_emit_z(const AnalysisArgs& a);
// analysis kernels that can emit the stage-1 rows in the blocked layout (AnalysisArgs::zblk)
bool analysis_can_emit_zblk(const AnalysisArgs& a);
// analysis shapes whose kernel reads with an input offset (AnalysisArgs::pad)
bool analysis_takes_offset(const AnalysisArgs& a);
// the fused kernel reads a stream carry through `pre` with `pad` (non-streaming shapes)
bool analysis_fused_takes_carry(const AnalysisArgs& a);

// Synthesis stage 1: per channelised time row, N-point inverse DFT across channels
// (after the combine permutation and per-channel gain).  See DESIGN.md §synthesis.
struct ChanIfftArgs {
  const float2* in;        // [pol][row][c], rows already offset to the first row
  int64_t in_pol_stride;
  float2* out;             // Z: [pol][row][t0]
  int64_t out_pol_stride;
  int64_t n_rows;
  int n_pol;
  int N;
  const int* perm;         // slot -> input channel (null = identity)
  const float* cgain;      // per-slot gain (null = 1)
  const float2* twN;
  int zblk = 1;            // Z rows in runs of zblk (1, 2, 4) per t0 (SynthBlockArgs::zblk)
};

// Synthesis stage 2: per block and group of t0, Nf-point FFT over time, kept-bin
// selection with deripple gain and four-step twiddle, W-point inverse FFT,
// overlap-discard and the 1/L * de/nu scale.
struct SynthBlockArgs {
  const float2* Z;         // [pol][row][t0] (chunk-local rows)
  int64_t z_pol_stride;
  float2* out;             // [pol][t]
  int64_t out_pol_stride;
  int64_t block0;          // global index of the chunk's first block
  int n_blocks;            // blocks in this chunk
  int n_pol;
  int N, Nf, W, keep, L, Lov, Lkeep, t1_lo, t1_hi;
  float scale;
  const float* window;     // Nf temporal window (device)
  int win_flat;            // 1: window[t] == 1 exactly for t in [48, 208) at Nf 256 / [128, 384) at
                           // Nf 512 (the wave kernels skip those taper multiplies)
  int spans;               // 1: spans Nyquist (signed-frequency bins), 0: critical
  const float2* tw4;       // [j'][t0] = gain[j'] e^{+2 pi i t0 expo[j'] / L} (W x N)
  const float2* twNf;      // e^{-2 pi i m / Nf}
  const float2* twW;       // e^{-2 pi i m / W}
  const float2* tw4s;      // tw4 x (de/nu) / L, rounded once (synth_wave_kernel)
  int64_t out_limit;       // samples per pol actually written (InverseFilterBank trim)
  int ranges;              // 0: one workgroup per block; -1 persistent auto; >0 persistent ranges
  int no_reuse;            // 1: re-read the 2 Ov overlap rows from HBM (PFB_SYNTH_NO_REUSE, A/B only)
  int xcd;                 // 1: XCD-aware workgroup -> (phase group, range) order (PFB_SYNTH_XCD)
  int timing_mask;         // experiments build only (PFB_TIMING_MASK, results invalid): bit0
                           // drop Z loads, bit1 drop output stores, bit2 drop tw4 loads; wave
                           // kernels: bit3 wave barriers for the block loop's workgroup
                           // barriers, bit4 a uniform twiddle for the LDS twiddle tables
  int zblk;                // Z layout of AnalysisArgs::zblk (0/1 rows, else ZB-row runs)
  // Recomputed stage-1 rows (the Nf = 256 round trip, synth_wave_kernel with fir_x set): the
  // analysis writes no Z; the synthesis evaluates each row it needs as N^2 x the streaming
  // analysis's FIR sums of the input series itself (same taps, same FMA order: bit-identical
  // rows).  fir_g[(s N + c) 16 + m] = N^2 x the folded tap of residue s, lag m < PE, column c
  // (pfb_ana_stream.hpp); Z row j is analysis row NU fir_q0 + j.
  const float2* fir_x;     // [pol][t] input series (null: read Z)
  int64_t fir_x_pol_stride;
  int64_t fir_n_dat;
  const float* fir_g;
  int64_t fir_q0;
  int fir_nu, fir_de, fir_pe;
  // wave kernels: workgroup -> (block range, phase group) order, 0 XCD-aware (xcd_tile), 1
  // linear (blockIdx.x: consecutive workgroups are the phase groups of one block range)
  int linear = 0;
};

// Synthesis with a non-identity spectral taper (pfb_spectral.hip): blocks [b0, b0 + nb)
// of the call, every polarisation, through two scratch buffers of nb N max(Nf, W) values.
struct SpectralArgs {
  const float2* in;        // [pol][row][c] channelised rows of the call (sample offset applied)
  int64_t in_pol_stride;
  float2* out;             // [pol][t]
  int64_t out_pol_stride;
  int64_t out_limit;
  int64_t b0, nb;
  int n_pol;
  int N, Nf, W, keep, L, Lov, Lkeep, t1_lo, t1_hi, spans;
  float scale;             // (de/nu) / L
  const float* window;     // Nf temporal window
  const float* cgain;      // per input channel gain (temporal 'hann' quirk) or null
  const int* perm;         // combine permutation (slot -> input channel) or null
  const float* gainj;      // W deripple gains in Matlab's FN row order
  const float* taper;      // L spectral taper coefficients
  const float2* twNf;      // e^{-2 pi i m / Nf}
  const float2* twN;       // e^{-2 pi i m / N}
  const float2* twW;       // e^{-2 pi i m / W}
  float2* buf0;
  float2* buf1;
};
bool spectral_synth_supported(int Nf, int W, int N);
hipError_t launch_spectral_synth(const SpectralArgs& a, hipStream_t s);

// SKA-Low CBF PST filterbank (polyphase_analysis_lowcbf.m / PSTFilterbank.m):
// 256 arms x 12 taps, step 192, forward FFT, fftshift, pi/2 derotation, 216 channels.
struct LowCbfArgs {
  const float2* in;        // [pol][t]
  int64_t in_pol_stride;
  int64_t n_dat;
  int64_t pad;             // leading zeros (1536 on the first call, else 0)
  float2* out;             // [pol][k][216]
  int64_t out_pol_stride;
  int64_t K;
  int n_pol;
  const float* taps;       // 3072 taps (device)
  const float2* tw;        // e^{-2 pi i m / 256}
  float scale;             // 2^28 / 2^9 / 128 = 2^12
};
hipError_t launch_lowcbf(const LowCbfArgs& a, hipStream_t s);

// Kernel timing (pfb_profile_*): when the C-ABI profiler arms these events, the next
// single-kernel launch records them in its own dispatch (hipExtLaunchKernelGGL), so the
// measured interval is the kernel alone, as a kernel trace sees it.
struct LaunchEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& armed_launch_events();
// name of the last kernel launched through armed events (pfb_profile_kernel_name)
const char*& launched_kernel_name();

// device-to-device strided copy of n_pol rows (pfb_layout.hip)
hipError_t launch_copy_rows(float2* dst, int64_t dps, const float2* src, int64_t sps, int64_t n, int n_pol,
                            hipStream_t s);

bool analysis_supported(int N, int P, int variant, bool* fused);
hipError_t launch_analysis(const AnalysisArgs& a, hipStream_t s);
bool chan_ifft_supported(int N);
hipError_t launch_chan_ifft(const ChanIfftArgs& a, hipStream_t s);
bool synth_block_supported(int Nf, int W);
// Nf = 256 synthesis with one output phase per 16 lanes and no barrier in the block loop
// (pfb_synth_wave.hip); launch_synth_block takes it where it applies
bool synth_wave_supported(const SynthBlockArgs& a);
// the same kernel with recomputed stage-1 rows (SynthBlockArgs::fir_x)
bool synth_wave_fir_supported(const SynthBlockArgs& a);
hipError_t launch_synth_wave(const SynthBlockArgs& a, hipStream_t s);
// Nf = 512, W = 448, keep 256 (SKA-Mid): one output phase per 32 lanes (pfb_synth_wave512.hip)
bool synth_wave512_supported(const SynthBlockArgs& a);
hipError_t launch_synth_wave512(const SynthBlockArgs& a, hipStream_t s);
hipError_t launch_synth_block(const SynthBlockArgs& a, hipStream_t s);

}  // namespace pfb
