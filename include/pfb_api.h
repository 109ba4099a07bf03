/*
 * pfb_api.h — C ABI of the MI355X-native oversampled polyphase filter bank (PFB).
 *
 * Drop-in boundary for the hot path of ska-telescope/ska-pst-dsp-model:
 *   polyphase_analysis        (matlab/polyphase_analysis.m:1-129, Bunton PFB)
 *   polyphase_analysis_padded (matlab/polyphase_analysis_padded.m:1-161, commutator PFB)
 *   polyphase_synthesis       (matlab/polyphase_synthesis.m:1-325, golden inversion)
 * and the stateful stream objects that call them
 *   FilterBank.execute        (matlab/FilterBank.m:65-128)
 *   InverseFilterBank.execute (matlab/InverseFilterBank.m:63-137)
 * which the reference selects by name (FilterBank.m:36 str2func(analysis_function))
 * or through the Python backend switch data_gen.channelize/synthesize
 * (python/data_gen/channelize.py:19-92, synthesize.py:27-95).
 *
 * Everything crossing this boundary is plain C: integers, doubles, pointers, sizes.
 * No C++ or torch types.  No exception crosses it: every entry point returns a
 * pfb_status and pfb_last_error() returns the thread-local message (mirrors the
 * reference's error(...) checks, e.g. InverseFilterBank.m:83-85).
 *
 * Data layout (complex float32, interleaved re/im = pfb_cf32):
 *   single-channel time series : in[pol * pol_stride + t]
 *   channelised data           : x[pol * pol_stride + t * n_chan + c]
 *                                (per polarisation the Matlab memory order of an
 *                                 (n_chan, n_dat) slice: channel fastest, then time)
 * Buffers are device pointers (PFB_MEM_DEVICE, zero copy on the given stream) or host
 * pointers (PFB_MEM_HOST, staged through the plan's device buffers; synchronous).
 *
 * Threading: a plan is bound to one device and is not thread safe (it carries the
 * streaming state).  Different plans are independent; multi-GPU = one plan per GPU.
 */
#ifndef PFB_API_H
#define PFB_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFB_API_VERSION 1

typedef struct pfb_cf32 {
  float re;
  float im;
} pfb_cf32;

typedef enum pfb_status {
  PFB_OK = 0,
  PFB_ERR_INVALID_ARG = 1,      /* e.g. N*de/nu, Ov*de/nu or Nf*de/nu not integral */
  PFB_ERR_UNSUPPORTED = 2,      /* size combination with no compiled kernel */
  PFB_ERR_HIP = 3,              /* HIP runtime error (message has hipGetErrorString) */
  PFB_ERR_OOM = 4,
  PFB_ERR_BUFFER_TOO_SMALL = 5, /* output capacity smaller than the required length */
  PFB_ERR_NO_DEVICE = 6
} pfb_status;

typedef enum pfb_analysis_variant {
  PFB_ANALYSIS_BUNTON = 0, /* polyphase_analysis.m */
  PFB_ANALYSIS_PADDED = 1, /* polyphase_analysis_padded.m */
  PFB_ANALYSIS_LOWCBF = 2  /* polyphase_analysis_lowcbf.m -> PSTFilterbank.m: the SKA-Low CBF
                              PST filterbank (n_chan 256, os 4/3, 3072 taps fixed); 216
                              output channels; 1536 zeros pre-padded on the plan's first call */
} pfb_analysis_variant;

typedef enum pfb_mem {
  PFB_MEM_DEVICE = 0,
  PFB_MEM_HOST = 1
} pfb_mem;

/* PFBWindow.m:10-16 lookup names, plus CUSTOM (explicit coefficients). */
typedef enum pfb_window_kind {
  PFB_WINDOW_NONE = 0,    /* no_window / identity_taper */
  PFB_WINDOW_TUKEY = 1,   /* PFBWindow.m:30-44 */
  PFB_WINDOW_TOP_HAT = 2, /* PFBWindow.m:63-68 */
  PFB_WINDOW_HANN = 3,    /* PFBWindow.m:72-99 (temporal: applied per channel row) */
  PFB_WINDOW_CUSTOM = 4   /* explicit coefficients (temporal: Nf values; spectral: L values) */
} pfb_window_kind;

/* ---------------------------------------------------------------- analysis */
typedef struct pfb_analysis_desc {
  int32_t variant;     /* pfb_analysis_variant */
  int32_t n_chan;      /* "block" = N channels (polyphase_analysis.m:3) */
  int32_t os_nu;       /* os_factor.nu */
  int32_t os_de;       /* os_factor.de */
  const double* taps;  /* prototype FIR taps (host memory, copied at create) */
  int64_t n_taps;
  int32_t n_pol;       /* polarisations processed per call */
  int32_t device;      /* HIP device ordinal */
} pfb_analysis_desc;

typedef struct pfb_analysis_plan pfb_analysis_plan;

/* Replaces: FilterBank constructor (FilterBank.m:26-63) + read_fir_filter_coeff. */
pfb_status pfb_analysis_plan_create(const pfb_analysis_desc* desc, pfb_analysis_plan** plan);
pfb_status pfb_analysis_plan_destroy(pfb_analysis_plan* plan);
/* The checks and host-side tables of pfb_analysis_plan_create without a device (nothing
 * allocated, nothing kept): the status create would return before touching the GPU. */
pfb_status pfb_analysis_plan_validate(const pfb_analysis_desc* desc);

/* Number of output samples per channel for n_dat input samples of a stateless call:
 * Bunton K = floor((n_dat - P*N)/M) (polyphase_analysis.m:62), padded K = floor(n_dat/M)
 * (polyphase_analysis_padded.m:75). */
int64_t pfb_analysis_output_length(const pfb_analysis_plan* plan, int64_t n_dat);

/* Channels per output row: n_chan, or 216 for PFB_ANALYSIS_LOWCBF
 * (polyphase_analysis_lowcbf.m:43, PSTFilterbank.m:44). */
int32_t pfb_analysis_output_channels(const pfb_analysis_plan* plan);

/* Stateless analysis — replaces polyphase_analysis(in, filt, block, os_factor) and
 * polyphase_analysis_padded(...).  in: n_pol series of n_dat samples; out: n_pol x
 * (K x n_chan).  *n_out receives K. */
pfb_status pfb_analysis_execute(pfb_analysis_plan* plan, const pfb_cf32* in,
                                int64_t in_pol_stride, int64_t n_dat, pfb_cf32* out,
                                int64_t out_pol_stride, int64_t out_capacity,
                                int64_t* n_out, int32_t mem, void* stream);

/* Stateful stream — replaces FilterBank.execute (FilterBank.m:65-128): prepends the
 * carried-over input, runs the analysis, trims the output to a multiple of nu and
 * keeps input[T_out*M:] for the next call.  Input rounding hooks (rndInput etc.) are
 * applied by the host mirror before this call.  Padded variant, device output: when
 * out_capacity covers all K computed rows (not just the *n_out = T_out kept ones), rows
 * [T_out, K) of each pol are used as scratch (the circular shift spans all K rows). */
pfb_status pfb_filterbank_execute(pfb_analysis_plan* plan, const pfb_cf32* in,
                                  int64_t in_pol_stride, int64_t n_in, pfb_cf32* out,
                                  int64_t out_pol_stride, int64_t out_capacity,
                                  int64_t* n_out, int32_t mem, void* stream);
int64_t pfb_filterbank_buffered(const pfb_analysis_plan* plan);
pfb_status pfb_filterbank_reset(pfb_analysis_plan* plan);
/* Rows the next pfb_filterbank_execute of n_in samples returns (the nu-trimmed T_out of
 * FilterBank.m:93-104 over the carried + new samples); -1 on a null plan. */
int64_t pfb_filterbank_output_rows(const pfb_analysis_plan* plan, int64_t n_in);

/* The same stream call writing the channelised product strided (device buffers only,
 * streaming Bunton kernel: N = 256): bin c of row k of polarisation p goes to
 * out[p * out_pol_stride + k * row_stride + j * chan_stride], j = c, or with sel_n > 0
 * the cascade's channel chomp j = c < sel_split ? c : c - sel_shift (bins in
 * [sel_split, sel_split + sel_shift) and j >= sel_n dropped).  Serves the two-stage
 * cascade (TwoStageFilterBank.m:92-110): stage 1 written channel-major (row_stride 1,
 * chan_stride = series length) is the per-channel input of stage 2 with no corner turn;
 * stage 2 written with row_stride nch1*nch2, out_pol_stride nch2 and the chomp
 * (sel_split nch2/2-1, sel_shift = dropped bins) is the assembled output of
 * TwoStageFilterBank.m:102-105 with no gather.  PFB_ERR_UNSUPPORTED for other kernels.
 * out_capacity is the number of pfb_cf32 elements available from `out`: a call whose
 * furthest written element ((n_pol-1) out_pol_stride + (rows-1) row_stride + (j_max)
 * chan_stride) lies beyond it fails with PFB_ERR_BUFFER_TOO_SMALL and writes nothing. */
pfb_status pfb_filterbank_execute_strided(pfb_analysis_plan* plan, const pfb_cf32* in,
                                          int64_t in_pol_stride, int64_t n_in, pfb_cf32* out,
                                          int64_t out_pol_stride, int64_t row_stride,
                                          int64_t chan_stride, int32_t sel_split,
                                          int32_t sel_shift, int32_t sel_n,
                                          int64_t out_capacity, int64_t* n_out, void* stream);

/* ---------------------------------------------------------------- synthesis */
typedef struct pfb_synthesis_desc {
  int32_t n_chan;             /* channels in the input */
  int32_t os_nu;
  int32_t os_de;
  int32_t input_fft_length;   /* Nf */
  int32_t input_overlap;      /* Ov */
  int32_t spans_nyquist;      /* input_fully_spans_Nyquist_zone (1 = oversampled Low/Mid) */
  int32_t combine;            /* coarse channels combined (polyphase_synthesis.m:198-239) */
  int32_t apply_deripple;     /* deripple.apply_deripple */
  const double* taps;         /* deripple.filter_coeff (host, copied) */
  int64_t n_taps;
  int32_t temporal_taper;     /* pfb_window_kind */
  const double* temporal_coeffs; /* CUSTOM: Nf coefficients */
  int32_t spectral_taper;     /* pfb_window_kind (NONE = identity_taper) */
  const double* spectral_coeffs; /* CUSTOM: L = Nf*de/nu*n_chan coefficients */
  int32_t n_pol;
  int32_t device;
} pfb_synthesis_desc;

typedef struct pfb_synthesis_plan pfb_synthesis_plan;

/* Replaces: InverseFilterBank constructor (InverseFilterBank.m:33-43) incl. the
 * PFBWindow lookup and the freqz-based deripple response (polyphase_synthesis.m:138-150). */
pfb_status pfb_synthesis_plan_create(const pfb_synthesis_desc* desc, pfb_synthesis_plan** plan);
pfb_status pfb_synthesis_plan_destroy(pfb_synthesis_plan* plan);
/* The checks and host-side tables (window, deripple gains, four-step twiddles) of
 * pfb_synthesis_plan_create without a device: the status create would return before
 * touching the GPU. */
pfb_status pfb_synthesis_plan_validate(const pfb_synthesis_desc* desc);

/* n_blocks * output_keep for n_dat channelised samples (polyphase_synthesis.m:112-131). */
int64_t pfb_synthesis_output_length(const pfb_synthesis_plan* plan, int64_t n_dat);

/* Stateless synthesis — replaces polyphase_synthesis(in, spans, Nf, os, deripple,
 * sample_offset, overlap, t_taper, s_taper, combine).  sample_offset is 1-based like
 * Matlab (:99).  in: n_pol x (n_dat x n_chan); out: n_pol series. */
pfb_status pfb_synthesis_execute(pfb_synthesis_plan* plan, const pfb_cf32* in,
                                 int64_t in_pol_stride, int64_t n_dat, int64_t sample_offset,
                                 pfb_cf32* out, int64_t out_pol_stride, int64_t out_capacity,
                                 int64_t* n_out, int32_t mem, void* stream);

/* Stateful stream — replaces InverseFilterBank.execute (InverseFilterBank.m:63-137):
 * carry-over of n_dat - B*keep samples rounded up to a multiple of nu. */
pfb_status pfb_inverse_filterbank_execute(pfb_synthesis_plan* plan, const pfb_cf32* in,
                                          int64_t in_pol_stride, int64_t n_in, pfb_cf32* out,
                                          int64_t out_pol_stride, int64_t out_capacity,
                                          int64_t* n_out, int32_t mem, void* stream);
int64_t pfb_inverse_filterbank_buffered(const pfb_synthesis_plan* plan);
pfb_status pfb_inverse_filterbank_reset(pfb_synthesis_plan* plan);
/* InverseFilterBank.sample_offset (InverseFilterBank.m:12, 0-based, default 0): every
 * pfb_inverse_filterbank_execute call synthesises the concatenated rows (carry + input)
 * from row sample_offset on — polyphase_synthesis(..., sample_offset+1, ...) at :92-96 —
 * while the carry still starts at the consumed blocks' end (:104-133), so the offset is
 * skipped again at the head of every call's concatenation, as the Matlab object does. */
pfb_status pfb_inverse_filterbank_set_sample_offset(pfb_synthesis_plan* plan, int64_t sample_offset);

/* Blocks processed per channel-IFFT/block-kernel chunk (scratch = chunk * keep rows). */
pfb_status pfb_synthesis_set_chunk_blocks(pfb_synthesis_plan* plan, int32_t blocks);

/* Where the fused round trip's synthesis gets its stage-1 rows (the channel IFFT of each
 * channelised row = N^2 x the analysis FIR sums).  STORED: the analysis kernel writes them
 * to the plan's scratch and the synthesis reads them back.  RECOMPUTED (N = 256 streaming
 * shapes, Nf 256): the analysis writes only the channelised product and the synthesis
 * evaluates the rows it needs from the input series — the same FIR sums in the same order,
 * so the output is bit-identical, with the stage-1 rows never crossing HBM.  AUTO: the
 * measured-faster one for the shape.  Shapes without a recomputing
 * kernel use STORED whatever is set.  Reference: polyphase_analysis.m:88-121 and
 * polyphase_synthesis.m:282-285 (the channel IFFT this factors). */
typedef enum pfb_stage1_rows {
  PFB_STAGE1_AUTO = 0,
  PFB_STAGE1_STORED = 1,
  PFB_STAGE1_RECOMPUTED = 2
} pfb_stage1_rows;
pfb_status pfb_synthesis_set_stage1_rows(pfb_synthesis_plan* plan, int32_t mode);
/* Where the plan's last synthesis launch got its stage-1 rows: PFB_STAGE1_STORED (read
 * from rows a channel IFFT or the analysis wrote), PFB_STAGE1_RECOMPUTED (evaluated from
 * the input series), 0 before any launch, -1 for a null plan.  A diagnostic: a caller that
 * asked for RECOMPUTED can tell whether the shape took it (no reference counterpart). */
int32_t pfb_synthesis_last_stage1_rows(const pfb_synthesis_plan* plan);

/* ---------------------------------------------------------------- round trip */
/* Analysis followed by synthesis of its output — replaces the analysis -> synthesis
 * sequence of test_data_pipeline.m:114,132 (and data_gen/pipeline.py:71-75).
 * Device memory only.  in: n_pol series of n_dat samples; chan: the full channelised
 * product (n_pol x K x n_chan, written as pfb_analysis_execute writes it); out: the
 * synthesis of chan(:, :, sample_offset:end) as pfb_synthesis_execute computes it.
 * When the analysis kernel can emit the synthesis stage-1 rows (N = 256 streaming
 * shapes, the N > 256 register-window FIR) and no chunk size is set, the two run fused:
 * `chan` is bit-identical to pfb_analysis_execute and `out` agrees with
 * pfb_synthesis_execute to ~1e-7 (the stage-1 rows are N^2 x the FIR sums, the exact
 * channel IFFT of the unrounded row).  Otherwise the call is pipelined in chunks of
 * synthesis blocks (pfb_synthesis_set_chunk_blocks, default 64) with the analysis on a
 * second stream, and both results are bit-identical to the separate calls.  Ordered
 * after prior work on `stream`; later work on `stream` sees all of it (graph-capturable). */
pfb_status pfb_roundtrip_execute(pfb_analysis_plan* analysis, pfb_synthesis_plan* synthesis,
                                 const pfb_cf32* in, int64_t in_pol_stride, int64_t n_dat,
                                 pfb_cf32* chan, int64_t chan_pol_stride, int64_t chan_capacity,
                                 int64_t* n_chan_rows, int64_t sample_offset, pfb_cf32* out,
                                 int64_t out_pol_stride, int64_t out_capacity, int64_t* n_out,
                                 void* stream);

/* The fused round trip above in two halves, for a caller that pipelines consecutive
 * blocks over two streams (block i's synthesis beside block i+1's analysis, each block on
 * its own plan pair).  pfb_roundtrip_analysis_execute runs the analysis kernel of the
 * fused path: it writes the channelised product (as pfb_roundtrip_execute does) and the
 * synthesis stage-1 rows into `synthesis`'s scratch.  pfb_roundtrip_synthesis_execute
 * turns those rows into the output; n_dat and sample_offset must be the analysis half's.
 * The halves' results equal pfb_roundtrip_execute's fused path bit for bit.  The caller
 * orders them (synthesis after the analysis, the next analysis on the same pair after
 * the synthesis), e.g. with events.  With recomputed stage-1 rows
 * (pfb_synthesis_set_stage1_rows) the analysis half writes no rows: the synthesis half
 * re-reads `in`, which must stay allocated and unchanged until it has run.
 * PFB_ERR_UNSUPPORTED when the plans take the chunked pipeline (see above);
 * PFB_ERR_INVALID_ARG from the synthesis half when the plan holds no analysis half of this
 * analysis plan with the same n_dat and sample_offset (another shape, another plan, or a
 * whole round trip ran on the pair since).  Reference: the same lines as
 * pfb_roundtrip_execute. */
pfb_status pfb_roundtrip_analysis_execute(pfb_analysis_plan* analysis, pfb_synthesis_plan* synthesis,
                                          const pfb_cf32* in, int64_t in_pol_stride, int64_t n_dat,
                                          pfb_cf32* chan, int64_t chan_pol_stride, int64_t chan_capacity,
                                          int64_t* n_chan_rows, int64_t sample_offset, void* stream);
pfb_status pfb_roundtrip_synthesis_execute(pfb_analysis_plan* analysis, pfb_synthesis_plan* synthesis,
                                           int64_t n_dat, int64_t sample_offset, pfb_cf32* out,
                                           int64_t out_pol_stride, int64_t out_capacity, int64_t* n_out,
                                           void* stream);

/* Round-trip output length estimate — replaces calc_output_nbins(nbins, channels,
 * os_factor, filter_taps, input_fft_length, input_overlap) (calc_output_nbins.m:17-27):
 * Matlab double arithmetic with its floor()s, so a non-integral normalize(os, n) gives the
 * same fractional result Matlab does.  Host-only arithmetic (no device needed). */
double pfb_calc_output_nbins(int64_t nbins, int32_t channels, int32_t os_nu, int32_t os_de,
                             int64_t filter_taps, int32_t input_fft_length, int32_t input_overlap);

/* ---------------------------------------------------------------- data formats */
/* Sample order of a DADA file's data section. */
typedef enum pfb_dada_order {
  PFB_DADA_TFP = 0,   /* time, channel, polarisation, re/im (reshape_dada_data.m:23-30,
                         write_dada_data.m:32-50) */
  PFB_DADA_LOWCBF = 1 /* heaps of 32 samples: [heap][chan][pol][sample], INSTRUMENT LowCBF
                         (reshape_low_cbf_data.m:14-43, DADARead.m:74-78) */
} pfb_dada_order;

/* DADA data section (device memory, NBIT 8/16/32/64 signed integer / float samples,
 * NDIM 1 or 2) -> [pol][t][chan] complex float32.  Replaces read_dada_file.m:36-47 +
 * reshape_dada_data.m (and DADARead.generate, DADARead.m:58-83, incl. its cast of
 * integer samples to floating point).  NBIT 64 is rounded to float32 (the engine's
 * arithmetic type).  Asynchronous on `stream`. */
pfb_status pfb_dada_unpack(const void* in, int32_t nbit, int32_t ndim, int32_t order,
                           int64_t n_dat, int32_t n_chan, int32_t n_pol, pfb_cf32* out,
                           int64_t out_pol_stride, void* stream);

/* [pol][t][chan] complex float32 -> DADA TFP data section (NDIM 2) of NBIT 8/16/32/64;
 * integer types follow Matlab's cast (round half away from zero, saturate).  Replaces
 * write_dada_data.m:32-50 (data written with the class write_dada_header.m:13-22
 * records as NBIT). */
pfb_status pfb_dada_pack(const pfb_cf32* in, int64_t in_pol_stride, int64_t n_dat, int32_t n_chan,
                         int32_t n_pol, void* out, int32_t nbit, void* stream);

/* Channel gather: out[o][t][j] = in[o][t][src0 + j + (j >= split ? shift : 0)] for
 * o < n_outer (<= 65535), t < n_rows, j < n_sel (strides in complex samples).
 * Replaces the stage-2 output assembly of TwoStageFilterBank.m:102-105 (shift = the
 * oversampled channels dropped in the middle) and the per-coarse-channel input slices
 * of TwoStageInverseFilterBank.m:124-126.  Device memory, asynchronous. */
pfb_status pfb_gather_channels(const pfb_cf32* in, int64_t in_outer_stride, int64_t in_row_stride,
                               pfb_cf32* out, int64_t out_outer_stride, int64_t out_row_stride,
                               int64_t n_outer, int64_t n_rows, int32_t n_sel, int32_t src0,
                               int32_t split, int32_t shift, void* stream);

/* Corner turn: out[o][c][r] = in[o][r][c] (r < n_rows, c < n_cols, o < n_outer).
 * Replaces the out1(1,ich,:) channel slices TwoStageFilterBank.m:94 feeds to stage 2
 * (channelised [t][chan] -> per-channel series).  Device memory, asynchronous. */
pfb_status pfb_corner_turn(const pfb_cf32* in, int64_t in_outer_stride, int64_t in_row_stride,
                           int64_t n_outer, int64_t n_rows, int64_t n_cols, pfb_cf32* out,
                           int64_t out_outer_stride, int64_t out_row_stride, void* stream);

/* Quantisation hook: out = round(single(scale) * in) with scale = rms / sqrt(var(in, 0,
 * "all")) over all n_pol x n samples, or 1 when rms <= 0 (Matlab round: half away from
 * zero).  Replaces FilterBank.m:75-83 (rndInput/rmsInput) and :106-113
 * (rndOutput/rmsOutput).  in == out is allowed.  Device memory; asynchronous unless
 * `scale` is non-null (then it receives the scale and the call synchronises). */
pfb_status pfb_quantize(const pfb_cf32* in, int64_t in_pol_stride, int64_t n, int32_t n_pol,
                        double rms, pfb_cf32* out, int64_t out_pol_stride, double* scale,
                        void* stream);

/* ---------------------------------------------------------------- utilities */
const char* pfb_last_error(void);
int32_t pfb_api_version(void);
int32_t pfb_device_count(void);
/* Device memory helpers for callers without their own allocator (ctypes harness). */
pfb_status pfb_device_malloc(int32_t device, int64_t bytes, void** ptr);
pfb_status pfb_device_free(void* ptr);
pfb_status pfb_memcpy_h2d(void* dst, const void* src, int64_t bytes, void* stream);
pfb_status pfb_memcpy_d2h(void* dst, const void* src, int64_t bytes, void* stream);
pfb_status pfb_stream_synchronize(void* stream);
/* Bandwidth probe (no reference counterpart; SURVEY §8(d) asks for the achievable
 * copy rate beside the HBM spec): device-to-device float4 copy kernel.  16-B aligned
 * pointers, n_bytes a multiple of 64.  Asynchronous on `stream`. */
pfb_status pfb_device_copy(void* dst, const void* src, int64_t n_bytes, void* stream);

/* Kernel timing: average duration (ms) of the named kernel class over the launches
 * recorded since the last reset, measured with HIP events on the plan's stream.
 * which: 0 = analysis, 1 = synthesis channel-IFFT, 2 = synthesis block kernel,
 *        3 = analysis fused with the synthesis channel IFFT (pfb_roundtrip_execute),
 *        4 / 5 = the FIR / the row FFT of the n_chan > 256 round trip (SKA-Mid), each
 *        launch timed alone; bytes: what each reads + writes once. */
pfb_status pfb_profile_enable(int32_t enable);
pfb_status pfb_profile_read(int32_t which, double* total_ms, int64_t* launches, double* bytes);
pfb_status pfb_profile_reset(void);
/* Name of the kernel whose launches class `which` recorded (the last one, demangled as a
 * kernel trace prints it, e.g. "void pfb::synth_block_kernel<256, 224, ...>(pfb::
 * SynthBlockArgs)"); "" when the class recorded no single-kernel launch.  Writes at most
 * `len` bytes including the terminating NUL. */
pfb_status pfb_profile_kernel_name(int32_t which, char* buf, int64_t len);

/* Build flags of the loaded library: bit 0 = experiments build (A/B knobs and timing
 * masks read from PFB_* environment variables; never a release or benchmark library). */
int32_t pfb_build_flags(void);

#ifdef __cplusplus
}
#endif

#endif /* PFB_API_H */
