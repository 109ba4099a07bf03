"""Purity metrics and alignment of the reference's verification harness
(``python/verify/util.py:15-43``, ``python/verify/purity.py:76-88,165-283``), so the
``hip`` backend can be scored exactly as the reference scores its backends.

Host-side NumPy on the (small) metric arrays; the data they score comes off the device.
"""
from __future__ import annotations

import numpy as np

from .config import as_rational

__all__ = ["spurious", "total_spurious", "mean_spurious", "max_spurious", "dB",
           "purity_alignment", "impulse_purity", "tone_purity", "pure_tone", "impulse",
           "comb_frequencies", "frequency_comb", "square_wave", "time_domain_offsets",
           "freq_domain_offsets", "frequency_comb_test", "purity_sweep", "zero_max_val",
           "max_spurious_power", "total_spurious_power", "mean_spurious_power",
           "temporal_difference", "temporal_performance", "spectral_performance", "chop",
           "performance_alignment", "complex_sinusoid", "time_domain_impulse", "sweep_vectors",
           "shard", "score_vector", "square_wave_contrast"]


def spurious(a):
    """util.py:15-18: the array with its largest element zeroed."""
    b = np.array(a, copy=True)
    b[np.argmax(b)] = 0.0
    return b


def dB(a):
    """util.py:39-43 (``a`` already in power)."""
    return 10.0 * np.log10(np.abs(np.array(a, copy=True)) + 1e-13)


def total_spurious(a):
    """util.py:21-24."""
    return dB(np.sum(spurious(np.abs(a) ** 2)))


def mean_spurious(a):
    """util.py:27-30."""
    return dB(np.mean(spurious(np.abs(a) ** 2)))


def max_spurious(a):
    """util.py:33-36."""
    return dB(np.amax(spurious(np.abs(a) ** 2)))


def purity_alignment(channels: int, os_factor, input_fft_length: int, input_overlap: int,
                     fir_filter_taps: int, blocks: int) -> dict:
    """purity.py:76-88: block size, sample counts and the shift between a test vector
    and the synthesised output (overlap discard + FIR group delay)."""
    o = as_rational(os_factor)
    block_size = input_fft_length * o.de // o.nu * channels
    output_sample_shift = input_overlap * o.de // o.nu * channels
    return {"normalize": input_fft_length * channels, "block_size": block_size,
            "fft_size": 2 * block_size, "n_samples": block_size * blocks,
            "output_sample_shift": output_sample_shift,
            "total_sample_shift": output_sample_shift + (fir_filter_taps - 1) // 2}


def impulse_purity(synth: np.ndarray, offset: int, total_sample_shift: int) -> dict:
    """Score a synthesised temporal impulse (TestImpulse.m:46-73 criteria): the output
    is aligned by ``total_sample_shift`` (purity.py:276-283) and the power outside the
    impulse sample is summarised by the util.py metrics."""
    y = np.asarray(synth).reshape(-1)
    pos = offset - total_sample_shift
    peak = int(np.argmax(np.abs(y)))
    p = np.abs(y) ** 2
    p = p / p.max()
    outside = p.copy()
    outside[max(peak - 1, 0):peak + 2] = 0.0  # TestImpulse.m:46-73: all but +-1 sample
    return {"peak_index": peak, "expected_index": pos,
            "max_outside_pm1_dB": float(dB(outside.max())),
            "total_spurious": float(total_spurious(np.sqrt(p))),
            "max_spurious": float(max_spurious(np.sqrt(p))),
            "mean_spurious": float(mean_spurious(np.sqrt(p)))}


def tone_purity(synth: np.ndarray) -> dict:
    """Score a synthesised tone (TestPureTone.m:55-89): spectrum power normalised to the
    tone bin, util.py metrics over the remaining bins."""
    y = np.asarray(synth).reshape(-1)
    spec = np.abs(np.fft.fft(y)) ** 2
    spec = spec / spec.max()
    return {"peak_bin": int(np.argmax(spec)), "total_spurious": float(total_spurious(np.sqrt(spec))),
            "max_spurious": float(max_spurious(np.sqrt(spec))),
            "mean_spurious": float(mean_spurious(np.sqrt(spec)))}


# ------------------------------------------------------------------ test-signal generators
def pure_tone(n: int, frequency: float, amplitude: float = 1.0, current: int = 0):
    """PureTone.m:1-30: amplitude e^{i 2 pi f (t + current)} (f in cycles per sample)."""
    t = np.arange(n, dtype=np.float64) + current
    return (amplitude * np.exp(2j * np.pi * frequency * t)).astype(np.complex64)


def impulse(n: int, offset: int, amplitude: float = 1.0, noise: float = 1e-6, rng=None):
    """Impulse.m:23-37 (its ``noise`` meant ``obj.noise`` = 1e-6)."""
    rng = np.random.default_rng(0) if rng is None else rng
    x = np.zeros(n, dtype=np.complex64)
    if noise:
        x += (noise * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    if 0 <= offset < n:
        x[offset] = amplitude
    return x


def comb_frequencies(nharmonic: int = 32, n_chan: int = 1, two_stage: bool = False,
                     invert: bool = False, comb: str = ""):
    """sgcht.m:394-431: harmonic frequencies (cycles per sample) and amplitudes
    linspace(1, sqrt 2) of the frequency-comb test signal."""
    amplitudes = np.linspace(1.0, np.sqrt(2.0), nharmonic)
    fmin = -0.5 + 1.0 / (nharmonic * 4)
    fmax = fmin + (nharmonic - 1.0) / nharmonic
    if comb == "coarse":
        fmin, fmax = fmin / n_chan, fmax / n_chan
    elif comb == "fine":
        fmin, fmax = fmin / n_chan ** 2, fmax / n_chan ** 2
    elif n_chan > 1:
        nch = n_chan ** 2 if two_stage else n_chan
        if invert:
            nch = nch / n_chan
        if nch > 1:
            fmin += 1.0 / (nch * 4)
            fmax += 1.0 / (nch * 4)
    return np.linspace(fmin, fmax, nharmonic), amplitudes


def frequency_comb(n: int, frequencies, amplitudes):
    """FrequencyComb.m:1-40: the sum of PureTone generators."""
    x = np.zeros(n, dtype=np.complex128)
    t = np.arange(n, dtype=np.float64)
    for f, a in zip(frequencies, amplitudes):
        x += a * np.exp(2j * np.pi * f * t)
    return x.astype(np.complex64)


def square_wave(n: int, period: int, duty_cycle: float = 0.5, on_amp: float = 1.0,
                off_amp: float = 0.0, rng=None, current: int = 0):
    """SquareWave.m:24-58: complex Gaussian noise of power on_amp during the first
    floor(period duty) samples of each period, off_amp otherwise."""
    rng = np.random.default_rng(0) if rng is None else rng
    ioff = int(np.floor(period * duty_cycle))
    phase = (np.arange(n) + current) % period
    amp = np.where(phase < ioff, np.sqrt(on_amp * 0.5), np.sqrt(off_amp * 0.5))
    noise = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    return (amp * noise).astype(np.complex64)


# ------------------------------------------------------------------ current_performance.m
# The C5 purity sweep as the reference's Matlab harness runs it (current_performance.m,
# DomainPerformance.m, ErrorAnalysis.m, chop.m): per test vector one analysis ->
# synthesis round trip, the output aligned with the input by chop, then scored.
def zero_max_val(a, domain: int = 0):
    """ErrorAnalysis.m:5-33: zero the maximum bin and ``domain`` bins either side."""
    a = np.array(a, copy=True)
    k = int(np.argmax(a))
    a[max(k - domain, 0):min(k + domain, len(a) - 1) + 1] = 0
    return a


def max_spurious_power(a, domain: int = 0):
    """ErrorAnalysis.m:39-42."""
    return float(np.max(zero_max_val(a, domain)))


def mean_spurious_power(a, domain: int = 0):
    """ErrorAnalysis.m:44-47."""
    return float(np.mean(zero_max_val(a, domain)))


def total_spurious_power(a, domain: int = 0):
    """ErrorAnalysis.m:49-52."""
    return float(np.sum(zero_max_val(a, domain)))


def temporal_difference(a, b):
    """DomainPerformance.m:7-64 (correct_phase = 0, no plots): [max, sum, mean] of |a-b|^2."""
    d = np.abs(np.asarray(a, np.complex128) - np.asarray(b, np.complex128)) ** 2
    return [float(d.max()), float(d.sum()), float(d.mean())]


def temporal_performance(a, domain: int = 0):
    """DomainPerformance.m:67-83: [max, total] spurious power of |a|^2."""
    p = np.abs(np.asarray(a, np.complex128)) ** 2
    return [max_spurious_power(p, domain), total_spurious_power(p, domain)]


def spectral_performance(a, fft_length: int, domain: int = 0):
    """DomainPerformance.m:85-100: |fft(a, fft_length) / fft_length|^2 (Matlab's fft(a, n)
    truncates or zero-pads a to n samples), [max, total] spurious power."""
    f = np.abs(np.fft.fft(np.asarray(a, np.complex128), int(fft_length)) / fft_length) ** 2
    return [max_spurious_power(f, domain), total_spurious_power(f, domain)]


def chop(input_series, inv_series, fir_offset: int, additional_offset: int = 0):
    """chop.m:13-46: drop ``additional_offset - fir_offset`` leading input samples and cut
    both series to the shorter length -> (input, inv)."""
    to_chomp = int(additional_offset) - int(fir_offset)
    sim = np.asarray(input_series).reshape(-1)[to_chomp:]
    inv = np.asarray(inv_series).reshape(-1)
    n = min(len(sim), len(inv))
    return sim[:n], inv[:n]


def performance_alignment(channels: int, os_factor, input_fft_length: int, input_overlap: int,
                          n_taps: int, blocks: int, fir_offset_direction: int,
                          kludge_offset: int) -> dict:
    """The constants of current_performance.m:203-235 and test_data_pipeline.m:136:
    block_size = normalize(os, Nf) N, nbins = blocks block_size, output_overlap =
    normalize(os, Ov) N - 1, filt_offset = round((L_h - 1) / 2), fir_offset =
    fir_offset_direction floor(L_h / 2), the chop offset output_overlap + kludge_offset,
    fft_length = 2 normalize(os, Nf) N (:179) and output_nbins (calc_output_nbins.m)."""
    o = as_rational(os_factor)
    block_size = input_fft_length * o.de // o.nu * channels
    output_overlap = input_overlap * o.de * channels // o.nu - 1
    nbins = blocks * block_size
    step = (channels * o.de) // o.nu
    nblocks_pfb = (nbins - n_taps) // step
    output_pfb = (step * nblocks_pfb) // channels
    keep = input_fft_length - 2 * input_overlap
    output_nbins = ((output_pfb - 2 * input_overlap) // keep) * (block_size - 2 * (output_overlap + 1))
    return {"block_size": block_size, "nbins": nbins, "output_overlap": output_overlap,
            "filt_offset": int(np.floor((n_taps - 1) / 2 + 0.5)),
            "fir_offset": int(fir_offset_direction) * (n_taps // 2),
            "additional_offset": output_overlap + int(kludge_offset),
            "fft_length": 2 * block_size, "output_nbins": output_nbins}


def time_domain_offsets(block_size: int, output_overlap: int, filt_offset: int, max_size: int,
                        npoints: int):
    """current_performance.m:60-74 (1-based impulse positions, Matlab colon ranges;
    ``output_overlap`` as passed there: normalize(os, Ov) N)."""
    jump = block_size - 2 * output_overlap
    spaced = list(range(filt_offset, max_size + 1, jump))
    p = list(spaced)
    p += [s - output_overlap for s in spaced[1:]]
    p += [s + output_overlap for s in spaced[:-1]]
    p += list(range(filt_offset, max_size + 1, block_size))
    p += list(range(1, max_size + 1, int(np.floor(max_size / npoints + 0.5))))
    return sorted(p)


def freq_domain_offsets(block_size: int, nblocks: int, npoints: int):
    """current_performance.m:77-81: tone frequencies (1:round(bs/np):bs) * nblocks, in
    cycles per nbins (complex_sinusoid.m)."""
    return [h * nblocks for h in range(1, block_size + 1, int(np.floor(block_size / npoints + 0.5)))]


def complex_sinusoid(n_bins: int, frequency: float, phase: float = np.pi / 4, bin_offset: float = 0.0):
    """complex_sinusoid.m:16-31 (double maths, single result)."""
    t = np.arange(n_bins, dtype=np.float64)
    return np.exp(1j * (2 * np.pi * (frequency + bin_offset) / n_bins * t + phase)).astype(np.complex64)


def time_domain_impulse(n_bins: int, offset: int, width: int = 1):
    """time_domain_impulse.m:13-24: ones at the 1-based positions offset .. offset+width-1."""
    x = np.zeros(n_bins, dtype=np.complex64)
    x[offset - 1:offset - 1 + width] = 1.0
    return x


def sweep_vectors(al: dict, npoints: int, blocks: int, domains=("time", "freq")):
    """The ordered (domain, parameter) list of the sweep: current_performance.m's impulse
    positions (time_domain_offsets with its arguments at :243-244) and tone frequencies."""
    out = []
    if "time" in domains:
        out += [("time", p) for p in time_domain_offsets(al["block_size"], al["output_overlap"] + 1,
                                                         al["filt_offset"], al["output_nbins"], npoints)]
    if "freq" in domains:
        out += [("freq", f) for f in freq_domain_offsets(al["block_size"], blocks, npoints)]
    return out


def shard(items, rank: int, world: int):
    """Round-robin share of rank ``rank`` (BASELINE configs[4]: vectors over 8 GPUs)."""
    return list(items)[rank::world]


def score_vector(domain: str, param: int, xin, y, al: dict) -> dict:
    """Score one round trip as current_performance.m does (time: temporal_performance(inv,
    30); freq: temporal_difference(input, inv) + spectral_performance(inv, fft_length)),
    plus the pass criteria of the reference's unit tests on the same aligned data:
    TestImpulse.m:46-73 (<= -60 dB outside +-1 sample of the EXPECTED index) and
    TestPureTone.m:55-89 (max spurious spectral power <= -60 dB of the tone)."""
    inp, inv = chop(xin, y, al["fir_offset"], al["additional_offset"])
    rec = {"domain": domain, "param": int(param), "n_chopped": int(len(inv))}
    if domain == "time":
        mx, tot = temporal_performance(inv, 30)
        rec.update(max_spurious_power=mx, total_spurious_power=tot,
                   max_spurious_dB=float(dB(mx)), total_spurious_dB=float(dB(tot)))
        e = int(param) - 1 - (al["additional_offset"] - al["fir_offset"])  # aligned index
        if 0 <= e < len(inv):
            a = np.abs(inv.astype(np.complex128))
            rec["expected_index"] = e
            rec["peak_index"] = int(np.argmax(a))
            rec["peak_amplitude"] = float(a[e])
            m = np.ones(len(a), bool)
            m[max(e - 1, 0):e + 2] = False
            rec["max_outside_pm1_dB"] = float(20 * np.log10(a[m].max() / max(a[e], 1e-30) + 1e-30))
    else:
        d = temporal_difference(inp, inv)
        sp = spectral_performance(inv, al["fft_length"])
        rec.update(max_diff_power=d[0], total_diff_power=d[1], mean_diff_power=d[2],
                   max_spurious_power=sp[0], total_spurious_power=sp[1],
                   max_spurious_dB=float(dB(sp[0])), total_spurious_dB=float(dB(sp[1])),
                   max_diff_dB=float(dB(d[0])))
    return rec


def square_wave_contrast(y, period: int, duty_cycle: float, shift: int, guard: int) -> dict:
    """Not a reference test (sgcht.m:380: 'Testing not implemented for square_wave'):
    mean output power in the on and off phases of the aligned square wave, ``guard``
    samples from each transition excluded."""
    y = np.asarray(y).reshape(-1)
    ph = (np.arange(len(y)) + shift) % period
    ioff = int(np.floor(period * duty_cycle))
    on = (ph >= guard) & (ph < ioff - guard)
    off = (ph >= ioff + guard) & (ph < period - guard)
    p = np.abs(y.astype(np.complex128)) ** 2
    return {"on_power": float(p[on].mean()), "off_power": float(p[off].mean())}


def frequency_comb_test(data, frequencies, os_factor="1/1", two_stage=False, invert=False,
                        critical=False) -> int:
    """TestFrequencyComb.m:1-86: every harmonic must appear with |FFT| >= 0.5 in the
    channel it falls in.  ``data`` is (n_pol, n_chan, n_dat).  Returns 0 or -1."""
    o = as_rational(os_factor)
    data = np.asarray(data)
    npol, nchan, _ = data.shape
    max_nfft = 8 * 1024
    for ipol in range(npol):
        for ichan in range(nchan):
            x = data[ipol, ichan, :]
            nfft = min(x.size, max_nfft)
            x = x[:nfft]
            fft_in = np.abs(np.fft.fft(x) / (nfft * nchan))
            level = 2 if two_stage else (1 if nchan > 1 else 0)
            level -= int(bool(invert)) + int(bool(critical))
            hfac = nchan * nfft
            for _ in range(max(level, 0)):
                hfac = hfac * o.de / o.nu
            for f in frequencies:
                jchan = (int(np.floor(f * nchan)) + nchan) % nchan
                if jchan == ichan:
                    offset = ichan / nchan
                    iharm = (int(np.floor((f - offset) * hfac)) + nfft) % nfft
                    if fft_in[iharm] < 0.5:
                        return -1
    return 0


# ------------------------------------------------------------------ the C5 sweep
def purity_sweep(device=0, npoints: int = 300, batch: int = 16, channels: int = 4096,
                 os_factor="8/7", input_fft_length: int = 512, input_overlap: int = 128,
                 taps=None, blocks: int = 3, analysis="polyphase_analysis_padded",
                 fir_offset_direction: int = 0, kludge_offset: int = 0, rank: int = 0,
                 world: int = 1, domains=("time", "freq"), extras: bool = True,
                 max_vectors: int = 0):
    """BASELINE configs[4]: the test_purity sweep of current_performance.m (sub-config
    'mid': padded bank, 4096 ch, 8/7, 100 353 two-stage taps, Nf 512, Ov 128, tukey,
    deripple, 3 blocks = 5 505 024 samples per vector, fir_offset_direction 0,
    kludge_offset 0; npoints 300) on the HIP engine — temporal impulses and tones scored
    exactly as the reference scores them (score_vector), plus the sgcht.m signals (the
    32-tone frequency comb with TestFrequencyComb.m, the square wave).  Vectors are
    dealt round-robin over ``world`` GPUs (this call runs rank ``rank``'s share) and
    batched ``batch`` at a time as the polarisations of ONE round-trip plan.  Returns
    one record per vector."""
    import torch
    from .core import AnalysisPlan, SynthesisPlan, roundtrip
    from .firio import design_PFB_FIR_filter_two_stage
    from .window import PFBWindow
    o = as_rational(os_factor)
    if taps is None:
        taps = design_PFB_FIR_filter_two_stage(channels, os_factor, 28)
    al = performance_alignment(channels, o, input_fft_length, input_overlap, len(taps), blocks,
                               fir_offset_direction, kludge_offset)
    n = al["nbins"]
    items = sweep_vectors(al, npoints, blocks, domains)
    if extras:
        items += [("comb", 32), ("square_wave", 3981)]
    if max_vectors:
        items = items[:max_vectors]
    items = shard(items, rank, world)
    f_comb, a_comb = comb_frequencies(n_chan=channels, invert=True)

    def make(kind, param):
        if kind == "time":
            return time_domain_impulse(n, param)
        if kind == "freq":
            return complex_sinusoid(n, param)
        if kind == "comb":
            return frequency_comb(n, f_comb, a_comb)
        return square_wave(n, param)

    dev = torch.device("cuda", int(device))
    win = PFBWindow().lookup["tukey"](input_fft_length, input_overlap)
    plans = {}
    out = []
    for i0 in range(0, len(items), batch):
        part = items[i0:i0 + batch]
        xs = [make(k, p) for k, p in part]
        x = torch.from_numpy(np.stack(xs)).to(dev)
        if len(part) not in plans:
            plans[len(part)] = (
                AnalysisPlan(taps, channels, o, analysis, len(part), int(device)),
                SynthesisPlan(channels, o, input_fft_length, input_overlap, True, 1, True, taps,
                              win, None, len(part), int(device)))
        ana, syn = plans[len(part)]
        _, y = roundtrip(ana, syn, x)
        y = y.cpu().numpy()
        for (kind, param), xin, yy in zip(part, xs, y):
            if kind in ("time", "freq"):
                rec = score_vector(kind, param, xin, yy, al)
            else:
                inp, inv = chop(xin, yy, al["fir_offset"], al["additional_offset"])
                rec = {"domain": kind, "param": int(param), "n_chopped": int(len(inv)),
                       "power_ratio": float(np.mean(np.abs(inv) ** 2) /
                                            max(np.mean(np.abs(inp) ** 2), 1e-30))}
                if kind == "comb":
                    rec["comb_test"] = frequency_comb_test(inv[None, None, :], f_comb, o, invert=True)
                else:
                    shift = al["additional_offset"] - al["fir_offset"]
                    rec.update(square_wave_contrast(inv, int(param), 0.5, shift, 64))
            rec["rank"] = rank
            out.append(rec)
    return out
