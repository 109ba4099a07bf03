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
           "freq_domain_offsets", "frequency_comb_test", "purity_sweep"]


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


def time_domain_offsets(block_size: int, output_overlap: int, filt_offset: int, max_size: int,
                        npoints: int):
    """current_performance.m:60-74: impulse positions across block boundaries and overlaps."""
    jump = block_size - 2 * output_overlap
    spaced = list(range(filt_offset, max_size + 1, jump))
    p = list(spaced)
    p += [s - output_overlap for s in spaced[1:]]
    p += [s + output_overlap for s in spaced[:-1]]
    p += list(range(filt_offset, max_size + 1, block_size))
    p += list(range(1, max_size + 1, int(round(max_size / npoints))))
    return sorted(p)


def freq_domain_offsets(block_size: int, nblocks: int, npoints: int):
    """current_performance.m:77-81: tone harmonic numbers (1:round(bs/np):bs) * nblocks."""
    return [h * nblocks for h in range(1, block_size + 1, int(round(block_size / npoints)))]


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
def purity_sweep(device=0, npoints: int = 8, batch: int = 8, channels: int = 4096,
                 os_factor="8/7", input_fft_length: int = 512, input_overlap: int = 128,
                 taps=None, blocks: int = 3, analysis="polyphase_analysis_padded"):
    """The test_purity sweep of BASELINE configs[4] (current_performance.m:35-81,
    sgcht.m:368-431) on the HIP engine: temporal impulses at the block-boundary and
    overlap positions, tones on the harmonic grid, the 32-tone frequency comb and a
    square wave, each a vector of blocks * Nf de/nu * N samples, run in batches of
    ``batch`` vectors as the polarisations of ONE round-trip plan.  Returns one record
    per vector (kind, parameter, metrics)."""
    import torch
    from .core import AnalysisPlan, SynthesisPlan, roundtrip
    from .firio import design_PFB_FIR_filter_two_stage
    from .window import PFBWindow
    o = as_rational(os_factor)
    if taps is None:
        taps = design_PFB_FIR_filter_two_stage(channels, os_factor, 28)
    al = purity_alignment(channels, o, input_fft_length, input_overlap, len(taps), blocks)
    n = al["n_samples"]
    vectors = []
    # impulse positions of the grid whose response lands inside the synthesised output
    # (blocks * L_keep samples starting total_sample_shift after the input)
    n_out = blocks * (al["block_size"] - 2 * al["output_sample_shift"])
    offs = [p for p in time_domain_offsets(al["block_size"], al["output_sample_shift"],
                                           al["total_sample_shift"], n - 1, npoints)
            if 0 <= p - al["total_sample_shift"] < n_out]
    pick = np.linspace(0, len(offs) - 1, min(npoints, len(offs))).round().astype(int)
    for off in sorted(set(offs[i] for i in pick)):
        vectors.append(("impulse", off, impulse(n, off)))
    for h in freq_domain_offsets(al["block_size"], blocks, npoints)[:npoints]:
        vectors.append(("tone", h, pure_tone(n, h / n)))
    f, a = comb_frequencies(n_chan=channels, invert=True)
    vectors.append(("comb", 32, frequency_comb(n, f, a)))
    vectors.append(("square_wave", 3981, square_wave(n, 3981)))
    dev = torch.device("cuda", int(device))
    win = PFBWindow().lookup["tukey"](input_fft_length, input_overlap)
    out = []
    for i0 in range(0, len(vectors), batch):
        part = vectors[i0:i0 + batch]
        x = torch.from_numpy(np.stack([v[2] for v in part])).to(dev)
        ana = AnalysisPlan(taps, channels, o, analysis, len(part), int(device))
        syn = SynthesisPlan(channels, o, input_fft_length, input_overlap, True, 1, True, taps,
                            win, None, len(part), int(device))
        _, y = roundtrip(ana, syn, x)
        y = y.cpu().numpy()
        for (kind, param, xin), yy in zip(part, y):
            rec = {"kind": kind, "param": int(param), "n_out": int(yy.size),
                   "power_ratio": float(np.mean(np.abs(yy) ** 2) /
                                        max(np.mean(np.abs(xin) ** 2), 1e-30))}
            if kind == "impulse":
                rec.update(impulse_purity(yy, int(param), al["total_sample_shift"]))
            elif kind == "tone":
                period = n / param
                span = int(np.floor(yy.size / period) * period) if period <= yy.size else yy.size
                rec.update(tone_purity(yy[:span]))
            elif kind == "comb":
                rec["comb_test"] = frequency_comb_test(yy[None, None, :], f, o, invert=True)
            out.append(rec)
    return out
