"""The reference's streaming test loop on the device: signal generator -> channelizer ->
(inverse) -> tester, in fixed-size chunks (matlab/sgcht.m:504-575, the primary call stack
of SURVEY §3.1), with the generator and tester objects it uses.

    PureTone        matlab/PureTone.m:13-27        (complex tone, phase carried across calls)
    Impulse         matlab/Impulse.m:14-38         (delta + optional noise, offset carried)
    TestPureTone    matlab/TestPureTone.m:13-90    (one FFT per block: peak bin, <= -60 dB)
    TestImpulse     matlab/TestImpulse.m:13-66     (<= -60 dB outside +-1 sample of the delta)
    sgcht           matlab/sgcht.m:269-575         (object set-up and the block loop)

The channelizers are the device stream objects of ``filterbank`` (FilterBank,
InverseFilterBank, TwoStageFilterBank, TwoStageInverseFilterBank): every block goes
through the HIP kernels and stays on the device between them; only the tester pulls the
block to the host (its FFT / magnitude checks are NumPy, as the Matlab ones are scalar
loops).  Generators run on the host (the reference generates single-precision blocks
with the Matlab RNG; here a seeded NumPy generator) and each block is copied to the
device once.

Reference quirks kept visible:
* ``Impulse.m:26`` tests ``noise`` (an undefined name in the class method) — the evident
  intent, ``obj.noise``, is used;
* TestPureTone/TestImpulse plot and pause (``figure; plot; pause``): not reproduced.
"""
from __future__ import annotations

import json
import math
import os
from types import SimpleNamespace

import numpy as np

from .config import as_rational, config_dir, default_config
from .firio import design_PFB_FIR_filter, design_PFB_FIR_filter_two_stage, read_fir_filter_coeff

__all__ = ["PureTone", "Impulse", "FrequencyComb", "SquareWave", "FrequencyWedge", "TestPureTone",
           "TestImpulse", "TestFrequencyComb", "comb_harmonics", "sgcht", "sgcht_config",
           "sgcht_filename", "header_template", "num2str"]


# ------------------------------------------------------------------ generators
class PureTone:
    """PureTone.m:13-27: x(1,1,:) = amplitude * exp(j 2 pi frequency (t + current)),
    computed in double and stored as single; ``current`` advances by nsample."""

    def __init__(self, frequency=1 / 26.5, amplitude=1.0):
        self.frequency = frequency
        self.amplitude = amplitude
        self.current = 0

    def generate(self, nsample: int):
        t = np.arange(nsample, dtype=np.float64) + self.current
        x = (self.amplitude * np.exp(1j * (2 * np.pi * self.frequency * t))).astype(np.complex64)
        self.current += nsample
        return self, x[None, None, :]


class Impulse:
    """Impulse.m:14-38: single-precision noise of rms ``noise`` per component, the delta
    of ``amplitude`` at absolute sample ``offset`` when it falls in this block, else
    sample 1 of the block set to 0 (as the Matlab else-branch does)."""

    def __init__(self, offset=0, amplitude=1.0, noise=1e-6, seed=0):
        self.offset = offset
        self.amplitude = amplitude
        self.noise = noise
        self.current = 0
        self._rng = np.random.default_rng(seed)

    def generate(self, nsample: int):
        x = np.zeros(nsample, dtype=np.complex64)
        if self.noise != 0:
            x = (self.noise * (self._rng.standard_normal(nsample, dtype=np.float32)
                               + 1j * self._rng.standard_normal(nsample, dtype=np.float32))
                 ).astype(np.complex64)
        off = self.offset - self.current
        if 0 <= off < nsample:
            x[off] = self.amplitude
        elif nsample:
            x[0] = 0.0
        self.current += nsample
        return self, x[None, None, :]


class FrequencyComb:
    """FrequencyComb.m:1-40: one PureTone per harmonic (amplitude, frequency), each
    carrying its own phase across calls; the block is the single-precision sum of the
    tones' single-precision blocks, accumulated in harmonic order as the Matlab loop
    does (``x = x + tmp``)."""

    def __init__(self, amplitudes, frequencies):
        self.tone = [PureTone(frequency=float(f), amplitude=float(a))
                     for a, f in zip(np.ravel(amplitudes), np.ravel(frequencies))]
        self.ntone = len(self.tone)

    def generate(self, nsample: int):
        x = np.zeros(nsample, dtype=np.complex64)
        for tone in self.tone:
            _, tmp = tone.generate(nsample)
            x = x + tmp[0, 0]
        return self, x[None, None, :]


def comb_harmonics(n_chan=1, two_stage=False, invert=False, comb="", nharmonic=32):
    """sgcht.m:394-431: (amplitudes, frequencies) of the frequency-comb test signal —
    linspace(1, sqrt 2) amplitudes; frequencies from -0.5 + 1/(4 nharmonic) in steps of
    1/nharmonic, scaled into one coarse or fine channel for ``comb`` 'coarse' / 'fine',
    otherwise moved a quarter channel of the output channels (n_chan, n_chan^2 two-stage,
    one stage fewer when inverting) off the DC bins."""
    amplitudes = np.linspace(1.0, math.sqrt(2.0), nharmonic)
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
    return amplitudes, np.linspace(fmin, fmax, nharmonic)


class SquareWave:
    """SquareWave.m:1-64: complex Gaussian noise of variance on_amp for the first
    floor(period duty_cycle) samples of every period, off_amp for the rest (zeros when the
    amplitude is 0); single precision, the phase carried across calls."""

    def __init__(self, period=26, duty_cycle=0.5, on_amp=1.0, off_amp=0.0, seed=0):
        self.period = int(period)
        self.duty_cycle = duty_cycle
        self.on_amp = on_amp
        self.off_amp = off_amp
        self.current = 0
        self._rng = np.random.default_rng(seed)

    def generate(self, nsample: int):
        ioff = int(math.floor(self.period * self.duty_cycle))
        x = np.zeros(nsample, dtype=np.complex64)
        nout = 0
        while nout < nsample:  # SquareWave.m:29-56
            iphase = self.current % self.period
            if iphase < ioff:
                n, a = ioff - iphase, math.sqrt(self.on_amp * 0.5)
            else:
                n, a = self.period - iphase, math.sqrt(self.off_amp * 0.5)
            n = min(n, nsample - nout)
            if a > 0:
                x[nout:nout + n] = (np.float32(a) * (self._rng.standard_normal(n, dtype=np.float32)
                                                     + 1j * self._rng.standard_normal(n, dtype=np.float32))
                                    ).astype(np.complex64)
            nout += n
            self.current += n
        return self, x[None, None, :]


class FrequencyWedge:
    """FrequencyWedge.m:1-66: blocks of ``resolution`` samples of complex noise whose
    spectrum has the amplitude slope sqrt(fftshift(linspace(0, 1, resolution))), i.e.
    ifft(slope .* (randn + i randn)) in single precision, streamed across calls."""

    def __init__(self, resolution=1024 * 1024, seed=0):
        self.resolution = int(resolution)
        self.slope = np.sqrt(np.fft.fftshift(np.linspace(0.0, 1.0, self.resolution))).astype(np.float32)
        self.current = 0
        self.buffer = None
        self._rng = np.random.default_rng(seed)

    def generate(self, nsample: int):
        x = np.zeros(nsample, dtype=np.complex64)
        nout = 0
        while nout < nsample:
            if self.current == 0:
                spec = (self._rng.standard_normal(self.resolution, dtype=np.float32)
                        + 1j * self._rng.standard_normal(self.resolution, dtype=np.float32))
                self.buffer = np.fft.ifft((self.slope * spec).astype(np.complex64)).astype(np.complex64)
            n = min(self.resolution - self.current, nsample - nout)
            x[nout:nout + n] = self.buffer[self.current:self.current + n]
            nout += n
            self.current += n
            if self.current == self.resolution:
                self.current = 0
        return self, x[None, None, :]


# ------------------------------------------------------------------ testers
def _host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


class TestPureTone:
    """TestPureTone.m:13-90 — per polarisation and channel: nfft = block length (at most
    8 Mi), the FFT peak must sit at bin frequency * nfft + 1 (1-based; the band-swapped
    bin nfft/2 + that is accepted), and every other bin <= dB_max relative to the peak."""

    __test__ = False  # not a pytest class

    def __init__(self, frequency=1 / 26.5, dB_max=-60.0):
        self.frequency = frequency
        self.dB_max = dB_max
        self.last = None  # diagnostics of the last block

    def test(self, x):
        x = _host(x)
        npol, nchan = x.shape[0], x.shape[1]
        max_nfft = 8 * 1024 * 1024
        worst = -np.inf
        for ipol in range(npol):
            for ichan in range(nchan):
                v = x[ipol, ichan, :].astype(np.complex128)
                nfft = min(v.shape[0], max_nfft)
                if nfft == 0:  # an empty block: Matlab's max([]) is empty and nothing fails
                    continue
                v = v[:nfft]
                exp_index = self.frequency * nfft + 1
                with np.errstate(divide="ignore"):
                    fft_dB = 20 * np.log10(np.abs(np.fft.fft(v) / nfft))
                a_index = int(np.argmax(fft_dB)) + 1
                fft_dB = fft_dB - fft_dB[a_index - 1]
                if a_index != exp_index and a_index != nfft / 2 + exp_index:
                    self.last = {"fail": "peak", "a_index": a_index, "exp_index": exp_index,
                                 "nfft": nfft}
                    return self, -1
                others = np.delete(fft_dB, a_index - 1)
                w = float(others.max()) if others.size else -np.inf
                worst = max(worst, w)
                if w > self.dB_max:
                    self.last = {"fail": "spurious", "dB": w, "nfft": nfft}
                    return self, -1
        self.last = {"max_spurious_dB": worst}
        return self, 0


class TestImpulse:
    """TestImpulse.m:13-66 — with off = offset - current + 1 (1-based in this block),
    every sample i outside [off - 1, off + 1] must be <= dB_max (20 log10 |x|, absolute);
    ``current`` advances by the block length."""

    __test__ = False

    def __init__(self, offset=0, dB_max=-60.0):
        self.offset = offset
        self.current = 0
        self.dB_max = dB_max
        self.last = None

    def test(self, x):
        x = _host(x)
        nsample = x.shape[2]
        off = self.offset - self.current + 1
        worst = -np.inf
        i = np.arange(1, nsample + 1)
        outside = (i < off - 1) | (i > off + 1)
        for ipol in range(x.shape[0]):
            for ichan in range(x.shape[1]):
                with np.errstate(divide="ignore"):
                    amp_dB = 20 * np.log10(np.abs(x[ipol, ichan, :].astype(np.complex128)))
                if outside.any():
                    w = float(amp_dB[outside].max())
                    worst = max(worst, w)
                    if w > self.dB_max:
                        # TestImpulse.m:67-70 returns without advancing obj.current
                        self.last = {"fail": "outside", "dB": w, "off": off}
                        return self, -1
        self.current += nsample
        self.last = {"max_outside_dB": worst, "off": off}
        return self, 0


class TestFrequencyComb:
    """TestFrequencyComb.m:15-118 — per polarisation and channel: nfft = block length (at
    most 8 Ki), |FFT(x)| / (nfft nchan); every harmonic that falls in this channel
    (jchan = floor(f nchan) mod nchan) must reach >= 0.5 at bin
    floor((f - ichan/nchan) hfac) mod nfft, where hfac = nchan nfft normalised by the
    oversampling factor once per analysis level left in the data (level = 2 two-stage, 1
    one stage with nchan > 1, minus one each for invert and critical).

    Each harmonic is checked in the one channel it falls in (the Matlab double loop over
    channels and harmonics visits exactly those pairs), so the verdict is the same."""

    __test__ = False

    def __init__(self, frequencies=(), os_factor="1/1", two_stage=False, invert=False,
                 critical=False):
        self.frequencies = np.ravel(np.asarray(frequencies, dtype=np.float64))
        self.os_factor = as_rational(os_factor)
        self.two_stage = two_stage
        self.invert = invert
        self.critical = critical
        self.last = None

    def test(self, x):
        x = _host(x)
        npol, nchan, n = x.shape
        nfft = min(n, 8 * 1024)
        if nfft == 0:
            self.last = {"min_level": None}
            return self, 0
        level = 2 if self.two_stage else (1 if nchan > 1 else 0)
        level -= int(bool(self.invert)) + int(bool(self.critical))
        hfac = nchan * nfft
        for _ in range(max(level, 0)):
            hfac = (self.os_factor.de * hfac) / self.os_factor.nu  # normalize.m
        f = self.frequencies
        jchan = np.mod(np.floor(f * nchan).astype(np.int64) + nchan, nchan)
        iharm = np.mod(np.floor((f - jchan / nchan) * hfac).astype(np.int64) + nfft, nfft)
        worst = np.inf
        for ipol in range(npol):
            spec = np.abs(np.fft.fft(x[ipol, jchan, :nfft].astype(np.complex128), axis=-1)
                          / (nfft * nchan))
            lv = spec[np.arange(f.size), iharm]
            worst = min(worst, float(lv.min()))
            bad = np.nonzero(lv < 0.5)[0]
            if bad.size:
                i = int(bad[0])
                self.last = {"fail": "harmonic", "harmonic": i, "frequency": float(f[i]),
                             "chan": int(jchan[i]), "bin": int(iharm[i]), "level": float(lv[i]),
                             "nfft": nfft}
                return self, -1
        self.last = {"min_level": worst, "nfft": nfft}
        return self, 0


# ------------------------------------------------------------------ set-up
def header_template(signal: str) -> dict:
    """config/<signal>_header.json (sgcht.m:286-288)."""
    with open(os.path.join(config_dir, f"{signal}_header.json")) as f:
        return json.load(f)


def sgcht_config(cfg: str):
    """default_config(cfg) with the FIR taps attached (``filt_coeff``): the tap file when it
    exists, else the configuration's ``fir_design`` (the reference's .npy tap files are not
    part of its repository)."""
    c = default_config(cfg)
    if os.path.exists(c.fir_filter_path):
        c.filt_coeff = read_fir_filter_coeff(c.fir_filter_path)
    else:
        d = getattr(c, "fir_design", {"kind": "single_stage", "taps_per_chan": 12})
        if d["kind"] == "file":  # a stand-in tap file of the package's config directory
            c.filt_coeff = read_fir_filter_coeff(os.path.join(config_dir, d["path"]))
        elif d["kind"] == "two_stage":
            c.filt_coeff = design_PFB_FIR_filter_two_stage(c.channels, c.os_factor, d["taps_per_chan"])
        else:
            c.filt_coeff = design_PFB_FIR_filter(c.channels, c.os_factor, d["taps_per_chan"])
    if not hasattr(c, "kept_channels"):
        c.kept_channels = 0
    return c


def num2str(x) -> str:
    """Matlab num2str of a scalar: integers as %d, otherwise %.{max(ceil(log10|x|), 1) + 4}g."""
    xf = float(x)
    if xf == int(xf) and abs(xf) < 1e15:
        return str(int(xf))
    digits = max(math.ceil(math.log10(abs(xf))), 1) + 4
    return f"{xf:.{digits}g}"


def sgcht_filename(signal, cfg="", cfg2="", comb="", two_stage=False, critical=False, invert=False,
                   f_taper="", combine=1, single=False, nbit=32, rndInput=False, rmsInput=0.0,
                   rndOutput=False, rmsOutput=0.0, directory="products"):
    """sgcht.m:101-163: the output file name, built from the options in the same order."""
    name = str(signal)
    if comb in ("coarse", "fine"):
        name += "_" + comb
    if cfg:
        name += "_" + cfg
    if cfg2:
        name += "_" + cfg2
    if two_stage:
        name += "_two_stage"
    if critical:
        name += "_critical"
    if invert:
        name += "_inverted"
    if f_taper:
        name += "_" + f_taper
    if combine > 1:
        name += "_" + str(int(combine))
    if single:
        name += "_single"
    if nbit != 32:
        name += "_" + str(int(nbit)) + "bit"
    rndIn = rndInput or rmsInput > 0.0
    if rndIn:
        name += "_rndIn"
    if rmsInput > 0.0:
        name += "_rmsIn=" + num2str(rmsInput)
    rndOut = rndOutput or rmsOutput > 0.0
    if rndOut:
        name += "_rndOut"
    if rmsOutput > 0.0:
        name += "_rmsOut=" + num2str(rmsOutput)
    return os.path.join(directory, name + ".dada")


def sgcht(signal="square_wave", cfg="", two_stage=False, invert=False, critical=False,
          combine=1, test=False, blocks=None, blocksz=None, device=0, collect=False,
          noise=1e-6, seed=0, comb="", single=False, f_taper="", nbit=32, scale=1.0,
          output_nchan=0, periods=0, rndInput=False, rmsInput=0.0, rndOutput=False,
          rmsOutput=0.0, output_dir=None):
    """sgcht.m: signal generator -> channeliser -> (inverse) -> tester or DADA file.

    Returns a namespace with ``result`` (0 pass, -1 fail, as sgcht returns), ``blocks``
    (blocks processed), ``tester`` (its ``last`` diagnostics), ``config``, ``header`` (the
    output DADA header, sgcht.m:314-356), ``filename`` and, with ``collect``, ``outputs``
    (the blocks after the channeliser / inverse, device tensors) and ``inputs`` (the
    generated host blocks).

    test=True (sgcht.m:442-459): complex_sinusoid (TestPureTone), temporal_impulse
    (TestImpulse) and frequency_comb (TestFrequencyComb; ``comb`` '', 'coarse' or 'fine',
    sgcht.m:394-432).  sgcht.m:439 assigns ``tester.os_factor = os_factor``, a name sgcht
    never defines (Matlab would stop there for any comb test with a cfg); the
    configuration's os_factor — the evident intent — is used.

    test=False (sgcht.m:540-575): each block is scaled by ``scale``, cast to ``nbit``
    (32: complex single; 16 / 8: Matlab's round-half-away, saturating cast, through
    pfb_dada_pack), cut to ``output_nchan`` channels and appended to the DADA file
    ``sgcht_filename(...)`` in ``output_dir`` — written only when ``output_dir`` is given
    (Matlab always writes ../products/<name>.dada; here a caller that only wants the blocks
    passes ``collect``).  Signals: square_wave (SquareWave.m, period from the header's
    CALFREQ, ``periods`` blocks of one period when set), frequency_wedge, frequency_comb,
    complex_sinusoid, temporal_impulse.  The header gets NBIT, TSAMP (scaled by the
    channelisation levels), PFB_DC_CHAN, NSTAGE, NCHAN_PFB_0, PFB_NCHAN, OS_FACTOR and the
    FIR (add_fir_filter_to_header.m, which resets NSTAGE to the number of filters, 1).

    Block size / count default to sgcht.m:480-500 (64 Ki samples x 2048 blocks single
    stage, 128 blocks for the comb, 64 Mi x 2 two-stage, doubled for 'mid'); tests pass
    smaller counts."""
    signals = ("square_wave", "frequency_wedge", "frequency_comb", "complex_sinusoid",
               "temporal_impulse")
    if signal not in signals:
        raise ValueError(f"Unrecognized signal: {signal}")
    if test and signal in ("square_wave", "frequency_wedge"):
        raise ValueError(f"Testing not implemented for {signal}")  # sgcht.m:376,385
    if comb and (not cfg or signal != "frequency_comb"):  # sgcht.m:106-114
        raise ValueError("Cannot specify comb spacing without analysis filterbank cfg "
                         "and a frequency_comb signal")
    from .filterbank import (FilterBank, InverseFilterBank, TwoStageFilterBank,
                             TwoStageInverseFilterBank)
    if two_stage and not cfg:
        raise ValueError("Cannot have two stages without analysis filterbank cfg")
    if critical and not two_stage:
        raise ValueError("Critically-sampled output implemented only for two-stage")
    if invert and not cfg:
        raise ValueError("Cannot invert without analysis filterbank cfg")
    if combine > 1 and not (two_stage and invert):
        raise ValueError("Cannot combine coarse channels without inverting a two-stage bank")
    if single and not two_stage:
        raise ValueError("Single-channel output implemented only for two-stage")
    header = header_template(signal)
    tsamp = float(header["TSAMP"])
    rndIn = rndInput or rmsInput > 0.0
    rndOut = rndOutput or rmsOutput > 0.0
    config = None
    filterbank = inverse = None
    n_chan = 1
    if cfg:
        config = sgcht_config(cfg)
        config.rndInput, config.rmsInput = rndIn, rmsInput
        config.rndOutput, config.rmsOutput = rndOut, rmsOutput
        n_chan = config.channels
        os1 = config.os_factor
        if two_stage:
            filterbank = TwoStageFilterBank(config, device=device)
            filterbank.critical = int(bool(critical))
            filterbank.single = int(bool(single))
            level = 2
        else:
            filterbank = FilterBank(config, device=device)
            level = 1
        pfb_nchan = n_chan
        if critical and level == 2:
            pfb_nchan = os1.normalize(n_chan)
        if invert:
            if two_stage:
                inverse = TwoStageInverseFilterBank(config, device=device)
                inverse.single = int(bool(single))
                inverse.combine = combine
                inverse.nch2 = int(pfb_nchan)
            else:
                inverse = InverseFilterBank(config, device=device)
            if f_taper:
                inverse = inverse.frequency_taper(f_taper)
            level -= 1
        if level != 0:  # sgcht.m:314-356
            def norm(v):  # normalize.m in double: (de * v) / nu
                return (os1.de * v) / os1.nu
            new_tsamp = tsamp
            if critical and level == 1:
                new_tsamp = new_tsamp * n_chan
            else:
                new_tsamp = norm(new_tsamp) * n_chan
                if level == 2:
                    new_tsamp = norm(new_tsamp) * n_chan
            new_tsamp = new_tsamp / combine
            header["NBIT"] = num2str(nbit)
            header["TSAMP"] = num2str(new_tsamp)
            header["PFB_DC_CHAN"] = "1"
            header["NSTAGE"] = num2str(level)
            header["NCHAN_PFB_0"] = num2str(n_chan)
            if getattr(config, "kept_channels", 0):
                pfb_nchan = config.kept_channels
            header["PFB_NCHAN"] = num2str(float(pfb_nchan))
            header["OS_FACTOR"] = f"{os1.nu}/{os1.de}"
            from .dada import add_fir_filter_to_header
            header = add_fir_filter_to_header(header, [config.filt_coeff], [os1])
    if blocksz is None:
        blocksz = 64 * 1024 * 1024 if two_stage else 64 * 1024
        if cfg == "mid":
            blocksz *= 2
    if blocks is None:
        blocks = 2 if two_stage else (128 if signal == "frequency_comb" else 2 * 1024)
    tester = None
    if signal == "square_wave":
        calfreq = float(header["CALFREQ"])  # Hz
        gen = SquareWave(period=round(1e6 / (calfreq * tsamp)), seed=seed)
        if periods > 0:
            blocks, blocksz = int(periods), gen.period  # sgcht.m:497-500
    elif signal == "frequency_wedge":
        gen = FrequencyWedge(seed=seed)
    elif signal == "frequency_comb":
        amps, freqs = comb_harmonics(n_chan, two_stage, invert, comb)
        gen = FrequencyComb(amps, freqs)
        tester = TestFrequencyComb(freqs)
        if config is not None:
            tester = TestFrequencyComb(freqs, config.os_factor, two_stage, invert, critical)
    elif signal == "complex_sinusoid":
        gen = PureTone(frequency=float(header["TONEFREQ"]) * tsamp / 1e6)  # sgcht.m:423-426
        tester = TestPureTone(frequency=gen.frequency)
    else:
        gen = Impulse(offset=20000, noise=noise, seed=seed)  # sgcht.m:436-438
        fir_offset = 0
        filter_offset = 0
        if config is not None:
            output_overlap = config.os_factor.normalize(config.input_overlap) * config.channels
            taps = len(config.filt_coeff)
            fir_offset = config.fir_offset_direction * (taps // 2)
            filter_offset = output_overlap - 1 + config.kludge_offset
        tester = TestImpulse(offset=int(gen.offset + fir_offset - filter_offset))
    filename = sgcht_filename(signal, cfg, "", comb, two_stage, critical, invert, f_taper, combine,
                              single, nbit, rndInput, rmsInput, rndOutput, rmsOutput,
                              directory=output_dir or "products")
    res = SimpleNamespace(result=0, blocks=0, tester=tester, config=config, n_chan=n_chan,
                          header=header, filename=filename if (output_dir and not test) else None,
                          outputs=[] if collect else None, inputs=[] if collect else None)
    writer = None
    if output_dir and not test:
        from .dada import DADAWrite
        os.makedirs(output_dir, exist_ok=True)
        writer = DADAWrite(filename, header, nbit=nbit).open(filename)
    torch = None
    if filterbank is not None or writer is not None:
        import torch
    try:
        for _ in range(int(blocks)):  # sgcht.m:504-575
            gen, x = gen.generate(int(blocksz))
            if x.shape[-1] == 0:
                break
            if collect:
                res.inputs.append(x)
            if torch is not None:  # one copy of the block to the device; it stays there
                x = torch.from_numpy(x).to(torch.device("cuda", int(device)))
            if filterbank is not None:
                filterbank, x = filterbank.execute(x)
            if inverse is not None:
                inverse, x = inverse.execute(x)
            if collect:
                res.outputs.append(x)
            res.blocks += 1
            if test:
                tester, r = tester.test(x)
                if r != 0:
                    res.result = -1
                    return res
            elif writer is not None:
                if scale != 1:
                    x = scale * x
                if output_nchan > 0:
                    x = x[:, :output_nchan, :]
                writer.write(x)
    finally:
        if writer is not None:
            writer.close()
    return res
