"""Stream-object surface: Channelizer / DeChannelizer / FilterBank / InverseFilterBank
and the two-stage cascades (matlab/Channelizer.m, DeChannelizer.m, FilterBank.m,
InverseFilterBank.m, TwoStageFilterBank.m, TwoStageInverseFilterBank.m).

``execute`` keeps the Matlab calling convention ``[obj, out] = execute(obj, in)``:
it returns ``(self, out)``.  The carry-over state (``FilterBank.m:13-14``) lives in
the device plan (``pfb_filterbank_execute`` / ``pfb_inverse_filterbank_execute``).
"""
from __future__ import annotations

import abc
from types import SimpleNamespace

import numpy as np

from . import _lib
from .config import as_rational
from .core import AnalysisPlan, SynthesisPlan, is_device_array
from .firio import read_fir_filter_coeff
from .window import PFBWindow, identity_taper

__all__ = ["Channelizer", "DeChannelizer", "FilterBank", "InverseFilterBank",
           "TwoStageFilterBank", "TwoStageInverseFilterBank"]


def _cfg(config, name, default=None):
    if isinstance(config, dict):
        return config.get(name, default)
    return getattr(config, name, default)


def _taps_from_config(config):
    taps = _cfg(config, "filt_coeff")
    if taps is None:
        taps = read_fir_filter_coeff(_cfg(config, "fir_filter_path"))
    return np.asarray(taps, dtype=np.float64).ravel()


class Channelizer(abc.ABC):
    """Channelizer.m:1-12 — abstract ``[obj, output] = execute(obj, input)``."""

    @abc.abstractmethod
    def execute(self, input):  # noqa: A002
        ...


class DeChannelizer(abc.ABC):
    """DeChannelizer.m:1-12 — abstract ``[obj, output] = execute(obj, input)``."""

    @abc.abstractmethod
    def execute(self, input):  # noqa: A002
        ...


def _npol(x):
    return 1 if len(tuple(x.shape)) == 1 else int(tuple(x.shape)[0])


def _quantize(x, rms):
    """round(scale * x) with scale = rms / std(x) (FilterBank.m:75-83,106-113)."""
    if is_device_array(x):
        import torch
        scale = 1.0
        if rms > 0:
            scale = rms / torch.sqrt(torch.var(x.reshape(-1).to(torch.complex128))).item()
        y = x * scale
        return torch.complex(torch.round(y.real), torch.round(y.imag)).to(torch.complex64)
    x = np.asarray(x)
    scale = 1.0
    if rms > 0:
        scale = rms / np.sqrt(np.var(x, ddof=1))
    return np.round(scale * x).astype(np.complex64)


class FilterBank(Channelizer):
    """FilterBank.m:1-130 — analysis PFB with input buffering and nu-trimming."""

    def __init__(self, config=None, n_pol: int = None, device: int = 0):
        self.pfb_analysis = "polyphase_analysis"
        self.os_factor = None
        self.filt_coeff = None
        self.n_chan = None
        self.rndInput = False
        self.rmsInput = 0.0
        self.rndOutput = False
        self.rmsOutput = 0.0
        self.device = device
        self._plan = None
        self._n_pol = n_pol
        if config is not None:
            self.pfb_analysis = _cfg(config, "analysis_function", "polyphase_analysis")
            self.filt_coeff = _taps_from_config(config)
            self.n_chan = int(_cfg(config, "channels", _cfg(config, "n_chan")))
            self.os_factor = as_rational(_cfg(config, "os_factor"))
            self.rndInput = bool(_cfg(config, "rndInput", False))
            self.rmsInput = float(_cfg(config, "rmsInput", 0.0))
            self.rndOutput = bool(_cfg(config, "rndOutput", False))
            self.rmsOutput = float(_cfg(config, "rmsOutput", 0.0))

    def _ensure_plan(self, n_pol):
        if self._plan is None or self._plan.n_pol != n_pol:
            if self._plan is not None and self._plan.buffered_samples:
                raise ValueError("n_pol changed while samples are buffered")
            self._plan = AnalysisPlan(self.filt_coeff, self.n_chan, self.os_factor,
                                      self.pfb_analysis, n_pol, self.device)
        return self._plan

    @property
    def buffered_samples(self) -> int:
        return 0 if self._plan is None else self._plan.buffered_samples

    def execute(self, input):  # noqa: A002
        x = input
        if self.rndInput:
            x = _quantize(x, self.rmsInput)
        plan = self._ensure_plan(_npol(x))
        out = plan.execute(x, stateful=True)  # (n_pol, T_out, n_chan)
        if self.rndOutput:
            out = _quantize(out, self.rmsOutput)
        view = out.transpose(1, 2) if is_device_array(out) else out.transpose(0, 2, 1)
        return self, view

    def reset(self):
        if self._plan is not None:
            self._plan.reset()


class InverseFilterBank(DeChannelizer):
    """InverseFilterBank.m:1-139 — synthesis with input buffering.

    The Matlab object forces ``deripple = false`` before every call
    (InverseFilterBank.m:90); ``honour_deripple=True`` applies the configured value
    instead (used by the test pipeline, which calls polyphase_synthesis directly with
    deripple on, test_data_pipeline.m:132)."""

    def __init__(self, config=None, device: int = 0, honour_deripple: bool = False):
        self.os_factor = as_rational("1/1")
        self.filt_coeff = None
        self.nchan = None
        self.n_fft = None
        self.overlap = None
        self.sample_offset = 0
        self.temporal_taper = None
        self.spectral_taper = identity_taper
        self.deripple = False
        self.critical = False
        self.combine = 1
        self.window_factory = PFBWindow()
        self.device = device
        self.honour_deripple = honour_deripple
        self._plan = None
        self._plan_key = None
        if config is not None:
            self.filt_coeff = _taps_from_config(config)
            self.n_fft = int(_cfg(config, "input_fft_length"))
            self.nchan = int(_cfg(config, "channels", _cfg(config, "n_chan")))
            self.os_factor = as_rational(_cfg(config, "os_factor"))
            self.overlap = int(_cfg(config, "input_overlap"))
            self.deripple = bool(_cfg(config, "deripple", False))
            factory = self.window_factory.lookup[_cfg(config, "temporal_taper", "no_window")]
            self.temporal_taper = factory(self.n_fft, self.overlap)

    def frequency_taper(self, name):
        """InverseFilterBank.m:48-61."""
        factory = self.window_factory.lookup[name]
        self.spectral_taper = factory(self.n_fft, self.overlap)
        return self

    def _ensure_plan(self, n_pol, n_chan):
        spans = not self.critical  # :89
        dr = self.deripple if self.honour_deripple else False  # :90
        key = (n_pol, n_chan, spans, dr, self.combine, id(self.temporal_taper),
               id(self.spectral_taper))
        if self._plan is None or key != self._plan_key:
            if self._plan is not None and self._plan.buffered_samples:
                raise ValueError("configuration changed while samples are buffered")
            self._plan = SynthesisPlan(n_chan, self.os_factor, self.n_fft, self.overlap, spans,
                                       self.combine, dr, self.filt_coeff, self.temporal_taper,
                                       self.spectral_taper, n_pol, self.device)
            self._plan_key = key
        return self._plan

    @property
    def buffered_samples(self) -> int:
        return 0 if self._plan is None else self._plan.buffered_samples

    def execute(self, input):  # noqa: A002
        shape = tuple(input.shape)
        if not is_device_array(input) and not np.iscomplexobj(np.asarray(input)):
            raise ValueError("polyphase_synthesis input data are real-valued!")
        if self.sample_offset != 0:
            raise NotImplementedError("stateful synthesis with sample_offset != 0")
        plan = self._ensure_plan(shape[0], shape[1])
        out = plan.execute(input, stateful=True)
        return self, out[:, None, :]

    def reset(self):
        if self._plan is not None:
            self._plan.reset()


class TwoStageFilterBank(Channelizer):
    """TwoStageFilterBank.m:1-118 — stage 2 cascaded over every stage-1 channel (pol 1)."""

    def __init__(self, config, device: int = 0):
        self.stage1 = FilterBank(config, device=device)
        self.config1 = config
        self.config2 = config
        self.nch1 = int(_cfg(config, "channels"))
        self.nch2 = int(_cfg(config, "channels"))
        self.critical = 0
        self.single = 0
        self.built = False
        self.stage2 = []
        self.device = device

    def set_stage2_config(self, config):
        self.config2 = config
        self.nch2 = int(_cfg(config, "channels"))
        return self

    def build(self):
        self.stage2 = [FilterBank(self.config2, device=self.device)
                       for _ in range(self.stage1.n_chan)]
        self.built = True
        return self

    def execute(self, input):  # noqa: A002
        _, out1 = self.stage1.execute(input)
        if not self.built:
            self.build()
        os_ = self.stage1.os_factor
        nch1 = self.stage1.n_chan
        nch2_orig = self.stage2[0].n_chan
        nch2 = (nch2_orig * os_.de) // os_.nu if self.critical else nch2_orig
        offset = nch2_orig - nch2
        if self.single == 1:
            nch1 = 1
        out = None
        dev = is_device_array(out1)
        for ich in range(nch1):
            _, tmp = self.stage2[ich].execute(out1[0:1, ich, :])
            if out is None:
                if dev:
                    import torch
                    out = torch.zeros((1, nch1 * nch2, tmp.shape[2]), dtype=torch.complex64,
                                      device=out1.device)
                else:
                    out = np.zeros((1, nch1 * nch2, tmp.shape[2]), dtype=np.complex64)
            base = ich * nch2
            # TwoStageFilterBank.m:104-105 (index nch2/2 written twice)
            out[0, base:base + nch2 // 2, :] = tmp[0, :nch2 // 2, :]
            out[0, base + nch2 // 2 - 1:base + nch2, :] = \
                tmp[0, nch2 // 2 - 1 + offset:nch2 + offset, :]
        return self, out


class TwoStageInverseFilterBank(DeChannelizer):
    """TwoStageInverseFilterBank.m:1-159 — stage-2 inversion per output coarse channel."""

    def __init__(self, config, device: int = 0):
        self.config1 = config
        self.config2 = config
        self.stage1 = InverseFilterBank(config, device=device)
        self.nch1 = int(_cfg(config, "channels"))
        self.nch2 = int(_cfg(config, "channels"))
        self.single = 0
        self.combine = 1
        self.built = False
        self.stage2 = []
        self.device = device

    def set_stage2_config(self, config):
        self.config2 = config
        self.nch2 = int(_cfg(config, "channels"))
        return self

    def build(self):
        self.stage2 = [InverseFilterBank(self.config2, device=self.device)
                       for _ in range(self.nch1)]
        self.built = True
        return self

    def frequency_taper(self, name):
        if not self.built:
            self.build()
        for st in self.stage2:
            st.frequency_taper(name)
        return self

    def execute(self, input):  # noqa: A002
        if not self.built:
            self.build()
        os_ = self.stage1.os_factor
        npol, nchan = int(input.shape[0]), int(input.shape[1])
        nch_out = nchan // self.nch2
        stage2_nchan = self.stage2[0].nchan
        critical_stage2_nchan = (stage2_nchan * os_.de) // os_.nu
        if self.nch2 == critical_stage2_nchan:
            critical = True
        elif self.nch2 == stage2_nchan:
            critical = False
            if self.combine > 1:
                raise ValueError("TwoStageInverseFilterBank::execute cannot combine "
                                 "oversampled coarse channels")
        else:
            raise ValueError("TwoStageInverseFilterBank::execute invalid nchan")
        nch_in = self.nch2 * self.combine
        nch_out = nch_out // self.combine
        if self.single:
            nch_out = 1
        out = None
        dev = is_device_array(input)
        for ich in range(nch_out):
            st = self.stage2[ich]
            st.critical = critical
            st.combine = self.combine
            _, tmp = st.execute(input[0:1, ich * nch_in:(ich + 1) * nch_in, :])
            if out is None:
                if dev:
                    import torch
                    out = torch.zeros((1, nch_out, tmp.shape[2]), dtype=torch.complex64,
                                      device=input.device)
                else:
                    out = np.zeros((1, nch_out, tmp.shape[2]), dtype=np.complex64)
            out[0, ich, :] = tmp[0, 0, :]
        return self, out
