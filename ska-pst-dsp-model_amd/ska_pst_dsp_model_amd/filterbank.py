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

from . import _lib, layout
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


def _to_device(x, device):
    """(array, was_host): host arrays go to the plan's device (torch as allocator)."""
    if is_device_array(x):
        return x, False
    import torch
    arr = np.ascontiguousarray(np.asarray(x), dtype=np.complex64)
    return torch.from_numpy(arr).to(torch.device("cuda", int(device))), True


def _to_host(x):
    return x.cpu().numpy()


def _quantize(x, rms, device=0):
    """round(rms / std(x) * x) (FilterBank.m:75-83,106-113) through pfb_quantize."""
    xd, host = _to_device(x, device)
    y = layout.quantize(xd, rms)
    return _to_host(y) if host else y


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
            x = _quantize(x, self.rmsInput, self.device)
        plan = self._ensure_plan(_npol(x))
        out = plan.execute(x, stateful=True)  # (n_pol, T_out, n_chan)
        if self.rndOutput:
            out = _quantize(out, self.rmsOutput, self.device)
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
        if int(self.sample_offset) < 0:
            raise ValueError("sample_offset is 0-based (>= 0)")
        plan = self._ensure_plan(shape[0], shape[1])
        # polyphase_synthesis(..., obj.sample_offset+1, ...) on every call (:92-96)
        plan.set_stream_sample_offset(int(self.sample_offset))
        out = plan.execute(input, stateful=True)
        return self, out[:, None, :]

    def reset(self):
        if self._plan is not None:
            self._plan.reset()


class TwoStageFilterBank(Channelizer):
    """TwoStageFilterBank.m:1-118 — stage 2 cascaded over every stage-1 channel (pol 1).

    The Matlab object runs nch1 independent FilterBank objects in a loop (:92-110).
    Here stage 2 is ONE batched plan whose "polarisations" are the nch1 stage-1
    channels (each keeps its own carry-over, as the separate objects do).  Stage 1
    writes its product channel-major, so pol 1's channels are the stage-2 series as
    they lie, and the batched stage 2 writes the assembled output with the oversampled
    channels chomped out (:102-105) straight from its FFT
    (``pfb_filterbank_execute_strided``, streaming kernel shapes); other shapes take a
    corner turn (``pfb_corner_turn``) and a gather (``pfb_gather_channels``)."""

    def __init__(self, config, device: int = 0):
        self.stage1 = FilterBank(config, device=device)
        self.config1 = config
        self.config2 = config
        self.nch1 = int(_cfg(config, "channels"))
        self.nch2 = int(_cfg(config, "channels"))
        self.critical = 0
        self.single = 0
        self.built = False
        self.stage2 = None
        self.device = device
        # both stages through pfb_filterbank_execute_strided where the kernels allow it
        # (no corner turn, no gather); False: the corner-turn / gather path
        self.strided = True

    def set_stage2_config(self, config):
        self.config2 = config
        self.nch2 = int(_cfg(config, "channels"))
        return self

    def build(self):
        self.stage2 = FilterBank(self.config2, device=self.device)
        self.built = True
        return self

    def execute(self, input):  # noqa: A002
        x, host = _to_device(input, self.device)
        if not self.built:
            self.build()
        view = self._execute_strided(x) if self.strided else None
        if view is None:
            _, out1 = self.stage1.execute(x)      # (n_pol, nch1, T1) view
            nch1 = 1 if self.single == 1 else self.stage1.n_chan
            # per-channel series of pol 1: (T1, nch1) rows -> (nch1, T1)
            rows = out1[0].transpose(0, 1)[:, :nch1]  # (T1, nch1) view of the engine buffer
            view = self._stage2(layout.corner_turn(rows), nch1)
        return self, (_to_host(view) if host else view)

    def _chomp(self):
        """(nch2 kept per stage-2 bank, dropped-bin count) of :81-85,102-105."""
        os_ = self.stage1.os_factor
        nch2_orig = self.stage2.n_chan
        nch2 = (nch2_orig * os_.de) // os_.nu if self.critical else nch2_orig
        return nch2, nch2_orig - nch2

    def _stage2(self, series, nch1):
        """Stage 2 over the (nch1, T1) series, then one gather assembles the output."""
        nch2, offset = self._chomp()
        _, tmp = self.stage2.execute(series)      # (nch1, nch2_orig, T2) view
        buf2 = tmp.transpose(1, 2)                # (nch1, T2, nch2_orig) engine buffer
        T2 = int(buf2.shape[1])
        import torch
        out = torch.empty((1, T2, nch1 * nch2), dtype=torch.complex64, device=buf2.device)
        # out[t][ich*nch2 + j] = tmp[ich][t][j (+ offset from j = nch2/2 - 1 on)]
        layout.gather_channels(buf2, n_outer=nch1, in_outer_stride=buf2.stride(0),
                               in_row_stride=buf2.stride(1), n_rows=T2, n_sel=nch2,
                               split=nch2 // 2 - 1, shift=offset, out=out,
                               out_outer_stride=nch2, out_row_stride=nch1 * nch2)
        return out.transpose(1, 2)                # (1, nch1*nch2, T2)

    def _execute_strided(self, x):
        """Both stages through pfb_filterbank_execute_strided: stage 1 writes its product
        channel-major, so pol 1's channels are already the stage-2 series (no corner
        turn), and stage 2 writes the assembled, chomped output (no gather).  Same
        kernels and arithmetic as the corner-turn / gather path (bit-identical).  None
        when stage 1 cannot take this path (its plan state is then untouched); a stage 2
        that cannot takes the gather path."""
        from ._lib import PFB_ERR_UNSUPPORTED, PfbError
        s1, s2 = self.stage1, self.stage2
        if s1.rndInput or s1.rndOutput or s2.rndInput or s2.rndOutput:
            return None
        import torch
        p1 = s1._ensure_plan(_npol(x))
        xs, _ = p1._prep_in(x)
        T1 = p1.stream_rows(int(xs.shape[1]))
        nch1_all = p1.out_chan
        T1c = max(16, (T1 + 15) // 16 * 16)  # 128-B aligned channel runs
        ser = torch.empty((p1.n_pol, nch1_all, T1c), dtype=torch.complex64, device=xs.device)
        try:
            T1 = p1.execute_strided(xs, ser, nch1_all * T1c, 1, T1c)
        except PfbError as e:
            if e.status == PFB_ERR_UNSUPPORTED:
                return None
            raise
        nch1 = 1 if self.single == 1 else nch1_all
        series = ser[0, :nch1, :T1]               # (nch1, T1), unit sample stride
        nch2, offset = self._chomp()
        p2 = s2._ensure_plan(nch1)
        T2 = p2.stream_rows(T1)
        out = torch.empty((1, max(T2, 1), nch1 * nch2), dtype=torch.complex64, device=xs.device)
        try:
            T2 = p2.execute_strided(series, out, nch2, nch1 * nch2, 1,
                                    (nch2 // 2 - 1, offset, nch2))
        except PfbError as e:
            if e.status == PFB_ERR_UNSUPPORTED:
                return self._stage2(series, nch1)
            raise
        return out[:, :T2, :].transpose(1, 2)     # (1, nch1*nch2, T2)


class TwoStageInverseFilterBank(DeChannelizer):
    """TwoStageInverseFilterBank.m:1-159 — stage-2 inversion per output coarse channel.

    The nch_out InverseFilterBank objects of the Matlab loop (:124-151) become ONE
    batched synthesis plan over nch_out "polarisations": one gather
    (``pfb_gather_channels``) slices the nch_in = nch2 * combine fine channels of every
    coarse channel, one synthesis call inverts them all."""

    def __init__(self, config, device: int = 0):
        self.config1 = config
        self.config2 = config
        self.stage1 = InverseFilterBank(config, device=device)
        self.nch1 = int(_cfg(config, "channels"))
        self.nch2 = int(_cfg(config, "channels"))
        self.single = 0
        self.combine = 1
        self.built = False
        self.stage2 = None
        self._ftaper = None
        self.device = device

    def set_stage2_config(self, config):
        self.config2 = config
        self.nch2 = int(_cfg(config, "channels"))
        return self

    def build(self):
        self.stage2 = InverseFilterBank(self.config2, device=self.device)
        if self._ftaper is not None:
            self.stage2.frequency_taper(self._ftaper)
        self.built = True
        return self

    def frequency_taper(self, name):
        self._ftaper = name
        if not self.built:
            self.build()
        self.stage2.frequency_taper(name)
        return self

    def execute(self, input):  # noqa: A002
        if not self.built:
            self.build()
        x, host = _to_device(input, self.device)
        if not x.is_complex():
            raise ValueError("input data are real !")
        os_ = self.stage1.os_factor
        npol, nchan, T = (int(v) for v in x.shape)
        nch_out = nchan // self.nch2
        stage2_nchan = self.stage2.nchan
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
        buf = x.transpose(1, 2)                   # (npol, T, nchan) engine order
        if buf.stride(2) != 1:
            buf = buf.contiguous()
        sliced = layout.gather_channels(buf[0], n_outer=nch_out, in_outer_stride=nch_in,
                                        in_row_stride=buf.stride(1), n_rows=T, n_sel=nch_in)
        st = self.stage2
        st.critical = critical
        st.combine = self.combine
        _, tmp = st.execute(sliced.transpose(1, 2))  # (nch_out, 1, T_out)
        out = tmp.reshape(1, nch_out, tmp.shape[2])
        return self, (_to_host(out) if host else out)
