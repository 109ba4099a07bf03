"""MI355X-native oversampled polyphase filter bank (analysis -> synthesis round trip).

Drop-in for the hot path of ska-telescope/ska-pst-dsp-model: the Matlab-shaped
functions ``polyphase_analysis``, ``polyphase_analysis_padded``,
``polyphase_synthesis`` and the stream objects ``FilterBank``, ``InverseFilterBank``,
``TwoStageFilterBank``, ``TwoStageInverseFilterBank``, ``PFBWindow``,
``Channelizer``, ``DeChannelizer``.  All compute runs in the hand-written HIP/CDNA4
kernels of ``lib/libpfb_hip.so`` (C ABI: ``include/pfb_api.h``).
"""
from ._lib import PfbError, device_count
from .config import Rational, default_config, load_config
from .core import (AnalysisPlan, SynthesisPlan, polyphase_analysis, polyphase_analysis_padded,
                   polyphase_analysis_lowcbf,
                   polyphase_synthesis, roundtrip, roundtrip_analysis, roundtrip_synthesis,
                   calc_output_nbins)
from .filterbank import (Channelizer, DeChannelizer, FilterBank, InverseFilterBank,
                         TwoStageFilterBank, TwoStageInverseFilterBank)
from .firio import (design_PFB_FIR_filter, design_PFB_FIR_filter_two_stage,
                    read_fir_filter_coeff)
from .window import PFBWindow, identity_taper
from .streaming import (FrequencyComb, Impulse, PureTone, TestFrequencyComb, TestImpulse,
                        TestPureTone, sgcht)
from . import dada, harness, layout, sharding, verify

__all__ = [
    "PfbError", "device_count", "Rational", "default_config", "load_config", "AnalysisPlan",
    "SynthesisPlan", "polyphase_analysis", "polyphase_analysis_padded", "polyphase_analysis_lowcbf", "polyphase_synthesis",
    "Channelizer", "DeChannelizer", "FilterBank", "InverseFilterBank", "TwoStageFilterBank",
    "TwoStageInverseFilterBank", "design_PFB_FIR_filter", "design_PFB_FIR_filter_two_stage",
    "read_fir_filter_coeff", "PFBWindow", "identity_taper", "roundtrip", "roundtrip_analysis",
    "roundtrip_synthesis", "calc_output_nbins",
    "sgcht", "PureTone", "Impulse", "FrequencyComb", "TestPureTone", "TestImpulse",
    "TestFrequencyComb",
]
