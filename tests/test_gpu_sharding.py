"""GPU check of the sharded path on the product itself.

tests/test_sharding.py proves the index arithmetic of ``ska_pst_dsp_model_amd.sharding``
with the CPU oracle standing in for the device.  Here every rank's slice runs through the
HIP library on one GPU (the ranks simulated one after another) and the concatenation of
the slices' outputs must equal the single-run HIP output BIT FOR BIT:

* Bunton analysis at the C2 shape (256 ch, 8/7, 3073 taps, 2^24 samples): row cuts at
  multiples of nu, each slice with its P N-sample halo (polyphase_analysis.m:83-121,
  FilterBank.m:93-104);
* padded analysis at the C3 shape (4096 ch, 8/7, 100 353 taps) at 2^22 samples: each
  slice starts >= ceil(P N / M) rows of history early, and the ranks holding the circular
  shift's tail (out[t] = FIR[(t + sds) mod K], polyphase_analysis_padded.m:156) compute
  those sds rows from a second slice at the start of the series;
* synthesis of the C2 channelised product (Nf 256, Ov 48) in block-aligned slices with a
  2 Ov-row overlap (polyphase_synthesis.m:112-131), and of the C3 product (Nf 512, Ov 128).
"""
import numpy as np
import pytest

from ska_pst_dsp_model_amd import sharding

pytestmark = pytest.mark.gpu


def _pfb():
    import ska_pst_dsp_model_amd as pfb
    return pfb


def _noise_t(torch, dev, n, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    re = torch.randn((1, n), device=dev, generator=g)
    im = torch.randn((1, n), device=dev, generator=g)
    return (torch.complex(re, im) / np.sqrt(2.0)).to(torch.complex64).contiguous()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bunton_analysis_and_synthesis_shards_bit_identical(gpu, world):
    import torch
    pfb = _pfb()
    n = 1 << 24
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    x = _noise_t(torch, gpu, n, 71)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, gpu.index or 0)
    full = ana.execute(x)                       # (1, K, 256) time-major
    parts = []
    for r in range(world):
        sh = sharding.analysis_shard(n, 256, "8/7", len(taps), world, r)
        y = ana.execute(x[:, sh.in_start:sh.in_stop].contiguous())
        assert y.shape[1] == sh.n_out
        parts.append(y)
    cat = torch.cat(parts, dim=1)
    torch.cuda.synchronize()
    assert torch.equal(cat, full), "sharded Bunton analysis differs from the single run"

    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, gpu.index or 0)
    y_full = syn.execute(full, layout="ptc")
    K = full.shape[1]
    outs = []
    for r in range(world):
        sh = sharding.synthesis_shard(K, 256, "8/7", 256, 48, world, r)
        o = syn.execute(full[:, sh.in_start:sh.in_stop].contiguous(), layout="ptc")
        assert o.shape[1] == sh.n_out
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs, dim=1), y_full), "sharded synthesis differs from the single run"


@pytest.mark.parametrize("world", [2, 3, 8])
def test_padded_analysis_shards_with_wrap_tail_bit_identical(gpu, world):
    """C3 parameters at 2^22 samples (1170 rows, sds 14): the last rank's tail rows wrap
    to FIR rows [0, sds) and come from a second, sds-row slice."""
    import torch
    pfb = _pfb()
    n = 1 << 22
    taps = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    x = _noise_t(torch, gpu, n, 73)
    ana = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 1, gpu.index or 0)
    full = ana.execute(x)
    K = full.shape[1]
    parts, wrapped = [], 0
    for r in range(world):
        sh = sharding.analysis_padded_shard(n, 4096, "8/7", len(taps), world, r)
        if sh.out_stop > sh.out_start:
            y = ana.execute(x[:, sh.in_start:sh.in_stop].contiguous())
            parts.append(y[:, sh.keep_start:sh.keep_start + sh.out_stop - sh.out_start])
        if sh.n_wrap:
            y = ana.execute(x[:, :sh.wrap_stop].contiguous())
            parts.append(y[:, sh.wrap_keep:sh.wrap_keep + sh.n_wrap])
            wrapped += sh.n_wrap
    cat = torch.cat(parts, dim=1)
    torch.cuda.synchronize()
    assert wrapped == 14, wrapped  # sds = ceil((100353 - 1) / 2 / 3584)
    assert cat.shape == full.shape
    assert torch.equal(cat, full), "sharded padded analysis differs from the single run"

    # the SKA-Mid synthesis of that product in block-aligned slices (Nf 512, Ov 128)
    win = pfb.PFBWindow().lookup["tukey"](512, 128)
    syn = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, taps, win, None, 1, gpu.index or 0)
    y_full = syn.execute(full, layout="ptc")
    outs = []
    for r in range(min(world, 3)):  # 4 blocks at this length
        sh = sharding.synthesis_shard(K, 4096, "8/7", 512, 128, min(world, 3), r)
        outs.append(syn.execute(full[:, sh.in_start:sh.in_stop].contiguous(), layout="ptc"))
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(outs, dim=1), y_full), "sharded SKA-Mid synthesis differs"
