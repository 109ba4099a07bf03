"""GPU tests of the pipelined round trip (pfb_roundtrip_execute) and full-size parity.

* The channelised product of the round trip is bit-identical to the separate analysis
  call.  The synthesised output is bit-identical to the separate synthesis call on the
  chunked pipeline (same kernels, same inputs per block; only the launch order
  differs).  On the fused path (chunk 0 with the streaming analysis shapes) the
  synthesis stage-1 rows are N^2 v_k taken before the analysis FFT instead of the
  channel IFFT of the rounded channelised row — the same quantity in exact arithmetic —
  so there the output agrees with the separate calls to the reference's 1e-6
  (relative to the peak), for both analysis variants, several chunk sizes, sample
  offsets and polarisations.
* At the BASELINE C2 size (2^24 samples, 256 ch, OS 8/7, 3073 taps, Nf 256, Ov 48,
  tukey, deripple) the round trip is compared with the float64 oracle at the
  reference's 1e-6 criterion (test_matlab_dspsr_pfb_inversion.py:35,151-152), and a
  size-independent property (linearity of the whole round trip) is checked too.
"""
import numpy as np
import pytest

from conftest import assert_pfb_close
from oracle import pfb_oracle as orc

pytestmark = pytest.mark.gpu


def _pfb():
    import ska_pst_dsp_model_amd as pfb
    return pfb


def _noise_t(torch, dev, shape, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    re = torch.randn(shape, device=dev, generator=g)
    im = torch.randn(shape, device=dev, generator=g)
    return (torch.complex(re, im) / np.sqrt(2.0)).to(torch.complex64).contiguous()


CASES = [
    # (N, os, taps/chan, Nf, Ov, variant, n_pol, n_dat, chunk_blocks, sample_offset)
    (256, "8/7", 12, 256, 48, "polyphase_analysis", 1, 1 << 20, 0, 1),
    (256, "8/7", 12, 256, 48, "polyphase_analysis", 2, 1 << 19, 1, 1),
    (256, "8/7", 12, 256, 48, "polyphase_analysis", 1, 1 << 19, 7, 5),
    (256, "8/7", 12, 256, 48, "polyphase_analysis_padded", 1, 1 << 19, 3, 1),
    (256, "8/7", 12, 256, 48, "polyphase_analysis_padded", 2, 1 << 19, 0, 9),
    (256, "4/3", 12, 256, 48, "polyphase_analysis", 1, 1 << 19, 5, 1),
    # chunk 0 with the streaming analysis shapes = the fused path (analysis kernel
    # emits the synthesis stage-1 rows)
    (256, "4/3", 12, 256, 48, "polyphase_analysis", 2, 1 << 19, 0, 3),
    (256, "8/7", 11, 256, 48, "polyphase_analysis", 1, (1 << 19) + 777, 0, 2),
    # sample offsets a multiple of nu
    (256, "8/7", 12, 256, 48, "polyphase_analysis", 2, 1 << 19, 0, 9),
    (256, "4/3", 12, 256, 48, "polyphase_analysis", 2, 1 << 19, 0, 5),
    (256, "8/7", 11, 256, 48, "polyphase_analysis", 1, (1 << 19) + 777, 0, 1),
    # N > 256: the register-window FIR emits the stage-1 rows (fused with chunk 0)
    (512, "8/7", 12, 128, 16, "polyphase_analysis", 2, 1 << 19, 0, 1),
    (512, "8/7", 12, 128, 16, "polyphase_analysis_padded", 1, 1 << 19, 0, 4),
    (1024, "4/3", 12, 256, 48, "polyphase_analysis_padded", 2, 1 << 19, 0, 1),
    (512, "8/7", 12, 128, 16, "polyphase_analysis_padded", 1, 1 << 19, 3, 1),
    # Nf 512 (4 phases per synthesis workgroup): phase-group-major stage-1 rows
    (512, "8/7", 12, 512, 128, "polyphase_analysis_padded", 2, 1 << 19, 0, 1),
    (512, "8/7", 12, 512, 128, "polyphase_analysis", 1, 1 << 19, 0, 3),
    (8, "8/7", 10, 128, 16, "polyphase_analysis", 2, 9000, 1, 1),
    (8, "8/7", 10, 128, 16, "polyphase_analysis_padded", 1, 9000, 2, 3),
]


@pytest.mark.parametrize("case", CASES)
def test_roundtrip_matches_separate_calls(gpu, case):
    import torch
    pfb = _pfb()
    N, os_, tpc, nf, ov, variant, n_pol, n_dat, cb, so = case
    taps = pfb.design_PFB_FIR_filter(N, os_, tpc)
    x = _noise_t(torch, gpu, (n_pol, n_dat), 7)
    ana = pfb.AnalysisPlan(taps, N, os_, variant, n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)
    syn = pfb.SynthesisPlan(N, os_, nf, ov, True, 1, True, taps, win, None, n_pol, 0)
    chan_ref = ana.execute(x)
    out_ref = syn.execute(chan_ref, sample_offset=so, layout="ptc")
    if cb:
        syn.set_chunk_blocks(cb)
    chan, out = pfb.roundtrip(ana, syn, x, sample_offset=so)
    torch.cuda.synchronize()
    assert chan.shape == chan_ref.shape and out.shape == out_ref.shape
    assert out.shape[1] > 0
    assert torch.equal(chan, chan_ref), "channelised product differs"
    fused = cb == 0 and ((N == 256 and variant == "polyphase_analysis" and tpc in (11, 12))
                         or N > 256)
    if fused:
        assert_pfb_close(out.cpu().numpy(), out_ref.cpu().numpy(), scale=1.0,
                         what="fused round trip (raw)")
    else:
        assert torch.equal(out, out_ref), "synthesised output differs"


@pytest.mark.parametrize("os_,n_pol", [("8/7", 1), ("4/3", 2)])
def test_roundtrip_wave_general_window(gpu, os_, n_pol):
    """The wave synthesis skips the taper multiply on rows [48, 208) when the window is
    exactly 1 there (tukey / top_hat / no_window at Ov 48: every other test); a window that
    is not runs the general taper.  Both against the separate calls (block kernel)."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, os_, 12)
    x = _noise_t(torch, gpu, (n_pol, 1 << 19), 11)
    t = np.arange(256)
    tukey = orc.tukey_window_coeffs(256, 48)
    for win in (tukey * (0.75 + 0.25 * np.cos(2 * np.pi * t / 256)), tukey):
        ana = pfb.AnalysisPlan(taps, 256, os_, "polyphase_analysis", n_pol, 0)
        syn = pfb.SynthesisPlan(256, os_, 256, 48, True, 1, True, taps, pfb.PFBWindow().custom(win),
                                None, n_pol, 0)
        out_ref = syn.execute(ana.execute(x), sample_offset=1, layout="ptc")
        _, out = pfb.roundtrip(ana, syn, x, sample_offset=1)
        torch.cuda.synchronize()
        assert out.shape == out_ref.shape and out.shape[1] > 0
        assert_pfb_close(out.cpu().numpy(), out_ref.cpu().numpy(), scale=1.0,
                         what=f"wave synthesis, {'tukey' if win is tukey else 'non-flat'} window")


def test_roundtrip_no_blocks_only_analysis(gpu):
    """Too short for one synthesis block: the channelised product is still produced."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    n_dat = 3328 + 224 * 50
    x = _noise_t(torch, gpu, (1, n_dat), 3)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    chan, out = pfb.roundtrip(ana, syn, x)
    assert out.shape == (1, 0)
    assert torch.equal(chan, ana.execute(x))


def test_roundtrip_rejects_mismatched_plans(gpu):
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    x = _noise_t(torch, gpu, (1, 1 << 16), 3)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](128, 16)
    t8 = pfb.design_PFB_FIR_filter(8, "8/7", 10)
    syn = pfb.SynthesisPlan(8, "8/7", 128, 16, True, 1, True, t8, win, None, 1, 0)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip(ana, syn, x)


@pytest.mark.parametrize("chunk_blocks", [4, 0])
def test_roundtrip_graph_capture(gpu, chunk_blocks):
    """The round-trip step replays correctly from a HIP graph: the pipelined form (two
    streams, chunk 4) and the fused form (chunk 0: one stream, analysis emits Z)."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    x = _noise_t(torch, gpu, (1, 1 << 19), 11)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    if chunk_blocks:
        syn.set_chunk_blocks(chunk_blocks)
    chan_ref, out_ref = pfb.roundtrip(ana, syn, x)  # eager reference (also the warm-up)
    chan_ref, out_ref = chan_ref.clone(), out_ref.clone()
    chan = torch.empty_like(chan_ref)
    out = torch.empty_like(out_ref)
    pfb.roundtrip(ana, syn, x, chan=chan, out=out)
    torch.cuda.synchronize()
    chan.zero_()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            pfb.roundtrip(ana, syn, x, chan=chan, out=out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(chan, chan_ref)
    assert torch.equal(out, out_ref)


def test_roundtrip_steps_in_flight(gpu):
    """bench.py's in-flight mode: 3 plan pairs, each step one graph replay on its pair's
    stream, steps dealt round-robin with nothing ordering one pair after another.  Every
    pair's outputs (channelised product and time series) after 7 overlapping steps on 3
    different units equal the eager single-stream round trip of that unit bit for bit."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    D, n = 3, 1 << 20
    pairs, refs = [], []
    for d in range(D):
        x = _noise_t(torch, gpu, (1, n), 40 + d)
        ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
        syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
        c_ref, o_ref = pfb.roundtrip(ana, syn, x)
        refs.append((c_ref.clone(), o_ref.clone()))
        chan, out = torch.empty_like(c_ref), torch.empty_like(o_ref)
        pairs.append((ana, syn, x, chan, out))
    torch.cuda.synchronize()
    graphs = []
    for ana, syn, x, chan, out in pairs:
        pfb.roundtrip(ana, syn, x, chan=chan, out=out)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            pfb.roundtrip(ana, syn, x, chan=chan, out=out)
        graphs.append(g)
        chan.zero_()
        out.zero_()
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(D)]
    for i in range(7):
        with torch.cuda.stream(streams[i % D]):
            graphs[i % D].replay()
    torch.cuda.synchronize()
    for (_, _, _, chan, out), (c_ref, o_ref) in zip(pairs, refs):
        assert torch.equal(chan, c_ref)
        assert torch.equal(out, o_ref)


@pytest.mark.parametrize("N,nf,ov,variant", [
    (256, 256, 48, "polyphase_analysis"),           # streaming analysis + wave synthesis
    (512, 512, 128, "polyphase_analysis_padded"),   # register-window FIR + row FFT + wave512
])
@pytest.mark.parametrize("so", [1, 17, 162])        # off 0 / 16: run layout; 161: row layout
@pytest.mark.parametrize("n_pol", [1, 2])
def test_roundtrip_split_halves(gpu, N, nf, ov, variant, so, n_pol):
    """pfb_roundtrip_analysis_execute + pfb_roundtrip_synthesis_execute (the halves bench.py
    pipelines over two streams) equal pfb_roundtrip_execute bit for bit — also when the
    halves run on two streams ordered by an event; the synthesis half of a fresh plan (no
    rows yet) and the halves of a chunked plan are rejected."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(N, "8/7", 12)
    x = _noise_t(torch, gpu, (n_pol, 1 << 20), 17)
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)

    def plans():
        return (pfb.AnalysisPlan(taps, N, "8/7", variant, n_pol, 0),
                pfb.SynthesisPlan(N, "8/7", nf, ov, True, 1, True, taps, win, None, n_pol, 0))
    ana, syn = plans()
    c_ref, o_ref = pfb.roundtrip(ana, syn, x, sample_offset=so)
    c_ref, o_ref = c_ref.clone(), o_ref.clone()
    ana2, syn2 = plans()
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(ana2, syn2, x.shape[1], sample_offset=so, device=gpu.index or 0)
    chan = pfb.roundtrip_analysis(ana2, syn2, x, sample_offset=so)
    sa, ss = torch.cuda.current_stream(), torch.cuda.Stream()
    ev = torch.cuda.Event()
    ev.record(sa)
    ss.wait_event(ev)
    with torch.cuda.stream(ss):
        out = pfb.roundtrip_synthesis(ana2, syn2, x.shape[1], sample_offset=so, device=gpu.index or 0)
    torch.cuda.synchronize()
    assert torch.equal(chan, c_ref)
    assert torch.equal(out, o_ref)
    syn2.set_chunk_blocks(2)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_analysis(ana2, syn2, x, sample_offset=so)


@pytest.mark.parametrize("N,nf,ov,variant", [
    (256, 256, 48, "polyphase_analysis"),
    (512, 512, 128, "polyphase_analysis_padded"),
])
def test_roundtrip_split_halves_reject_mismatch(gpu, N, nf, ov, variant):
    """The synthesis half checks that the stage-1 rows in its scratch came from the analysis
    half of THIS analysis plan with the same n_dat and sample_offset: another
    n_dat, another offset, another analysis plan, or rows overwritten by a whole round trip
    on the pair are rejected with PfbError instead of synthesising stale rows."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(N, "8/7", 12)
    x = _noise_t(torch, gpu, (1, 1 << 19), 23)
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)
    ana = pfb.AnalysisPlan(taps, N, "8/7", variant, 1, 0)
    ana_b = pfb.AnalysisPlan(taps, N, "8/7", variant, 1, 0)
    syn = pfb.SynthesisPlan(N, "8/7", nf, ov, True, 1, True, taps, win, None, 1, 0)
    dev = gpu.index or 0
    pfb.roundtrip_analysis(ana, syn, x, sample_offset=17)
    for kw in (dict(n_dat=x.shape[1] - 4096, sample_offset=17), dict(n_dat=x.shape[1], sample_offset=1)):
        with pytest.raises(pfb.PfbError):
            pfb.roundtrip_synthesis(ana, syn, kw["n_dat"], sample_offset=kw["sample_offset"], device=dev)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(ana_b, syn, x.shape[1], sample_offset=17, device=dev)
    # the matching call still works after the rejected ones
    out = pfb.roundtrip_synthesis(ana, syn, x.shape[1], sample_offset=17, device=dev)
    _, o_ref = pfb.roundtrip(ana_b, syn, x, sample_offset=17)
    torch.cuda.synchronize()
    assert torch.equal(out, o_ref)
    # the whole round trip just reused the pair's rows: the synthesis half alone is refused
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(ana_b, syn, x.shape[1], sample_offset=17, device=dev)


def test_plan_close_refused_during_capture(gpu):
    """A plan whose launches a stream capture recorded cannot be closed while that capture
    is open (its device buffers are referenced by the graph: the round-3 use-after-free);
    after the capture ends and the graph is replayed and dropped, close() works."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    x = _noise_t(torch, gpu, (1, 1 << 18), 29)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    chan, out = pfb.roundtrip(ana, syn, x)  # warm-up: allocates the plan scratch
    ref = out.clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        try:
            pfb.roundtrip(ana, syn, x, chan=chan, out=out)
            with pytest.raises(RuntimeError):
                ana.close()
            with pytest.raises(RuntimeError):
                syn.close()
        finally:
            g.capture_end()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    del g
    ana.close()
    syn.close()


# ------------------------------------------------------------------ BASELINE C2 size
@pytest.fixture(scope="module")
def c2(gpu):
    """C2 round trip on 2^24 noise samples (seed 0), device and oracle results."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    assert len(taps) == 3073
    n = 1 << 24
    rng = np.random.default_rng(0)
    x = ((rng.standard_normal((1, 1, n)) + 1j * rng.standard_normal((1, 1, n))) /
         np.sqrt(2)).astype(np.complex64)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    xd = torch.from_numpy(x[:, 0, :]).to(gpu)
    chan, out = pfb.roundtrip(ana, syn, xd)
    torch.cuda.synchronize()
    return dict(pfb=pfb, taps=taps, x=x, xd=xd, ana=ana, syn=syn,
                chan=chan.cpu().numpy(), out=out.cpu().numpy())


def test_c2_full_size_matches_oracle(c2):
    """BASELINE configs[1] at full size: channelised data and output vs the oracle."""
    taps, x = c2["taps"], c2["x"]
    ref_chan = orc.polyphase_analysis(x, taps, 256, "8/7")       # (1, 256, K) float64 maths
    assert_pfb_close(c2["chan"].transpose(0, 2, 1), ref_chan, what="C2 analysis")
    win = orc.pfb_window("tukey", 256, 48)
    ref = orc.polyphase_synthesis(ref_chan, 1, 256, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 48, win)
    assert c2["out"].shape == (1, 16737280)
    assert_pfb_close(c2["out"][:, None, :], ref, scale=1.0, what="C2 round trip (raw)")


def test_c2_full_size_standalone_synthesis(c2):
    """The synthesis alone on the WHOLE C2 channelised product (74 883 rows, 467 blocks)
    — ``SynthesisPlan.execute(chan)``, the path bench.py's ``synthesis_only`` times (the
    PST production case: InverseFilterBank.m:92-96 -> polyphase_synthesis.m:163-316; row
    FFT stage 1 + synth_wave_kernel) — against the oracle synthesis of the same
    channelised product, every output sample (16 737 280) at the raw 1e-6 criterion."""
    import torch
    pfb = _pfb()
    taps, chan = c2["taps"], c2["chan"]                       # (1, K, 256) from the GPU
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    out = syn.execute(torch.from_numpy(chan).to(c2["xd"].device), 1, layout="ptc")
    torch.cuda.synchronize()
    assert syn.last_stage1_rows == "stored"
    ref = orc.polyphase_synthesis(chan.transpose(0, 2, 1), 1, 256, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 48,
                                  orc.pfb_window("tukey", 256, 48))
    assert out.shape == (1, 16737280)
    assert_pfb_close(out.cpu().numpy()[:, None, :], ref, scale=1.0, what="C2 synthesis only (raw)")
    syn.close()


def test_c2_full_size_inverse_filterbank_stream(c2):
    """InverseFilterBank streaming over the whole C2 channelised product in three device
    chunks (InverseFilterBank.m:73-135: carry-over rounded up to a multiple of nu,
    deripple forced off at :90) against InverseFilterBankOracle on the same chunks."""
    import torch
    pfb = _pfb()
    taps, chan = c2["taps"], c2["chan"]
    cfg = dict(filt_coeff=taps, channels=256, os_factor="8/7", input_fft_length=256,
               input_overlap=48, deripple=True, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg)
    oifb = orc.InverseFilterBankOracle(taps, 256, "8/7", 256, 48, "tukey", deripple=True)
    cd = torch.from_numpy(chan).to(c2["xd"].device)
    K = chan.shape[1]
    cuts = [0, 30001, 55555, K]
    total = 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        ifb, got = ifb.execute(cd[:, a:b, :].transpose(1, 2))   # (n_pol, n_chan, n) view
        ref = oifb.execute(chan[:, a:b, :].transpose(0, 2, 1))
        assert tuple(got.shape) == ref.shape, (a, b, tuple(got.shape), ref.shape)
        assert_pfb_close(got.cpu().numpy(), ref, scale=1.0, what=f"C2 inverse stream rows [{a}, {b})")
        assert ifb.buffered_samples == oifb.buffered_samples
        total += ref.shape[2]
    assert total > 16_000_000


def test_c2_full_size_linearity(c2):
    """Size-independent property: RT(a x1 + b x2) = a RT(x1) + b RT(x2)."""
    import torch
    pfb = _pfb()
    x1 = c2["xd"]
    x2 = torch.roll(x1, 12345, dims=1).contiguous()
    a, b = 0.75, -1.25j
    _, y1 = pfb.roundtrip(c2["ana"], c2["syn"], x1)
    _, y2 = pfb.roundtrip(c2["ana"], c2["syn"], x2)
    _, y = pfb.roundtrip(c2["ana"], c2["syn"], (a * x1 + b * x2).to(torch.complex64))
    lhs = y.cpu().numpy()
    rhs = (a * y1 + b * y2).cpu().numpy()
    assert_pfb_close(lhs, rhs, tol=2e-6, scale=1.0, what="linearity (raw)")


def test_c2_series_beyond_2gib(gpu):
    """Maximum-size case: one 2^28 + 2^20 + 12345-sample series (over 2 GiB of input and
    of output per polarisation, 2.4 GB of stage-1 rows) through the fused round trip, where every
    kernel's per-workgroup buffer descriptor covers only its own range (kRsrcMaxBytes).
    Blocks are local (rows b keep .. b keep + Nf, each row reading x[k M, k M + P N)), so
    the first and the last blocks are checked against the oracle run on the matching
    slices of the series (the tail slice starts on a commutator period, k0 a multiple of
    nu, as the sharding helpers cut it)."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    n = (1 << 28) + (1 << 20) + 12345
    g = torch.Generator(device=gpu).manual_seed(7)
    xd = torch.complex(torch.randn((1, n), device=gpu, generator=g),
                       torch.randn((1, n), device=gpu, generator=g)).to(torch.complex64) / np.sqrt(2.0)
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    _, out = pfb.roundtrip(ana, syn, xd)
    torch.cuda.synchronize()
    M, PN, keep, lkeep = 224, 13 * 256, 160, 35840
    K = (n - PN) // M
    B = (K - 96) // keep
    assert out.shape == (1, B * lkeep) and B * lkeep * 8 > (1 << 31)
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    w = orc.pfb_window("tukey", 256, 48)

    def ref_from(s0, s1):
        xs = xd[:, s0:s1].cpu().numpy()[:, None, :]
        chan = orc.polyphase_analysis(xs, taps, 256, "8/7")
        return orc.polyphase_synthesis(chan, 1, 256, "8/7", dr, 1, 48, w)[:, 0, :]

    head = ref_from(0, 1 << 21)
    assert_pfb_close(out[:, :head.shape[1]].cpu().numpy(), head, scale=1.0, what="beyond 2 GiB: head")
    b0 = B - 40
    k0 = b0 * keep
    assert k0 % 8 == 0
    tail = ref_from(k0 * M, n)
    assert tail.shape[1] == 40 * lkeep
    assert_pfb_close(out[:, b0 * lkeep:].cpu().numpy(), tail, scale=1.0, what="beyond 2 GiB: tail")


# ------------------------------------------------------------------ BASELINE C3 / C4 units
def _np_noise(seed, n):
    rng = np.random.default_rng(seed)
    return ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)


def _mid_taps(pfb):
    taps = pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    assert len(taps) == 100353
    return taps


def test_c3_parameters_match_oracle(gpu):
    """BASELINE configs[2] parameters exactly (SKA-Mid padded, 4096 ch, 8/7, 100 353
    two-stage taps, Nf 512, Ov 128, tukey, deripple) at a reduced length (2^22 samples:
    1170 channelised rows, 3 synthesis blocks) through the production round trip —
    fir_window_kernel<PADDED> writing the stage-1 rows, row_fft_kernel<4096>,
    synth_block_kernel<512,448> — compared with orc.polyphase_analysis_padded ->
    orc.polyphase_synthesis (polyphase_analysis_padded.m:106-156,
    polyphase_synthesis.m:163-316): channelised product at unit amplitude (RMS), the
    synthesised series raw."""
    import torch
    pfb = _pfb()
    taps = _mid_taps(pfb)
    n = 1 << 22
    x = _np_noise(1, n)[None, None, :]
    ana = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](512, 128)
    syn = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, taps, win, None, 1, 0)
    chan, out = pfb.roundtrip(ana, syn, torch.from_numpy(x[:, 0, :]).to(gpu))
    torch.cuda.synchronize()
    ref_chan = orc.polyphase_analysis_padded(x, taps, 4096, "8/7")
    assert ref_chan.shape == (1, 4096, 1170)
    assert_pfb_close(chan.cpu().numpy().transpose(0, 2, 1), ref_chan, what="C3 analysis")
    ref = orc.polyphase_synthesis(ref_chan, 1, 512, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 128,
                                  orc.pfb_window("tukey", 512, 128))
    assert ref.shape == (1, 1, 3 * 917504)
    assert_pfb_close(out.cpu().numpy()[:, None, :], ref, scale=1.0, what="C3 round trip (raw)")


def test_c3_dual_pol_unit(gpu):
    """The SKA-Mid `mid` sub-config's dual-polarisation unit (config/test.config.json:104-128,
    n_pol 2) with the BASELINE configs[2] parameters at 2^22 samples per pol: one fused
    round trip over both pols (the FIR / row FFT / synthesis kernels index the pols by
    blockIdx.y) equals each pol's own single-pol round trip bit for bit — pol 0 is the
    input test_c3_parameters_match_oracle compares with the oracle — and the channelised
    product of pol 1 agrees with the oracle."""
    import torch
    pfb = _pfb()
    taps = _mid_taps(pfb)
    n = 1 << 22
    x = np.stack([_np_noise(1, n), _np_noise(2, n)])
    win = pfb.PFBWindow().lookup["tukey"](512, 128)
    ana = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 2, 0)
    syn = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, taps, win, None, 2, 0)
    chan, out = pfb.roundtrip(ana, syn, torch.from_numpy(x).to(gpu))
    ana1 = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 1, 0)
    syn1 = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, taps, win, None, 1, 0)
    for p in range(2):
        c1, o1 = pfb.roundtrip(ana1, syn1, torch.from_numpy(x[p:p + 1]).to(gpu))
        assert torch.equal(c1[0], chan[p]), f"pol {p} channelised product differs from its single-pol run"
        assert torch.equal(o1[0], out[p]), f"pol {p} output differs from its single-pol run"
    ref_chan = orc.polyphase_analysis_padded(x[1:2, None, :], taps, 4096, "8/7")
    assert_pfb_close(chan[1:2].cpu().numpy().transpose(0, 2, 1), ref_chan, what="C3 dual-pol analysis (pol 1)")
    for pl in (ana, syn, ana1, syn1):
        pl.close()


def test_c4_unit_matches_oracle(gpu):
    """BASELINE configs[3]'s unit: one dual-polarisation DADA time block with the C2
    parameters (256 ch, 8/7, 3073 taps, Nf 256, Ov 48, tukey, deripple), pols drawn
    from seeds 100 and 101, through the fused streaming round trip
    (analysis_stream_kernel indexes the pols by blockIdx.y and z_pol_stride),
    compared with the oracle per polarisation (2^22 samples per pol)."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    n = 1 << 22
    x = np.stack([_np_noise(100, n), _np_noise(101, n)])[:, None, :]
    ana = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 2, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 2, 0)
    chan, out = pfb.roundtrip(ana, syn, torch.from_numpy(x[:, 0, :]).to(gpu))
    torch.cuda.synchronize()
    ref_chan = orc.polyphase_analysis(x, taps, 256, "8/7")
    assert_pfb_close(chan.cpu().numpy().transpose(0, 2, 1), ref_chan, what="C4 analysis")
    ref = orc.polyphase_synthesis(ref_chan, 1, 256, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 48,
                                  orc.pfb_window("tukey", 256, 48))
    assert ref.shape[0] == 2 and ref.shape[2] > 4_000_000
    assert_pfb_close(out.cpu().numpy()[:, None, :], ref, scale=1.0, what="C4 round trip (raw)")
    # the two polarisations are independent units: each equals its own single-pol run
    ana1 = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    syn1 = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    for p in range(2):
        _, o1 = pfb.roundtrip(ana1, syn1, torch.from_numpy(x[p:p + 1, 0, :]).to(gpu))
        assert torch.equal(o1[0], out[p]), f"pol {p} differs from its single-pol run"


# C3 round-trip delay of an impulse: the analysis commutator repeats every N de = 28 672
# input samples and the synthesis blocks every keep * M = 917 504, so an impulse at any
# position congruent modulo 917 504 comes back with the same delay.  The oracle fixes
# it on a 2^22-sample vector (test_oracle.py pins the same number on the CPU).
C3_BLOCK_PERIOD = 256 * 3584


def c3_impulse_delay_from_oracle(pfb, taps, off_full):
    n = 1 << 22
    pos = off_full % C3_BLOCK_PERIOD + 2 * C3_BLOCK_PERIOD
    x = np.zeros((1, 1, n), np.complex64)
    x[0, 0, pos] = 1.0
    ch = orc.polyphase_analysis_padded(x, taps, 4096, "8/7")
    y = orc.polyphase_synthesis(ch, 1, 512, "8/7", {"apply_deripple": 1, "filter_coeff": taps},
                                1, 128, orc.pfb_window("tukey", 512, 128))
    return pos - int(np.argmax(np.abs(y[0, 0])))


def test_c3_full_size_impulse_and_linearity(gpu):
    """BASELINE configs[2] (SKA-Mid padded, 4096 ch, 8/7, 100 353 two-stage taps,
    2^26 samples, Nf 512, Ov 128) at full size, through the fused generic round trip:
    size-independent properties (the float64 oracle at 2^26 x 4096 is too slow; the
    same parameters at 2^22 are compared sample by sample in
    test_c3_parameters_match_oracle):
    * an impulse comes back at the oracle-derived position (TestImpulse.m:46-73: mask
      +-1 sample around the EXPECTED index, <= -60 dB everywhere else);
    * the channelised product equals the separate analysis call bit for bit;
    * linearity of the whole round trip."""
    import torch
    pfb = _pfb()
    taps = _mid_taps(pfb)
    n = 1 << 26
    off = 40_000_000
    delay = c3_impulse_delay_from_oracle(pfb, taps, off)
    assert delay == 458751  # output overlap Ov de/nu N = 458 752, minus the padded bank's 1
    ana = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](512, 128)
    syn = pfb.SynthesisPlan(4096, "8/7", 512, 128, True, 1, True, taps, win, None, 1, 0)
    x = torch.zeros((1, n), dtype=torch.complex64, device=gpu)
    x[0, off] = 1.0
    chan, y = pfb.roundtrip(ana, syn, x)
    assert torch.equal(chan, ana.execute(x)), "channelised product differs"
    yy = y[0].abs().cpu().numpy().astype(np.float64)
    expected = off - delay
    assert int(np.argmax(yy)) == expected, (int(np.argmax(yy)), expected)
    amp = 20 * np.log10(yy / yy[expected] + 1e-30)
    mask = np.ones(len(yy), bool)
    mask[expected - 1:expected + 2] = False
    assert amp[mask].max() <= -60.0, amp[mask].max()
    assert abs(yy[expected] - 1.0) < 1e-3, yy[expected]  # unit round-trip gain
    # linearity on noise (same plan, different input)
    g = torch.Generator(device=gpu).manual_seed(3)
    x1 = torch.complex(torch.randn((1, n), device=gpu, generator=g),
                       torch.randn((1, n), device=gpu, generator=g)).to(torch.complex64)
    _, y1 = pfb.roundtrip(ana, syn, x1)
    y1 = y1.clone()
    _, y2 = pfb.roundtrip(ana, syn, (x1 * 0.5 + x * 3.0).to(torch.complex64))
    lhs = y2.cpu().numpy()
    rhs = (0.5 * y1 + 3.0 * y).cpu().numpy()
    assert_pfb_close(lhs, rhs, tol=2e-6, scale=1.0, what="C3 linearity (raw)")


RECOMPUTE_CASES = [
    # (os, taps/chan, n_pol, n_dat, sample_offset): streaming-analysis shapes of the fused
    # round trip (Bunton, N 256, Nf 256 / Ov 48)
    ("8/7", 12, 1, 1 << 20, 1),
    ("8/7", 12, 2, 1 << 19, 17),
    ("8/7", 11, 1, 300_000, 1),
    ("4/3", 12, 2, 1 << 19, 1),
    ("4/3", 12, 1, 200_001, 9),
    ("8/7", 12, 1, 90_000, 1),    # a handful of blocks: ranges of 0 or 1 block
    ("8/7", 12, 3, 1 << 18, 1),
]


@pytest.mark.parametrize("case", RECOMPUTE_CASES)
def test_roundtrip_fused_and_chunked_paths_agree(gpu, case):
    """pfb_roundtrip_execute has two internal paths: the fused one (the analysis kernel
    writes the synthesis stage-1 rows as N^2 x its FIR sums) and the chunked pipeline
    (an explicit chunk size: separate analysis and synthesis kernels, bit-identical to the
    separate calls).  The channelised product is bit-identical on both; the outputs agree
    within the reference's 1e-6 (include/pfb_api.h)."""
    import torch
    pfb = _pfb()
    os_, tpc, n_pol, n_dat, so = case
    taps = pfb.design_PFB_FIR_filter(256, os_, tpc)
    x = _noise_t(torch, gpu, (n_pol, n_dat), 11)
    ana = pfb.AnalysisPlan(taps, 256, os_, "polyphase_analysis", n_pol, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    syn = pfb.SynthesisPlan(256, os_, 256, 48, True, 1, True, taps, win, None, n_pol, 0)
    chan_f, out_f = pfb.roundtrip(ana, syn, x, sample_offset=so)
    torch.cuda.synchronize()
    syn.set_chunk_blocks(3)
    chan_c, out_c = pfb.roundtrip(ana, syn, x, sample_offset=so)
    torch.cuda.synchronize()
    assert out_f.shape == out_c.shape and out_f.shape[1] > 0
    assert torch.equal(chan_f, chan_c)
    assert_pfb_close(out_f.cpu().numpy(), out_c.cpu().numpy(), scale=1.0,
                     what="fused vs chunked round trip (raw)")


def test_mid_external_matches_oracle(gpu):
    """Reference sub-config 'mid_external' (config/test.config.json: SKA-Mid padded analysis,
    4096 ch, 8/7, 100 353 taps, Nf 256, Ov 32 — so W = 224 at N = 4096, keep 192,
    L_ov = 114 688) through the production round trip, 2^22 samples (1170 channelised
    rows, 5 synthesis blocks), against orc.polyphase_analysis_padded ->
    orc.polyphase_synthesis: channelised product at unit amplitude (RMS), output raw."""
    import torch
    pfb = _pfb()
    cfg = pfb.default_config("mid_external")
    assert (cfg.channels, cfg.input_fft_length, cfg.input_overlap) == (4096, 256, 32)
    taps = _mid_taps(pfb)
    n = 1 << 22
    x = _np_noise(9, n)[None, None, :]
    ana = pfb.AnalysisPlan(taps, 4096, "8/7", "polyphase_analysis_padded", 1, 0)
    win = pfb.PFBWindow().lookup["tukey"](256, 32)
    syn = pfb.SynthesisPlan(4096, "8/7", 256, 32, True, 1, True, taps, win, None, 1, 0)
    chan, out = pfb.roundtrip(ana, syn, torch.from_numpy(x[:, 0, :]).to(gpu))
    torch.cuda.synchronize()
    ref_chan = orc.polyphase_analysis_padded(x, taps, 4096, "8/7")
    assert ref_chan.shape == (1, 4096, 1170)
    assert_pfb_close(chan.cpu().numpy().transpose(0, 2, 1), ref_chan, what="mid_external analysis")
    ref = orc.polyphase_synthesis(ref_chan, 1, 256, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 32,
                                  orc.pfb_window("tukey", 256, 32))
    assert ref.shape == (1, 1, 5 * (917504 - 2 * 114688))
    assert_pfb_close(out.cpu().numpy()[:, None, :], ref, scale=1.0,
                     what="mid_external round trip (raw)")


# ------------------------------------------------------------------ recomputed stage-1 rows
@pytest.mark.parametrize("os_,tpc,n,so,n_pol", [
    ("8/7", 12, 1 << 20, 1, 1),        # C2 shape (P 13)
    ("8/7", 11, 1 << 20, 17, 2),       # P 12, offset, two polarisations
    ("4/3", 12, 1 << 20, 1, 1),        # C2' shape ('low')
    ("4/3", 11, 777_777, 33, 2),       # ragged length, offset
    ("8/7", 12, 1 << 24, 1, 1),        # full C2 unit
])
def test_roundtrip_recomputed_stage1_rows_bit_identical(gpu, os_, tpc, n, so, n_pol):
    """pfb_synthesis_set_stage1_rows(RECOMPUTED): the synthesis evaluates the stage-1 rows
    from the input (the analysis writes only the channelised product).  The rows are the
    same FIR sums in the same FMA order with taps pre-scaled by N^2 (a power of two), so
    the channelised product and the output equal the stored-rows round trip bit for bit —
    whole calls and split halves (the synthesis half re-reads the input)."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, os_, tpc)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    x = _noise_t(torch, gpu, (n_pol, n), 31)

    def pair(mode):
        a = pfb.AnalysisPlan(taps, 256, os_, "polyphase_analysis", n_pol, 0)
        s = pfb.SynthesisPlan(256, os_, 256, 48, True, 1, True, taps, win, None, n_pol, 0)
        s.set_stage1_rows(mode)
        return a, s
    a0, s0 = pair("stored")
    c_ref, o_ref = pfb.roundtrip(a0, s0, x, sample_offset=so)
    assert s0.last_stage1_rows == "stored"
    a1, s1 = pair("recomputed")
    c1, o1 = pfb.roundtrip(a1, s1, x, sample_offset=so)
    torch.cuda.synchronize()
    # the recomputing kernel ran (not a silent fall-back to stored rows, which would give
    # the same bits)
    assert s1.last_stage1_rows == "recomputed"
    assert torch.equal(c1, c_ref)
    assert torch.equal(o1, o_ref)
    # split halves on two streams
    chan = pfb.roundtrip_analysis(a1, s1, x, sample_offset=so)
    ss = torch.cuda.Stream()
    ss.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(ss):
        out = pfb.roundtrip_synthesis(a1, s1, x.shape[1], sample_offset=so, device=gpu.index or 0)
    torch.cuda.synchronize()
    assert s1.last_stage1_rows == "recomputed"
    assert torch.equal(chan, c_ref)
    assert torch.equal(out, o_ref)
    # the analysis half of one mode is not continued by the other
    pfb.roundtrip_analysis(a1, s1, x, sample_offset=so)
    s1.set_stage1_rows("stored")
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(a1, s1, x.shape[1], sample_offset=so, device=gpu.index or 0)


def test_roundtrip_recomputed_rows_reject_mismatch(gpu):
    """The recomputed-rows synthesis half checks the analysis plan, n_dat and offset of the
    analysis half, as the stored-rows one does."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    x = _noise_t(torch, gpu, (1, 1 << 19), 37)
    a = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    b = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    s = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    s.set_stage1_rows("recomputed")
    dev = gpu.index or 0
    pfb.roundtrip_analysis(a, s, x)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(a, s, x.shape[1] - 2048, device=dev)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(b, s, x.shape[1], device=dev)
    with pytest.raises(pfb.PfbError):
        pfb.roundtrip_synthesis(a, s, x.shape[1], sample_offset=17, device=dev)
    out = pfb.roundtrip_synthesis(a, s, x.shape[1], device=dev)
    _, o_ref = pfb.roundtrip(b, s, x)
    torch.cuda.synchronize()
    assert torch.equal(out, o_ref)


@pytest.mark.parametrize("kind", ["complex128", "strided"])
def test_roundtrip_recomputed_split_temporary_input(gpu, kind):
    """Split round trip with recomputed stage-1 rows whose input is NOT a contiguous
    complex64 tensor: _prep_in makes a temporary, which the synthesis half re-reads after
    roundtrip_analysis has returned.  The plan keeps it alive until roundtrip_synthesis has
    been enqueued (and records it on that stream), so allocations in between — which the
    caching allocator would serve from a freed temporary — cannot overwrite it."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, "8/7", 12)
    win = pfb.PFBWindow().lookup["tukey"](256, 48)
    n = 1 << 20
    x64 = _noise_t(torch, gpu, (1, n), 41)
    if kind == "complex128":
        xin = x64.to(torch.complex128)
    else:
        big = torch.zeros((1, 2 * n), dtype=torch.complex64, device=gpu)
        big[:, ::2] = x64
        xin = big[:, ::2]
        assert not xin.is_contiguous()
    a0 = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    s0 = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    _, o_ref = pfb.roundtrip(a0, s0, x64)
    a1 = pfb.AnalysisPlan(taps, 256, "8/7", "polyphase_analysis", 1, 0)
    s1 = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, True, taps, win, None, 1, 0)
    s1.set_stage1_rows("recomputed")
    pfb.roundtrip_analysis(a1, s1, xin)
    # allocations of the temporary's size, filled with garbage, on the same stream
    junk = [torch.full((1, n), 7.0 + 3.0j, dtype=torch.complex64, device=gpu) for _ in range(4)]
    out = pfb.roundtrip_synthesis(a1, s1, n, device=gpu.index or 0)
    torch.cuda.synchronize()
    del junk
    assert s1.last_stage1_rows == "recomputed"
    assert torch.equal(out, o_ref)
