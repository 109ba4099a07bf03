"""GPU parity of the HIP kernels (through the C ABI) against the oracle.

Sizes are chosen so the float64 oracle finishes in seconds; the BASELINE C2 size and
the C3/C4 parameters are compared with the oracle in test_gpu_roundtrip.py, which also
holds the full-size C3 size-independent properties (impulse position, linearity).
Tolerance: the reference's np.isclose(atol=1e-6, rtol=1e-6) on unit-amplitude data —
raw for round trips of unit-amplitude inputs, else both sides divided by the oracle's
RMS magnitude (conftest.assert_pfb_close, which also reports max / RMS error).
"""
import numpy as np
import pytest

from conftest import assert_pfb_close
from oracle import pfb_oracle as orc

pytestmark = pytest.mark.gpu


def _pfb():
    import ska_pst_dsp_model_amd as pfb
    return pfb


def _taps(kind):
    pfb = _pfb()
    if kind == "test":
        return pfb.design_PFB_FIR_filter(8, "8/7", 10)
    if kind == "low87":
        return pfb.design_PFB_FIR_filter(256, "8/7", 12)
    if kind == "low43":
        return pfb.design_PFB_FIR_filter(256, "4/3", 12)
    if kind == "pst":
        return pfb.read_fir_filter_coeff(pfb.config.config_dir + "/PST_filtertaps.txt")
    if kind == "mid":
        return pfb.design_PFB_FIR_filter_two_stage(4096, "8/7", 28)
    raise KeyError(kind)


def _noise(rng, shape):
    return ((rng.standard_normal(shape) + 1j * rng.standard_normal(shape)) /
            np.sqrt(2)).astype(np.complex64)


def _tone(n, freq_bins, n_pol=1, phase=np.pi / 4):
    t = np.arange(n)
    x = np.exp(1j * (2 * np.pi * freq_bins / n * t + phase)).astype(np.complex64)
    return np.repeat(x[None, None, :], n_pol, axis=0)


# ----------------------------------------------------------------------------- analysis
@pytest.mark.parametrize("case", [
    ("test", 8, "8/7", 2, 4096, "bunton"),
    ("low87", 256, "8/7", 1, 1 << 18, "bunton"),
    ("low43", 256, "4/3", 2, 1 << 17, "bunton"),
    ("pst", 256, "4/3", 1, 1 << 17, "bunton"),
    ("test", 8, "8/7", 2, 4096, "padded"),
    ("low87", 256, "8/7", 1, 1 << 17, "padded"),
])
def test_analysis_matches_oracle(gpu, case):
    import torch
    pfb = _pfb()
    kind, N, os_, n_pol, n_dat, variant = case
    taps = _taps(kind)
    rng = np.random.default_rng(1234)
    x = _noise(rng, (n_pol, 1, n_dat))
    if variant == "bunton":
        ref = orc.polyphase_analysis(x, taps, N, os_)
        got = pfb.polyphase_analysis(torch.from_numpy(x).to(gpu), taps, N, os_)
    else:
        ref = orc.polyphase_analysis_padded(x, taps, N, os_)
        got = pfb.polyphase_analysis_padded(torch.from_numpy(x).to(gpu), taps, N, os_)
    assert_pfb_close(got.cpu().numpy(), ref, what=f"analysis {case}")


def test_analysis_host_memory_path(gpu):
    """PFB_MEM_HOST staging gives the same answer as device pointers."""
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(7), (2, 1, 3000))
    ref = orc.polyphase_analysis(x, taps, 8, "8/7")
    got = pfb.polyphase_analysis(x, taps, 8, "8/7")
    assert isinstance(got, np.ndarray)
    assert_pfb_close(got, ref)


def test_analysis_tone_closed_form(gpu):
    """Known answer (polyphase_analysis.m:105-120 closed form): a tone x = e^{j w n}
    gives out[c, k] = N e^{-j 2 pi c r_k / N} e^{j w M k} sum_i f[i] e^{j (w - 2 pi c / N) i}."""
    import torch
    pfb = _pfb()
    N, M = 8, 7
    taps = _taps("test")
    n = 4096
    w = 2 * np.pi * 0.0371
    x = np.exp(1j * w * np.arange(n)).astype(np.complex64)[None, None, :]
    got = pfb.polyphase_analysis(torch.from_numpy(x).to(gpu), taps, N, "8/7").cpu().numpy()[0]
    f = orc.pad_filter(taps, N)
    i = np.arange(len(f))
    c = np.arange(N)
    H = np.array([np.sum(f * np.exp(1j * (w - 2 * np.pi * cc / N) * i)) for cc in c])
    K = got.shape[1]
    k = np.arange(K)
    r = (M * k) % N
    ref = N * np.exp(-2j * np.pi * np.outer(c, r) / N) * np.exp(1j * w * M * k)[None, :] * H[:, None]
    assert_pfb_close(got, ref, tol=2e-6)


@pytest.mark.parametrize("N,os_,ppc", [(256, "32/27", 24), (64, "8/7", 20)])
def test_analysis_many_taps_fused(gpu, N, os_, ppc):
    """P in (16, 32]: the PMAX=32 instantiation of the fused kernel."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(N, os_, ppc)
    x = _noise(np.random.default_rng(3), (1, 1, 40000))
    ref = orc.polyphase_analysis(x, taps, N, os_)
    got = pfb.polyphase_analysis(torch.from_numpy(x).to(gpu), taps, N, os_).cpu().numpy()
    assert_pfb_close(got, ref)


@pytest.mark.parametrize("N,os_,ppc,variant", [
    (512, "8/7", 12, "bunton"),    # register-window FIR, PW 13, DE 7
    (512, "4/3", 12, "padded"),    # PW 13, DE 3
    (1024, "4/3", 24, "bunton"),   # PW 25
    (512, "8/7", 19, "padded"),    # PW 25 (P 20)
    (512, "8/7", 28, "bunton"),    # PW 32 (P 29)
    (512, "32/27", 12, "padded"),  # DE 27
    (768, "8/7", 12, "bunton"),    # no row-FFT size for 768 -> rejected at plan time
])
def test_analysis_generic_path(gpu, N, os_, ppc, variant):
    """N > 256 goes through the FIR (register-window kernel) + row-FFT kernels, two
    polarisations, an input length that is not a multiple of anything."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(N, os_, ppc)
    x = _noise(np.random.default_rng(5), (2, 1, 60000 + 37))
    fn_o = orc.polyphase_analysis if variant == "bunton" else orc.polyphase_analysis_padded
    fn_g = pfb.polyphase_analysis if variant == "bunton" else pfb.polyphase_analysis_padded
    if N == 768:
        with pytest.raises(pfb.PfbError):
            fn_g(torch.from_numpy(x).to(gpu), taps, N, os_)
        return
    ref = fn_o(x, taps, N, os_)
    got = fn_g(torch.from_numpy(x).to(gpu), taps, N, os_).cpu().numpy()
    assert_pfb_close(got, ref)


def test_analysis_padded_mid(gpu):
    """SKA-Mid commutator PFB: 4096 channels, 100353 two-stage taps (C3, reduced length)."""
    import torch
    pfb = _pfb()
    taps = _taps("mid")
    assert len(taps) == 100353
    x = _noise(np.random.default_rng(11), (1, 1, 1 << 20))
    ref = orc.polyphase_analysis_padded(x, taps, 4096, "8/7")
    got = pfb.polyphase_analysis_padded(torch.from_numpy(x).to(gpu), taps, 4096, "8/7")
    assert_pfb_close(got.cpu().numpy(), ref)


@pytest.mark.parametrize("variant", ["polyphase_analysis", "polyphase_analysis_padded"])
def test_analysis_4096_persistent_row_fft(gpu, variant):
    """4096 channels with more than 2048 output rows: the row FFT after the FIR runs as
    row_fft_persist_kernel (contiguous row ranges per workgroup, next row prefetched),
    compared with the oracle (the C3 test at 2^22 samples stays below that row count)."""
    import torch
    pfb = _pfb()
    taps = np.random.default_rng(41).standard_normal(4096 * 12 + 1) / 64.0
    n_dat = 2100 * 3584 + 13 * 4096
    x = _noise(np.random.default_rng(42), (1, 1, n_dat))
    ref = getattr(orc, variant)(x, taps, 4096, "8/7")
    assert ref.shape[2] >= 2100
    got = getattr(pfb, variant)(torch.from_numpy(x).to(gpu), taps, 4096, "8/7")
    assert_pfb_close(got.cpu().numpy(), ref, what=f"{variant} 4096 ch, {ref.shape[2]} rows")


def test_analysis_short_input(gpu):
    """n_dat shorter than the filter: zero output rows (polyphase_analysis.m:62)."""
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(0), (1, 1, 50))
    got = pfb.polyphase_analysis(x, taps, 8, "8/7")
    assert got.shape == (1, 8, 0)


# ----------------------------------------------------------------------------- synthesis
def _synth_case(pfb, x, spans, nf, os_, deripple, taps, ov, taper, combine=1, sample_offset=1):
    import torch
    t_orc = orc.pfb_window(taper, nf, ov)
    t_gpu = pfb.PFBWindow().lookup[taper](nf, ov)
    dr = {"apply_deripple": deripple, "filter_coeff": taps}
    ref = orc.polyphase_synthesis(x, spans, nf, os_, dr, sample_offset, ov, t_orc, None, combine)
    got = pfb.polyphase_synthesis(torch.from_numpy(x).cuda(), spans, nf, os_, dr, sample_offset,
                                  ov, t_gpu, None, combine)
    return got.cpu().numpy(), ref


@pytest.mark.parametrize("spans", [1, 0])
@pytest.mark.parametrize("deripple", [1, 0])
@pytest.mark.parametrize("taper", ["tukey", "no_window", "top_hat", "hann"])
def test_synthesis_small_matches_oracle(gpu, spans, deripple, taper):
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(21), (2, 8, 96 * 7 + 32 + 5))
    got, ref = _synth_case(pfb, x, spans, 128, "8/7", deripple, taps, 16, taper)
    assert_pfb_close(got, ref, what=f"synthesis spans={spans} dr={deripple} {taper}")


def test_synthesis_literal_agreement_small(gpu):
    """GPU vs the literal (statement-by-statement) transliteration."""
    import torch
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(22), (1, 8, 96 * 3 + 32))
    t_orc = orc.pfb_window("tukey", 128, 16)
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    ref = orc.polyphase_synthesis_literal(x, 1, 128, "8/7", dr, 1, 16, t_orc)
    got = pfb.polyphase_synthesis(torch.from_numpy(x).cuda(), 1, 128, "8/7", dr, 1, 16,
                                  pfb.PFBWindow().lookup["tukey"](128, 16)).cpu().numpy()
    assert_pfb_close(got, ref)


@pytest.mark.parametrize("combine", [2, 4])
def test_synthesis_combine(gpu, combine):
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(23 + combine), (1, 8, 96 * 4 + 32))
    got, ref = _synth_case(pfb, x, 0, 128, "8/7", 0, taps, 16, "tukey", combine=combine)
    assert_pfb_close(got, ref)


def test_synthesis_sample_offset(gpu):
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(24), (1, 8, 96 * 4 + 32 + 9))
    got, ref = _synth_case(pfb, x, 1, 128, "8/7", 1, taps, 16, "tukey", sample_offset=7)
    assert_pfb_close(got, ref)


def test_synthesis_execute_into_out_buffer(gpu):
    """SynthesisPlan.execute(..., out=buf) (the bench's graph-captured synthesis-only leg)
    writes the same samples as the allocating call, bit for bit, into a wider buffer's
    rows; a buffer too short is refused before any launch."""
    import torch
    pfb = _pfb()
    taps = _taps("low87")
    N, nf, ov = 256, 256, 48
    x = _noise(np.random.default_rng(31), (2, 6 * 160 + 2 * ov + 3, N)).astype(np.complex64)
    win = pfb.PFBWindow().lookup["tukey"](nf, ov)
    syn = pfb.SynthesisPlan(N, "8/7", nf, ov, True, 1, True, taps, win, None, 2, 0)
    chan = torch.from_numpy(x).cuda()
    ref = syn.execute(chan, layout="ptc").cpu().numpy()
    buf = torch.full((2, ref.shape[1] + 5), complex(7.0, -7.0), dtype=torch.complex64, device="cuda")
    got = syn.execute(chan, layout="ptc", out=buf)
    torch.cuda.synchronize()
    assert got.data_ptr() == buf.data_ptr()
    np.testing.assert_array_equal(got.cpu().numpy(), ref)
    assert (buf[:, ref.shape[1]:].cpu().numpy() == np.complex64(7 - 7j)).all()
    with pytest.raises(ValueError):
        syn.execute(chan, layout="ptc", out=buf[:, : ref.shape[1] - 1].contiguous())
    syn.close()


@pytest.mark.parametrize("N,os_,nf,ov,blocks", [
    (256, "8/7", 256, 48, 12),
    (256, "4/3", 256, 48, 10),
    (4096, "8/7", 512, 128, 3),
])
def test_synthesis_baseline_shapes(gpu, N, os_, nf, ov, blocks):
    pfb = _pfb()
    taps = _taps({"8/7": "low87", "4/3": "low43"}[os_]) if N == 256 else _taps("mid")
    keep = nf - 2 * ov
    x = _noise(np.random.default_rng(N + blocks), (1, N, blocks * keep + 2 * ov + 3))
    got, ref = _synth_case(pfb, x, 1, nf, os_, 1, taps, ov, "tukey")
    assert_pfb_close(got, ref, what=f"synthesis N={N} {os_}")


@pytest.mark.parametrize("N", [8, 64])
@pytest.mark.parametrize("spans", [1, 0])
@pytest.mark.parametrize("deripple,taper", [(1, "tukey"), (0, "hann"), (1, "top_hat")])
def test_synthesis_nf512_wave_kernel(gpu, N, spans, deripple, taper):
    """The SKA-Mid synthesis shape (Nf 512, W 448, Ov 128: synth_wave512_kernel) at small
    channel counts: spans and critical kept-bin orders, deripple on/off, three tapers, two
    polarisations, a sample offset and a ragged tail, against the oracle."""
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(N, "8/7", 12)
    x = _noise(np.random.default_rng(60 + N + 3 * spans), (2, N, 7 * 256 + 256 + 11))
    got, ref = _synth_case(pfb, x, spans, 512, "8/7", deripple, taps, 128, taper, sample_offset=3)
    assert_pfb_close(got, ref, what=f"synthesis Nf 512 N={N} spans={spans} dr={deripple} {taper}")


@pytest.mark.parametrize("spans", [1, 0])
def test_synthesis_nf512_wave_kernel_non_flat_window(gpu, spans):
    """The wave kernels skip the taper multiply where the window is exactly 1 (rows
    [128, 384) at Nf 512: tukey, top_hat, no_window); an explicit window that is not runs
    the general taper — against the oracle with the same coefficients."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(64, "8/7", 12)
    x = _noise(np.random.default_rng(77 + spans), (2, 64, 7 * 256 + 256 + 11))
    t = np.arange(512)
    win = orc.tukey_window_coeffs(512, 128)
    win = win * (0.75 + 0.25 * np.cos(2 * np.pi * t / 512))
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    ref = orc.polyphase_synthesis(x, spans, 512, "8/7", dr, 3, 128, lambda a, nf, ov: a * win[None, :])
    got = pfb.polyphase_synthesis(torch.from_numpy(x).cuda(), spans, 512, "8/7", dr, 3, 128,
                                  pfb.PFBWindow().custom(win))
    assert_pfb_close(got.cpu().numpy(), ref, what=f"synthesis Nf 512 non-flat window spans={spans}")


@pytest.mark.parametrize("taper,combine", [("tukey", 1), ("hann", 1), ("tukey", 2)])
def test_synthesis_4096_persistent_chan_ifft(gpu, taper, combine):
    """4096-channel synthesis with more than 2048 channelised rows in one chunk: the
    stage-1 channel IFFT runs as row_fft_persist_kernel, plain, with the temporal 'hann'
    per-channel gain (GAIN) and with the combine permutation (PERM)."""
    pfb = _pfb()
    taps = _taps("mid")
    x = _noise(np.random.default_rng(43), (1, 4096, 8 * 256 + 256 + 3))
    got, ref = _synth_case(pfb, x, 1, 512, "8/7", 1, taps, 128, taper, combine=combine)
    assert_pfb_close(got, ref, what=f"synthesis 4096 ch, {taper}, combine {combine}")


def test_synthesis_chunking_invariant(gpu):
    """Chunked channel-IFFT/block kernels give identical output for any chunk size."""
    import torch
    pfb = _pfb()
    x = torch.from_numpy(_noise(np.random.default_rng(31), (1, 256, 160 * 11 + 96))).cuda()
    plan = pfb.SynthesisPlan(256, "8/7", 256, 48, True, 1, False, None, "tukey", None, 1)
    a = plan.execute(x)
    plan.set_chunk_blocks(3)
    b = plan.execute(x)
    plan.set_chunk_blocks(1)
    c = plan.execute(x)
    assert torch.equal(a, b) and torch.equal(a, c)


def test_synthesis_nf512_chunking_invariant(gpu):
    """The SKA-Mid wave synthesis over chunks of 1, 2 and 5 blocks (block0 > 0, ranges
    shorter than the reuse window) equals the one-chunk call bit for bit, two pols."""
    import torch
    pfb = _pfb()
    x = torch.from_numpy(_noise(np.random.default_rng(32), (2, 64, 256 * 11 + 256 + 7))).cuda()
    plan = pfb.SynthesisPlan(64, "8/7", 512, 128, True, 1, False, None, "tukey", None, 2)
    a = plan.execute(x)
    for cb in (5, 2, 1):
        plan.set_chunk_blocks(cb)
        assert torch.equal(plan.execute(x), a), f"chunk {cb}"


def test_synthesis_rejects_real_input(gpu):
    pfb = _pfb()
    with pytest.raises(ValueError):
        pfb.polyphase_synthesis(np.zeros((1, 8, 400), dtype=np.float32), 1, 128, "8/7")


def test_synthesis_invalid_args(gpu):
    pfb = _pfb()
    x = _noise(np.random.default_rng(0), (1, 8, 400))
    with pytest.raises(pfb.PfbError):
        # Nf*de/nu not integral
        pfb.polyphase_synthesis(x, 1, 100, "8/7", None, 1, 16)


# ----------------------------------------------------------------------------- round trip
def test_round_trip_test_config(gpu):
    """C1: 'test' config, complex sinusoid (bin 3, pi/4) through analysis -> synthesis."""
    import torch
    pfb = _pfb()
    cfg = pfb.default_config("test")
    taps = _taps("test")
    n = 3 * 112 * 8 + 1000
    x = _tone(n, 3, n_pol=2)
    chan = pfb.polyphase_analysis(torch.from_numpy(x).cuda(), taps, 8, cfg.os_factor)
    win = pfb.PFBWindow().lookup["tukey"](128, 16)
    out = pfb.polyphase_synthesis(chan, 1, 128, cfg.os_factor,
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 16, win)
    ref_chan = orc.polyphase_analysis(x, taps, 8, "8/7")
    ref = orc.polyphase_synthesis(ref_chan, 1, 128, "8/7",
                                  {"apply_deripple": 1, "filter_coeff": taps}, 1, 16,
                                  orc.pfb_window("tukey", 128, 16))
    assert_pfb_close(out.cpu().numpy(), ref, scale=1.0, what="C1 round trip (raw)")


# ----------------------------------------------------------------------------- streaming
def test_filterbank_streaming_matches_oracle(gpu):
    pfb = _pfb()
    taps = _taps("test")
    cfg = dict(analysis_function="polyphase_analysis", filt_coeff=taps, channels=8,
               os_factor="8/7")
    fb = pfb.FilterBank(cfg)
    ofb = orc.FilterBankOracle(taps, 8, "8/7")
    rng = np.random.default_rng(41)
    for n in (1000, 777, 2048, 5, 3001):
        x = _noise(rng, (2, 1, n))
        fb, got = fb.execute(x)
        ref = ofb.execute(x)
        assert got.shape == ref.shape
        if ref.size:
            assert_pfb_close(got, ref)
        assert fb.buffered_samples == ofb.buffered_samples


def test_filterbank_stream_equals_one_shot(gpu):
    """Carry-over makes chunked Bunton analysis identical to a single call."""
    import torch
    pfb = _pfb()
    taps = _taps("low87")
    cfg = dict(analysis_function="polyphase_analysis", filt_coeff=taps, channels=256,
               os_factor="8/7")
    x = torch.from_numpy(_noise(np.random.default_rng(42), (1, 1, 1 << 17))).cuda()
    fb = pfb.FilterBank(cfg)
    parts = []
    for a, b in ((0, 40000), (40000, 90001), (90001, 1 << 17)):
        fb, y = fb.execute(x[:, :, a:b])
        parts.append(y)
    streamed = torch.cat(parts, dim=2)
    whole = pfb.polyphase_analysis(x, taps, 256, "8/7")
    assert torch.equal(streamed, whole[:, :, :streamed.shape[2]])


@pytest.mark.parametrize("os_,tpc", [("8/7", 12), ("4/3", 12), ("8/7", 11)])
def test_filterbank_stream_carry_in_place(gpu, os_, tpc):
    """Streaming FilterBank on the 256-channel streaming kernel with carried samples: the
    rows that read only the new input run on it in place (the carry as a read offset),
    the first ones on a small stitched buffer (pfb_filterbank_execute).  Chunks include
    ones shorter than the carry (the concatenating path) and two polarisations; the
    result equals the one-shot analysis bit for bit and the streaming oracle at 1e-6."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, os_, tpc)
    cfg = dict(analysis_function="polyphase_analysis", filt_coeff=taps, channels=256,
               os_factor=os_)
    n_tot = 70000 + 5 + 3001 + 40000 + 123457
    x = torch.from_numpy(_noise(np.random.default_rng(43), (2, 1, n_tot))).cuda()
    fb = pfb.FilterBank(cfg)
    ofb = orc.FilterBankOracle(taps, 256, os_)
    parts, a = [], 0
    for n in (70000, 5, 3001, 40000, 123457):
        fb, y = fb.execute(x[:, :, a:a + n])
        ref = ofb.execute(x[:, :, a:a + n].cpu().numpy())
        assert y.shape == ref.shape and fb.buffered_samples == ofb.buffered_samples
        if ref.size:
            assert_pfb_close(y.cpu().numpy(), ref, what=f"stream chunk {n}")
        parts.append(y)
        a += n
    streamed = torch.cat(parts, dim=2)
    whole = pfb.polyphase_analysis(x, taps, 256, os_)
    assert torch.equal(streamed, whole[:, :, :streamed.shape[2]])


@pytest.mark.parametrize("os_", ["8/7", "4/3"])
def test_filterbank_stream_long_carry_one_launch(gpu, os_):
    """Carries longer than P N (up to P N + NU M samples: the nu-trimmed rows' samples stay
    buffered, FilterBank.m:93-104,119-126) are read through the streaming kernel's carry
    descriptor in its first register window (DE 16/NU + P rows) — one launch per call,
    no stitched rows (round 5; the bound was P N).  Every call must equal the one-shot
    analysis bit for bit, and the chunk lengths are chosen so that such carries occur."""
    import torch
    pfb = _pfb()
    taps = pfb.design_PFB_FIR_filter(256, os_, 12)
    cfg = dict(analysis_function="polyphase_analysis", filt_coeff=taps, channels=256,
               os_factor=os_)
    fb = pfb.FilterBank(cfg)
    nu, de = (8, 7) if os_ == "8/7" else (4, 3)
    M, P = 256 * de // nu, -(-len(taps) // 256)
    chunks = [50000 + 977 * i for i in range(12)]
    x = torch.from_numpy(_noise(np.random.default_rng(44), (1, 1, sum(chunks)))).cuda()
    parts, a, long_carries = [], 0, 0
    for n in chunks:
        b = fb.buffered_samples
        if P * 256 < b <= (de * 16 // nu + P) * 256:
            long_carries += 1
        fb, y = fb.execute(x[:, :, a:a + n])
        parts.append(y)
        a += n
    assert long_carries >= 2, long_carries
    streamed = torch.cat(parts, dim=2)
    whole = pfb.polyphase_analysis(x, taps, 256, os_)
    assert torch.equal(streamed, whole[:, :, :streamed.shape[2]])


def test_filterbank_stream_padded(gpu):
    """Streaming FilterBank on the SKA-Mid padded (commutator) analysis: 4096 channels,
    100 353 two-stage taps, 8/7 (FilterBank.m:85-126 calling polyphase_analysis_padded).
    The Matlab object calls the padded analysis on carry + chunk every time, so each call
    restarts the commutator with zero history (polyphase_analysis_padded.m:101-102) and
    circularly shifts its own rows by -sds (:156) — the reference defect SURVEY §8(c)
    names; the engine reproduces it by running the analysis over the concatenated call
    input (pfb_filterbank_execute: all K rows, the nu-trimmed Kt copied out).  Chunks are
    shorter than M (3584: no output row, everything carried), shorter and longer than
    P N (102 400), and two polarisations; every chunk is compared with the oracle object
    and the carry lengths must match."""
    import torch
    pfb = _pfb()
    taps = _taps("mid")
    cfg = dict(analysis_function="polyphase_analysis_padded", filt_coeff=taps, channels=4096,
               os_factor="8/7")
    fb = pfb.FilterBank(cfg)
    ofb = orc.FilterBankOracle(taps, 4096, "8/7", "polyphase_analysis_padded")
    rng = np.random.default_rng(47)
    chunks = (3000, 131072, 50000, 2000, 262144, 100000, 1 << 17)
    for i, n in enumerate(chunks):
        x = _noise(rng, (2, 1, n))
        xd = torch.from_numpy(x).to(gpu) if i % 2 else x  # device and host inputs
        fb, got = fb.execute(xd)
        ref = ofb.execute(x)
        got = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
        assert got.shape == ref.shape, (n, got.shape, ref.shape)
        if ref.size:
            assert_pfb_close(got, ref, what=f"padded stream chunk {i} ({n} samples)")
        assert fb.buffered_samples == ofb.buffered_samples, (n, fb.buffered_samples,
                                                             ofb.buffered_samples)


def test_inverse_filterbank_streaming_matches_oracle(gpu):
    pfb = _pfb()
    taps = _taps("test")
    cfg = dict(filt_coeff=taps, channels=8, os_factor="8/7", input_fft_length=128,
               input_overlap=16, deripple=True, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg)
    oifb = orc.InverseFilterBankOracle(taps, 8, "8/7", 128, 16, "tukey", deripple=True)
    rng = np.random.default_rng(43)
    for n in (500, 333, 1000, 20, 777):
        x = _noise(rng, (2, 8, n))
        ifb, got = ifb.execute(x)
        ref = oifb.execute(x)
        assert got.shape == ref.shape, (got.shape, ref.shape)
        if ref.size:
            assert_pfb_close(got, ref)
        assert ifb.buffered_samples == oifb.buffered_samples


@pytest.mark.parametrize("N,nf,ov,chunks", [
    (8, 128, 16, (500, 333, 1000, 20, 777)),
    (256, 256, 48, (1000, 161, 5000, 3, 2222)),
])
def test_inverse_filterbank_stream_carry_in_place(gpu, N, nf, ov, chunks):
    """Streaming InverseFilterBank on device tensors with carried rows: blocks that read
    only the new input run on it in place (a row shift), the first ones on a small
    stitched buffer (pfb_inverse_filterbank_execute); every chunk against the oracle."""
    import torch
    pfb = _pfb()
    taps = _taps("test") if N == 8 else _taps("low87")
    cfg = dict(filt_coeff=taps, channels=N, os_factor="8/7", input_fft_length=nf,
               input_overlap=ov, deripple=True, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg)
    oifb = orc.InverseFilterBankOracle(taps, N, "8/7", nf, ov, "tukey", deripple=True)
    rng = np.random.default_rng(44)
    for n in chunks:
        x = _noise(rng, (2, N, n))
        try:
            ref = oifb.execute(x)
        except ValueError:
            # no complete block and the carry rounded past the data (InverseFilterBank.m:
            # 104-122 indexes before the first sample): rejected, state unchanged
            with pytest.raises(pfb.PfbError):
                ifb.execute(torch.from_numpy(x).to(gpu))
            continue
        ifb, got = ifb.execute(torch.from_numpy(x).to(gpu))
        assert tuple(got.shape) == ref.shape, (got.shape, ref.shape)
        if ref.size:
            assert_pfb_close(got.cpu().numpy(), ref, what=f"inverse stream N={N} chunk {n}")
        assert ifb.buffered_samples == oifb.buffered_samples


@pytest.mark.parametrize("N,nf,ov,so,chunks,device", [
    (8, 128, 16, 5, (500, 333, 1000, 20, 777), False),
    (8, 128, 16, 37, (300, 2000, 96, 1234), True),
    (8, 128, 16, 200, (150, 700, 2100), True),          # offset longer than a block
    (256, 256, 48, 17, (1000, 161, 5000, 3, 2222), True),
])
def test_inverse_filterbank_sample_offset_matches_oracle(gpu, N, nf, ov, so, chunks, device):
    """InverseFilterBank.sample_offset != 0 (InverseFilterBank.m:12,92-96): every call
    synthesises the concatenated carry + input from row sample_offset on, and the carry
    starts at the consumed blocks' end (:104-133) — against InverseFilterBankOracle (its
    literal restatement) over several chunkings, host and device inputs, with the carry
    in place (row shift) and stitched."""
    import torch
    pfb = _pfb()
    taps = _taps("test") if N == 8 else _taps("low87")
    cfg = dict(filt_coeff=taps, channels=N, os_factor="8/7", input_fft_length=nf,
               input_overlap=ov, deripple=True, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg)
    ifb.sample_offset = so
    oifb = orc.InverseFilterBankOracle(taps, N, "8/7", nf, ov, "tukey", deripple=True, sample_offset=so)
    rng = np.random.default_rng(45 + so)
    produced = 0
    for n in chunks:
        x = _noise(rng, (2, N, n))
        xin = torch.from_numpy(x).to(gpu) if device else x
        try:
            ref = oifb.execute(x)
        except ValueError:
            with pytest.raises(pfb.PfbError):
                ifb.execute(xin)
            continue
        ifb, got = ifb.execute(xin)
        got = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
        assert got.shape == ref.shape, (n, got.shape, ref.shape)
        if ref.size:
            assert_pfb_close(got, ref, what=f"inverse stream offset {so} N={N} chunk {n}")
        produced += ref.shape[2]
        assert ifb.buffered_samples == oifb.buffered_samples
    assert produced > 0


# ----------------------------------------------------------------------------- spectral taper
# polyphase_synthesis.m:282 (FFFF = spectral_taper(FFFF, L, Ov)) through
# InverseFilterBank.frequency_taper (InverseFilterBank.m:48-61); 'hann' on the L-vector
# is circshift(hann(L), L/2) (PFBWindow.m:83-95).  GPU path: pfb_spectral.hip.
@pytest.mark.parametrize("spans", [1, 0])
@pytest.mark.parametrize("deripple", [1, 0])
def test_synthesis_spectral_hann_matches_oracle(gpu, spans, deripple):
    import torch
    pfb = _pfb()
    taps = _taps("test")
    x = _noise(np.random.default_rng(51), (2, 8, 96 * 5 + 32 + 3))
    dr = {"apply_deripple": deripple, "filter_coeff": taps}
    ref = orc.polyphase_synthesis(x, spans, 128, "8/7", dr, 1, 16, orc.pfb_window("tukey", 128, 16),
                                  orc.pfb_window("hann", 128, 16))
    w = pfb.PFBWindow()
    got = pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), spans, 128, "8/7", dr, 1, 16,
                                  w.lookup["tukey"](128, 16), w.lookup["hann"](128, 16))
    assert_pfb_close(got.cpu().numpy(), ref, what=f"spectral hann spans={spans} dr={deripple}")


def test_synthesis_spectral_hann_c2prime(gpu):
    """C2' shape (SKA-Low 256 ch, 4/3, Nf 256, Ov 48, deripple) with the hann spectral taper."""
    import torch
    pfb = _pfb()
    taps = _taps("low43")
    x = _noise(np.random.default_rng(52), (1, 256, 160 * 6 + 96 + 7))
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    ref = orc.polyphase_synthesis(x, 1, 256, "4/3", dr, 1, 48, orc.pfb_window("tukey", 256, 48),
                                  orc.pfb_window("hann", 256, 48))
    w = pfb.PFBWindow()
    got = pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), 1, 256, "4/3", dr, 1, 48,
                                  w.lookup["tukey"](256, 48), w.lookup["hann"](256, 48))
    assert_pfb_close(got.cpu().numpy(), ref, what="C2' spectral hann")


def test_synthesis_spectral_custom_and_combine(gpu):
    """Explicit L spectral coefficients (API extension), critical + combine 2."""
    import torch
    pfb = _pfb()
    taps = _taps("test")
    L = 112 * 8
    coeffs = np.random.default_rng(53).uniform(0.2, 1.0, L)
    x = _noise(np.random.default_rng(54), (1, 8, 96 * 4 + 32))

    def taper(a, *args):
        return coeffs[:, None] * a

    ref = orc.polyphase_synthesis(x, 0, 128, "8/7", None, 1, 16, orc.pfb_window("tukey", 128, 16),
                                  taper, 2)
    w = pfb.PFBWindow()
    got = pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), 0, 128, "8/7", None, 1, 16,
                                  w.lookup["tukey"](128, 16), w.custom(coeffs), 2)
    assert_pfb_close(got.cpu().numpy(), ref, what="custom spectral taper, combine 2")
    with pytest.raises(ValueError):
        pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), 0, 128, "8/7", None, 1, 16,
                                None, w.custom(coeffs[:100]))
    with pytest.raises(pfb.PfbError):  # tukey has no meaning on the L-vector
        pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), 0, 128, "8/7", None, 1, 16,
                                None, w.lookup["tukey"](128, 16))


@pytest.mark.parametrize("so,chunks", [(5, (500, 333, 1000)), (200, (150, 700, 2100))])
@pytest.mark.parametrize("device", [False, True])
def test_inverse_filterbank_sample_offset_spectral_taper(gpu, so, chunks, device):
    """sample_offset != 0 together with frequency_taper('hann') (InverseFilterBank.m:48-61,
    92-96): the spectral-taper path takes the offset as a negative row shift into the
    concatenated carry + input (pfb_api.hip synthesis_chunk) — against
    InverseFilterBankOracle over several chunks, host and device input."""
    import torch
    pfb = _pfb()
    taps = _taps("test")
    cfg = dict(filt_coeff=taps, channels=8, os_factor="8/7", input_fft_length=128,
               input_overlap=16, deripple=False, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg).frequency_taper("hann")
    ifb.sample_offset = so
    oifb = orc.InverseFilterBankOracle(taps, 8, "8/7", 128, 16, "tukey",
                                       sample_offset=so).frequency_taper("hann")
    rng = np.random.default_rng(57 + so)
    produced = 0
    for n in chunks:
        x = _noise(rng, (2, 8, n))
        xin = torch.from_numpy(x).to(gpu) if device else x
        try:
            ref = oifb.execute(x)
        except ValueError:
            with pytest.raises(pfb.PfbError):
                ifb.execute(xin)
            continue
        ifb, got = ifb.execute(xin)
        got = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
        assert got.shape == ref.shape, (n, got.shape, ref.shape)
        if ref.size:
            assert_pfb_close(got, ref, what=f"inverse hann offset {so} chunk {n}")
        produced += ref.shape[2]
        assert ifb.buffered_samples == oifb.buffered_samples
    assert produced > 0


def test_inverse_filterbank_frequency_taper_stream(gpu):
    """InverseFilterBank.frequency_taper('hann') (InverseFilterBank.m:48-61) streaming."""
    pfb = _pfb()
    taps = _taps("test")
    cfg = dict(filt_coeff=taps, channels=8, os_factor="8/7", input_fft_length=128,
               input_overlap=16, deripple=False, temporal_taper="tukey")
    ifb = pfb.InverseFilterBank(cfg).frequency_taper("hann")
    oifb = orc.InverseFilterBankOracle(taps, 8, "8/7", 128, 16, "tukey").frequency_taper("hann")
    rng = np.random.default_rng(55)
    for n in (500, 333, 1000):
        x = _noise(rng, (2, 8, n))
        ifb, got = ifb.execute(x)
        ref = oifb.execute(x)
        assert got.shape == ref.shape
        if ref.size:
            assert_pfb_close(got, ref, what=f"inverse filterbank hann n={n}")


@pytest.mark.parametrize("N,os_,nf,ov,spans", [
    (256, "32/27", 256, 48, 1),   # 'sps': normalize(os, Ov) = 40.5 -> L_ov = 10368 = 40.5 N
    (8, "32/27", 256, 16, 1),     # L_ov = 108 = 13.5 N (the pair-store block kernel)
    (8, "8/7", 128, 7, 0),        # L_ov = 49: odd (single-sample stores), critical
])
def test_synthesis_fractional_output_overlap(gpu, N, os_, nf, ov, spans):
    """output_overlap = normalize(os, Ov) * n_chan (polyphase_synthesis.m:117) need not be a
    multiple of n_chan: the kept samples iFFFF(output_overlap + 1 : L - output_overlap)
    (:302) then start mid-way through a t1 row.  The kernels discard sample-exactly
    (offset t0 + N t1 - L_ov, range-checked)."""
    import torch
    pfb = _pfb()
    tpc = 24 if os_ == "32/27" and N == 256 else 10
    taps = pfb.design_PFB_FIR_filter(N, os_, tpc)
    x = _noise(np.random.default_rng(61), (2, N, (nf - 2 * ov) * 7 + 2 * ov + 5))
    dr = {"apply_deripple": 1, "filter_coeff": taps}
    win = orc.pfb_window("tukey", nf, ov)
    ref = orc.polyphase_synthesis(x, spans, nf, os_, dr, 1, ov, win)
    got = pfb.polyphase_synthesis(torch.from_numpy(x).to(gpu), spans, nf, os_, dr, 1, ov,
                                  pfb.PFBWindow().lookup["tukey"](nf, ov))
    assert_pfb_close(got.cpu().numpy(), ref, what=f"synthesis {N} ch {os_} Ov {ov}")
