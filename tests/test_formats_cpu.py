"""CPU tests of the data-format host logic: DADA header read/write (read_header.m,
write_header.m semantics), the oracle's layout restatements and Matlab rounding,
and the harness' naming helpers.  No device needed."""
import io

import numpy as np
import pytest

from oracle import pfb_oracle as orc


def _dada():
    from ska_pst_dsp_model_amd import dada
    return dada


def test_header_round_trip_and_order():
    dada = _dada()
    hdr = {"NCHAN": "256", "HDR_SIZE": "4096", "OS_FACTOR": "8/7", "A_KEY": "1"}
    f = io.BytesIO()
    dada.write_header(f, hdr)
    raw = f.getvalue()
    assert len(raw) == 4096
    text = raw.rstrip(b"\0").decode()
    lines = text.strip("\n").split("\n")
    assert lines[0] == "HDR_SIZE 4096"
    assert lines[1:] == ["A_KEY 1", "NCHAN 256", "OS_FACTOR 8/7"]  # containers.Map order
    assert dada.read_header(io.BytesIO(raw)) == hdr


def test_header_grows_when_too_long():
    dada = _dada()
    hdr = {"HDR_SIZE": "4096", "COEFF_0": ",".join(["1.000000E+00"] * 500)}
    f = io.BytesIO()
    dada.write_header(f, hdr)
    raw = f.getvalue()
    assert len(raw) == 8192
    h = dada.read_header(io.BytesIO(raw + b"\x01" * 100))
    assert h["HDR_SIZE"] == "8192" and h["COEFF_0"] == hdr["COEFF_0"]


def test_header_comments_and_missing_size():
    dada = _dada()
    text = b"# comment line\nHDR_VERSION 1.0\nNBIT 8 trailing words\n"
    h = dada.read_header(io.BytesIO(text))
    assert h == {"HDR_VERSION": "1.0", "NBIT": "8"}


def test_add_fir_filter_to_header():
    dada = _dada()
    h = dada.add_fir_filter_to_header({}, np.array([0.5, -1.25e-3]), "8/7")
    assert h == {"NSTAGE": "1", "COEFF_0": "5.000000E-01,-1.250000E-03", "OVERSAMP_0": "8/7",
                 "NTAP_0": "2"}


def test_matlab_round_half_away_from_zero():
    v = np.array([0.5, -0.5, 1.5, -1.5, 2.5, -2.5, 0.49999997, 2.0])
    assert np.array_equal(orc.matlab_round(v), [1, -1, 2, -2, 3, -3, 0, 2])


def test_oracle_dada_layouts():
    # TFP: sample index = p + P (c + C t), re/im interleaved
    P, C, T = 2, 3, 5
    x = np.arange(P * C * T) * (1 + 2j)
    x = x.reshape((P, C, T), order="F")
    flat = orc.write_dada_data(x, 64)
    for p in range(P):
        for c in range(C):
            for t in range(T):
                e = p + P * (c + C * t)
                assert flat[2 * e] == x[p, c, t].real and flat[2 * e + 1] == x[p, c, t].imag
    assert np.array_equal(orc.reshape_dada_data(flat, 2, P, C), x)
    # LowCBF heap: [heap][chan][pol][sample]
    raw = np.arange(2 * P * C * 32 * 2, dtype=np.float64)
    y = orc.reshape_low_cbf_data(raw, 2, P, C)
    h, c, p, s = 1, 2, 1, 7
    e = ((h * C + c) * P + p) * 32 + s
    assert y[p, c, h * 32 + s] == raw[2 * e] + 1j * raw[2 * e + 1]


def test_oracle_write_saturates_integers():
    x = np.array([[[300.4 - 300.6j, 127.5 + 0.5j, -128.5 - 0.49j]]])
    assert orc.write_dada_data(x, 8).tolist() == [127, -128, 127, 1, -128, 0]


def test_harness_names():
    from ska_pst_dsp_model_amd import harness
    assert harness.create_output_file_names(None, "a.b") == ("a.b", "a.b.log", "a.b.dump")
    assert harness.create_output_file_names("x.dump", "q") == ("x", "x.log", "x.dump")
    assert harness._num2str(241.92) == "241.92"
    assert harness._num2str(2.0) == "2"
    assert harness._num2str(1.0 / 7) == "0.14286"


def test_verify_metrics_match_util_definitions():
    from ska_pst_dsp_model_amd import verify
    a = np.array([1.0, 0.1, 0.01, 3.0])
    assert np.array_equal(verify.spurious(a), [1.0, 0.1, 0.01, 0.0])
    p = np.abs(a) ** 2
    assert np.isclose(verify.total_spurious(a), 10 * np.log10(1 + 0.01 + 1e-4 + 1e-13))
    assert np.isclose(verify.max_spurious(a), 10 * np.log10(1 + 1e-13))
    assert np.isclose(verify.mean_spurious(a), 10 * np.log10((p.sum() - 9) / 4 + 1e-13))
    al = verify.purity_alignment(8, "8/7", 128, 16, 81, 3)
    assert al == {"normalize": 1024, "block_size": 896, "fft_size": 1792, "n_samples": 2688,
                  "output_sample_shift": 112, "total_sample_shift": 152}


# ------------------------------------------------------------------ C5 purity scoring
def test_c5_alignment_constants_mid():
    """current_performance.m:203-235 + test_data_pipeline.m:136 for sub-config 'mid'
    (fir_offset_direction 0, kludge_offset 0): the chop offset equals the padded bank's
    round-trip delay pinned in test_oracle.test_c3_impulse_delay_and_gain (458 751)."""
    from ska_pst_dsp_model_amd import verify
    al = verify.performance_alignment(4096, "8/7", 512, 128, 100353, 3, 0, 0)
    assert al["block_size"] == 1835008 and al["nbins"] == 5505024
    assert al["additional_offset"] - al["fir_offset"] == 458751
    assert al["filt_offset"] == 50176 and al["fft_length"] == 3670016
    items = verify.sweep_vectors(al, 300, 3)
    t = [p for d, p in items if d == "time"]
    f = [p for d, p in items if d == "freq"]
    assert len(f) == 300 and f[0] == 3 and f[1] == 6118 * 3
    assert t[0] == 1 and 50176 in t and 50176 + 917504 in t
    # round-robin over 8 GPUs covers every vector exactly once
    shares = [verify.shard(items, r, 8) for r in range(8)]
    assert sorted(sum(shares, [])) == sorted(items)


def test_c5_scoring_matches_reference_on_oracle():
    """The C5 scoring (chop.m, DomainPerformance.m, ErrorAnalysis.m) on oracle round
    trips of the reference's 'low' sub-config (Bunton, 256 ch, 4/3, fir_offset_direction
    -1, kludge_offset 1): every impulse whose response lies in the output comes back at
    its aligned index with <= -60 dB outside +-1 sample (TestImpulse.m:46-73), every
    grid tone has <= -60 dB spurious spectral power (TestPureTone.m:55-89)."""
    from oracle import pfb_oracle as orc
    from ska_pst_dsp_model_amd import firio, verify
    taps = firio.design_PFB_FIR_filter(256, "4/3", 12)
    al = verify.performance_alignment(256, "4/3", 256, 48, len(taps), 3, -1, 1)
    win = orc.pfb_window("tukey", 256, 48)
    items = verify.sweep_vectors(al, 4, 3)
    scored = 0
    for kind, p in items:
        x = verify.time_domain_impulse(al["nbins"], p) if kind == "time" else \
            verify.complex_sinusoid(al["nbins"], p)
        ch = orc.polyphase_analysis(x[None, None, :], taps, 256, "4/3")
        y = orc.polyphase_synthesis(ch, 1, 256, "4/3", {"apply_deripple": 1, "filter_coeff": taps},
                                    1, 48, win)[0, 0]
        r = verify.score_vector(kind, p, x, y, al)
        if kind == "time" and "expected_index" in r:
            assert r["peak_index"] == r["expected_index"], r
            assert r["max_outside_pm1_dB"] <= -60.0, r
            scored += 1
        elif kind == "freq":
            assert r["max_spurious_dB"] <= -60.0, r
            scored += 1
    assert scored >= 8


# ------------------------------------------------------------------ sgcht testers
def test_sgcht_generators_carry_state():
    """PureTone.m / Impulse.m: the phase (and the delta position) continue across calls."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    g = sgcht.PureTone(frequency=0.25)
    _, a = g.generate(6)
    _, b = g.generate(6)
    whole = sgcht.PureTone(frequency=0.25).generate(12)[1]
    assert np.array_equal(np.concatenate([a, b], axis=2), whole)
    imp = sgcht.Impulse(offset=7, noise=0.0)
    _, x1 = imp.generate(5)
    _, x2 = imp.generate(5)
    assert not x1.any() and x2[0, 0, 2] == 1.0 and np.count_nonzero(x2) == 1


def test_sgcht_testers_match_matlab_rules():
    """TestPureTone.m: peak at frequency * nfft + 1 (1-based), else fail; every other bin
    <= -60 dB re the peak.  TestImpulse.m: nothing above -60 dB (absolute) outside +-1 of
    offset - current + 1; current advances by the block length."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    t = np.arange(1024)
    tone = np.exp(2j * np.pi * 0.25 * t)[None, None, :]
    assert sgcht.TestPureTone(frequency=0.25).test(tone)[1] == 0
    assert sgcht.TestPureTone(frequency=0.125).test(tone)[1] == -1          # wrong bin
    spur = tone + 2e-3 * np.exp(2j * np.pi * 0.5 * t)[None, None, :]        # -54 dB
    assert sgcht.TestPureTone(frequency=0.25).test(spur)[1] == -1
    x = np.zeros((1, 1, 100), np.complex64)
    x[0, 0, 40] = 1.0
    x[0, 0, 41] = 0.5
    ti = sgcht.TestImpulse(offset=40)   # 1-based off = 41: samples 40..42 (1-based) exempt
    assert ti.test(x)[1] == 0 and ti.current == 100
    x2 = np.zeros((1, 1, 100), np.complex64)
    x2[0, 0, 45] = 2e-3                  # -54 dB, next block
    assert sgcht.TestImpulse(offset=40).test(x2)[1] == -1


def test_sgcht_without_channelizer_passes():
    """sgcht(signal=..., test=true) with no cfg: the generators straight into the testers
    (the first case of test_sgcht.m) — no device needed."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    assert sgcht.sgcht(signal="complex_sinusoid", test=True, blocks=3, blocksz=4096).result == 0
    r = sgcht.sgcht(signal="temporal_impulse", test=True, blocks=3, blocksz=16384)
    assert r.result == 0 and r.tester.current == 3 * 16384


def test_test_impulse_does_not_advance_on_failure():
    """TestImpulse.m:67-70 returns -1 without advancing obj.current."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    x = np.zeros((1, 1, 100), np.complex64)
    x[0, 0, 70] = 1.0
    t = sgcht.TestImpulse(offset=10)
    assert t.test(x)[1] == -1 and t.current == 0


def test_frequency_comb_generator_and_harmonics():
    """FrequencyComb.m: the single-precision sum of its PureTones, phase carried across
    calls; sgcht.m:394-431's harmonic grid with the quarter-channel offsets."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    amps, f = sgcht.comb_harmonics()
    assert f.size == 32 and np.isclose(f[0], -0.5 + 1 / 128) and np.isclose(f[1] - f[0], 1 / 32)
    assert np.isclose(amps[0], 1.0) and np.isclose(amps[-1], np.sqrt(2))
    _, f1 = sgcht.comb_harmonics(256)
    assert np.isclose(f1[0] - f[0], 1 / 1024)
    _, f2 = sgcht.comb_harmonics(256, two_stage=True, invert=True)
    assert np.allclose(f2, f1)
    _, fc = sgcht.comb_harmonics(256, comb="coarse")
    assert np.allclose(fc, f / 256)
    g = sgcht.FrequencyComb(amps, f)
    _, a = g.generate(100)
    _, b = g.generate(60)
    whole = sgcht.FrequencyComb(amps, f).generate(160)[1]
    assert np.array_equal(np.concatenate([a, b], axis=2), whole)
    ref = np.zeros(160, np.complex64)
    for ai, fi in zip(amps, f):
        ref = ref + (ai * np.exp(2j * np.pi * fi * np.arange(160))).astype(np.complex64)
    assert np.array_equal(whole[0, 0], ref)


def test_frequency_comb_tester_equals_literal_loop():
    """TestFrequencyComb (one FFT per harmonic's channel) gives the verdict of the literal
    channel x harmonic loop of TestFrequencyComb.m:15-118 (verify.frequency_comb_test) on
    the comb itself (level 0, passing and failing) and on oracle channelised combs
    (level 1)."""
    from ska_pst_dsp_model_amd import streaming as sgcht
    from ska_pst_dsp_model_amd import verify
    from ska_pst_dsp_model_amd.firio import design_PFB_FIR_filter
    from oracle import pfb_oracle as orc
    amps, f = sgcht.comb_harmonics()
    x = sgcht.FrequencyComb(amps, f).generate(8192)[1]
    t = sgcht.TestFrequencyComb(f)
    assert t.test(x)[1] == 0 == verify.frequency_comb_test(x, f)
    # drop one harmonic: both fail
    x_bad = sgcht.FrequencyComb(amps[1:], f[1:]).generate(8192)[1]
    assert t.test(x_bad)[1] == -1 == verify.frequency_comb_test(x_bad, f)
    taps = design_PFB_FIR_filter(16, "8/7", 10)
    amps, f = sgcht.comb_harmonics(16)
    xc = sgcht.FrequencyComb(amps, f).generate(16 * 14 * 600)[1]
    ch = orc.polyphase_analysis(xc, taps, 16, "8/7")
    for scale in (1.0, 1e-3):
        got = sgcht.TestFrequencyComb(f, "8/7").test(scale * ch)[1]
        assert got == verify.frequency_comb_test(scale * ch, f, "8/7")
    # (channel k of the Bunton bank is centred on k/N while the tester assigns harmonic f to
    # channel floor(f N): the harmonics at k + 7/8 lie outside their channel's passband, so
    # the channelised comb fails TestFrequencyComb in the reference's own rules too)
    assert sgcht.TestFrequencyComb(f, "8/7").test(ch)[1] == -1


def test_sgcht_frequency_comb_without_channelizer_passes():
    from ska_pst_dsp_model_amd import streaming as sgcht
    r = sgcht.sgcht(signal="frequency_comb", test=True, blocks=3, blocksz=8192)
    assert r.result == 0 and r.blocks == 3


def test_sgcht_generators_square_wave_and_wedge():
    """SquareWave.m: noise of variance on_amp in the first floor(period duty) samples of
    each period, zeros in the rest (off_amp 0), phase carried across calls;
    FrequencyWedge.m: blocks of `resolution` samples with a |spectrum| slope rising from DC
    to the band edges (fftshift of linspace(0, 1))."""
    from ska_pst_dsp_model_amd import streaming as sg
    g = sg.SquareWave(period=10, seed=1)
    _, a = g.generate(7)
    _, b = g.generate(13)
    x = np.concatenate([a, b], axis=2)[0, 0]
    on = (np.arange(20) % 10) < 5
    assert np.all(x[~on] == 0) and np.all(x[on] != 0) and g.current == 20
    w = sg.FrequencyWedge(resolution=1 << 14, seed=2)
    _, y = w.generate(3 << 14)
    p = np.abs(np.fft.fft(y[0, 0, :1 << 14])) ** 2
    h = len(p) // 2
    # power follows fftshift(linspace(0, 1)): ~1 just below index n/2, ~0 just above it,
    # ~0.5 at DC
    hi, lo, dc = p[h - 600:h - 100].mean(), p[h + 100:h + 600].mean(), p[:500].mean()
    assert hi > 10 * lo and 0.3 < dc / hi < 0.7


def test_num2str_matches_matlab():
    from ska_pst_dsp_model_amd.streaming import num2str
    assert num2str(3) == "3" and num2str(1.0) == "1"
    assert num2str(np.pi) == "3.1416" and num2str(123.456) == "123.456"
    assert num2str(0.001234567) == "0.0012346" and num2str(1.14285714) == "1.1429"


def test_sgcht_filename_and_header_without_gpu():
    """sgcht.m:101-163 output names; the header of a 'low' analysis (sgcht.m:314-356):
    TSAMP x os de/nu x n_chan, NSTAGE reset to 1 by add_fir_filter_to_header."""
    from ska_pst_dsp_model_amd import streaming as sg
    assert sg.sgcht_filename("square_wave", "low", two_stage=True, invert=True, critical=True,
                             combine=16, nbit=8, directory="p") == \
        "p/square_wave_low_two_stage_critical_inverted_16_8bit.dada"
    assert sg.sgcht_filename("frequency_comb", "mid", comb="coarse", rmsOutput=2.5) == \
        "products/frequency_comb_coarse_mid_rndOut_rmsOut=2.5.dada"


@pytest.mark.parametrize("name,N,os_,func", [
    ("sps", 256, "32/27", "polyphase_analysis"),
    ("lowpsi", 256, "4/3", "polyphase_analysis_lowcbf"),
    ("lowpsi_old", 256, "4/3", "polyphase_analysis_lowcbf"),
    ("low_alt", 256, "4/3", "polyphase_analysis"),
    ("low", 256, "4/3", "polyphase_analysis"),
    ("mid", 4096, "8/7", "polyphase_analysis_padded"),
    ("low_external", 256, "4/3", "polyphase_analysis"),
    ("mid_external", 4096, "8/7", "polyphase_analysis_padded"),
])
def test_every_reference_sub_config_loads(name, N, os_, func):
    """Every sub-config of the reference's config/test.config.json (default_config.m /
    load_config) exists here with its analysis function, channels and OS factor, and
    sgcht_config attaches taps (the tap file, else the documented stand-in)."""
    from ska_pst_dsp_model_amd import streaming as sg
    c = sg.sgcht_config(name)
    assert c.channels == N and str(c.os_factor) == os_ and c.analysis_function == func
    assert len(c.filt_coeff) > 0
    if func == "polyphase_analysis_lowcbf":
        assert len(c.filt_coeff) == 3072
