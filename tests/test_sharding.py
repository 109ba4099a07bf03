"""Multi-process (gloo, world_size 2, CPU) tests of the sharded path.

Each rank computes its shard of one long series (index ranges from
``ska_pst_dsp_model_amd.sharding``) with the CPU oracle as a stand-in for the device
(no GPU here); rank 0 gathers the pieces and checks that their concatenation equals the
single-run result exactly.  No collective sits on the data path in production — the
gather exists only to check the result.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import pfb_oracle as orc
from ska_pst_dsp_model_amd import sharding

N_CHAN, OS, NF, OV = 8, "8/7", 128, 16


def _taps():
    rng = np.random.default_rng(3)
    return rng.standard_normal(81)


def _series(n):
    rng = np.random.default_rng(5)
    return (rng.standard_normal((1, 1, n)) + 1j * rng.standard_normal((1, 1, n))) / np.sqrt(2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_dat, err_file):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        taps = _taps()
        taps_mid = np.random.default_rng(4).standard_normal(20 * N_CHAN + 1)  # sds = 12 rows
        x = _series(n_dat)
        # analysis shard
        sa = sharding.analysis_shard(n_dat, N_CHAN, OS, len(taps), world, rank)
        ya = orc.polyphase_analysis(x[:, :, sa.in_start:sa.in_stop], taps, N_CHAN, OS)
        assert ya.shape[2] == sa.n_out
        # synthesis shard of the full channelised series
        chan = orc.polyphase_analysis(x, taps, N_CHAN, OS)
        ss = sharding.synthesis_shard(chan.shape[2], N_CHAN, OS, NF, OV, world, rank)
        win = orc.pfb_window("tukey", NF, OV)
        dr = {"apply_deripple": 1, "filter_coeff": taps}
        ys = orc.polyphase_synthesis(chan[:, :, ss.in_start:ss.in_stop], 1, NF, OS, dr, 1, OV, win)
        assert ys.shape[2] == ss.n_out
        # padded (commutator) analysis shard: main slice + the circular shift's tail
        sp = sharding.analysis_padded_shard(n_dat, N_CHAN, OS, len(taps_mid), world, rank)
        yp = []
        if sp.out_stop > sp.out_start:
            y = orc.polyphase_analysis_padded(x[:, :, sp.in_start:sp.in_stop], taps_mid, N_CHAN, OS)
            yp.append(y[:, :, sp.keep_start:sp.keep_start + sp.out_stop - sp.out_start])
        if sp.n_wrap:
            y = orc.polyphase_analysis_padded(x[:, :, :sp.wrap_stop], taps_mid, N_CHAN, OS)
            yp.append(y[:, :, sp.wrap_keep:sp.wrap_keep + sp.n_wrap])
        yp = np.concatenate(yp, axis=2) if yp else np.zeros((1, N_CHAN, 0), complex)
        parts = [None] * world
        dist.all_gather_object(parts, (ya, ys, yp))
        if rank == 0:
            full_a = orc.polyphase_analysis(x, taps, N_CHAN, OS)
            full_s = orc.polyphase_synthesis(chan, 1, NF, OS, dr, 1, OV, win)
            cat_a = np.concatenate([p[0] for p in parts], axis=2)
            cat_s = np.concatenate([p[1] for p in parts], axis=2)
            assert np.array_equal(cat_a, full_a), "analysis shards differ from the single run"
            assert np.array_equal(cat_s, full_s), "synthesis shards differ from the single run"
            full_p = orc.polyphase_analysis_padded(x, taps_mid, N_CHAN, OS)
            cat_p = np.concatenate([p[2] for p in parts], axis=2)
            assert np.array_equal(cat_p, full_p), "padded analysis shards differ from the single run"
    except Exception as e:  # report to the parent
        with open(err_file, "a") as f:
            f.write(f"rank {rank}: {e!r}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_round_trip_gloo(tmp_path, world):
    err = tmp_path / "err.txt"
    n_dat = 7 * 8 * 90 + 333
    mp.start_processes(_worker, args=(world, _free_port(), n_dat, str(err)), nprocs=world,
                       join=True, start_method="spawn")
    assert not err.exists() or err.read_text() == ""


def test_shard_ranges_cover_exactly():
    """Shards tile the output without gaps or overlap; analysis cuts are multiples of nu."""
    for world in (1, 2, 3, 8):
        a = [sharding.analysis_shard(1 << 16, 256, "8/7", 3073, world, r) for r in range(world)]
        assert a[0].out_start == 0
        for s, t in zip(a, a[1:]):
            assert s.out_stop == t.out_start
            assert t.out_start % 8 == 0  # nu
        K = (((1 << 16) - 13 * 256) // 224)
        assert a[-1].out_stop == K
        s_ = [sharding.synthesis_shard(74880, 256, "8/7", 256, 48, world, r) for r in range(world)]
        for s, t in zip(s_, s_[1:]):
            assert s.out_stop == t.out_start
            assert t.in_start == s.in_stop - 2 * 48
        assert s_[-1].out_stop == ((74880 - 96) // 160) * 35840


def test_padded_shards_match_single_run():
    """Padded (commutator) analysis, polyphase_analysis_padded.m:56-156: the ranks' main
    slices plus the circular shift's tail (FIR rows [0, sds) recomputed from the first
    sds M samples) concatenate to the single-run output exactly, for rank counts where
    one or several ranks hold wrapped rows."""
    rng = np.random.default_rng(1)
    for n_taps in (16 * 6 + 1, 16 * 20 + 1):
        taps = rng.standard_normal(n_taps)
        for n_dat in (14 * 40 + 5, 14 * 200 + 13):
            x = rng.standard_normal((1, 1, n_dat)) + 1j * rng.standard_normal((1, 1, n_dat))
            full = orc.polyphase_analysis_padded(x, taps, 16, "8/7")
            for world in (1, 2, 5, 8):
                parts = []
                for r in range(world):
                    sh = sharding.analysis_padded_shard(n_dat, 16, "8/7", n_taps, world, r)
                    if sh.out_stop > sh.out_start:
                        y = orc.polyphase_analysis_padded(x[:, :, sh.in_start:sh.in_stop], taps, 16, "8/7")
                        parts.append(y[:, :, sh.keep_start:sh.keep_start + sh.out_stop - sh.out_start])
                    if sh.n_wrap:
                        y = orc.polyphase_analysis_padded(x[:, :, :sh.wrap_stop], taps, 16, "8/7")
                        parts.append(y[:, :, sh.wrap_keep:sh.wrap_keep + sh.n_wrap])
                assert np.array_equal(np.concatenate(parts, axis=2), full), (n_taps, n_dat, world)


def test_padded_shard_ranges_c3():
    """C3 (SKA-Mid: 4096 ch, 8/7, 100 353 taps, 2^26 samples) over 8 ranks: output rows
    tile [0, K); only the last rank holds the sds = 14 wrapped rows; every main slice
    starts on a commutator-period boundary (M k_s, k_s a multiple of nu)."""
    n_dat, N, taps = 1 << 26, 4096, 100353
    M = N * 7 // 8
    K = n_dat // M
    sh = [sharding.analysis_padded_shard(n_dat, N, "8/7", taps, 8, r) for r in range(8)]
    rows = []
    for s in sh:
        rows += list(range(s.out_start, s.out_stop)) + list(range(s.out_stop, s.out_stop + s.n_wrap))
        assert s.in_start % (8 * M) == 0
    assert rows == list(range(K))
    assert [s.n_wrap for s in sh] == [0] * 7 + [14]
