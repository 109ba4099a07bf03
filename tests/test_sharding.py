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
        parts = [None] * world
        dist.all_gather_object(parts, (ya, ys))
        if rank == 0:
            full_a = orc.polyphase_analysis(x, taps, N_CHAN, OS)
            full_s = orc.polyphase_synthesis(chan, 1, NF, OS, dr, 1, OV, win)
            cat_a = np.concatenate([p[0] for p in parts], axis=2)
            cat_s = np.concatenate([p[1] for p in parts], axis=2)
            assert np.array_equal(cat_a, full_a), "analysis shards differ from the single run"
            assert np.array_equal(cat_s, full_s), "synthesis shards differ from the single run"
    except Exception as e:  # report to the parent
        with open(err_file, "a") as f:
            f.write(f"rank {rank}: {e!r}\n")
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
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
