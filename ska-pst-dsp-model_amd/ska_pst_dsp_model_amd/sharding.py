"""Exact partitioning of one long series across GPUs.

The round trip shards without any collective: polarisations and independent DADA time
blocks are independent units (``polyphase_analysis.m:83``, ``polyphase_synthesis.m:164``)
and ``bench.py`` runs one unit per rank.  A *single* long series can also be split, and
the concatenation of the per-rank outputs is identical to the single-run output, when
the cut points respect the streaming granularity the reference itself uses:

* Bunton analysis (``polyphase_analysis.m:83-121``): output row k reads
  x[M k, M k + P N) and its phase rotation is (M k) mod N.  Cutting the output rows at
  multiples of nu (as ``FilterBank.m:93-104`` trims its output) makes M k0 a multiple
  of N, so a rank that starts its input at M k0 computes the same rotations.  Each
  rank reads a halo of P N samples past its last row's step (the reference's row
  count K = floor((n - P N) / M) needs M K + P N samples).
* Synthesis (``polyphase_synthesis.m:112-131``): block b reads channelised rows
  [b keep, b keep + Nf) and writes output samples [b L_keep, (b+1) L_keep); blocks are
  independent, ranks overlap by 2 Ov input rows.

These helpers only compute index ranges (host logic, no device work).
"""
from __future__ import annotations

from dataclasses import dataclass

from .config import as_rational


@dataclass(frozen=True)
class Shard:
    """Rank-local slice: input [in_start, in_stop), output rows/samples [out_start, out_stop)."""
    in_start: int
    in_stop: int
    out_start: int
    out_stop: int

    @property
    def n_in(self) -> int:
        return self.in_stop - self.in_start

    @property
    def n_out(self) -> int:
        return self.out_stop - self.out_start


def _split(n_units: int, world: int, rank: int, quantum: int = 1):
    """Contiguous split of n_units into world parts whose cut points are multiples of quantum."""
    q = max(1, int(quantum))
    chunks = n_units // q
    lo = (chunks * rank // world) * q
    hi = (chunks * (rank + 1) // world) * q if rank < world - 1 else n_units
    return lo, hi


def analysis_shard(n_dat: int, n_chan: int, os_factor, n_taps: int, world: int, rank: int) -> Shard:
    """Input/output ranges of rank's part of a stateless Bunton analysis of n_dat samples."""
    os_ = as_rational(os_factor)
    M = n_chan * os_.de // os_.nu
    P = -(-n_taps // n_chan)
    K = max(0, (n_dat - P * n_chan) // M)  # polyphase_analysis.m:62
    k0, k1 = _split(K, world, rank, os_.nu)
    if k1 <= k0:
        return Shard(M * k0, M * k0, k0, k0)
    # K = floor((n - P N) / M) rows need n = M K + P N samples (the reference's count)
    return Shard(M * k0, M * k1 + P * n_chan, k0, k1)


def synthesis_shard(n_dat: int, n_chan: int, os_factor, nf: int, ov: int, world: int,
                    rank: int) -> Shard:
    """Channelised-row and output-sample ranges of rank's part of a stateless synthesis."""
    os_ = as_rational(os_factor)
    keep = nf - 2 * ov
    B = max(0, (n_dat - 2 * ov) // keep)  # polyphase_synthesis.m:114
    W = nf * os_.de // os_.nu
    l_keep = n_chan * W - 2 * (ov * os_.de // os_.nu) * n_chan
    b0, b1 = _split(B, world, rank)
    if b1 <= b0:
        return Shard(b0 * keep, b0 * keep, b0 * l_keep, b0 * l_keep)
    return Shard(b0 * keep, b1 * keep + 2 * ov, b0 * l_keep, b1 * l_keep)
