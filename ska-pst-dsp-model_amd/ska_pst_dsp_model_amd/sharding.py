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
* Padded (commutator) analysis (``polyphase_analysis_padded.m:56-156``): FIR row q reads
  x[q M - P N, q M) with zero history before t = 0, its barrel index depends on q mod nu,
  and the output is circularly shifted, out[t] = FIR[(t + sds) mod K].  A rank producing
  output rows [t0, t1) runs the same analysis on the slice starting at row k_s (a
  multiple of nu, at least ceil(P N / M) rows before the FIR rows it needs, or 0), so
  its FIR rows past the history are the global ones; it keeps the local output rows that
  map to [t0, t1 - wrap).  The last sds output rows wrap round to FIR rows [0, sds): the
  last rank computes them from the first sds M samples (a second, tiny slice whose own
  zero history is the true one).  ``analysis_padded_shard`` returns both slices.
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


@dataclass(frozen=True)
class PaddedShard:
    """Rank-local work of a sharded padded analysis.

    main: run polyphase_analysis_padded on x[in_start, in_stop) and keep its output rows
    [keep_start, keep_start + out_stop - out_start) -> global output rows [out_start, out_stop).
    wrap (n_wrap > 0: ranks holding the circular shift's tail): run it on x[0, wrap_stop)
    (sds rows) and keep its rows [wrap_keep, wrap_keep + n_wrap) -> global output rows
    [out_stop, out_stop + n_wrap).
    """
    in_start: int
    in_stop: int
    keep_start: int
    out_start: int
    out_stop: int
    wrap_stop: int = 0
    wrap_keep: int = 0
    n_wrap: int = 0


def analysis_padded_shard(n_dat: int, n_chan: int, os_factor, n_taps: int, world: int,
                          rank: int) -> PaddedShard:
    """Slices of rank's part of a stateless padded (commutator) analysis of n_dat samples."""
    os_ = as_rational(os_factor)
    M = n_chan * os_.de // os_.nu
    P = -(-n_taps // n_chan)
    K = max(0, n_dat // M)                            # polyphase_analysis_padded.m:59
    sds = min(K, -(-(n_taps - 1) // (2 * M)))         # :89, ceil((Lh - 1) / 2 / M)
    t0, t1 = _split(K, world, rank, os_.nu)
    hist = -(-(P * n_chan) // M)                      # rows of input history a FIR row reads
    m1 = min(t1, K - sds)                             # output rows [t0, m1): FIR rows + sds
    if m1 > t0:
        k_s = max(0, ((t0 + sds - hist) // os_.nu) * os_.nu)
        main = (k_s * M, (m1 + sds) * M, t0 - k_s, t0, m1)
    else:
        main = (0, 0, 0, t0, t0)
    w0 = max(t0, K - sds)                             # output rows [w0, t1) wrap to FIR rows
    if t1 > w0:                                       # [w0 + sds - K, t1 + sds - K)
        # a slice of sds rows: its output row t' is FIR row t' (own zero history = true one)
        return PaddedShard(*main[:4], w0, sds * M, w0 + sds - K, t1 - w0)
    return PaddedShard(*main)
