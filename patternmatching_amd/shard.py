"""Splitting one stream across ranks.

A position's answer depends only on the max_len-1 bytes before it
(DESIGN.md §1), so rank r scans positions [lo, hi) of the stream with the
preceding max_len-1 bytes (clipped at the stream start) as read-only
context.  Shards are exact at every seam; the only exchange is the final
sum of match counts (an all-reduce).
"""
from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    ctx_lo: int   # first byte this rank reads (context start)
    lo: int       # first position it answers for
    hi: int       # one past the last


def shard_plan(n: int, world: int, rank: int, max_len: int, align: int = 16) -> Shard:
    """Contiguous, `align`-aligned split of n positions over `world` ranks."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-n // world)
    per = -(-per // align) * align
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    ctx = max(0, max_len - 1)
    return Shard(ctx_lo=max(0, lo - ctx), lo=lo, hi=hi)


def scan_shard(scan_fn, text, shard: Shard):
    """Run scan_fn(bytes_with_context, n_context) and keep the shard's part.

    scan_fn must return one answer per input byte for a stream that starts at
    the first byte it is given (e.g. a fresh read_block after reset)."""
    part = text[shard.ctx_lo:shard.hi]
    res = scan_fn(part)
    return res[shard.lo - shard.ctx_lo:]
