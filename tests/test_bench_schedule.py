"""bench.py's step schedule (round 6): encode calls from the library's launch plan, decode calls of
262 144 frames as soon as that many chunks are encoded, the rest at the end.  CPU only: the schedule
is host arithmetic; tests/test_gpu_config5_shard.py runs it on the GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _check(enc, dec_sub):
    ops = bench.schedule(enc, dec_sub)
    n = sum(enc)
    # every chunk is encoded once and decoded once, both in order, each decode after its encodes
    e_next = d_next = 0
    pending_max = 0
    for kind, lo, m in ops:
        if kind == "enc":
            assert lo == e_next
            e_next += m
        else:
            assert lo == d_next and lo + m <= e_next and 0 < m <= dec_sub
            d_next += m
        pending_max = max(pending_max, e_next - d_next)
    assert e_next == d_next == n
    # the ring bench.SnappyRoundTrip allocates holds every encoded, not yet decoded chunk
    assert pending_max <= max(enc) + dec_sub - 1
    return ops


def test_schedule_100gib_one_gpu():
    ops = _check([327680] * 5, 262144)
    dec = [m for k, _, m in ops if k == "dec"]
    assert dec == [262144] * 6 + [65536]
    assert [k for k, _, _ in ops] == ["enc", "dec", "enc", "dec", "enc", "dec", "enc", "dec", "dec", "enc", "dec", "dec"]


def test_schedule_per_rank_shapes():
    for enc in ([294912, 262144, 262144], [196608, 212992], [204800], [262144] * 4, [64, 64, 64, 8], [1], [96, 96, 108]):
        for dec_sub in (262144, 64, 1, 100):
            _check(enc, dec_sub)


def test_schedule_aligned_calls_alternate():
    ops = bench.schedule([64, 64, 64, 8], 64)
    assert ops == [("enc", 0, 64), ("dec", 0, 64), ("enc", 64, 64), ("dec", 64, 64), ("enc", 128, 64), ("dec", 128, 64),
                   ("enc", 192, 8), ("dec", 192, 8)]
