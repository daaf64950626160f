"""CPU check of bench.py's framed-stream layout (bench_frame_scan): the streams it builds in device
memory are valid SnappyFrameEncoder output whose chunks the oracle's frame scan lists and decodes
with matching checksums.  Runs the layout code on CPU tensors with the device calls stubbed."""
import os
import sys

import pytest

torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Done(Exception):
    pass


class _Event:  # torch.cuda.Event stand-in: the layout code records events before the first device call
    def __init__(self, **kw):
        pass

    def record(self):
        pass


def test_bench_frame_layout(oracle, monkeypatch):
    import bench

    monkeypatch.setattr(torch.cuda, "Event", _Event)

    m, per, cap = 10, 4, 2048
    raw = [oracle.textgen_chunk(i, 1000 + 37 * i) for i in range(m)]
    chunks = [oracle.snappy_encode(r) for r in raw]
    enc = torch.zeros(m * cap, dtype=torch.uint8)
    for i, c in enumerate(chunks):
        enc[i * cap:i * cap + len(c)] = torch.tensor(list(c), dtype=torch.uint8)
    eoff = torch.arange(m, dtype=torch.int64) * cap
    elen = torch.tensor([len(c) for c in chunks], dtype=torch.int32)
    crc = torch.tensor([oracle.snappy_checksum(r) for r in raw], dtype=torch.int64).to(torch.int32)
    seen = {}

    class FakeB:
        @staticmethod
        def gather(src, src_off, length, dst=None, dst_off=None):
            for a, n, d in zip(src_off.tolist(), length.tolist(), dst_off.tolist()):
                dst[d:d + n] = src[a:a + n]

        @staticmethod
        def snappy_frame_scan(buf, ss, slen, state, cap_):
            b = bytes(buf.tolist())
            k = 0
            for s, n in zip(ss.tolist(), slen.tolist()):
                ents, consumed, st, res = oracle.snappy_frame_scan(b[s:s + n])
                assert res == 0 and consumed == n and st == 1
                for typ, o, ln, c in ents:
                    status, out, _ = oracle.snappy_decode(b[s + o:s + o + ln], 65536)
                    assert typ == 0 and status >= 0 and out == raw[k] and oracle.snappy_checksum(out) == c
                    k += 1
            seen["chunks"] = k
            raise _Done()

    class Leg:  # the fields of bench.SnappyRoundTrip that bench_frame_scan reads
        src, dec, sub, n = None, None, m, m

    leg = Leg()
    leg.enc, leg.eoff, leg.elen, leg.crc = enc, eoff, elen, crc
    with pytest.raises(_Done):
        bench.bench_frame_scan(torch, FakeB, torch.device("cpu"), leg, m, per, reps=1)
    assert seen["chunks"] == m
