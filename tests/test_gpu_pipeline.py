"""Host-memory pipeline (pinned → H2D → encode/pack → D2H and back): byte parity of the packed
compressed stream with the oracle's Snappy.encode of each chunk, and identity after decode."""
import pytest

pytestmark = pytest.mark.gpu


def test_host_pipeline_round_trip(oracle):
    import torch
    from netty_amd.pipeline import SnappyHostPipeline
    n, sub, ch = 37, 8, 65536
    pipe = SnappyHostPipeline("cuda:0", sub_chunks=sub)
    h_src = torch.empty(n * ch, dtype=torch.uint8, pin_memory=True)
    chunks = [oracle.textgen_chunk(i, ch) for i in range(n)]
    h_src.copy_(torch.frombuffer(bytearray(b"".join(chunks)), dtype=torch.uint8))
    h_comp = torch.empty(n * pipe.cap, dtype=torch.uint8, pin_memory=True)
    h_len = torch.empty(n, dtype=torch.int32, pin_memory=True)
    h_crc = torch.empty(n, dtype=torch.int32, pin_memory=True)
    total = pipe.encode(h_src, n, h_comp, h_len, h_crc)
    want = [oracle.snappy_encode(c) for c in chunks]
    assert [int(x) for x in h_len] == [len(w) for w in want]
    assert bytes(h_comp[:total].numpy()) == b"".join(want)
    assert [int(x) & 0xFFFFFFFF for x in h_crc] == [oracle.snappy_checksum(c) for c in chunks]
    h_out = torch.empty(n * ch, dtype=torch.uint8, pin_memory=True)
    st = pipe.decode(h_comp, h_len, h_crc, n, h_out)
    assert int((st != 0).sum()) == 0
    assert torch.equal(h_out, h_src)
