"""Host-memory pipeline: pinned host chunks → H2D → kernels → D2H, double-buffered on two HIP
streams (the north_star's end-to-end rate).

Netty's path starts and ends in host memory: a pooled direct ByteBuf off a socket
(ByteBuf.memoryAddress(), ByteBuf.java:2395-2403) goes into SnappyFrameEncoder.encode and the
framed bytes go back out in a ByteBuf (MessageToByteEncoder.java:105-117); the decoder does the
reverse.  Here a batch of chunks moves as sub-batches: while sub-batch k computes on one stream,
sub-batch k+1 uploads on the other and k-1's results download.  Encoded chunks are gathered into
one contiguous run on the device (nx_pack_batch) so each sub-batch needs exactly one D2H copy of
exactly its compressed bytes; the host learns that size from a 4-byte pinned read-back, which is
the only point where the host waits, and it waits on the previous sub-batch only.
"""
from __future__ import annotations

import time

import torch

from . import batch as B

CHUNK = 65536


class SnappyHostPipeline:
    """Encode/decode many 64 KiB chunks held in pinned host memory through the GPU."""

    def __init__(self, device, sub_chunks: int = 32768, chunk: int = CHUNK):
        # The encoder runs one chunk per lane: a sub-batch needs tens of thousands of chunks to
        # fill the GPU (262 144 = 16 waves per CU), so sub-batches are large.
        self.dev = torch.device(device)
        self.sub = sub_chunks
        self.chunk = chunk
        self.cap = (B.snappy_max_compressed_length(chunk) + 15) // 16 * 16
        self.streams = [torch.cuda.Stream(self.dev) for _ in range(2)]
        sub, dev = sub_chunks, self.dev
        self.d_in = [torch.empty(sub * chunk, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.d_enc = [torch.empty(sub * self.cap, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.d_pack = [torch.empty(sub * self.cap, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.in_off = torch.arange(sub, dtype=torch.int64, device=dev) * chunk
        self.enc_off = torch.arange(sub, dtype=torch.int64, device=dev) * self.cap
        self.pin_total = torch.zeros(2, dtype=torch.int64, pin_memory=True)
        torch.cuda.synchronize(dev)  # the constant tensors above were made on the current stream

    # ------------------------------------------------------------------ encode
    def encode(self, h_src, n: int, h_comp, h_len, h_crc):
        """h_src: pinned uint8[n*chunk].  Writes the compressed chunks back to back into pinned
        h_comp, their lengths into h_len (int32[n]) and masked CRC32Cs into h_crc (int32[n]).
        Returns total compressed bytes."""
        sub, ch = self.sub, self.chunk
        pos = 0
        pending = None  # (k, slot, event, m)
        nb = (n + sub - 1) // sub
        for k in range(nb + 1):
            if k < nb:
                s = k % 2
                st = self.streams[s]
                lo, m = k * sub, min(sub, n - k * sub)
                with torch.cuda.stream(st):
                    din = self.d_in[s][: m * ch]
                    din.copy_(h_src[lo * ch:(lo + m) * ch], non_blocking=True)
                    ln = torch.full((m,), ch, dtype=torch.int32, device=self.dev)
                    crc = B.crc32c_masked(din, self.in_off[:m], ln)
                    elen, est = B.snappy_encode(din, self.in_off[:m], ln, self.d_enc[s], self.enc_off[:m])
                    dpk, dst_off = self._pack(self.d_enc[s], self.enc_off[:m], elen, self.d_pack[s], s)
                    h_len[lo:lo + m].copy_(elen, non_blocking=True)
                    h_crc[lo:lo + m].copy_(crc, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(st)
                cur = (k, s, ev, m)
            else:
                cur = None
            if pending is not None:
                pk, ps, pev, pm = pending
                pev.synchronize()  # previous sub-batch's packed size is now in pinned memory
                total = int(self.pin_total[ps])
                with torch.cuda.stream(self.streams[ps]):
                    h_comp[pos:pos + total].copy_(self.d_pack[ps][:total], non_blocking=True)
                pos += total
            pending = cur
        for st in self.streams:
            st.synchronize()
        return pos

    def _pack(self, src, src_off, elen, dst, slot):
        m = elen.numel()
        dst_off = torch.zeros(m, dtype=torch.int64, device=self.dev)
        if m > 1:
            torch.cumsum(elen[:-1].to(torch.int64), 0, out=dst_off[1:])
        B.gather(src, src_off, elen, dst, dst_off)
        tot = dst_off[-1:] + elen[-1:].to(torch.int64)
        self.pin_total[slot:slot + 1].copy_(tot, non_blocking=True)
        return dst, dst_off

    # ------------------------------------------------------------------ decode
    def decode(self, h_comp, h_len, h_crc, n: int, h_out):
        """Inverse of encode(): pinned h_comp (back-to-back chunks), lengths h_len, expected
        masked CRCs h_crc → pinned h_out[n*chunk].  Returns the per-chunk status tensor (host)."""
        sub, ch = self.sub, self.chunk
        starts = torch.zeros(n + 1, dtype=torch.int64)
        starts[1:] = torch.cumsum(h_len[:n].to(torch.int64), 0)
        status = torch.empty(n, dtype=torch.int32, pin_memory=True)
        nb = (n + sub - 1) // sub
        for k in range(nb):
            s = k % 2
            st = self.streams[s]
            lo, m = k * sub, min(sub, n - k * sub)
            c0, c1 = int(starts[lo]), int(starts[lo + m])
            with torch.cuda.stream(st):
                dc = self.d_pack[s][: max(c1 - c0, 1)]
                dc[: c1 - c0].copy_(h_comp[c0:c1], non_blocking=True)
                off = (starts[lo:lo + m] - c0).to(self.dev, non_blocking=True)
                ln = h_len[lo:lo + m].to(self.dev, non_blocking=True)
                exp = h_crc[lo:lo + m].to(self.dev, non_blocking=True)
                dout = self.d_in[s][: m * ch]
                dst = B.snappy_decode(dc, off, ln, dout, self.in_off[:m], expected_crc=exp)["status"]
                h_out[lo * ch:(lo + m) * ch].copy_(dout, non_blocking=True)
                status[lo:lo + m].copy_(dst, non_blocking=True)
        for st in self.streams:
            st.synchronize()
        return status


def measure(device, n: int = 131072, sub: int = 65536):
    """End-to-end GiB/s (uncompressed bytes) of host→device→host Snappy encode and decode of n
    text-like 64 KiB chunks, plus raw pinned H2D/D2H copy rates for context."""
    dev = torch.device(device)
    pipe = SnappyHostPipeline(dev, sub)
    ch = pipe.chunk
    h_src = torch.empty(n * ch, dtype=torch.uint8, pin_memory=True)
    tmp = torch.empty(sub * ch, dtype=torch.uint8, device=dev)
    for k in range(0, n, sub):
        m = min(sub, n - k)
        B.textgen(tmp, k, m, ch)
        h_src[k * ch:(k + m) * ch].copy_(tmp[: m * ch])
    torch.cuda.synchronize(dev)
    h_comp = torch.empty(n * pipe.cap, dtype=torch.uint8, pin_memory=True)
    h_len = torch.empty(n, dtype=torch.int32, pin_memory=True)
    h_crc = torch.empty(n, dtype=torch.int32, pin_memory=True)
    h_out = torch.empty(n * ch, dtype=torch.uint8, pin_memory=True)
    pipe.encode(h_src[: sub * ch], min(n, sub), h_comp, h_len, h_crc)  # warm-up
    t0 = time.perf_counter()
    ctot = pipe.encode(h_src, n, h_comp, h_len, h_crc)
    t1 = time.perf_counter()
    status = pipe.decode(h_comp, h_len, h_crc, n, h_out)
    t2 = time.perf_counter()
    ok = bool((status == 0).all()) and bool(torch.equal(h_out, h_src))
    # raw pinned copy rates
    d = torch.empty(n * ch, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    a = time.perf_counter()
    d.copy_(h_src, non_blocking=True)
    torch.cuda.synchronize(dev)
    b = time.perf_counter()
    h_out.copy_(d, non_blocking=True)
    torch.cuda.synchronize(dev)
    c = time.perf_counter()
    U = n * ch
    gib = 2.0 ** 30
    return {
        "chunks": n, "sub_batch_chunks": sub, "bytes": U, "compressed_bytes": ctot,
        "encode_gib_s": round(U / (t1 - t0) / gib, 3), "decode_gib_s": round(U / (t2 - t1) / gib, 3),
        "round_trip_gib_s": round(U / (t2 - t0) / gib, 3),
        "h2d_gib_s": round(U / (b - a) / gib, 3), "d2h_gib_s": round(U / (c - b) / gib, 3),
        "verified": ok,
    }
