"""Lifetime stress of the handle / batcher C-ABI (diagnostics, not a test): sync decoders and
encoders of every codec, batchers with validating and plain decoders, jobs left in flight, handles and
batchers freed in random orders, and cyclic garbage collected at random points.  Run with
NX_SEGV_TRACE=1 so a native crash prints its stack.

    NX_SEGV_TRACE=1 python scripts/experiments/handle_lifetime_stress.py [iterations]
"""
import gc
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import netty_amd as nx  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    rng = random.Random(5)
    data = [O.textgen_chunk(i, rng.randint(100, 70000)) for i in range(16)]
    framed = [O.snappy_frame_encode(d)[0] for d in data]
    fl = [O.fastlz_frame_encode(d[:60000], level=1, checksum=True) for d in data]
    live = []
    for it in range(iters):
        op = rng.randrange(8)
        if op == 0:
            live.append(nx.Batcher())
        elif op == 1 or op == 2:
            d = nx.SnappyFrameDecoder(rng.random() < 0.5)
            s = framed[rng.randrange(len(framed))]
            if rng.random() < 0.3:
                s = s[:rng.randrange(len(s))] + bytes([rng.randrange(256)]) + s[rng.randrange(len(s)):]
            try:
                d.channel_read(s)
            except nx.DecoderException:
                pass
            live.append(d)
        elif op == 3:
            bs = [x for x in live if isinstance(x, nx.Batcher)]
            if bs:
                b = rng.choice(bs)
                ds = [nx.SnappyFrameDecoder(rng.random() < 0.5) for _ in range(rng.randint(1, 6))]
                ts = []
                for d in ds:
                    s = framed[rng.randrange(len(framed))]
                    q = rng.randrange(len(s) + 1)
                    ts.append(b.submit_decode(d, s[:q]))
                    ts.append(b.submit_decode(d, s[q:]))
                if rng.random() < 0.7:
                    b.flush()
                live.extend(ds)
                if rng.random() < 0.5:
                    for t in ts:
                        try:
                            b.wait(t)
                            b.result(t)
                        except nx.DecoderException as e:
                            live.append(e)  # a traceback cycle, freed by the collector later
        elif op == 4:
            d = nx.FastLzFrameDecoder(True)
            try:
                d.channel_read(fl[rng.randrange(len(fl))])
            except nx.DecoderException:
                pass
            live.append(d)
        elif op == 5:
            e = nx.SnappyFrameEncoder()
            e.encode(data[rng.randrange(len(data))])
            live.append(e)
        elif op == 6 and live:
            rng.shuffle(live)
            del live[:rng.randint(1, len(live))]
        else:
            gc.collect()
        if it % 50 == 0:
            print("iteration", it, "live", len(live), flush=True)
    del live
    gc.collect()
    print("done", flush=True)


if __name__ == "__main__":
    main()
