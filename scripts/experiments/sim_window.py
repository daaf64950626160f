"""Model of the sliding-window record expander (k_expand, round 2 design) on the bench corpus.

One wave holds up to 64 pending records (one per lane).  Each pass: free lanes take the next records
in stream order (subject to the ring limit), a copy is ready when the bytes it reads are below the
frontier F (start of the lowest pending record), every ready lane produces up to K bytes, and finished
lanes free up.  Counts passes, 8-byte pieces and far (HBM) copies per frame.
Usage: python scripts/experiments/sim_window.py [frames] [K] [R]
"""
import sys

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from oracle import pyoracle as O  # noqa: E402


def records(block: bytes):
    i, _ = 0, 0
    while block[i] & 0x80:
        i += 1
    i += 1
    op = 0
    out = []
    n = len(block)
    while i < n:
        t = block[i]
        i += 1
        ty = t & 3
        if ty == 0:
            c = t >> 2
            if c >= 60:
                nb = c - 59
                ln = int.from_bytes(block[i:i + nb], "little") + 1
                i += nb
            else:
                ln = c + 1
            k = 0
            while k < ln:
                m = min(64, ln - k)
                out.append((False, m, i + k, op))
                op += m
                k += m
            i += ln
        else:
            if ty == 1:
                ln = 4 + ((t >> 2) & 7)
                off = ((t & 0xE0) << 3) | block[i]
                i += 1
            elif ty == 2:
                ln = 1 + (t >> 2)
                off = block[i] | (block[i + 1] << 8)
                i += 2
            else:
                ln = 1 + (t >> 2)
                off = int.from_bytes(block[i:i + 4], "little")
                i += 4
            out.append((True, ln, off, op))
            op += ln
    return out, op


def simulate(recs, K=16, R=4096, B=512, lanes=64):
    N = len(recs)
    k = 0
    Emax = 0
    flushed = 0
    pend = []  # [isc, rem, x, dst]
    passes = pieces_sum = piece_iters = far = ready_sum = 0
    while True:
        limit = flushed + R - B - 64
        while len(pend) < lanes and k < N:
            isc, ln, x, dst = recs[k]
            if dst + ln > limit:
                break
            pend.append([isc, ln, x, dst])
            Emax = dst + ln
            k += 1
        if not pend:
            break
        passes += 1
        F = min(p[3] for p in pend)
        flushed = max(flushed, (F // B) * B)
        maxp = 0
        nxt = []
        for p in pend:
            isc, rem, x, dst = p
            if isc:
                s = dst - x
                need = min(s + rem, dst)
                if need > F:
                    nxt.append(p)
                    continue
                if s < Emax - R:
                    far += 1
            n = min(rem, K)
            npc = ((dst + n + 7) // 8) - (dst // 8)
            pieces_sum += npc
            maxp = max(maxp, npc)
            ready_sum += 1
            if rem > n:
                p[1] = rem - n
                p[3] = dst + n
                if not isc:
                    p[2] = x + n
                nxt.append(p)
        piece_iters += maxp
        pend = nxt
    return dict(passes=passes, ready_per_pass=ready_sum / max(passes, 1), piece_iters=piece_iters,
                pieces=pieces_sum, far=far, records=N)


if __name__ == "__main__":
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    tot = {}
    for f in range(frames):
        blk = O.snappy_encode(O.textgen_chunk(f, 65536))
        recs, olen = records(blk)
        assert olen == 65536
        r = simulate(recs, K=K, R=R)
        for a, b in r.items():
            tot[a] = tot.get(a, 0) + b
    print({a: round(b / frames, 2) for a, b in tot.items()})
