"""CPU model of copy-source redirection in k_parse: how many producer-map passes,
dependency rounds and far (HBM) piece reads k_expand would see on the bench corpus if k_parse rewrote

  * a copy whose source lies wholly inside one of the last H tags' output that was a LITERAL into a
    literal record reading the compressed input (no in-pass producer, no ring read), and
  * a copy whose source lies wholly inside a recent COPY's output into a copy of that copy's source
    (out[q + i] == out[q - off + i] for every byte of a copy tag, overlapping ones included),
    repeated up to D times.

Pieces and passes follow expand_tags (snappy_decode.hip): a piece is a tag's bytes within one output
dword, a pass is 64 consecutive pieces, a piece whose source bytes lie in the pass's own output waits
one round past the deepest piece producing them.  Not product code.

    python scripts/experiments/redirect_model.py [frames] [H] [D]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from oracle import pyoracle as O  # noqa: E402

RING = 4096


def tags_of(comp):
    """(out_start, len, kind, x): kind 0 literal (x = input position), 1 copy (x = offset)"""
    ip, shift, n = 0, 0, 0
    while True:
        b = comp[ip]
        ip += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if b < 0x80:
            break
    op, out = 0, []
    while ip < len(comp):
        t = comp[ip]
        ip += 1
        k = t & 3
        if k == 0:
            ln = (t >> 2) + 1
            if ln > 60:
                nb = ln - 60
                ln = int.from_bytes(comp[ip:ip + nb], "little") + 1
                ip += nb
            out.append((op, ln, 0, ip))
            ip += ln
        else:
            if k == 1:
                ln = ((t >> 2) & 7) + 4
                off = ((t >> 5) << 8) | comp[ip]
                ip += 1
            elif k == 2:
                ln = (t >> 2) + 1
                off = comp[ip] | (comp[ip + 1] << 8)
                ip += 2
            else:
                ln = (t >> 2) + 1
                off = int.from_bytes(comp[ip:ip + 4], "little")
                ip += 4
            out.append((op, ln, 1, off))
        op += ln
    assert op == n
    return out


def redirect(tags, H, D):
    out, hist, nlit, ncopy = [], [], 0, 0
    for (p, ln, kind, x) in tags:
        if kind == 1 and x >= ln:  # non-overlapping copy
            s = p - x
            for _ in range(D):
                T = next((t for t in reversed(hist) if t[0] <= s and s + ln <= t[0] + t[1]), None)
                if T is None:
                    break
                if T[2] == 0:
                    kind, x = 0, T[3] + (s - T[0])
                    nlit += 1
                    break
                s -= T[3]
                ncopy += 1
            if kind == 1:
                x = p - s
        out.append((p, ln, kind, x))
        hist.append((p, ln, tags and kind if False else kind, x) if False else (p, ln, kind, x))
        if len(hist) > H:
            hist.pop(0)
    return out, nlit, ncopy


def pieces_of(tags):
    ps = []
    for ti, (p, ln, kind, x) in enumerate(tags):
        a = p
        while a < p + ln:
            b = min((a & ~3) + 4, p + ln)
            ps.append((a, b, ti))
            a = b
    return ps


def model(tags):
    ps = pieces_of(tags)
    passes = rounds = map_passes = far = 0
    for P0 in range(0, len(ps), 64):
        grp = ps[P0:P0 + 64]
        lo, hi = grp[0][0], grp[-1][1]
        producer = {}
        depth = []
        any_dep = False
        for i, (a, b, ti) in enumerate(grp):
            p, ln, kind, x = tags[ti]
            d = 0
            if kind == 1:
                if x < ln:  # overlapping: reads [p - x, p)
                    sa, sb = p - x, p
                else:
                    sa, sb = a - x, b - x
                if sb > lo:
                    mx = max(depth[producer[q]] for q in range(max(sa, lo), sb) if q in producer) if any(
                        q in producer for q in range(max(sa, lo), sb)) else -1
                    d = mx + 1 if mx >= 0 else 0
                    any_dep = any_dep or d > 0 or sb > lo
                elif x < ln:
                    pass
                elif hi - RING > sa:  # older than the ring: an HBM read
                    far += 1
            for q in range(a, b):
                producer[q] = i
            depth.append(d)
        passes += 1
        map_passes += any_dep
        rounds += 1 + max(depth)
    return {"passes": passes, "map_passes": map_passes, "rounds": rounds, "far_pieces": far, "pieces": len(ps)}


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    base = {}
    red = {}
    nl = nc = ntag = 0
    for f in range(frames):
        data = O.textgen_chunk(f * 40961, 65536)
        comp = O.snappy_encode(data)
        t = tags_of(comp)
        ntag += len(t)
        r, a, b = redirect(t, H, D)
        nl += a
        nc += b
        for k, v in model(t).items():
            base[k] = base.get(k, 0) + v
        for k, v in model(r).items():
            red[k] = red.get(k, 0) + v
    per = lambda d: {k: round(v / frames, 1) for k, v in d.items()}
    print(json.dumps({"frames": frames, "history": H, "hops": D, "tags_per_frame": round(ntag / frames, 1),
                      "to_literal_per_frame": round(nl / frames, 1), "copy_hops_per_frame": round(nc / frames, 1),
                      "baseline": per(base), "redirected": per(red)}))


if __name__ == "__main__":
    main()
