"""CPU model of k_expand's pass structure (round 6; experiments only, uses the oracle as the encoder).

Encodes configs[4]-style text chunks with the oracle, cuts each Snappy stream into k_parse's records
(literals and copies split at 64 bytes), the output into pieces (record ∩ aligned dword) and the pieces
into passes of 64, ignoring window boundaries, and counts per frame: pieces, passes, dependency rounds
(a near copy waits for the pieces producing its source bytes in the same pass; overlapping copies read
their period from before the record), passes holding an overlapping copy (has_ov), and of those, passes
in which some overlapping piece's 4 bytes wrap around its period.
    python scripts/experiments/expand_model.py [frames]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import pyoracle as O  # noqa: E402


def records(z):
    i, n = 0, 0
    while z[i] & 0x80:
        i += 1
    i += 1
    op = 0
    out = []
    while i < len(z):
        t = z[i]
        i += 1
        ty = t & 3
        if ty == 0:
            L = t >> 2
            if L >= 60:
                nb = L - 59
                L = int.from_bytes(z[i:i + nb], "little")
                i += nb
            L += 1
            for k in range(0, L, 64):
                m = min(64, L - k)
                out.append((op, m, None))
                op += m
            i += L
        else:
            if ty == 1:
                L = 4 + ((t >> 2) & 7)
                off = ((t & 0xE0) << 3) | z[i]
                i += 1
            elif ty == 2:
                L = 1 + (t >> 2)
                off = int.from_bytes(z[i:i + 2], "little")
                i += 2
            else:
                L = 1 + (t >> 2)
                off = int.from_bytes(z[i:i + 4], "little")
                i += 4
            for k in range(0, L, 64):
                m = min(64, L - k)
                out.append((op, m, off))
                op += m
    return out, op


def model(z):
    recs, O_ = records(z)
    pieces = []  # (x0, x1, rec)
    for r, (s, m, off) in enumerate(recs):
        x = s
        while x < s + m:
            e = min((x // 4 + 1) * 4, s + m)
            pieces.append((x, e, r))
            x = e
    st = dict(pieces=len(pieces), passes=0, rounds=0, dep_passes=0, ov_passes=0, wrap_passes=0, ov_pieces=0, wrap_pieces=0)
    for p0 in range(0, len(pieces), 64):
        P = pieces[p0:p0 + 64]
        ps, pe = P[0][0], P[-1][1]
        owner = {}
        for j, (a, b, r) in enumerate(P):
            for x in range(a, b):
                owner[x] = j
        depth = [0] * len(P)
        has_ov = has_wrap = False
        dep_any = False
        for j, (a, b, r) in enumerate(P):
            s, m, off = recs[r]
            if off is None:
                continue
            overlap = off < m
            if overlap:
                has_ov = True
                st["ov_pieces"] += 1
                n0 = a - s
                if (n0 % off) + (b - a) > off:
                    has_wrap = True
                    st["wrap_pieces"] += 1
                lo, hi = s - off, s
            else:
                lo, hi = a - off, b - off
            if hi <= ps or (pe > 4096 and lo < pe - 4096 and not overlap):
                continue
            d = 0
            for x in range(max(lo, ps), hi):
                if x in owner:
                    d = max(d, depth[owner[x]] + 1)
            depth[j] = d
            dep_any = dep_any or d > 0
        st["passes"] += 1
        st["rounds"] += 1 + max(depth)
        st["dep_passes"] += dep_any
        st["ov_passes"] += has_ov
        st["wrap_passes"] += has_wrap
    return st


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    O.build()
    tot = {}
    for i in range(n):
        z = O.snappy_encode(O.textgen_chunk(i * (1638400 // n), 65536))
        for k, v in model(z).items():
            tot[k] = tot.get(k, 0) + v
    print({k: round(v / n, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
