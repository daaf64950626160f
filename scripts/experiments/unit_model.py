"""Model of a unit-lane Snappy record expander on the bench corpus (round 5 design study).

A wave expands one frame in groups of 64 aligned 16-byte output units (1 KiB), lane = unit.  A unit's
bytes come from its SEGMENTS (record ∩ unit), applied in stream order from a per-lane cursor; a segment
is ready when the bytes it reads are final: a literal always, a copy when its source lies before the
group, inside the lane's own unit (earlier bytes, already applied), or in a unit of the group that was
final at the start of the round.  Rounds repeat until every unit of the group is final.

Counts per frame: groups, rounds, segment iterations (the wave runs max-over-lanes iterations per round),
segments per unit, far segments (source older than the LDS history H).
Usage: python scripts/experiments/unit_model.py [frames] [unit] [group_units] [H]
"""
import sys

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from oracle import pyoracle as O  # noqa: E402
from scripts.experiments.sim_window import records  # noqa: E402


def model(recs, total, U=16, GU=64, H=16384):
    # per-byte owner record index
    starts = [r[3] for r in recs]
    lens = [r[1] for r in recs]
    isc = [r[0] for r in recs]
    src = [r[2] for r in recs]
    nunits = (total + U - 1) // U
    # segments of each unit: list of record indices
    segs = [[] for _ in range(nunits)]
    for i, (o, ln) in enumerate(zip(starts, lens)):
        for u in range(o // U, (o + ln - 1) // U + 1):
            segs[u].append(i)
    G = U * GU
    stats = dict(groups=0, rounds=0, iters=0, iters_r0=0, segs=0, far=0, maxsegs=0, applied_r0=0)
    for g0 in range(0, nunits, GU):
        units = range(g0, min(nunits, g0 + GU))
        Gs = g0 * U
        cur = {u: 0 for u in units}
        final = set()
        stats["groups"] += 1
        rnd = 0
        while len(final) < len(units):
            newly = set()
            it_max = 0
            for u in units:
                if u in final:
                    continue
                its = 0
                L = segs[u]
                while cur[u] < len(L):
                    i = L[cur[u]]
                    its += 1
                    if isc[i]:
                        o, d = starts[i], src[i]
                        q0 = max(o, u * U)
                        q1 = min(o + lens[i], (u + 1) * U)
                        lo = q0 - d if q0 - d < o else o - d
                        hi = min(q1 - d, o)
                        if hi <= lo:
                            hi = o
                        ok = True
                        for v in range(lo // U, (hi - 1) // U + 1):
                            if v * U + U <= Gs or v < g0:
                                continue
                            if v == u or v in final:
                                continue
                            ok = False
                        if not ok:
                            break
                        if rnd == 0 and lo < Gs + G - H:
                            stats["far"] += 1
                    cur[u] += 1
                    if rnd == 0:
                        stats["applied_r0"] += 1
                if cur[u] == len(L):
                    newly.add(u)
                it_max = max(it_max, its)
            final |= newly
            stats["iters"] += it_max
            if rnd == 0:
                stats["iters_r0"] += it_max
            rnd += 1
            if rnd > 10000:
                raise RuntimeError("stuck")
        stats["rounds"] += rnd
    stats["segs"] = sum(len(s) for s in segs)
    stats["maxsegs"] = max(len(s) for s in segs)
    return stats


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    U = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    GU = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    H = int(sys.argv[4]) if len(sys.argv) > 4 else 16384
    acc = {}
    for f in range(frames):
        data = O.textgen_chunk(f * 6553 + 17)
        blk = O.snappy_encode(data)
        recs, total = records(blk)
        s = model(recs, total, U, GU, H)
        s["records"] = len(recs)
        for k, v in s.items():
            acc[k] = acc.get(k, 0) + v
    print({k: round(v / frames, 1) for k, v in acc.items()})


if __name__ == "__main__":
    main()
