"""A second, independent restatement of FastLz.compress / FastLz.decompress
(codec-compression/src/main/java/io/netty/handler/codec/compression/FastLz.java:96-557), written
as a token emitter rather than a transcription of the Java control flow, cross-checks the C
oracle (oracle/netty_oracle.c orc_fastlz_compress / orc_fastlz_decompress).  The reference holds
no FastLZ byte vectors (FastLzIntegrationTest only round-trips), so two restatements that agree
byte for byte on every input below — including the readU16 quirk (:552-557), far matches
(level 2, :211-228, :310-331), runs (:165-176, :247-256) and level-1 long matches (:334-342) —
is the pin.  CPU only; the GPU kernels are checked against the C oracle elsewhere.
"""
import random

import pytest

MAX_DISTANCE = 8191                        # FastLz.java:31
MAX_FARDISTANCE = 65535 + MAX_DISTANCE - 1  # :32
HASH_MASK = (1 << 13) - 1                  # :34-36


def _literal_runs(lits):
    """Pending literals as FastLZ literal runs: at most 32 bytes each, header = count - 1."""
    out = bytearray()
    for i in range(0, len(lits), 32):
        run = lits[i:i + 32]
        out.append(len(run) - 1)
        out += run
    return out


def _match_token(level, length, dist):
    """One match: `length` = matched bytes - 2 (Java's biased len), `dist` = distance - 1."""
    t = bytearray()
    if level == 2:
        far = dist >= MAX_DISTANCE
        d = dist - MAX_DISTANCE if far else dist
        hi = 31 if far else d >> 8
        if length < 7:
            t.append((length << 5) | hi)
        else:
            t.append((7 << 5) | hi)
            length -= 7
            while length >= 255:
                t.append(255)
                length -= 255
            t.append(length)
        if far:
            t += bytes([255, d >> 8, d & 255])
        else:
            t.append(d & 255)
        return t
    while length > 262:  # MAX_LEN - 2: a level-1 token holds at most 264 bytes
        t += bytes([(7 << 5) | (dist >> 8), 253, dist & 255])
        length -= 262
    if length < 7:
        t += bytes([(length << 5) | (dist >> 8), dist & 255])
    else:
        t += bytes([(7 << 5) | (dist >> 8), length - 7, dist & 255])
    return t


def fastlz_compress_py(data: bytes, level: int, u16_limit=None, tail: bytes = b"") -> bytes:
    n = len(data)
    buf = bytes(data) + bytes(tail)
    lim = n if u16_limit is None else u16_limit
    if level == 0:
        level = 1 if n < 65536 else 2
    if n < 4:
        return b"" if n == 0 else bytes([n - 1]) + bytes(data)

    def u16(o):  # readU16 compares the index with readableBytes, not with the chunk end
        return buf[o] if o + 1 >= lim else buf[o] | (buf[o + 1] << 8)

    def hsh(o):
        v = u16(o)
        return (v ^ u16(o + 1) ^ (v >> 3)) & HASH_MASK

    table = [0] * (HASH_MASK + 1)
    out = bytearray()
    lits = bytearray(buf[0:2])
    ip, end_match, end_scan = 2, n - 2, n - 12
    while ip < end_scan:
        anchor = ip
        if level == 2 and buf[ip] == buf[ip - 1] and u16(ip - 1) == u16(ip + 1):
            dist, ref, mlen = 1, anchor + 2, 3  # a run of the previous byte
        else:
            slot = hsh(ip)
            cand = table[slot]
            table[slot] = anchor
            dist = anchor - cand
            limit = MAX_DISTANCE if level == 1 else MAX_FARDISTANCE
            ok = 0 < dist < limit and buf[cand:cand + 3] == buf[anchor:anchor + 3]
            mlen = 3
            if ok and level == 2 and dist >= MAX_DISTANCE:  # far: five bytes must match
                ok = buf[cand + 3:cand + 5] == buf[anchor + 3:anchor + 5]
                mlen = 5
            if not ok:
                lits.append(buf[anchor])
                ip = anchor + 1
                continue
            ref = cand + mlen
        ip = anchor + mlen
        dist -= 1
        if dist == 0:
            x = buf[ip - 1]
            while ip < end_match and buf[ref] == x:
                ref += 1
                ip += 1
        else:
            k = 0
            while k < 8:  # the first eight bytes unconditionally (the outer bound keeps them in the chunk)
                same = buf[ref] == buf[ip]
                ref += 1
                ip += 1
                k += 1
                if not same:
                    break
            else:
                while ip < end_match:
                    same = buf[ref] == buf[ip]
                    ref += 1
                    ip += 1
                    if not same:
                        break
        out += _literal_runs(lits)
        lits = bytearray()
        ip -= 3
        out += _match_token(level, ip - anchor, dist)
        for _ in range(2):  # hash the two positions after the match
            table[hsh(ip)] = ip
            ip += 1
    lits += buf[ip:n]
    out += _literal_runs(lits)
    if level == 2:
        out[0] |= 1 << 5
    return bytes(out)


def fastlz_decompress_py(src: bytes, out_len: int):
    """Java's return value (0 on a bad stream or short output) and the bytes produced."""
    level = (src[0] >> 5) + 1
    if level not in (1, 2):
        return -1, b""
    out = bytearray()
    ip = 1
    ctrl = src[0] & 31
    while True:
        if ctrl >= 32:
            length = (ctrl >> 5) - 1
            back = (ctrl & 31) << 8
            if length == 6:
                if level == 1:
                    length += src[ip]
                    ip += 1
                else:
                    while True:
                        c = src[ip]
                        ip += 1
                        length += c
                        if c != 255:
                            break
            c = src[ip]
            ip += 1
            back += c
            if level == 2 and c == 255 and (ctrl & 31) == 31:
                back = ((src[ip] << 8) | src[ip + 1]) + MAX_DISTANCE
                ip += 2
            if len(out) + length + 3 > out_len or len(out) - back - 1 < 0:
                return 0, bytes(out)
            start = len(out) - back - 1
            for i in range(length + 3):  # byte by byte: overlapping copies repeat their period
                out.append(out[start + i])
            if ip >= len(src):
                break
            ctrl = src[ip]
            ip += 1
        else:
            cnt = ctrl + 1
            if len(out) + cnt > out_len or ip + cnt > len(src):
                return 0, bytes(out)
            out += src[ip:ip + cnt]
            ip += cnt
            if ip >= len(src):
                break
            ctrl = src[ip]
            ip += 1
    return len(out), bytes(out)


def _corpus():
    rng = random.Random(7)
    words = [bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(rng.randint(2, 9))) for _ in range(300)]
    text = b" ".join(rng.choice(words) for _ in range(30000))
    cases = [b"", b"a", b"ab", b"abc", b"abcd", bytes(5), bytes(40), b"x" * 1000, b"ab" * 700]
    cases += [bytes(rng.getrandbits(8) for _ in range(n)) for n in (4, 13, 31, 32, 33, 100, 4096)]
    cases += [text[:n] for n in (12, 13, 14, 64, 1000, 8191, 8192, 65535, 65536, 70000, len(text))]
    block = bytes(rng.getrandbits(8) for _ in range(3000))
    for gap in (8100, 8189, 8190, 8191, 8192, 8193, 20000, 65000, 73000):  # far and out-of-reach repeats
        filler = bytes(rng.getrandbits(8) for _ in range(gap - len(block)))
        cases.append(block + filler + block + block[:100] + bytes(2000))
    cases.append(bytes(rng.getrandbits(8) for _ in range(500)) * 20)  # matches longer than 264 bytes
    cases.append(b"z" * 70000)  # one long run
    return cases


@pytest.mark.parametrize("level", [1, 2])
def test_fastlz_compress_restatements_agree(oracle, level):
    for data in _corpus():
        mine = fastlz_compress_py(data, level)
        assert mine == oracle.fastlz_compress(data, level), (level, len(data))
        if data:
            r, out = fastlz_decompress_py(mine, len(data))
            assert (r, out) == (len(data), data)


def test_fastlz_auto_level_restatements_agree(oracle):
    for data in _corpus():
        assert fastlz_compress_py(data, 0) == oracle.fastlz_compress(data, 0)


def test_fastlz_readu16_quirk_restatements_agree(oracle):
    """readU16 compares the ABSOLUTE index with readableBytes (FastLz.java:552-557): with a reader
    index > 0 the limit sits short of (or, with bytes after the chunk, past) the chunk end."""
    rng = random.Random(11)
    for data in _corpus()[9:]:
        n = len(data)
        tail = bytes(rng.getrandbits(8) for _ in range(8))
        for lim in (0, 1, n // 2, max(n - 3, 0), n - 1, n + 1, n + 4):
            for level in (1, 2):
                mine = fastlz_compress_py(data, level, u16_limit=lim, tail=tail)
                assert mine == oracle.fastlz_compress(data, level, u16_limit=lim, tail=tail), (n, lim, level)


def test_fastlz_decompress_restatements_agree(oracle):
    rng = random.Random(5)
    for data in _corpus():
        if not data:
            continue
        for level in (1, 2):
            comp = oracle.fastlz_compress(data, level)
            assert fastlz_decompress_py(comp, len(data)) == oracle.fastlz_decompress(comp, len(data))
            short = rng.randint(0, len(data) - 1)  # output buffer too small: Java returns 0
            assert fastlz_decompress_py(comp, short)[0] == oracle.fastlz_decompress(comp, short)[0] == 0
