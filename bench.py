"""bench.py — BASELINE.json metric: "GiB/s device-resident Snappy encode+decode, 64 KiB chunks, 1/2/4/8 MI355X".

One step = one pass of the hot path over every chunk of the job, device-resident:
    encode leg: masked CRC32C of every 64 KiB chunk (SnappyFrameEncoder.calculateAndWriteChecksum)
                + Snappy.encode of every chunk            (configs[1])
    decode leg: Snappy.decode of every chunk + CRC32C verify against the stored checksum (configs[2])
value = Σ uncompressed bytes of all ranks / (max over ranks of the timed wall time) / 2^30,
i.e. the round-trip rate Σ U / (t_enc + t_dec) of SURVEY.md §8d.

Workload (`value`): configs[4] — 100 GiB = 1 638 400 text-like 64 KiB chunks split across the ranks
(STRONG scaling: the job is the same 100 GiB at N = 1, 2, 4, 8).  Each rank generates its contiguous
shard of chunk indices on its own device (no host transfer) and runs it in sub-batches that fit HBM;
the inputs of the whole shard are resident before the timed region starts.  A second, separate leg
(`weak_1m_per_gpu`) runs configs[1]+[2] as stated: 1 048 576 chunks per GPU.

Multi-GPU: `python bench.py --gpus N` with no WORLD_SIZE in the environment starts N worker
processes itself (spawn, before any GPU call in the parent); under torchrun (WORLD_SIZE set) each
process is one rank.  Ranks talk over RCCL (backend "nccl") only for the timing barrier, the
max-over-ranks reduction and one all-gather of per-rank compressed byte totals (the offset exchange
that lays the shards out as one stream, netty_amd/shard.py), all outside the data path.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--total-chunks C] [--no-cpu-baseline]
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident Snappy encode+decode, 64 KiB chunks, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CHUNK = 65536
CONFIG5_CHUNKS = 1638400  # 100 GiB of 64 KiB chunks
# kernels whose PMC traffic backs roofline.traffic; the summary must have been taken on these sources
PMC_SOURCES = ("netty_amd/csrc/snappy_encode.hip", "netty_amd/csrc/snappy_decode.hip", "netty_amd/csrc/crc32c.hip",
               "netty_amd/csrc/nx_common.hpp", "netty_amd/csrc/workspace.hpp")  # (workspace.hpp: the launch geometry)
# the alt-codec legs' kernels (their parses share the Snappy decoder's translation unit and expander)
ALT_PMC_SOURCES = ("netty_amd/csrc/fastlz.hip", "netty_amd/csrc/lzf.hip", "netty_amd/csrc/lz4.hip",
                   "netty_amd/csrc/snappy_decode.hip", "netty_amd/csrc/nx_common.hpp", "netty_amd/csrc/workspace.hpp")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--total-chunks", type=int, default=CONFIG5_CHUNKS,
                    help="64 KiB chunks of the whole job, split across ranks (configs[4]: 1 638 400 = 100 GiB)")
    ap.add_argument("--sub-chunks", type=int, default=0,
                    help="chunks per encode and decode call (0: the library's encode plan, decode calls of 262 144)")
    ap.add_argument("--weak-chunks", type=int, default=1 << 20,
                    help="chunks per GPU of the separate configs[1]+[2] leg (0 = skip)")
    ap.add_argument("--weak-steps", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-sample", type=int, default=32768,
                    help="first-sub-batch chunks the cpu_baseline leg checks against the oracle byte for byte")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (H2D/D2H) end-to-end measurement")
    ap.add_argument("--e2e-channels", type=int, default=256, help="C-ABI end-to-end: channels (handler pairs)")
    ap.add_argument("--e2e-messages", type=int, default=256, help="C-ABI end-to-end: 64 KiB messages per channel")
    ap.add_argument("--e2e-chunks", type=int, default=131072, help="chunks through the torch host pipeline (8 GiB)")
    ap.add_argument("--e2e-sub", type=int, default=65536, help="chunks per pipelined sub-batch")
    ap.add_argument("--no-alt", action="store_true", help="skip the FastLZ/LZF/LZ4 (configs[3]) measurement")
    ap.add_argument("--no-probe-ceiling", action="store_true", help="skip the live random-access ceiling of the encoder")
    ap.add_argument("--alt-chunks", type=int, default=262144)
    ap.add_argument("--hc-chunks", type=int, default=1024, help="chunks of the LZ4 HC (highCompressor) leg (0 = skip)")
    ap.add_argument("--no-latency", action="store_true", help="skip the per-batch-size latency leg")
    ap.add_argument("--no-frame-scan", action="store_true", help="skip the framed-stream (§8f row 1) measurement")
    ap.add_argument("--scan-chunks", type=int, default=131072, help="chunks laid out as framed streams")
    ap.add_argument("--scan-per-stream", type=int, default=64, help="chunks per stream (one cumulation each)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------- CPU baseline
def host_cores() -> int:
    """CPUs this process may actually use: the affinity mask, capped by a cgroup CPU quota (on the GPU
    box the affinity mask shows the whole machine while the job's share is a quota)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def take_gpu_sample(torch, B, leg, k: int):
    """Every (m // k)-th chunk of the leg's first decode call as the GPU left it (compressed bytes and
    masked CRC32C), on the host: the input of cpu_baseline's parity check.  No oracle here."""
    lo, m = leg.run_prefix()  # the first decode call's chunks, encoded as the timed steps encode them
    k = max(1, min(k, m))
    step = m // k
    idx = torch.arange(0, step * k, step, dtype=torch.int64, device=leg.dev)
    packed, poff = B.gather(leg.enc, leg.eoff[lo + idx], leg.elen[lo + idx])
    torch.cuda.synchronize()
    return {"first": leg.first + lo, "step": step, "index": idx.cpu().tolist(), "bytes": packed.cpu().numpy().tobytes(),
            "off": poff.cpu().tolist(), "len": leg.elen[lo + idx].cpu().tolist(),
            "crc": [c & 0xFFFFFFFF for c in leg.crc[lo + idx].cpu().tolist()]}


def parity_check(O, sample, threads: int):
    """The oracle's Snappy.encode and masked CRC32C of each sampled chunk (regenerated from its index,
    include/netty_amd_textgen.h) against the GPU's bytes, on `threads` host threads."""
    from concurrent.futures import ThreadPoolExecutor
    idx, buf = sample["index"], sample["bytes"]

    def one(j):
        src = O.textgen_chunk(sample["first"] + idx[j], CHUNK)
        want = O.snappy_encode(src)
        got = buf[sample["off"][j]:sample["off"][j] + sample["len"][j]]
        return (got != want), (O.snappy_checksum(src) != sample["crc"][j])

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, range(len(idx))))
    bad = sum(1 for a, _ in res if a)
    badc = sum(1 for _, c in res if c)
    return {"chunks": len(idx), "stride": sample["step"], "compressed_bytes": len(buf), "encode_mismatches": bad,
            "crc_mismatches": badc, "verified": bad == 0 and badc == 0, "seconds": round(time.perf_counter() - t0, 2),
            "note": "bench workload chunks (first sub-batch, every stride-th) encoded by the GPU in the timed path "
                    "vs the oracle's Snappy.encode and masked CRC32C, byte for byte"}


def cpu_baseline(seconds: float, gpu_sample=None):
    """The oracle (C restatement of Snappy.encode/decode + Crc32c, byte-at-a-time CRC like Crc32c.java)
    timed on this host: encode+CRC then decode+CRC-verify of text-like 64 KiB chunks, one thread per
    available core; plus configs[0] (1 MiB java.util.Random(42) frame round trip) and a per-codec
    configs[3] sample, single-thread.  With `gpu_sample` (take_gpu_sample) the oracle also checks
    those GPU outputs (`gpu_parity_sample`)."""
    import ctypes as C
    from concurrent.futures import ThreadPoolExecutor

    from oracle import pyoracle as O

    L = O.lib()
    nchunk = 64
    chunks = [O.textgen_chunk(i, CHUNK) for i in range(nchunk)]
    cap = L.orc_snappy_max_compressed_length(CHUNK)

    def work(deadline):
        out = (C.c_uint8 * cap)()
        dec = (C.c_uint8 * CHUNK)()
        olen, cons = C.c_size_t(0), C.c_size_t(0)
        done = 0
        i = 0
        while time.perf_counter() < deadline:
            c = chunks[i % nchunk]
            crc = L.orc_snappy_checksum(c, CHUNK)
            n = L.orc_snappy_encode(c, CHUNK, out)
            st = L.orc_snappy_decode(C.cast(out, C.c_char_p), n, dec, CHUNK, C.byref(olen), C.byref(cons))
            crc2 = L.orc_snappy_checksum(C.cast(dec, C.c_char_p), olen.value)
            assert st == 0 and olen.value == CHUNK and crc == crc2
            done += 1
            i += 1
        return done

    t0 = time.perf_counter()
    d1 = work(t0 + seconds / 4)
    t1 = time.perf_counter()
    single = d1 * CHUNK / (t1 - t0) / 2**30
    threads = host_cores()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL during the C calls
        counts = list(ex.map(work, [t0 + seconds / 2] * threads))
    t1 = time.perf_counter()
    multi = sum(counts) * CHUNK / (t1 - t0) / 2**30
    out = {"value": round(multi, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
           "sample": f"oracle/netty_oracle.c encode+CRC32C then decode+verify of text-like 64 KiB chunks, "
                     f"{sum(counts)} chunks on {threads} threads in {t1 - t0:.1f}s (+ {d1} chunks single-thread)",
           "single_thread_value": round(single, 4),
           "config1_frame_round_trip": config1_cpu(O, seconds / 8),
           "config4_per_codec": config4_cpu(O, seconds / 8)}
    if gpu_sample is not None:
        out["gpu_parity_sample"] = parity_check(O, gpu_sample, threads)
    return out


def config1_cpu(O, seconds: float):
    """configs[0]: SnappyFrameEncoder then SnappyFrameDecoder (validating) over the 1 MiB
    java.util.Random(42) message of AbstractIntegrationTest.java:106-112, default (32767-byte slices)
    and jumbo (65535) framing; identity checked; single thread; GiB/s of the 1 MiB message."""
    data = O.java_random_bytes(42, 1 << 20)
    res = {}
    for name, jumbo in (("default", False), ("jumbo", True)):
        reps, t0 = 0, time.perf_counter()
        while True:
            framed, _ = O.snappy_frame_encode(data, jumbo=jumbo)
            out = bytearray()
            p = 10  # stream identifier
            while p < len(framed):
                typ, ln = framed[p], int.from_bytes(framed[p + 1:p + 4], "little")
                crc = int.from_bytes(framed[p + 4:p + 8], "little")
                body = framed[p + 8:p + 4 + ln]
                if typ == 0:
                    st, dec, _ = O.snappy_decode(body, 65536)
                    assert st == 0
                else:
                    dec = body
                assert O.snappy_checksum(dec) == crc
                out += dec
                p += 4 + ln
            assert bytes(out) == data
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds / 2:
                break
        res[name] = {"gib_s": round(reps * len(data) / dt / 2**30, 4), "round_trips": reps,
                     "framed_bytes": len(framed)}
    return res


def config4_cpu(O, seconds: float):
    """configs[3] CPU beside-rate per codec and direction: the oracle on a mixed sample (sizes uniform in
    [4096, 65535], half text-like, half random), single thread, GiB/s of uncompressed bytes."""
    import random
    rnd = random.Random(1234)
    sample = []
    for i in range(16):
        n = rnd.randrange(4096, 65536)
        sample.append(O.textgen_chunk(i, n) if i % 2 == 0 else rnd.randbytes(n))
    U = sum(len(s) for s in sample)
    per = seconds / 8

    def rate(fn, inputs):
        reps, t0 = 0, time.perf_counter()
        while True:
            for x in inputs:
                fn(x)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= per:
                return round(reps * U / dt / 2**30, 4)

    res = {"sample": "16 chunks, sizes uniform [4096, 65535], half text-like, half random", "threads": 1}
    for lv in (1, 2):
        enc = [O.fastlz_compress(s, lv) for s in sample]
        res[f"fastlz_l{lv}"] = {"encode_gib_s": rate(lambda s: O.fastlz_compress(s, lv), sample),
                                "decode_gib_s": rate(lambda e: O.fastlz_decompress(e[0], e[1]),
                                                     [(e, len(s)) for e, s in zip(enc, sample)])}
    lz = [O.lzf_compress_body(s) for s in sample]
    res["lzf"] = {"encode_gib_s": rate(O.lzf_compress_body, sample),
                  "decode_gib_s": rate(lambda e: O.lzf_decode_chunk(e[0], e[1]), [(e, len(s)) for e, s in zip(lz, sample)])}
    z4 = [O.lz4_compress(s) for s in sample]
    res["lz4"] = {"encode_gib_s": rate(O.lz4_compress, sample),
                  "decode_gib_s": rate(lambda e: O.lz4_decompress(e[0], e[1]), [(e, len(s)) for e, s in zip(z4, sample)])}
    # LZ4 HC (Lz4FrameEncoder(highCompressor = true): LZ4_compress_HC level 9), single thread and on every
    # host core (the beside-rate the GPU's alt_codecs.lz4_hc leg is compared with)
    from concurrent.futures import ThreadPoolExecutor
    threads = host_cores()

    def hc_worker(deadline):
        done = 0
        while time.perf_counter() < deadline:
            for x in sample:
                O.lz4hc_compress(x)
            done += 1
        return done

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:  # ctypes releases the GIL inside the C call
        reps = sum(ex.map(hc_worker, [t0 + 2 * per] * threads))
    t1 = time.perf_counter()
    res["lz4_hc"] = {"encode_gib_s": rate(O.lz4hc_compress, sample),
                     "encode_gib_s_all_cores": round(reps * U / (t1 - t0) / 2**30, 4), "cores": threads,
                     "note": "oracle/netty_oracle.c orc_lz4hc_compress (liblz4 level 9 restated, pinned byte-equal to liblz4)"}
    try:  # the library lz4-java's highCompressor() wraps: liblz4 level 9 (pyarrow's bundled copy), same sample
        import pyarrow as pa
        z = pa.Codec("lz4_raw", compression_level=9)

        def lib_worker(deadline):
            done = 0
            while time.perf_counter() < deadline:
                for x in sample:
                    z.compress(x)
                done += 1
            return done

        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            reps = sum(ex.map(lib_worker, [t0 + 2 * per] * threads))
        t1 = time.perf_counter()
        res["lz4_hc"]["liblz4_level9"] = {"encode_gib_s": rate(lambda x: z.compress(x), sample),
                                          "encode_gib_s_all_cores": round(reps * U / (t1 - t0) / 2**30, 4),
                                          "library": "liblz4 1.10.0 in pyarrow " + pa.__version__}
    except ImportError:
        pass
    return res


# ---------------------------------------------------------------------------------------- PMC traffic
def source_digest(paths=PMC_SOURCES) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(os.path.join(ROOT, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def alt_source_digest() -> str:
    return source_digest(ALT_PMC_SOURCES)


def load_alt_traffic():
    """HBM bytes per call of each alt-codec leg's encode / decode from the newest committed
    alt_traffic.json (scripts/pmc_alt_traffic.sh) taken on these kernel sources, else (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "alt_traffic.json"), recursive=True),
                   key=os.path.getmtime)
    want = alt_source_digest()
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("source_digest") == want:
            return d["legs"], os.path.relpath(f, ROOT)
    return None, f"no alt-codec PMC summary for kernel sources {want} (run scripts/pmc_alt_traffic.sh)"


def load_traffic():
    """Per-chunk HBM bytes per kernel from the newest committed PMC summary (scripts/pmc_traffic.sh:
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench's workload).  The summary
    records the digest of the kernel sources it was taken on; a summary of other sources is stale and
    is not used (roofline.traffic is then null with the reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "pmc_traffic.json"), recursive=True),
                   key=os.path.getmtime)
    want = source_digest()
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("source_digest") == want:
            return {k: v["hbm_bytes_per_chunk"] for k, v in d["kernels"].items()}, os.path.relpath(f, ROOT)
    return None, f"no PMC summary for kernel sources {want} (run scripts/pmc_traffic.sh)"


def load_issue():
    """Per-kernel issue counters (scripts/pmc_issue.sh: instruction mix per chunk, VALU busy, wave-state
    split) from the newest committed pmc_issue.json taken on these kernel sources, else (None, reason)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "pmc_issue.json"), recursive=True), key=os.path.getmtime)
    want = source_digest()
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("source_digest") == want:
            return d["kernels"], os.path.relpath(f, ROOT)
    return None, f"no issue-counter summary for kernel sources {want} (run scripts/pmc_issue.sh)"


CLOCK_GHZ = 2.4  # MI355X max engine clock (MI355X_MICROARCH.md): the issue capacity's upper bound


def issue_ceiling(issue, kernels, frames_per_launch: int, ms_per_launch: float, simds: int):
    """roofline_decode.issue: the decoder's instruction stream against the chip's
    issue capacity.  Per frame: wave-instructions by type summed over the kernels (PMC); live: VALU
    busy = 2 cycles per wave64 VALU instruction x instructions per launch / (SIMDs x 2.4 GHz x the
    launch's HIP-event time), a lower bound on the busy fraction (the chip runs below 2.4 GHz under load);
    per kernel: VALU busy and the wave-state split measured in the profiled run itself."""
    ks, src = issue
    if not ks:
        return {"source": src}
    per = {}
    rows = {}
    for name, v in ks.items():
        base = name.split("<")[0]
        if not any(base == k.split("<")[0] for k in kernels):
            continue
        for t, x in v["insts_per_chunk"].items():
            per[t] = per.get(t, 0.0) + x
        rows[base] = {"valu_busy_profiled": round(v["valu_busy"], 4) if v.get("valu_busy") is not None else None,
                      "insts_per_simd_cycle_profiled": round(v["insts_per_simd_cycle"], 4) if v.get("insts_per_simd_cycle") else None,
                      "wave_split": {k: round(x, 4) for k, x in v.get("wave_split", {}).items()},
                      "insts_per_frame": {t: round(x) for t, x in v["insts_per_chunk"].items()}}
    if not per:
        return {"source": src}
    valu_cycles = 2.0 * per.get("VALU", 0.0) * frames_per_launch
    cap = simds * CLOCK_GHZ * 1e9 * (ms_per_launch / 1e3)
    return {"bound": "issue", "unit": "wave-instructions per frame", "insts_per_frame": {t: round(x) for t, x in per.items()},
            "valu_salu_lds_per_frame": round(per.get("VALU", 0) + per.get("SALU", 0) + per.get("LDS", 0)),
            "frames_per_launch": frames_per_launch, "ms_per_launch": round(ms_per_launch, 3),
            "valu_busy_live": round(valu_cycles / cap, 4) if cap else None,
            "all_insts_per_simd_cycle_live": round(sum(per.values()) * frames_per_launch / cap, 4) if cap else None,
            "clock_ghz_assumed": CLOCK_GHZ, "simds": simds, "kernels": rows, "source": src}


# ---------------------------------------------------------------------------------------- the GPU leg
DEC_SUB = 262144  # frames per decode call: one k_parse / k_expand pair (snappy_decode.hip kSubBatch)


class SnappyRoundTrip:
    """One rank's shard [first, first + n) of text-like 64 KiB chunks: the whole shard's inputs are
    generated on the device up front; a step runs CRC32C + encode and decode/verify over them as a
    schedule of calls (`ops`) whose buffers are reused.

    Encode calls follow the library's launch plan (nx_snappy_encode_plan: equal full-occupancy
    launches, e.g. 5 x 327 680 chunks per 100 GiB on 256 CUs; round 6), so each
    call is one launch of the dense encoder.  Decode calls take DEC_SUB frames at a time as soon as
    that many are encoded (one parse/expand pair each; the last call takes the rest), reading the
    compressed chunks from a ring of encode slots that holds every chunk between its encode and its
    decode.  `sub` (tests, --sub-chunks) fixes both sizes instead.  The compressed bytes of every chunk
    are kept only as per-chunk lengths; the decoded bytes are checked against the inputs after the
    timed region."""

    def __init__(self, torch, dev, first: int, n: int, sub: int = 0, dec_sub: int = DEC_SUB, enc_sizes=None):
        from netty_amd import batch as B
        from netty_amd import _lib
        self.torch, self.B, self.dev = torch, B, dev
        self.first, self.n = first, n
        self.cap = (B.snappy_max_compressed_length(CHUNK) + 15) // 16 * 16
        L = _lib.load()
        st = torch.cuda.current_stream(dev).cuda_stream
        if enc_sizes:  # tests: an explicit schedule
            assert sum(enc_sizes) == n
            self.enc_sizes, self.dec_sub = list(enc_sizes), max(1, min(dec_sub, n))
        elif sub:
            sub = max(1, min(sub, n))
            self.enc_sizes = [min(sub, n - lo) for lo in range(0, n, sub)]
            self.dec_sub = sub
        else:
            self.enc_sizes = encode_plan(n)
            self.dec_sub = max(1, min(dec_sub, n))
        # place the encoder's table workspace before the shard's buffers take the memory its
        # placement choice draws candidates from (as a server would at start-up).  This
        # process owns the device, so the placement may draw as many candidates as memory allows.
        assert L.nx_workspace_placement_config(2**64 - 1, 0) == 0
        rc = L.nx_snappy_encoder_reserve(max(self.enc_sizes), st)
        assert rc == 0, f"nx_snappy_encoder_reserve: {rc}"
        if not sub and not enc_sizes:
            assert encode_plan(n) == self.enc_sizes, "the plan changed with the reserved workspace"
        self.ops = schedule(self.enc_sizes, self.dec_sub)
        self.sub = next(m for kind, _, m in self.ops if kind == "dec")  # the first decode call's frames
        # encode ring: chunk c's compressed bytes live in slot c mod R until their decode
        R = min(n, max(self.enc_sizes) + self.dec_sub - 1)
        self.ring = R
        self.src = torch.empty(n * CHUNK, dtype=torch.uint8, device=dev)
        tg = max(self.enc_sizes)
        for lo in range(0, n, tg):  # textgen in pieces keeps its temporaries small
            B.textgen(self.src[lo * CHUNK:], first + lo, min(tg, n - lo), CHUNK)
        w = max(max(self.enc_sizes), self.dec_sub)
        self.off = torch.arange(w, dtype=torch.int64, device=dev) * CHUNK
        self.soff = torch.arange(n, dtype=torch.int64, device=dev) * CHUNK  # chunk c's input at c * CHUNK
        self.ln = torch.full((w,), CHUNK, dtype=torch.int32, device=dev)
        self.enc = torch.empty(R * self.cap, dtype=torch.uint8, device=dev)
        self.eoff = (torch.arange(n, dtype=torch.int64, device=dev) % R) * self.cap
        self.dec = torch.empty(self.dec_sub * CHUNK, dtype=torch.uint8, device=dev)
        self.elen = torch.empty(n, dtype=torch.int32, device=dev)
        self.est = torch.empty(n, dtype=torch.int32, device=dev)
        self.crc = torch.empty(n, dtype=torch.int32, device=dev)
        self.dlen = torch.empty(n, dtype=torch.int32, device=dev)
        self.dst = torch.empty(n, dtype=torch.int32, device=dev)
        self.ev = {k: [] for k in ("crc", "enc", "dec")}
        torch.cuda.synchronize(dev)

    def plan_info(self):
        return {"encode_calls": self.enc_sizes, "decode_calls": [m for kind, _, m in self.ops if kind == "dec"],
                "encode_ring_slots": self.ring}

    def batches(self):
        """the encode calls' chunk ranges"""
        for kind, lo, m in self.ops:
            if kind == "enc":
                yield lo, m

    def enc_op(self, lo, m, record=False):
        torch, B = self.torch, self.B
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if record else None
        if record:
            e[0].record()
        B.crc32c_masked(self.src, self.soff[lo:lo + m], self.ln[:m], out=self.crc[lo:lo + m])
        if record:
            e[1].record()
        B.snappy_encode(self.src, self.soff[lo:lo + m], self.ln[:m], self.enc, self.eoff[lo:lo + m], out_len=self.elen[lo:lo + m],
                        status=self.est[lo:lo + m])
        if record:
            e[2].record()
            self.ev["crc"].append((e[0], e[1]))
            self.ev["enc"].append((e[1], e[2]))

    def dec_op(self, lo, m, record=False, expected=None):
        torch, B = self.torch, self.B
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if record else None
        if record:
            e[0].record()
        B.snappy_decode(self.enc, self.eoff[lo:lo + m], self.elen[lo:lo + m], self.dec, self.off[:m],
                        expected_crc=self.crc[lo:lo + m] if expected is None else expected,
                        out_len=self.dlen[lo:lo + m], status=self.dst[lo:lo + m])
        if record:
            e[1].record()
            self.ev["dec"].append((e[0], e[1]))

    def run_op(self, op, record=False, expected=None):
        kind, lo, m = op
        if kind == "enc":
            self.enc_op(lo, m, record)
        else:
            self.dec_op(lo, m, record, expected)

    def run_sub(self, lo, m):
        """encode then decode chunks [lo, lo + m) (m <= the decode buffer's frames), outside the schedule"""
        assert m <= self.dec_sub and m <= self.ring
        self.enc_op(lo, m)
        self.dec_op(lo, m)

    def run_prefix(self, expected=None):
        """the schedule up to and including its first decode call (its frames' compressed bytes are then
        in the ring and their decoded bytes in `dec`); `expected` replaces that call's CRCs"""
        for op in self.ops:
            self.run_op(op, expected=expected if op[0] == "dec" else None)
            if op[0] == "dec":
                return op[1], op[2]

    def step(self, record=False):
        for op in self.ops:
            self.run_op(op, record)

    def kernel_ms_per_step(self, steps: int):
        def tot(pairs):
            return sum(a.elapsed_time(b) for a, b in pairs) / max(1, steps)
        return tot(self.ev["crc"]), tot(self.ev["enc"]), tot(self.ev["dec"])

    def verify(self, rank: int):
        """Outside the timed region: every status 0 and length right, decode(encode(x)) == x for every
        chunk, and a 2 % subset with corrupted expected CRCs flagged (and nothing else)."""
        torch = self.torch
        ok = True
        for op in self.ops:
            self.run_op(op)
            kind, lo, m = op
            if kind == "dec":
                ok = ok and bool(torch.equal(self.dec[:m * CHUNK], self.src[lo * CHUNK:(lo + m) * CHUNK]))
        ok = (ok and int((self.est != 0).sum()) == 0 and int((self.dst != 0).sum()) == 0
              and bool(torch.equal(self.dlen, torch.full_like(self.dlen, CHUNK))))
        m = self.sub
        g = torch.Generator(device=self.dev).manual_seed(77 + rank)
        bad = torch.rand(m, device=self.dev, generator=g) < 0.02
        crc = self.crc[:m].clone()
        self.run_prefix(expected=torch.where(bad, crc ^ 1, crc))
        d = self.dst[:m]
        detect = bool(torch.equal(d != 0, bad)) and bool(torch.equal(d[bad], torch.full_like(d[bad], -7)))
        self.run_prefix()  # leave the first decode call's buffers decoded with the right CRCs
        return ok and detect, detect

    def comp_bytes(self) -> int:
        return int(self.elen.to(self.torch.int64).sum().item())


def encode_plan(n: int):
    """The library's encode launches for n chunks on the current device (nx_snappy_encode_plan)."""
    import ctypes
    from netty_amd import _lib
    L = _lib.load()
    cap = 4096
    sizes = (ctypes.c_uint32 * cap)()
    cnt = ctypes.c_uint32(0)
    assert L.nx_snappy_encode_plan(n, sizes, cap, ctypes.byref(cnt)) == 0
    assert 0 < cnt.value <= cap
    out = [sizes[i] for i in range(cnt.value)]
    assert sum(out) == n
    return out


def schedule(enc_sizes, dec_sub: int):
    """The step's calls in order: each encode call, then a decode call of dec_sub frames whenever that
    many are encoded and not yet decoded, the rest after the last encode.  [(kind, first chunk, chunks)]"""
    ops, enc_done, dec_done = [], 0, 0
    for m in enc_sizes:
        ops.append(("enc", enc_done, m))
        enc_done += m
        while enc_done - dec_done >= dec_sub:
            ops.append(("dec", dec_done, dec_sub))
            dec_done += dec_sub
    if enc_done > dec_done:
        ops.append(("dec", dec_done, enc_done - dec_done))
    return ops


def copy_rate_gbs(torch, a, b):
    ts = []
    for _ in range(3):
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x.record()
        b.copy_(a)
        y.record()
        torch.cuda.synchronize()
        ts.append(x.elapsed_time(y))
    return 2 * a.numel() / (min(ts) / 1e3) / 1e9


def roofline(algo_bytes, ms, n_chunks, kernels, traffic, copy_gbs):
    a = algo_bytes / (ms / 1e3) / 1e9
    tr, src = traffic
    per_chunk = (sum(v for k2, v in tr.items() if any(k2.split("<")[0] == k.split("<")[0] for k in kernels))
                 if tr else None)
    return {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(a / HBM_PEAK_GBS, 4),
            "traffic": round(per_chunk * n_chunks) if per_chunk else None,
            "traffic_per_chunk": round(per_chunk) if per_chunk else None,
            "traffic_source": src,
            "algorithmic_per_chunk": round(algo_bytes / n_chunks),
            "achievable_copy_gbs": round(copy_gbs, 1) if copy_gbs else None,
            "frac_of_achievable": round(a / copy_gbs, 4) if copy_gbs else None,
            "kernel": " + ".join(kernels)}


ENC_KERNELS = ["nx::enc::k_snappy_encode"]
# Snappy.encode's random table traffic per 64 KiB chunk of the bench corpus: table probes (one
# exchange of a random 64-bit slot each), inserts (one store after each match, :187-188) and first
# reads of a candidate's input (with the wide table entries — exact word + 3 following bytes — only
# matches of 7+ bytes read the candidate).  Pinned by tests/test_bench_census.py to the oracle's
# census (oracle/netty_oracle.c orc_snappy_encode_census) over chunks spread across configs[4]: the
# bench itself runs no oracle code outside its cpu_baseline leg.
ENC_PROBES_PER_CHUNK = 16546
ENC_INSERTS_PER_CHUNK = 7724
ENC_CANDIDATE_LOADS_PER_CHUNK = 4275


def probe_ceiling(torch, dev, lanes=None, steps=16384):
    """The random-access ceiling of the encoder's request pattern on this GPU (netty_amd/tools/
    probe_ceiling.hip: per lane a serial chain of 64-bit table exchanges + the encoder's share of
    dependent input loads over its own regions, with and without the encoder's share of insert
    stores, at the encoder's resident lane count).  Returns {"with_inserts", "no_inserts"} probes/s,
    or None."""
    import ctypes
    path = os.path.join(ROOT, "netty_amd", "libnx_probe_ceiling.so")
    if not os.path.exists(path):
        return None
    if lanes is None:  # the encoder's resident lanes: 20 waves per CU (snappy_encode.hip)
        lanes = torch.cuda.get_device_properties(dev).multi_processor_count * 20 * 64
    lib = ctypes.CDLL(path)
    lib.nx_probe_ceiling.restype = ctypes.c_int32
    lib.nx_probe_ceiling.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
    # The rate depends on where the table lands; the encoder's workspace is the best of
    # six placements (nx_common.hpp alloc_placed_workspace), so the ceiling is too: the fastest of up
    # to six tables held at once (each drawn while the others stay allocated; fewer if memory is short).
    # With three, a box whose three draws all landed slowly reported a ceiling below the encoder's rate.
    inp = torch.empty(lanes * 16384, dtype=torch.int32, device=dev)
    sink = torch.empty(lanes, dtype=torch.int32, device=dev)
    loads = round(1000 * ENC_CANDIDATE_LOADS_PER_CHUNK / ENC_PROBES_PER_CHUNK)
    inserts = round(1000 * ENC_INSERTS_PER_CHUNK / ENC_PROBES_PER_CHUNK)
    tabs, best, per = [], {}, []
    for k in range(6):
        if k and torch.cuda.mem_get_info(dev)[0] < lanes * 16384 * 8 + (8 << 30):
            break
        tabs.append(torch.empty(lanes * 16384, dtype=torch.int64, device=dev))
        for key, ins in (("no_inserts", 0), ("with_inserts", inserts)):
            ms = ctypes.c_float(0.0)
            rc = lib.nx_probe_ceiling(tabs[-1].data_ptr(), inp.data_ptr(), sink.data_ptr(), lanes, steps, loads, ins,
                                      ctypes.byref(ms), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
            if rc == 0 and ms.value > 0:
                rate = lanes * steps / (ms.value / 1e3)
                best[key] = max(best.get(key, 0.0), rate)
                if key == "with_inserts":
                    per.append(round(rate / 1e9, 2))
    del tabs, inp, sink
    torch.cuda.empty_cache()
    if best:
        best["placements_gprobes_per_s"] = per  # with inserts, one per table placement tried
        best["lanes"] = lanes
    return best or None


def encoder_placement():
    """Probe times of the candidate placements the encoder's workspace was chosen from."""
    import ctypes
    from netty_amd import _lib
    L = _lib.load()
    ms = (ctypes.c_float * 32)()
    n, pick = ctypes.c_int32(0), ctypes.c_int32(-1)
    if L.nx_snappy_encode_placement(ms, 32, ctypes.byref(n), ctypes.byref(pick)) != 0:
        return None
    return {"note": "k_ws_probe ms per candidate workspace (256 dependent exchanges per lane), four draws of up to six; the encoder keeps the fastest",
            "probe_ms": [round(ms[k], 3) for k in range(n.value)], "pick": pick.value}


DEC_KERNELS = ["nx::dec::k_parse", "nx::dec::k_expand"]


def timed_legs(torch, leg, steps, warmup, sync, S, dev, cdev=None):
    """W untimed steps, then exactly K steps bracketed by barrier + device synchronize on both sides;
    the job's time is the max over ranks (reduced on cdev, default dev)."""
    dsync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    for _ in range(warmup):
        leg.step(False)
    dsync()
    sync()
    dsync()
    t0 = time.perf_counter()
    for _ in range(steps):
        leg.step(True)
    dsync()
    sync()
    t1 = time.perf_counter()
    return S.max_over_ranks(t1 - t0, device=dev if cdev is None else cdev)


def run_rank(args, rank: int, world: int, local: int, backend: str = "nccl", leg_factory=None, emit=print):
    """One rank of the job.  `leg_factory(first, n)` builds the rank's work (default: the GPU
    SnappyRoundTrip); the CPU test of the N>1 path passes its own over gloo.  Returns the JSON line
    (rank 0) or None."""
    import torch
    import torch.distributed as dist

    from netty_amd import shard as S

    gpu = leg_factory is None
    if gpu:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    # the device of the few collective tensors: the GPU under RCCL; the host under gloo (the CPU tests,
    # and the GPU test that runs two ranks' GPU legs on one device)
    cdev = dev if backend == "nccl" else torch.device("cpu")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gpu and backend == "nccl":
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        world = dist.get_world_size()  # the ranks the backend actually sees

    def sync():
        if world > 1:
            dist.barrier()

    lo, hi = S.shard_range(args.total_chunks, rank, world)
    n = hi - lo
    leg = SnappyRoundTrip(torch, dev, lo, n, args.sub_chunks) if gpu else leg_factory(lo, n)
    elapsed = timed_legs(torch, leg, args.steps, args.warmup, sync, S, dev, cdev)
    ok, crc_detect = leg.verify(rank)
    comp_bytes = leg.comp_bytes()
    my_off, total_comp, totals_all = S.exchange_offsets(comp_bytes, device=cdev)
    t_crc, t_enc, t_dec = leg.kernel_ms_per_step(args.steps)
    U, C_ = n * CHUNK, comp_bytes
    copy_gbs = copy_rate_gbs(torch, leg.src[:min(n, leg.dec_sub) * CHUNK], leg.dec[:min(n, leg.dec_sub) * CHUNK]) if gpu else None
    traffic = load_traffic() if gpu else (None, "cpu test leg")
    r_dec = roofline(C_ + U, t_dec, n, DEC_KERNELS, traffic, copy_gbs)  # decode: C_in + U_out per chunk
    r_enc = roofline(U + C_, t_enc, n, ENC_KERNELS, traffic, copy_gbs)  # encode: U_in + C_out per chunk
    if gpu and t_dec:
        simds = torch.cuda.get_device_properties(dev).multi_processor_count * 4
        # the decode calls' frames per launch: DEC_SUB; their time per frame from this run's events
        fpl = min(getattr(leg, "dec_sub", n), n)
        r_dec["issue"] = issue_ceiling(load_issue(), DEC_KERNELS, fpl, t_dec * fpl / n, simds)
        if t_enc:
            fpe = max(leg.enc_sizes) if hasattr(leg, "enc_sizes") else n
            r_enc["issue"] = issue_ceiling(load_issue(), ENC_KERNELS, fpe, t_enc * fpe / n, simds)
    def fill_random_access():
        ceil = probe_ceiling(torch, dev) or {}
        got = ENC_PROBES_PER_CHUNK * n / (t_enc / 1e3)
        cw, cn = ceil.get("with_inserts"), ceil.get("no_inserts")
        r_enc["random_access"] = {
            "note": "the encoder's bound: serial chains of random table exchanges + insert stores + candidate loads per lane",
            "probes_per_chunk": ENC_PROBES_PER_CHUNK, "inserts_per_chunk": ENC_INSERTS_PER_CHUNK,
            "candidate_loads_per_chunk": ENC_CANDIDATE_LOADS_PER_CHUNK,
            "census_source": "tests/test_bench_census.py (oracle census of configs[4] chunks, within 1 %)",
            "achieved_probes_per_s": round(got / 1e9, 3) * 1e9,
            "ceiling_probes_per_s": round(cw / 1e9, 3) * 1e9 if cw else None,
            "frac": round(got / cw, 4) if cw else None,
            "ceiling_no_inserts_probes_per_s": round(cn / 1e9, 3) * 1e9 if cn else None,
            "frac_no_inserts": round(got / cn, 4) if cn else None,
            "ceiling_placements_gprobes_per_s": ceil.get("placements_gprobes_per_s"),
            "ceiling_source": "netty_amd/tools/probe_ceiling.hip, the same request mix without compute (exchanges, "
                              "insert stores and candidate loads in the census proportions; and without the stores), "
                              f"{ceil.get('lanes')} lanes (the encoder's resident lanes), timed live, fastest of up to 6 table "
                              "placements (as the encoder chooses its workspace), drawn after the job's buffers are freed at N=1"}

    want_ceiling = bool(gpu and t_enc and not args.no_probe_ceiling)
    if want_ceiling and not (rank == 0 and world == 1):
        fill_random_access()
    if gpu:
        r_enc["workspace_placement"] = encoder_placement()
    dominant = r_enc if t_enc >= t_dec else r_dec
    value = args.total_chunks * CHUNK / elapsed * args.steps / 2**30
    line = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic text-like 64 KiB chunks (include/netty_amd_textgen.h: 4096-word Zipf(1.1) vocabulary), "
                "generated on device",
        "config": {"workload": "configs[4]: Snappy encode (+frame CRC32C) then decode + CRC32C verify of "
                               f"{args.total_chunks} text-like 64 KiB chunks ({args.total_chunks * CHUNK / 2**30:.0f} GiB) "
                               f"split across {world} GPU(s), device-resident",
                   "chunk_bytes": CHUNK, "global_chunks": args.total_chunks, "chunks_per_gpu": n,
                   "calls": leg.plan_info() if hasattr(leg, "plan_info") else None,
                   "parallelism": f"dp{world} (independent chunk shards, no data-path collective)"},
        "roofline": dominant,
        "roofline_decode": r_dec, "roofline_encode": r_enc,
        "encode_gib_s": round(U / ((t_crc + t_enc) / 1e3) / 2**30, 3) if t_enc else None,
        "decode_gib_s": round(U / (t_dec / 1e3) / 2**30, 3) if t_dec else None,
        "kernel_ms_per_step": {"crc32c": round(t_crc, 3), "encode": round(t_enc, 3), "decode_crc": round(t_dec, 3)},
        "compression_ratio": round(C_ / U, 4) if U else None,
        "shard": {"first_chunk": lo, "chunks": n, "stream_offset": my_off, "stream_bytes": total_comp},
        "compressed_bytes_per_rank": totals_all,
        "crc_corruption_subset_detected": crc_detect,
    }
    ok = S.all_true(ok, device=cdev)
    line["verified"] = ok
    if rank == 0:  # progress on stderr (the JSON line comes at the end, after the extra legs)
        print(f"[bench] strong leg: {line['value']} GiB/s, {line['ms_per_step']} ms/step, kernel ms/step "
              f"{line['kernel_ms_per_step']}, verified {ok}", file=sys.stderr, flush=True)
    if gpu and rank == 0:
        line["device"] = device_info(torch, dev)
    if gpu and args.weak_chunks > 0:
        del leg
        torch.cuda.empty_cache()
        wk = SnappyRoundTrip(torch, dev, rank * args.weak_chunks, args.weak_chunks, args.sub_chunks)
        wel = timed_legs(torch, wk, args.weak_steps, 1 if args.warmup else 0, sync, S, dev, cdev)
        wok, _ = wk.verify(rank)
        wok = S.all_true(wok, device=cdev)
        _, we, wd = wk.kernel_ms_per_step(args.weak_steps)
        line["weak_1m_per_gpu"] = {
            "workload": "configs[1]+configs[2]: the same step over chunks_per_gpu chunks on every GPU (weak scaling)",
            "chunks_per_gpu": args.weak_chunks, "steps": args.weak_steps,
            "value": round(world * args.weak_chunks * CHUNK / wel * args.weak_steps / 2**30, 3), "unit": "GiB/s",
            "ms_per_step": round(wel / args.weak_steps * 1e3, 3), "encode_ms": round(we, 3), "decode_crc_ms": round(wd, 3),
            "scaling": "weak", "verified": wok}
        ok = ok and wok
        line["verified"] = ok
        leg = wk
        del wk  # `leg` is the only reference: `del leg` below frees the weak leg's buffers
    if gpu and rank == 0 and world == 1:
        from netty_amd import batch as B
        # a strided sample of the first sub-batch's GPU outputs (compressed bytes, masked CRCs), taken to
        # the host now; the cpu_baseline leg checks it against the oracle byte for byte
        gpu_sample = None if args.no_cpu_baseline else take_gpu_sample(torch, B, leg, args.parity_sample)
        if not args.no_frame_scan:
            line["frame_scan"] = bench_frame_scan(torch, B, dev, leg, args.scan_chunks, args.scan_per_stream)
            ok = ok and line["frame_scan"]["verified"]
            torch.cuda.empty_cache()
        del leg
        torch.cuda.empty_cache()
        if want_ceiling:  # with the job's buffers freed, the ceiling can draw as many placements as the encoder
            fill_random_access()
        if not args.no_alt:
            line["alt_codecs"] = bench_alt_codecs(torch, B, dev, args.alt_chunks, hc_n=args.hc_chunks)
            torch.cuda.empty_cache()
        if not args.no_latency:
            line["latency"] = bench_latency(torch, B, dev)
            torch.cuda.empty_cache()
        if not args.no_e2e:
            # host memory in, host memory out, through the C-ABI a JNI caller binds (never `value`)
            link = link_budget(torch, dev)
            line["end_to_end"] = e2e_capi(args.e2e_channels, args.e2e_messages)
            e2e = line["end_to_end"]
            if "decode_gib_s" in e2e and e2e.get("compressed_bytes") and e2e.get("uncompressed_bytes"):
                r = e2e["compressed_bytes"] / e2e["uncompressed_bytes"]
                # every decoded byte crosses the link once, with r compressed bytes the other way
                link["decode_bound_gib_s"] = round(link["both_gb_s_total"] * 1e9 / (1 + r) / 2**30, 2)
                link["decode_frac_of_bound"] = round(e2e["decode_gib_s"] / link["decode_bound_gib_s"], 3)
                link["encode_bound_gib_s"] = link["decode_bound_gib_s"]  # the same bytes, the other way round
                link["encode_frac_of_bound"] = round(e2e["encode_gib_s"] / link["encode_bound_gib_s"], 3)
            e2e["link"] = link
            # the same round trip driven from torch (pinned tensors, two streams): netty_amd/pipeline.py
            from netty_amd import pipeline as P
            line["end_to_end_torch_pipeline"] = P.measure(dev, n=args.e2e_chunks, sub=args.e2e_sub)
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, gpu_sample)
            ok = ok and line["cpu_baseline"].get("gpu_parity_sample", {}).get("verified", True)
            hc_gpu = line.get("alt_codecs", {}).get("lz4_hc", {}).get("encode_gib_s")
            hc_cpu = line["cpu_baseline"].get("config4_per_codec", {}).get("lz4_hc", {})
            if hc_gpu and hc_cpu:
                # highCompressor = true: below the host's own liblz4 on all cores, it stays on the JVM
                # (DESIGN.md §5); the ratio makes that visible in every line
                lib = hc_cpu.get("liblz4_level9", {}).get("encode_gib_s_all_cores")
                hc_cpu["gpu_over_oracle_all_cores"] = round(hc_gpu / hc_cpu["encode_gib_s_all_cores"], 3)
                if lib:
                    hc_cpu["gpu_over_liblz4_all_cores"] = round(hc_gpu / lib, 3)
        line["verified"] = ok
    if rank == 0:
        emit(json.dumps(line))
        sys.stdout.flush()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return line if rank == 0 else None, ok


# ---------------------------------------------------------------------------------------- extra legs
def device_info(torch, dev):
    """What the box is: device properties (the encoder's speed differs by up to ~15 % between boxes of
    this pool; recorded so runs can be compared).  No rocm-smi: it is a Python script, and a child
    process of a GPU-initialised program may not exec an interpreter on this pool."""
    p = torch.cuda.get_device_properties(dev)
    info = {"name": p.name, "arch": p.gcnArchName, "cus": p.multi_processor_count, "hbm_gib": round(p.total_memory / 2**30, 1),
            "pci_bus_id": getattr(p, "pci_bus_id", None)}
    return info


def link_budget(torch, dev, mib: int = 512, reps: int = 3):
    """The host link the end-to-end legs share: pinned host -> device and device -> host copy rates
    alone and issued together on two streams.  On the pool's boxes the two directions share one
    ~57 GB/s budget (together they take the sum of their times alone: profiles/r05/s31), so a decode
    that moves r compressed bytes in per decoded byte out is bounded by budget / (1 + r)."""
    import time
    n = mib << 20
    hs = torch.empty(n, dtype=torch.uint8).pin_memory()
    hd = torch.empty(n, dtype=torch.uint8).pin_memory()
    da = torch.empty(n, dtype=torch.uint8, device=dev)
    db = torch.zeros(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def timed(fn):
        best = None
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        return best

    def h2d():
        with torch.cuda.stream(s1):
            da.copy_(hs, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            hd.copy_(db, non_blocking=True)

    def both():
        h2d()
        d2h()

    th, td, tb = timed(h2d), timed(d2h), timed(both)
    del hs, hd, da, db
    torch.cuda.empty_cache()
    gb = n / 1e9
    return {"h2d_gb_s": round(gb / th, 2), "d2h_gb_s": round(gb / td, 2), "both_gb_s_total": round(2 * gb / tb, 2),
            "both_over_sum_of_alone": round(tb / (th + td), 3), "bytes_per_copy": n,
            "note": "pinned copies on two streams; both_over_sum_of_alone ~1 means the directions share one budget"}


def e2e_capi(channels: int, messages: int, timeout: float = 240.0, dec_flush_mib: int = 64):
    """Host-to-host Snappy frame round trip through the asynchronous batcher C-ABI
    (netty_amd/tools/e2e_capi.cpp): `channels` SnappyFrameEncoder/Decoder pairs, `messages` 65535-byte
    text messages each in registered host memory; encode in one flush, decode auto-flushed every
    `dec_flush_mib` MiB (the batches rotate over four streams and take disjoint record slots, so one
    batch's PCIe gather and decode overlap the previous one's result writes; round 4, one box:
    23.3 GiB/s with one flush, 25.3 at 256 MiB, 26.6 at 512 MiB, 23.1 at 1 GiB; round 5, with batches
    of <= 32 768 frames on the wave-parallel fused decoder: 30.9-31.0 at 64 MiB, 27.5-30.1 at 128,
    27.3-28.7 at 256, 25.6-26.3 at 512, profiles/r05/s8, s10).  Workspaces and pinned arenas are reserved before the timed rounds;
    `arena_allocs_after_round0` counts pinned allocations after the first round (0: none on the submit
    path).  Run as a child process (its own HIP context); returns its JSON, or the failure."""
    import subprocess
    exe = os.path.join(ROOT, "netty_amd", "e2e_capi")
    if not os.path.exists(exe):
        return {"error": "netty_amd/e2e_capi not built (make -C netty_amd)"}
    # 16 hardware queues for the child's HIP streams (HIP's default is 4): with 4, the batcher's four
    # streams share queues with the null stream and a batch's kernels wait behind another stream's
    # result copy (round 4, one box, three runs each: decode 25.4-27.1 GiB/s with 4, 28.2-28.7 with
    # 16; profiles/r04/s4/e2e_hwq.log).  A caller's setting of 16 or more is kept.
    env = dict(os.environ)
    if int(env.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:  # (the GPU boxes export HIP's default, 4)
        env["GPU_MAX_HW_QUEUES"] = "16"
    try:
        r = subprocess.run([exe, str(channels), str(messages), "65535", "3", "0", str(dec_flush_mib)], capture_output=True, text=True,
                           timeout=timeout, env=env)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout}s"}
    try:
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    d["gpu_max_hw_queues"] = int(env["GPU_MAX_HW_QUEUES"])
    d["path"] = ("pooled-direct-ByteBuf stand-in (registered host memory) -> nx_snappy_frame_encoder_submit x N -> one flush "
                 "-> framed bytes in mapped pinned memory -> (network: copied, untimed, into a registered receive buffer) -> "
                 "nx_snappy_frame_decoder_submit_registered x N (auto-flush every decode_flush_mib) -> messages; decode_copied_*: the same through "
                 "nx_snappy_frame_decoder_submit (payloads copied at submit)")
    return d


def bench_frame_scan(torch, B, dev, leg, m: int, per_stream: int, reps: int = 3):
    """§8f row 1: the first sub-batch's encoded chunks laid out as SnappyFrameEncoder streams in HBM
    (stream identifier, then one COMPRESSED_DATA chunk per 64 KiB: type 0, 24-bit length, masked CRC,
    payload), one stream per connection cumulation; nx_snappy_frame_scan_batch lists their chunks and
    nx_snappy_decode_batch decodes straight from that list with CRC verification."""
    m = min(m, leg.sub, leg.n)
    if hasattr(leg, "run_prefix"):
        leg.run_prefix()  # the first decode call's chunks: compressed in the ring, decoded in `dec`
    src, enc, eoff, elen, crc, dec = leg.src, leg.enc, leg.eoff, leg.elen, leg.crc, leg.dec
    ns = (m + per_stream - 1) // per_stream
    fs = elen[:m].to(torch.int64) + 8
    sid = torch.arange(m, dtype=torch.int64, device=dev) // per_stream
    hp = torch.cumsum(fs, 0) - fs + 10 * (sid + 1)          # chunk header positions
    first = torch.arange(ns, dtype=torch.int64, device=dev) * per_stream
    ss = hp[first] - 10                                        # stream starts
    ends = torch.cat([ss[1:], (hp[-1] + fs[-1]).view(1)])
    slen = ends - ss
    total = int(ends[-1].item())
    buf = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    ident = torch.tensor(list(b"\xff\x06\x00\x00sNaPpY"), dtype=torch.uint8, device=dev)
    buf[(ss.view(-1, 1) + torch.arange(10, device=dev)).view(-1)] = ident.repeat(ns)
    clen = fs - 4
    c32 = crc[:m].to(torch.int64) & 0xFFFFFFFF
    hdr = torch.stack([torch.zeros_like(clen), clen & 255, (clen >> 8) & 255, (clen >> 16) & 255,
                       c32 & 255, (c32 >> 8) & 255, (c32 >> 16) & 255, (c32 >> 24) & 255], 1).to(torch.uint8)
    buf[(hp.view(-1, 1) + torch.arange(8, device=dev)).view(-1)] = hdr.view(-1)
    B.gather(enc, eoff[:m], elen[:m], dst=buf, dst_off=hp + 8)
    state = torch.zeros(ns, dtype=torch.int32, device=dev)
    t_scan, t_all = [], []
    for _ in range(reps):
        state.zero_()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        e[0].record()
        r = B.snappy_frame_scan(buf, ss, slen, state, m)
        e[1].record()
        idx = r["stream"][:m].to(torch.int64) * per_stream + r["seq"][:m].to(torch.int64)
        d = B.snappy_decode(buf, r["data_off"][:m], r["data_len"][:m], dec, idx * CHUNK, expected_crc=r["masked_crc"][:m])
        e[2].record()
        torch.cuda.synchronize()
        t_scan.append(e[0].elapsed_time(e[1]))
        t_all.append(e[0].elapsed_time(e[2]))
    cnt = r["counts"].tolist()
    ok = (cnt == [m, 0, m] and int((r["status"] != 0).sum()) == 0 and bool(torch.equal(r["consumed"], slen))
          and int((d["status"] != 0).sum()) == 0 and bool(torch.equal(dec[:m * CHUNK], src[:m * CHUNK])))
    ts, ta = min(t_scan), min(t_all)
    # §8f row 1 follow-up: the first streams up to 1 GiB as ONE cumulation (their stream identifiers
    # in between are legal chunks): the lane walk (one lane, ~35 K dependent header loads) against the
    # segmented walk (nx_snappy_frame_scan_long); both lists must be equal
    kk = max(1, int((ends <= (1 << 30)).sum().item()))
    L1, m1 = int(ends[kk - 1].item()), kk * per_stream
    st1 = torch.zeros(1, dtype=torch.int32, device=dev)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    lens = torch.tensor([L1], dtype=torch.int64, device=dev)

    def best(fn):
        fn()
        torch.cuda.synchronize()
        tt = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st1.zero_()
            a.record()
            box["r"] = fn()
            b.record()
            torch.cuda.synchronize()
            tt.append(a.elapsed_time(b))
        return min(tt)

    box = {}
    t_lane = best(lambda: B.snappy_frame_scan(buf, zero, lens, st1, m1))
    rl = box["r"]
    t_long = best(lambda: B.snappy_frame_scan_long(buf, L1, st1, m1))
    rg = box["r"]
    same = all(bool(torch.equal(rl[k][:m1], rg[k][:m1])) for k in ("data_off", "data_len", "masked_crc", "seq"))
    long_ok = (same and rg["counts"].tolist() == [m1, 0, m1] and int(rg["consumed"].item()) == L1 and int(rg["status"].item()) == 0)
    ok = ok and long_ok
    long_res = {"bytes": L1, "chunks": m1, "lane_walk_ms": round(t_lane, 3), "segmented_walk_ms": round(t_long, 3),
                "speedup": round(t_lane / t_long, 1), "verified": long_ok,
                "note": "one cumulation; the segmented walk's list equals the lane walk's"}
    return {"streams": ns, "chunks_per_stream": per_stream, "chunks": m, "framed_bytes": total, "long_stream": long_res,
            "scan_ms": round(ts, 3), "scan_chunks_per_s": round(m / (ts / 1e3)),
            "scan_decode_ms": round(ta, 3), "framed_decode_gib_s": round(m * CHUNK / (ta / 1e3) / 2**30, 2),
            "note": "scan = one lane per stream walking its chunk headers (it reads the 8-byte headers only, "
                    "so it is reported in chunks/s, not bytes); the list it writes is the decode batch's "
                    "in_off / in_len / expected CRC as is",
            "verified": ok}


def bench_alt_codecs(torch, B, dev, n: int, reps: int = 2, hc_n: int = 1024):
    """configs[3]: FastLZ (level 1 and 2) and LZF encode/decode of a mixed batch — sizes uniform in
    [4096, 65535], half text-like, half random — device-resident.  GiB/s of uncompressed bytes."""
    g = torch.Generator(device=dev).manual_seed(1234)
    CH = CHUNK
    src = torch.empty(n * CH, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, n, CH)
    view = src.view(n, CH)
    view[1::2] = torch.randint(0, 256, (len(range(1, n, 2)), CH), dtype=torch.uint8, device=dev, generator=g)
    ln = torch.randint(4096, 65536, (n,), dtype=torch.int32, device=dev, generator=g)
    off = torch.arange(n, dtype=torch.int64, device=dev) * CH
    U = int(ln.to(torch.int64).sum())
    res = {"chunks": n, "bytes": U, "sizes": "uniform [4096, 65535]", "data": "50% text-like, 50% random",
           "roofline_note": "per leg: algorithmic bytes U + C (uncompressed + compressed, SURVEY.md section 8d) / the "
                            "leg's HIP-event time, against 8 TB/s HBM"}

    alt_tr, alt_src = load_alt_traffic()
    res["traffic_source"] = alt_src

    def roof(nbytes, ms, leg=None, phase=None):
        """algorithmic bytes / time against HBM peak; with a digest-matched PMC summary (taken over this
        same leg at the default --alt-chunks), also the measured HBM bytes per call and the fraction of
        HBM bandwidth they occupied over the call's time"""
        a = nbytes / (ms / 1e3) / 1e9
        r = {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(a / HBM_PEAK_GBS, 4)}
        t = (alt_tr or {}).get(leg, {}).get(phase)
        if t and n == 262144:
            hb = t["hbm_bytes_per_call"]
            r.update({"traffic": round(hb), "traffic_per_chunk": round(hb / n), "traffic_over_algorithmic": round(hb / nbytes, 2),
                      "traffic_frac": round(hb / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)})
        else:
            r["traffic"] = None
        return r

    def same(rows, lens):
        """every decoded chunk equals its source (rows: chunk indices), 16384 chunks at a time"""
        col = torch.arange(CH, device=dev)
        for a in range(0, rows.numel(), 16384):
            r = rows[a:a + 16384]
            m = col.view(1, -1) < lens[a:a + 16384].view(-1, 1)
            if not torch.equal(dec.view(n, CH)[r][m], src.view(n, CH)[r][m]):
                return False
        return True

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return min(ts)

    fcap = (B.fastlz_max_compressed_length(CH) + 15) // 16 * 16
    fout = torch.empty(n * fcap, dtype=torch.uint8, device=dev)
    foff = torch.arange(n, dtype=torch.int64, device=dev) * fcap
    dec = torch.empty_like(src)
    for level in (1, 2):
        dec.zero_()
        lv = torch.full((n,), level, dtype=torch.int32, device=dev)
        box = {}

        def enc():
            box["r"] = B.fastlz_compress(src, off, ln, fout, foff, level=lv)

        te = timed(enc)
        flen, fst = box["r"]

        def dcm():
            box["d"] = B.fastlz_decompress(fout, foff, flen, dec, off, ln)

        td = timed(dcm)
        ok = bool(torch.equal(box["d"], ln)) and int((fst != 0).sum()) == 0
        ok = ok and same(torch.arange(n, device=dev), ln)
        C = int(flen.to(torch.int64).sum())
        res[f"fastlz_l{level}"] = {"encode_gib_s": round(U / te * 1e3 / 2**30, 3), "decode_gib_s": round(U / td * 1e3 / 2**30, 3),
                                   "ratio": round(C / U, 4), "verified": ok,
                                   "roofline_encode": roof(U + C, te, f"fastlz_l{level}", "encode"),
                                   "roofline_decode": roof(U + C, td, f"fastlz_l{level}", "decode")}
    del fout
    lcap = (B.lzf_max_compressed_length(CH) + 15) // 16 * 16
    lout = torch.empty(n * lcap, dtype=torch.uint8, device=dev)
    loff = torch.arange(n, dtype=torch.int64, device=dev) * lcap
    box = {}

    def lenc():
        box["r"] = B.lzf_encode(src, off, ln, lout, loff)

    te = timed(lenc)
    llen, lst = box["r"]
    # compressed "ZV" blocks (type 1): body at +7, compressed length at +3 (big-endian)
    typ = lout[loff + 2]
    idx = torch.nonzero(typ == 1).flatten()
    boff = loff[idx] + 7
    blen = (lout[loff[idx] + 3].to(torch.int32) << 8) | lout[loff[idx] + 4].to(torch.int32)
    uo = off[idx]
    ul = ln[idx]
    Ud = int(ul.to(torch.int64).sum())

    def ldec():
        box["d"] = B.lzf_decode(lout, boff, blen, dec, uo, ul)

    dec.zero_()
    td = timed(ldec)
    ok = int((lst != 0).sum()) == 0 and int((box["d"] != 0).sum()) == 0
    ok = ok and same(idx, ul)
    Cl = int(llen.to(torch.int64).sum())
    Cd = int(blen.to(torch.int64).sum())
    res["lzf"] = {"encode_gib_s": round(U / te * 1e3 / 2**30, 3),
                  "decode_gib_s": round(Ud / td * 1e3 / 2**30, 3) if idx.numel() else None,
                  "decoded_chunks": int(idx.numel()), "ratio": round(Cl / U, 4), "verified": ok,
                  "roofline_encode": roof(U + Cl, te, "lzf", "encode"),
                  "roofline_decode": roof(Ud + Cd, td, "lzf", "decode") if idx.numel() else None}
    del lout
    # LZ4 blocks (§8f row 4): GPU block encoder, then decode through the parse/expand kernels
    zcap = (B.lz4_max_compressed_length(CH) + 15) // 16 * 16
    zout = torch.empty(n * zcap, dtype=torch.uint8, device=dev)
    zoff = torch.arange(n, dtype=torch.int64, device=dev) * zcap

    def zenc():
        box["z"] = B.lz4_encode(src, off, ln, zout, zoff)

    te = timed(zenc)
    zlen, zst = box["z"]

    def zdec():
        box["zd"] = B.lz4_decode(zout, zoff, zlen, dec, off, ln)

    dec.zero_()
    td = timed(zdec)
    ok = (int((zst != 0).sum()) == 0 and int((box["zd"] != 0).sum()) == 0 and same(torch.arange(n, device=dev), ln))
    Cz = int(zlen.to(torch.int64).sum())
    res["lz4"] = {"encode_gib_s": round(U / te * 1e3 / 2**30, 3), "decode_gib_s": round(U / td * 1e3 / 2**30, 3),
                  "ratio": round(Cz / U, 4), "verified": ok,
                  "roofline_encode": roof(U + Cz, te, "lz4", "encode"), "roofline_decode": roof(U + Cz, td, "lz4", "decode")}
    # LZ4 HC (Lz4FrameEncoder(highCompressor = true): LZ4_compress_HC level 9, one lane per block with
    # 256 KiB of hash/chain tables in HBM) on the first hc_n chunks of the same mix; decoded back
    hn = min(n, hc_n)
    if hn:
        Uh = int(ln[:hn].to(torch.int64).sum())

        def henc():
            box["h"] = B.lz4_encode(src, off[:hn], ln[:hn], zout, zoff[:hn], high=True)

        th = timed(henc)
        hlen, hst = box["h"]

        def hdec():
            box["hd"] = B.lz4_decode(zout, zoff[:hn], hlen, dec, off[:hn], ln[:hn])

        dec.zero_()
        thd = timed(hdec)
        ok = (int((hst != 0).sum()) == 0 and int((box["hd"] != 0).sum()) == 0 and same(torch.arange(hn, device=dev), ln[:hn]))
        Ch = int(hlen.to(torch.int64).sum())
        res["lz4_hc"] = {"chunks": hn, "encode_gib_s": round(Uh / th * 1e3 / 2**30, 4), "encode_ms": round(th, 2),
                         "decode_gib_s": round(Uh / thd * 1e3 / 2**30, 3), "ratio": round(Ch / Uh, 4), "verified": ok,
                         "roofline_encode": roof(Uh + Ch, th), "roofline_decode": roof(Uh + Ch, thd),
                         "note": "LZ4_compress_HC level 9 (256-candidate hash chains) per lane: a compatibility path"}
    del zout
    # LZ4 frame (Lz4FrameEncoder / Lz4FrameDecoder with validateChecksums): XXH32, frame blocks into
    # slots, gathered into 4096 contiguous streams (64 blocks each), then device scan -> block decode -> XXH32 verify.
    def xh():
        box["h"] = B.xxhash32(src, off, ln)

    th = timed(xh)
    fzcap = (21 + B.lz4_max_compressed_length(CH) + 15) // 16 * 16
    fz = torch.empty(n * fzcap, dtype=torch.uint8, device=dev)
    fzoff = torch.arange(n, dtype=torch.int64, device=dev) * fzcap

    def fenc():
        box["f"] = B.lz4_frame_encode(src, off, ln, fz, fzoff, 6)

    tfe = timed(fenc)
    fzlen, fzst = box["f"]
    streams = max(1, min(4096, n // 64))
    packed, poff = B.gather(fz, fzoff, fzlen)
    del fz
    per = n // streams
    s_off = poff[::per][:streams].contiguous()
    s_end = torch.cat([s_off[1:], (poff[-1] + fzlen[-1].to(torch.int64)).reshape(1)])
    s_len = s_end - s_off
    fstate = torch.zeros(streams, dtype=torch.int32, device=dev)

    def fdec():
        fstate.zero_()
        sc = B.lz4_frame_scan(packed, s_off, s_len, fstate, n)
        box["fd"] = (sc, B.lz4_frame_decode(packed, sc, n))

    tfd = timed(fdec)
    sc, fd = box["fd"]
    nc, nu = (int(v) for v in sc["counts"][:2].tolist())
    ok = (int((fzst != 0).sum()) == 0 and nc + nu == n and int((sc["status"] != 0).sum()) == 0
          and int((fd["compressed"][2] != 0).sum()) == 0 and int((fd["raw"][2] != 0).sum()) == 0)
    res["lz4_frame"] = {"xxhash32_gib_s": round(U / th * 1e3 / 2**30, 3), "encode_gib_s": round(U / tfe * 1e3 / 2**30, 3),
                        "scan_decode_verify_gib_s": round(U / tfd * 1e3 / 2**30, 3), "streams": streams,
                        "framed_bytes": int(fzlen.to(torch.int64).sum()), "compressed_blocks": nc,
                        "non_compressed_blocks": nu, "verified": ok,
                        "note": "decode leg = scan + LZ4 block decode + XXH32 of every block vs its header (one host sync for the list counts)"}
    return res


def bench_latency(torch, B, dev, sizes=(1, 64, 1024, 4096, 16384), reps: int = 3):
    """Per-batch latency of the Snappy encode (+ CRC32C) and decode (+ verify) batch calls, as a
    handler call or a batcher flush of that many 64 KiB text chunks sees it: best of `reps` HIP-event
    timings on the current stream, outputs checked against the sources."""
    nmax = max(sizes)
    src = torch.empty(nmax * CHUNK, dtype=torch.uint8, device=dev)
    B.textgen(src, 0, nmax, CHUNK)
    cap = (B.snappy_max_compressed_length(CHUNK) + 15) // 16 * 16
    enc = torch.empty(nmax * cap, dtype=torch.uint8, device=dev)
    dec = torch.empty(nmax * CHUNK, dtype=torch.uint8, device=dev)
    rows = []

    def best(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        return min(ts)

    for m in sizes:
        off = torch.arange(m, dtype=torch.int64, device=dev) * CHUNK
        ln = torch.full((m,), CHUNK, dtype=torch.int32, device=dev)
        eoff = torch.arange(m, dtype=torch.int64, device=dev) * cap
        box = {}

        def e():
            box["crc"] = B.crc32c_masked(src, off, ln)
            box["e"] = B.snappy_encode(src, off, ln, enc, eoff)

        te = best(e)
        elen, est = box["e"]

        def d():
            box["d"] = B.snappy_decode(enc, eoff, elen, dec, off, expected_crc=box["crc"])

        td = best(d)
        ok = (int((est != 0).sum()) == 0 and int((box["d"]["status"] != 0).sum()) == 0
              and torch.equal(dec[:m * CHUNK], src[:m * CHUNK]))
        rows.append({"chunks": m, "encode_ms": round(te, 3), "decode_verify_ms": round(td, 3), "verified": ok})
    return {"sizes": rows, "note": "one nx_crc32c_masked_batch + nx_snappy_encode_batch call, and one nx_snappy_decode_batch "
                                   "call with CRC verify (fused decoder up to 32768 frames), per batch of 64 KiB text chunks"}


# ---------------------------------------------------------------------------------------- launcher
def _spawned_rank(local: int, argv, world: int, port: int):
    os.environ.update({"RANK": str(local), "LOCAL_RANK": str(local), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    args = parse(argv)
    _, ok = run_rank(args, local, world, local)
    if not ok:
        sys.exit(3)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start one process per GPU ourselves; nothing in this parent has touched the GPU
        import torch.multiprocessing as mp
        mp.start_processes(_spawned_rank, args=(argv, args.gpus, free_port()), nprocs=args.gpus, join=True,
                           start_method="spawn")
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    _, ok = run_rank(args, rank, world, local)
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
