"""The two-phase encoder model (scripts/experiments/enc_chain_model.c): its chain
walker, which replaces Snappy.encode's table by "the last written position with the same hash", makes
exactly the reference's choices — the bytes equal the oracle's Snappy.encode on bench-corpus chunks —
and its census equals the oracle's (probes, inserts).  The model is what decided against building
the kernel; this keeps its counts honest."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chain_model_is_bit_exact_and_counts(tmp_path, oracle):
    exe = tmp_path / "enc_chain_model"
    subprocess.check_call(["gcc", "-O2", "-DWITH_ORACLE", "-o", str(exe), os.path.join(ROOT, "scripts/experiments/enc_chain_model.c"),
                           "-I", os.path.join(ROOT, "include"), "-L", os.path.join(ROOT, "oracle"), "-loracle",
                           "-Wl,-rpath," + os.path.join(ROOT, "oracle"), "-lm"])
    out = subprocess.run([str(exe), "8", "34133"], check=True, capture_output=True, text=True).stdout
    r = json.loads(out)
    assert r["tag_streams_identical"] is True
    probes = inserts = 0
    for k in range(8):
        _, c = oracle.snappy_encode_census(oracle.textgen_chunk(k * 34133, 65536))
        probes += c["probes"]
        inserts += c["inserts"]
    assert abs(r["per_chunk"]["probes"] - probes / 8) < 0.2
    assert abs(r["per_chunk"]["inserts"] - inserts / 8) < 0.2
    assert r["per_chunk"]["hops_per_probe"] > 0.5  # every probe walks ~1 unwritten position on this corpus
