"""The per-chunk table-traffic figures bench.py reports beside the encoder's random-access ceiling
(bench.ENC_*_PER_CHUNK) against the oracle's census of Snappy.encode (Snappy.java:104-158,
oracle/netty_oracle.c orc_snappy_encode_census) over chunks spread across configs[4]'s 1 638 400."""
import bench


def test_encoder_census_matches_bench_constants(oracle):
    n = 48
    tot = {"probes": 0, "inserts": 0, "matches": 0, "matches_7plus": 0}
    for i in range(n):
        chunk = oracle.textgen_chunk(i * (1638400 // n), 65536)
        z, c = oracle.snappy_encode_census(chunk)
        assert z == oracle.snappy_encode(chunk)  # the census does not change the encoding
        for k in tot:
            tot[k] += c[k]
    avg = {k: v / n for k, v in tot.items()}
    assert abs(avg["probes"] / bench.ENC_PROBES_PER_CHUNK - 1) < 0.01, avg
    assert abs(avg["inserts"] / bench.ENC_INSERTS_PER_CHUNK - 1) < 0.01, avg
    assert abs(avg["matches_7plus"] / bench.ENC_CANDIDATE_LOADS_PER_CHUNK - 1) < 0.01, avg
    assert avg["inserts"] <= avg["matches"]  # one insert per match that does not end the chunk
