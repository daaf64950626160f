"""Driver for scripts/pmc_alt_traffic.sh: bench.py's configs[3] alt-codec leg alone (FastLZ L1/L2, LZF,
LZ4 block encode + decode over the same mixed batch), one timed call per phase after one warm-up, so
that the rocprofv3 --pmc passes see each codec's encode and decode dispatches in a fixed order."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netty_amd import batch as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
res = bench.bench_alt_codecs(torch, B, torch.device("cuda:0"), n, reps=1, hc_n=0)
print(json.dumps({k: v for k, v in res.items() if isinstance(v, dict)}))
