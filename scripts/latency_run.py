"""bench.py's latency leg alone (Snappy encode + CRC32C and decode + verify per batch size)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from netty_amd import batch as B  # noqa: E402

print(json.dumps(bench.bench_latency(torch, B, torch.device("cuda:0"))))
