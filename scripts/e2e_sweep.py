"""End-to-end host pipeline sweep: python scripts/e2e_sweep.py N SUB [SUB ...]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netty_amd import pipeline as P
n = int(sys.argv[1])
for sub in map(int, sys.argv[2:]):
    print(json.dumps(P.measure(torch.device("cuda:0"), n=n, sub=sub)), flush=True)
