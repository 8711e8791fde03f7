"""Probe: the Ulysses N = 8 per-rank self-attention launch (3 CFG rows x 10 752 queries x 3 heads over 21 504 keys)
as one launch vs the same work split over the keys (each query row twice / 4x, against half / a quarter of the keys:
the workgroup count a key-split launch would have, minus its merge pass).  usage: python scripts/attn_split_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import ops  # noqa: E402

dev = "cuda"
B, Lq, Lk, H, D = 3, 10752, 21504, 3, 128
q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)


def segs_for(split):
    kl = Lk // split
    return torch.tensor([[b * Lq, Lq, b * Lk + s * kl, kl] for b in range(B) for s in range(split)],
                        dtype=torch.int32, device=dev)


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {}
for split in (1, 2, 3, 4):
    sg = segs_for(split)
    for kern in (1, 2):
        res[f"split{split}_k{kern}_ms"] = round(t(lambda: ops.attention(q, k, v, o, sg, B * split, Lq, H, kernel=kern)), 4)
print(json.dumps({"probe": "attn_key_split_n8", **res}), flush=True)
