"""Self-attention launch time at the per-rank shapes of each Ulysses SP degree (config 2, 12 heads, L = 21 504,
B = 3 CFG rows): N = 1 (12 heads, all queries), 2 (6 heads), 4 (3 heads), 8 (3 heads, half the queries).
Prints the time per launch and the ideal time (the N = 1 launch / N) to expose work-group quantization."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import ops  # noqa: E402
from stableavatar_amd.kbench import _time  # noqa: E402

L, D, B = 21504, 128, 3
res = {}
base = None
for N, hg, R in ((1, 12, 1), (2, 6, 1), (4, 3, 1), (8, 3, 2)):
    Lq = L // R
    q = torch.randn(B * Lq, hg * D, device="cuda").bfloat16()
    kv = torch.randn(B * L, 2 * hg * D, device="cuda").bfloat16()
    o = torch.empty_like(q)
    segs = torch.tensor([[b * Lq, Lq, b * L, L] for b in range(B)], dtype=torch.int32, device="cuda")
    t = {k_: _time(lambda: ops.attention(q, kv[:, :hg * D], kv[:, hg * D:], o, segs, B, Lq, hg, kernel=k_),
                   iters=5, warmup=2) for k_ in (1, 2, 0)}  # 256-row, 128-row workgroups, auto
    base = base or t[1]
    res[f"N{N}"] = {"ms_wg256": round(t[1], 3), "ms_wg128": round(t[2], 3), "ms_auto": round(t[0], 3),
                    "ideal_ms": round(base / N, 3), "workgroups_256": B * hg * -(-Lq // 256),
                    "efficiency_auto": round(base / N / t[0], 3)}
    del q, kv, o
print(json.dumps(res), flush=True)
