"""The sequence-parallel per-rank GEMM shapes (N = 8: M = 8 064; per-row QKV 2 688; N = 4: 16 128) timed per
persistent tile height (kernel 2: 256 rows, 3: 192) and tile raster run length (group_m), one process."""
import json
import math
import sys

import torch

from stableavatar_amd import ops


def t(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


dev = "cuda"
torch.manual_seed(0)
for (M, N, K, epi, name) in [(8064, 1536, 8960, ops.EPI_RES_F32, "ffn_down_n8"), (8064, 8960, 1536, ops.EPI_GELU_TANH_BF16, "ffn_up_n8"),
                             (8064, 1536, 1536, ops.EPI_RES_F32, "o_proj_n8"), (2688, 4608, 1536, ops.EPI_BF16, "qkv_row_n8"),
                             (16128, 1536, 8960, ops.EPI_RES_F32, "ffn_down_n4")]:
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev)
    out = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == ops.EPI_RES_F32 else torch.bfloat16)
    gate = torch.randn(3, N, device=dev)
    r = {"kernel": name, "M": M, "N": N, "K": K}
    for kern in (2, 3):
        for gm in (1, 2, 4, 8, 16, 64):
            if epi == ops.EPI_RES_F32:
                fn = lambda: ops.linear(x, w, b, epi, out=out, residual=out, gate=gate, rows_per_batch=M // 3,
                                        kernel=kern, group_m=gm)
            else:
                fn = lambda: ops.linear(x, w, b, epi, out=out, kernel=kern, group_m=gm)
            r[f"k{kern}_g{gm}"] = round(t(fn) * 1e3, 1)
    print(json.dumps(r), flush=True)
