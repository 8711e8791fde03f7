"""sha256 of the DiT GEMM outputs on seeded inputs (every epilogue), to check two library builds bit for bit:
SA_LIB=<lib> python scripts/gemm_hash.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import ops  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(7)
M = 3 * 21504
for name, N, K, epi in [("qkv", 4608, 1536, ops.EPI_BF16), ("o_proj", 1536, 1536, ops.EPI_RES_F32),
                        ("ffn_up", 8960, 1536, ops.EPI_GELU_TANH_BF16), ("ffn_down", 1536, 8960, ops.EPI_RES_F32)]:
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev, generator=g) * 0.1
    if epi == ops.EPI_RES_F32:
        y = torch.randn(M, N, device=dev, generator=g)
        gate = torch.randn(3, N, device=dev, generator=g)
        ops.linear(x, w, b, epi, out=y, residual=y, gate=gate, rows_per_batch=21504)
    else:
        y = ops.linear(x, w, b, epi)
    torch.cuda.synchronize()
    print(name, hashlib.sha256(y.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
