"""Bit-identity probe for GEMM epilogue A/Bs: runs the config-2 gated-residual GEMMs (O-proj, FFN-down) on
seeded inputs with the library SA_LIB points at and prints a hash of each fp32 output."""
import hashlib
import math

import torch

from stableavatar_amd import ops

dev = "cuda"
torch.manual_seed(0)
M = 3 * 21504
for name, N, K in (("o_proj", 1536, 1536), ("ffn_down", 1536, 8960)):
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev)
    gate = torch.randn(3, N, device=dev)
    out = torch.randn(M, N, device=dev)
    ops.linear(x, w, b, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=21504)
    # a per-row gate (tiles straddling CFG rows) as well
    out2 = torch.randn(M, N, device=dev)
    ops.linear(x, w, b, ops.EPI_RES_F32, out=out2, residual=out2, gate=gate, rows_per_batch=21500)
    torch.cuda.synchronize()
    h = hashlib.sha256(out.cpu().numpy().tobytes() + out2.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"hash {name} {h}", flush=True)
