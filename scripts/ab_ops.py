"""Per-op outputs (fixed seed) for an A/B of two builds: run from each tree's root, then compare the saved
tensors.  usage: python scripts/ab_ops.py <out.pt>"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from stableavatar_amd import ops  # noqa: E402
from stableavatar_amd.transformer import rope_table  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
out = {}
C, L, B = 1536, 120, 3
qkv = torch.randn(B * L, 3 * C, device=dev).bfloat16()
wq, wk = torch.randn(C, device=dev), torch.randn(C, device=dev)
x = qkv.clone()
ops.qk_rmsnorm_rope(x, 0, C, wq, wk, C, 1e-6, rope=rope_table(128).to(dev), rows_per_batch=L, grid=(5, 4, 6),
                    head_dim=128, n_frame_pairs=22, n_height_pairs=21)
out["qk"] = x.clone()
segs = torch.tensor([[b * L, L, b * L, L] for b in range(B)], dtype=torch.int32, device=dev)
o = torch.empty(B * L, C, device=dev, dtype=torch.bfloat16)
for kern in (1, 2):
    ops.attention(x[:, :C], x[:, C:2 * C], x[:, 2 * C:], o, segs, B, L, 12, kernel=kern)
    out[f"attn{kern}"] = o.clone()
w = torch.randn(C, C, device=dev).bfloat16()
bias = torch.randn(C, device=dev)
gate = torch.randn(B, C, device=dev)
res = torch.randn(B * L, C, device=dev)
y = res.clone()
ops.linear(o, w, bias, ops.EPI_RES_F32, out=y, residual=y, gate=gate, rows_per_batch=L)
out["gemm_res"] = y
out["gemm_bf16"] = ops.linear(o, w, bias, ops.EPI_BF16)
out["gemm_gelu"] = ops.linear(o, w, bias, ops.EPI_GELU_TANH_BF16)
torch.cuda.synchronize()
torch.save({k: v.cpu() for k, v in out.items()}, sys.argv[1])
print("saved", list(out))
