"""debug: the V^T path pieces at the config-2 shape (QKV split GEMMs, EPI_BF16_TP32, attention kernel 3)"""
import torch
from stableavatar_amd import ops
from stableavatar_amd.kbench import vt_layout

dev = "cuda"
torch.manual_seed(0)
B, L, H, D = 3, 21504, 12, 128
M, dim = B * L, H * D
x = torch.randn(M, dim, device=dev).bfloat16()
w = (torch.randn(3 * dim, dim, device=dev) / dim ** 0.5).bfloat16()
b = torch.randn(3 * dim, device=dev) * 0.1
qkv = ops.linear(x, w, b, ops.EPI_BF16)
qkv2 = torch.empty_like(qkv)
ops.linear(x, w[:2 * dim], b[:2 * dim], ops.EPI_BF16, out=qkv2[:, :2 * dim])
Rv = (M + 63) // 64 * 64
vt = torch.zeros(dim, Rv, device=dev, dtype=torch.bfloat16)
ops.linear(x, w[2 * dim:], b[2 * dim:], ops.EPI_BF16_TP32, out=vt)
vt_ref = vt_layout(qkv[:, 2 * dim:].contiguous(), 3)
vt_nat = torch.zeros(dim, Rv, device=dev, dtype=torch.bfloat16)
ops.linear(x, w[2 * dim:], b[2 * dim:], ops.EPI_BF16_T, out=vt_nat)
torch.cuda.synchronize()
print("qk equal", torch.equal(qkv2[:, :2 * dim], qkv[:, :2 * dim]))
print("vt natural equal", torch.equal(vt_nat[:, :M], qkv[:, 2 * dim:].t()))
print("vt p32 equal", torch.equal(vt, vt_ref), (vt.float() - vt_ref.float()).abs().max().item())
bad = (vt != vt_ref).nonzero()
print("mismatches", bad.shape[0], bad[:10].tolist())
segs = torch.tensor([[i * L, L, i * L, L] for i in range(B)], dtype=torch.int32, device=dev)
o1 = torch.empty(M, dim, device=dev, dtype=torch.bfloat16)
o3 = torch.empty_like(o1)
ops.attention(qkv[:, :dim], qkv[:, dim:2 * dim], qkv[:, 2 * dim:], o1, segs, B, L, H, kernel=1)
ops.attention(qkv[:, :dim], qkv[:, dim:2 * dim], vt, o3, segs, B, L, H, kernel=3)
torch.cuda.synchronize()
print("attn equal", torch.equal(o1, o3), ((o1.float() - o3.float()).norm() / o1.float().norm()).item())
