"""GEMM probe: hipBLASLt (torch.nn.functional.linear) vs our persistent kernel on the DiT's GEMM
shapes, a fixed number of launches each, for rocprofv3 (kernel names / durations / PMC passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import ops  # noqa: E402

M = 64512
SHAPES = {"cross_q": (1536, 1536), "qkv": (4608, 1536), "ffn_up": (8960, 1536), "ffn_down": (1536, 8960)}
which = sys.argv[1].split(",") if len(sys.argv) > 1 else list(SHAPES)
iters = int(os.environ.get("PROBE_ITERS", "10"))
dev = "cuda"
for name in which:
    N, K = SHAPES[name]
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev)
    bb = b.bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(iters):
        torch.nn.functional.linear(x, w, bb)
    for _ in range(iters):
        ops.linear(x, w, b, ops.EPI_BF16, out=out, kernel=2)
    torch.cuda.synchronize()
    print(name, "done", flush=True)
