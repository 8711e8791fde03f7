"""Which hipBLASLt kernels does torch pick for the DiT GEMM shapes (bf16 x @ w^T, with and without bias)?
Run under rocprofv3 --kernel-trace --stats; prints per-shape timing so the trace can be matched."""
import torch
import torch.nn.functional as F

torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"
shapes = {"qkv": (64512, 4608, 1536), "o": (64512, 1536, 1536), "ffn_up": (64512, 8960, 1536),
          "ffn_down": (64512, 1536, 8960)}
for name, (M, N, K) in shapes.items():
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev).bfloat16()
    for bias in (False, True):
        for _ in range(3):
            y = F.linear(x, w, b if bias else None)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            y = F.linear(x, w, b if bias else None)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name} bias={bias} M={M} N={N} K={K}: {ms:.3f} ms = {2 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
