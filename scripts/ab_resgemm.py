"""Time the DiT's gated-residual GEMM shapes (O-proj / cross-O: K=1536; FFN-down: K=8960) in one
process; run twice with SA_GEMM_TILEGATE=1/0 for the tile-uniform-gate epilogue A/B."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    M, L = 64512, 21504
    res = {"tilegate": os.environ.get("SA_GEMM_TILEGATE", "1")}
    for name, N, K in (("o_proj", 1536, 1536), ("ffn_down", 1536, 8960)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=dev)
        gate = torch.randn(3, N, device=dev)
        out = torch.randn(M, N, device=dev)
        ref = out.clone()
        for _ in range(3):
            ops.linear(x, w, b, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=L)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.linear(x, w, b, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=L)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        # correctness of one application vs torch on a fresh residual
        out2 = ref.clone()
        ops.linear(x, w, b, ops.EPI_RES_F32, out=out2, residual=out2, gate=gate, rows_per_batch=L)
        y = (x.float() @ w.float().t() + b).bfloat16().float()
        exp = ref + y * gate.repeat_interleave(L, 0)
        err = ((out2 - exp).norm() / exp.norm()).item()
        res[name] = {"ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1), "rel_err": err}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
