"""Where a persistent GEMM tile's time goes, per config-2 DiT shape: s_memtime sums over every wave of the first K-step
pair of each tile (it holds the wait for the previous tile's epilogue stores), the rest of the K loop and the epilogue,
for the default kernel and the no-epilogue measurement kernel (8).  Needs the SA_GEMM_STAMPS build
(scripts/build_variant.sh gstamps -DSA_GEMM_STAMPS) loaded through SA_LIB; each stamp waits lgkmcnt(0)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import _lib, ops  # noqa: E402

dev = "cuda"
M = 3 * 21504
lib = ctypes.CDLL(str(_lib.LIB_PATH))
buf = (ctypes.c_ulonglong * 8)()
for (N, K, epi, name) in [(4608, 1536, ops.EPI_BF16, "qkv"), (1536, 1536, ops.EPI_BF16, "cross_q"),
                          (8960, 1536, ops.EPI_GELU_TANH_BF16, "ffn_up"), (1536, 1536, ops.EPI_RES_F32, "o_proj"),
                          (1536, 8960, ops.EPI_RES_F32, "ffn_down")]:
    x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev)
    out = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == ops.EPI_RES_F32 else torch.bfloat16)
    gate = torch.randn(3, N, device=dev)
    r = {"kernel": f"gemm_{name}", "M": M, "N": N, "K": K}
    for kern in (0, 8):
        if epi == ops.EPI_RES_F32:
            fn = lambda: ops.linear(x, w, b, epi, out=out, residual=out, gate=gate, rows_per_batch=21504, kernel=kern)
        else:
            fn = lambda: ops.linear(x, w, b, epi, out=out, kernel=kern)
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        lib.sa_debug_gemm_stamps(buf, 1)
        n = 5
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(n):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        lib.sa_debug_gemm_stamps(buf, 1)
        first, rest, epil, tiles = buf[0], buf[1], buf[2], max(buf[3], 1)
        r[f"k{kern}"] = {"ms": round(ev0.elapsed_time(ev1) / n, 4), "tiles_per_wave_launch": round(tiles / n / 1024, 2),
                         "cyc_first_pair": round(first / tiles), "cyc_rest_kloop": round(rest / tiles),
                         "cyc_epilogue": round(epil / tiles)}
    print(json.dumps(r), flush=True)
