"""Phase anatomy of the ping-pong self-attention (kernel 5) at the config-2 shape: s_memtime sums per wave group of
barrier 1 / work 1 / barrier 2 / MFMA phase.  Needs the SA_V13_STAMPS build (scripts/build_variant.sh stamps
-DSA_V13_STAMPS with SRC=attention) loaded through SA_LIB."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import _lib, ops  # noqa: E402
from stableavatar_amd.kbench import vt_layout  # noqa: E402

L, H, D = 21504, 12, 128
dev = "cuda"
qkv = torch.randn(3 * L, 3 * H * D, device=dev).bfloat16()
segs = torch.tensor([[b * L, L, b * L, L] for b in range(3)], dtype=torch.int32, device=dev)
q, k, v_ = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
vt = vt_layout(v_, 3)
o = torch.empty(3 * L, H * D, device=dev, dtype=torch.bfloat16)
lib = ctypes.CDLL(str(_lib.LIB_PATH))
buf = (ctypes.c_ulonglong * 12)()
ops.attention(q, k, vt, o, segs, 3, L, H, kernel=5)
torch.cuda.synchronize()
lib.sa_debug_v13_stamps(buf, 1)
n = 3
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(n):
    ops.attention(q, k, vt, o, segs, 3, L, H, kernel=5)
ev1.record()
torch.cuda.synchronize()
lib.sa_debug_v13_stamps(buf, 1)
waves = 3 * H * (L // 256) * 4 * n  # per group
blocks = L // 64
names = ["barrier1", "work1", "barrier2", "mfma_phase", "wait_dma_A", "stage_A"]
r = {"ms_per_launch": round(ev0.elapsed_time(ev1) / n, 3), "cycles_per_block": {}}
for gi, gname in enumerate(("A", "B")):
    r["cycles_per_block"][gname] = {nm: round(buf[gi * 6 + i] / waves / blocks, 1) for i, nm in enumerate(names)}
print(json.dumps(r))
