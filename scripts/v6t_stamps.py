"""Barrier / DMA-wait anatomy of the V^T self-attention (kernel 3) at the config-2 shape: s_memtime sums per wave
group (waves 0-3, 4-7) of the per-block DMA wait (vmcnt(0)), the workgroup barrier and the whole block loop.  Needs the
SA_V6T_STAMPS build (scripts/build_variant.sh v6tstamps -DSA_V6T_STAMPS with SRC=attention) loaded through SA_LIB;
the stamps themselves cost ~10 % (each waits lgkmcnt(0))."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stableavatar_amd import _lib, ops  # noqa: E402
from stableavatar_amd.kbench import vt_layout  # noqa: E402

L, H, D = 21504, 12, 128
KERN = int(os.environ.get("SA_STAMPS_KERNEL", "3"))  # the V^T kernel to stamp (3: v6t)
dev = "cuda"
qkv = torch.randn(3 * L, 3 * H * D, device=dev).bfloat16()
segs = torch.tensor([[b * L, L, b * L, L] for b in range(3)], dtype=torch.int32, device=dev)
q, k, v_ = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
vt = vt_layout(v_, 3)
o = torch.empty(3 * L, H * D, device=dev, dtype=torch.bfloat16)
lib = ctypes.CDLL(str(_lib.LIB_PATH))
buf = (ctypes.c_ulonglong * 12)()
ops.attention(q, k, vt, o, segs, 3, L, H, kernel=KERN)
torch.cuda.synchronize()
lib.sa_debug_v13_stamps(buf, 1)
n = 3
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(n):
    ops.attention(q, k, vt, o, segs, 3, L, H, kernel=KERN)
ev1.record()
torch.cuda.synchronize()
lib.sa_debug_v13_stamps(buf, 1)
r = {"kernel": KERN, "ms_per_launch": round(ev0.elapsed_time(ev1) / n, 3), "groups": {}}
for gi, gname in enumerate(("waves0-3", "waves4-7")):
    dma, bar, loop, blocks = (buf[gi * 6 + i] for i in range(4))
    r["groups"][gname] = {"cycles_per_block": round(loop / blocks, 1), "dma_wait": round(dma / blocks, 1),
                          "barrier": round(bar / blocks, 1), "barrier_frac": round(bar / loop, 3),
                          "dma_frac": round(dma / loop, 3)}
print(json.dumps(r))
