"""VAE decode timing + per-conv breakdown source for rocprofv3 (config 2: 21 latent frames at 64x64 ->
81 frames at 512x512), synthetic weights.  usage: python scripts/kb_vae.py [iters]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from stableavatar_amd import synthetic  # noqa: E402
from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes, param_shapes  # noqa: E402

dev = torch.device("cuda")
vae = AutoencoderKLWan().to(dev)
vae.load_state_dict(synthetic.fill_state_dict(dict(param_shapes(), **encoder_param_shapes()), 1, backend="torch",
                                              device=dev))
lat = torch.randn(16, 21, 64, 64, generator=torch.Generator().manual_seed(0)).to(dev)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
with torch.no_grad():
    out = vae.decode_clip(lat, post=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        vae.decode_clip(lat, post=True)
    torch.cuda.synchronize()
ms = (time.perf_counter() - t) / iters * 1e3
# checksum of the output bytes: an A/B of two library builds with the same K order must agree exactly
h = int(out.float().contiguous().view(torch.int32).to(torch.int64).sum().item())
print(json.dumps({"kernel": "vae_decode_81f_512", "ms": round(ms, 1), "out_checksum": h}))
