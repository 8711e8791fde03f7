"""Compute-only time of ONE Ulysses rank's DiT forward at SP degree N on one MI355X (config 2 shape), with the
point-to-point exchanges and the head all-gather stubbed out (no data moves; the exchange buffers hold random
values so the kernels see ordinary data).  Measures what sequence parallelism costs in kernel efficiency alone
(GEMM tiles and attention workgroups per rank at 1/N of the tokens), i.e. the upper bound of the N-GPU
speedup before any xGMI time.  usage: python scripts/sp_rank_compute.py [N ...]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from stableavatar_amd import sp, synthetic  # noqa: E402
from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes  # noqa: E402

degrees = [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8]
dev = "cuda"
cfg = dict(model_type="i2v", dim=1536, ffn_dim=8960, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
           num_heads=12, num_layers=30, text_len=512)
m = WanTransformer3DFantasyModel(**cfg)
m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), 0, backend="torch", device=dev))
m = m.to(dev)
g = torch.Generator(device=dev).manual_seed(0)
lat = torch.randn(1, 16, 21, 64, 64, device=dev, generator=g).bfloat16()
y = torch.randn(1, 20, 21, 64, 64, device=dev, generator=g).bfloat16().expand(3, -1, -1, -1, -1).contiguous()
ctx = [torch.randn(n, 4096, device=dev, generator=g) for n in (120, 120, 60)]
clip = torch.randn(3, 257, 1280, device=dev, generator=g)
voc = torch.randn(3, 167, 768, device=dev, generator=g)
t = torch.tensor([990.0], device=dev)

sp._p2p = lambda sends, recvs, group: sp.Pending(None)
_orig_gather = sp.gather_tokens


def fake_gather(local, B, Lc, world, group=None):
    return torch.zeros(B * world * Lc, local.shape[1], device=local.device, dtype=local.dtype)


sp.gather_tokens = fake_gather


shared = os.environ.get("SA_SPRC_SHARED", "1") != "0"  # the pipeline's CFG rows: equal inputs (shared_rows)


def fwd():
    return m.forward_window(lat, 0, True, 3, t, ctx, 21504, clip, y, voc, 81, shared_rows=shared)


res = []
modes = os.environ.get("SA_SPRC_MODES", "1").split(",")  # SA_SP_OVERLAP values to time at each degree > 1
with torch.no_grad():
    for N, ov in [(n, o) for n in degrees for o in (modes if n > 1 else ["1"])]:
        os.environ["SA_SP_OVERLAP"] = ov
        if N == 1:
            m.disable_multi_gpus_inference()
        else:
            m.sp_group, m.sp_world_size, m.sp_world_rank, m._sp_enabled = None, N, 0, True
        fwd()  # builds the exchange buffers at this degree
        if N > 1:
            ex = m._sp_ex[1]
            for buf in (ex.q, ex.kv, ex.obuf):
                buf.normal_()
        for _ in range(2):
            fwd()
        torch.cuda.synchronize()
        ts, hs = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            fwd()
            hs.append((time.perf_counter() - t0) * 1e3)  # host enqueue time of the forward (no sync inside)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        r = {"kernel": "sp_rank_forward", "degree": N, "sp_overlap": ov, "ms": round(sorted(ts)[1], 2),
             "host_enqueue_ms": round(sorted(hs)[1], 2)}
        res.append(r)
        print(json.dumps(r), flush=True)
base = res[0]["ms"] if res[0]["degree"] == 1 else None
if base:
    for r in res:
        r["ideal_ms"] = round(base / r["degree"], 2)
        r["compute_efficiency"] = round(base / r["degree"] / r["ms"], 3)
    print(json.dumps({"kernel": "sp_rank_summary", "rows": res}), flush=True)
