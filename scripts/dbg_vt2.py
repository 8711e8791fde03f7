"""debug: 1-layer full-width DiT at L = 21 504, V^T path vs V rows: capture the self-attention call's inputs"""
import os
import sys
import torch
sys.path.insert(0, "tests/golden")
from golden_cases import DIT_FULL
from stableavatar_amd import ops, synthetic
from stableavatar_amd.kbench import vt_layout
from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes

dev = "cuda"
L = 21504
cfg = dict(DIT_FULL, num_layers=1)
m = WanTransformer3DFantasyModel(**cfg)
m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), 53))
m = m.to(dev)
lat = synthetic.seeded_normal((1, 16, 21, 64, 64), 521)
x = torch.cat([lat] * 3).to(dev).bfloat16()
y = synthetic.seeded_normal((3, 20, 21, 64, 64), 522).to(dev).bfloat16()
ctx = [c.to(dev) for c in [synthetic.seeded_normal((24, 4096), 523)] * 2 + [synthetic.seeded_normal((31, 4096), 524)]]
clip = synthetic.seeded_normal((1, 257, 1280), 525).expand(3, -1, -1).contiguous().to(dev)
a = synthetic.seeded_normal((1, 167, 768), 526)
voc = torch.cat([torch.zeros_like(a), a, a]).to(dev)
t = torch.full((3,), 937.5, device=dev)
cap = {}
orig = ops.attention


def spy(q, k, v, out, segs, nseg, mq, heads, **kw):
    r = orig(q, k, v, out, segs, nseg, mq, heads, **kw)
    if q.shape[0] == 3 * L and k.shape[0] == 3 * L:
        torch.cuda.synchronize()
        cap[os.environ["SA_ATTN_VT"]] = (q.clone(), k.clone(), v.clone(), out.clone(), kw.get("kernel"), segs.clone())
    return r


ops.attention = spy
outs = {}
rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
for i, vt in enumerate(("0", "1", "0", "1")):
    os.environ["SA_ATTN_VT"] = vt
    with torch.no_grad():
        outs[i] = m(x=x, t=t, context=ctx, seq_len=L, clip_fea=clip, y=y, vocal_embeddings=voc,
                    video_sample_n_frames=81).float()
    torch.cuda.synchronize()
print("0 vs 2 (rows twice)", rel(outs[0], outs[2]), "1 vs 3 (vt twice)", rel(outs[1], outs[3]),
      "0 vs 1", rel(outs[1], outs[0]), "2 vs 3", rel(outs[3], outs[2]))
q1, k1, v1, o1, kern1, s1 = cap["1"]
q0, k0, v0, o0, kern0, s0 = cap["0"]
print("kernels", kern1, kern0, "segs", s1.tolist(), s0.tolist(), "v shapes", v1.shape, v0.shape, v1.stride(), v0.stride())
print("q equal", torch.equal(q1, q0), "k equal", torch.equal(k1, k0))
vref = vt_layout(v0.contiguous(), 3)
print("vt equal", torch.equal(v1, vref), rel(v1, vref))
print("attn out rel", rel(o1, o0), torch.equal(o1, o0))
