import torch, json, time
from stableavatar_amd import ops
dev = "cuda"
# vocal projector call at config 2: 21 frames x 32 queries, 8 heads of 192, 1024 keys per frame
Fn, nper, G, H, D = 21, 32, 1024, 8, 192
q = torch.randn(Fn * nper, H * D, device=dev).bfloat16()
kv = torch.randn(Fn * G, 2 * H * D, device=dev).bfloat16()
o = torch.empty(Fn * nper, H * D, device=dev, dtype=torch.bfloat16)
segs = torch.tensor([[f * nper, nper, f * G, G] for f in range(Fn)], dtype=torch.int32, device=dev)
fn = lambda: ops.attention_small(q, kv[:, :H * D], kv[:, H * D:], o, segs, Fn, nper, G, H, D)
for _ in range(3): fn()
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): fn()
torch.cuda.synchronize(); ms = (time.perf_counter() - t) / 20 * 1e3
print(json.dumps({"kernel": "attn_small_vocal", "ms": round(ms, 4)}))
