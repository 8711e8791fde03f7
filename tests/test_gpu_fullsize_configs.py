"""Parity at the sizes BASELINE.json's other configurations name:

* the examples/case-1 windowed loop at full size (config 2's long-clip form: 512x512, T_lat 42, 5 windows of 21
  latent frames at overlap 15 per step) with a 1-layer full-width DiT for 2 of the 50 sampling steps, through
  pipeline.denoise on the HIP path, vs oracle/pipeline.py's loop (tests/golden/case1_fullsize.npz,
  gen_case1_fullsize.py): the window gather, CFG, Euler step, overlap blend and scatter at full size;
* config 4's 14B shapes at 720x1280x81f (L = 75 600, B = 3, 40 heads of 128): the self-attention launch on
  sampled query rows of several heads vs fp32 softmax(QK^T/sqrt(D))V over all 75 600 keys, and the block GEMMs
  (M = 226 800; QKV 5120 -> 15360, O 5120 -> 5120 + gated residual, FFN 5120 -> 13824 + GELU, 13824 -> 5120 +
  gated residual) on sampled rows, including the last, partial tile, vs fp32 matmul
  (wan_fantasy_transformer3d_14B.py's WanAttentionBlock at dim 5120, ffn 13824)."""
import math
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import CASE1_FULL, case1_fullsize_inputs  # noqa: E402

from stableavatar_amd import synthetic  # noqa: E402

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double().to(a.device)
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.timeout(300)
def test_case1_windows_fullsize_vs_oracle():
    """latents rel-L2 <= 3e-2 (the pipeline contract) after 2 steps x 5 windows at 512x512, T_lat 42"""
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, audio_window, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    C = CASE1_FULL
    g = np.load(os.path.join(HERE, "golden", "case1_fullsize.npz"))
    ref = torch.from_numpy(g["latents_bf16"]).view(torch.bfloat16).float()
    cfg = {k: v for k, v in C["dit"].items() if k != "seed"}
    dit = WanTransformer3DFantasyModel(**cfg)
    dit.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), C["dit"]["seed"]))
    pipe = WanI2VTalkingInferenceLongPipeline(transformer=dit.to(dev))
    inp = case1_fullsize_inputs(C)
    T, fpb = C["T"], (C["clip_length"] - 1) // 4 + 1
    wins = window_schedule(T, fpb, C["overlap"])
    assert len(wins) == 5 and int(g["forwards"]) == 5 * C["run_steps"]
    audio = inp["audio"]
    feats = {}
    for (s, e, _) in wins:
        a = synthetic.fake_wav2vec_features(audio[audio_window(s, e, T, 640, audio.shape[0])][None])
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a]).to(dev)
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(C["steps"], device=dev)
    h = C["size"] // 8
    seq_len = math.ceil(h * h / 4 * fpb)
    with torch.no_grad():
        lat = pipe.denoise(inp["latents"].to(dev), inp["y"].to(dev), [c.to(dev) for c in inp["context"]],
                           inp["clip"].to(dev), feats, sched.timesteps[:C["run_steps"]],
                           sched.sigmas[:C["run_steps"] + 1], clip_length=C["clip_length"], seq_len=seq_len,
                           overlap=C["overlap"], text_guide_scale=C["text_guide"], audio_guide_scale=C["audio_guide"])
    torch.cuda.synchronize()
    out = lat.float().cpu()
    e = rel(out, ref)
    # the frames only the later windows write (and the blended overlaps) on their own
    e_tail = rel(out[:, :, 21:], ref[:, :, 21:])
    print(f"case-1 full size ({len(wins)} windows x {C['run_steps']} steps): latents rel-L2 {e:.2e} "
          f"(frames 21-41 {e_tail:.2e})")
    assert out.shape == ref.shape == (1, 16, T, h, h)
    assert e <= 3e-2 and e_tail <= 3e-2, (e, e_tail)


L14, H14, D = 75600, 40, 128
M14 = 3 * L14


@pytest.mark.timeout(300)
def test_attention_14b_720p_sampled_rows():
    """one sa_attn_fwd launch at B = 3, L = 75 600, 40 heads; 4 heads x 3 batch rows x 320 query rows (256 random +
    the last 64, the partial query block) vs fp32 over all keys: rel-L2 <= 1e-2 per (row, head) set"""
    from stableavatar_amd import ops
    gen = torch.Generator(device=dev).manual_seed(14)
    qkv = torch.randn(M14, 3 * H14 * D, device=dev, generator=gen, dtype=torch.bfloat16)
    q, k, v = qkv[:, :H14 * D], qkv[:, H14 * D:2 * H14 * D], qkv[:, 2 * H14 * D:]
    o = torch.empty(M14, H14 * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * L14, L14, b * L14, L14] for b in range(3)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, 3, L14, H14)
    torch.cuda.synchronize()
    rows = torch.cat([torch.randperm(L14 - 64, generator=torch.Generator().manual_seed(5))[:256],
                      torch.arange(L14 - 64, L14)]).to(dev)
    worst = 0.0
    for b in range(3):
        for h in (0, 13, 27, 39):
            cs = slice(h * D, (h + 1) * D)
            kb, vb = k[b * L14:(b + 1) * L14, cs].float(), v[b * L14:(b + 1) * L14, cs].float()
            qb = q[b * L14 + rows, cs].float()
            ref = torch.softmax((qb @ kb.t()) * D ** -0.5, -1) @ vb
            worst = max(worst, rel(o[b * L14 + rows, cs].float(), ref))
    print(f"attention 14B 720p L={L14}: worst rel-L2 over 12 (batch, head) row sets {worst:.2e}")
    assert worst <= 1e-2, worst


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,N,K,epi", [("qkv", 15360, 5120, "bf16"), ("o_proj", 5120, 5120, "res"),
                                          ("ffn_up", 13824, 5120, "gelu"), ("ffn_down", 5120, 13824, "res")])
def test_dit14_gemm_720p_sampled_rows(name, N, K, epi):
    """M = 226 800 (885.9 256-row tiles: a partial last tile) through the auto-selected persistent kernel; 2 048
    random rows + the last 300 vs fp32 (bf16 outputs 1e-2, gated fp32 residual 2e-3)"""
    from stableavatar_amd import ops
    gen = torch.Generator(device=dev).manual_seed(15)
    x = torch.randn(M14, K, device=dev, generator=gen, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=dev, generator=gen) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev, generator=gen) * 0.1
    rows = torch.cat([torch.randperm(M14 - 300, generator=torch.Generator().manual_seed(6))[:2048],
                      torch.arange(M14 - 300, M14)]).to(dev)
    ref = x[rows].float() @ w.float().t() + b
    if epi == "bf16":
        y = ops.linear(x, w, b, ops.EPI_BF16)
        tol = 1e-2
    elif epi == "gelu":
        y = ops.linear(x, w, b, ops.EPI_GELU_TANH_BF16)
        ref = torch.nn.functional.gelu(ref.bfloat16().float(), approximate="tanh")
        tol = 1e-2
    else:
        gate = torch.randn(3, N, device=dev, generator=gen)
        y = torch.randn(M14, N, device=dev, generator=gen)
        res_rows = y[rows].clone()
        ops.linear(x, w, b, ops.EPI_RES_F32, out=y, residual=y, gate=gate, rows_per_batch=L14)
        ref = res_rows + ref.bfloat16().float() * gate[rows // L14]
        tol = 2e-3
    torch.cuda.synchronize()
    e = rel(y[rows].float(), ref)
    print(f"gemm 14B {name} M={M14} N={N} K={K}: rel-L2 {e:.2e} on {rows.numel()} rows")
    assert e < tol, e
