"""Parity at the benchmarked size (BASELINE config 2: B=3 CFG rows, 512x512x81f -> L = 21 504 tokens,
d 1536, 12 heads x 128, ffn 8960) and at config 1 through the drop-in pipeline's own __call__.

* self-attention: one sa_attn_fwd launch over the full 336 x 84 key/query blocks per head vs fp32
  softmax(QK^T/sqrt(D))V computed on the GPU in query chunks (the reference SDPA, 1B:158-207);
* the persistent GEMMs at M = 64 512 for the QKV, O-proj + gated residual, FFN-up + GELU and FFN-down +
  gated residual shapes vs fp32 matmul (1B:376-379,412,644-646,679,691);
* one full DiT block (a 1-layer model at full width, with the patch embedding, vocal projector and head
  at full size) vs the CPU oracle (oracle/dit.py, pinned to the reference);
* BASELINE config 1 (full 30-layer DiT + full VAE, 256x256, 5 steps, 2 windows/step) and the small
  pipeline golden through WanI2VTalkingInferenceLongPipeline.__call__ with the fake encoders the
  reference golden was made with (its y came from the reference's VAE encode; ours from the HIP encode).
Tolerances (bf16 MFMA vs fp32 reference) are stated per test."""
import json
import math
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import (DIT_FULL, PIPE, PIPE_C1, PIPE_C1_VIDEO_FRAMES, fake_encoders,  # noqa: E402
                          pipe_fixed_inputs, ref_image)

from stableavatar_amd import synthetic  # noqa: E402

pytestmark = pytest.mark.gpu
dev = "cuda"
B, L, H, D = 3, 21504, 12, 128
M = B * L


def rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double().to(a.device)
    return ((a - b).norm() / b.norm()).item()


def psnr(a, b, peak):
    mse = ((torch.as_tensor(a).double().cpu() - torch.as_tensor(b).double().cpu()) ** 2).mean().item()
    return 10 * math.log10(peak * peak / max(mse, 1e-30))


def _attn_errors(q, k, v, o, rows, heads, chunk=4096):
    """per-(row, head) rel-L2 of o vs fp32 softmax(q k^T / sqrt(D)) v, and the max abs error"""
    errs, mx = [], 0.0
    for b in rows:
        for h in heads:
            sl = slice(b * L, (b + 1) * L)
            cs = slice(h * D, (h + 1) * D)
            qh, kh, vh, oh = q[sl, cs].float(), k[sl, cs].float(), v[sl, cs].float(), o[sl, cs].float()
            num = den = 0.0
            for c in range(0, L, chunk):
                ref = torch.softmax((qh[c:c + chunk] @ kh.t()) * D ** -0.5, -1) @ vh
                d = oh[c:c + chunk] - ref
                num += d.pow(2).sum().item()
                den += ref.pow(2).sum().item()
                mx = max(mx, d.abs().max().item())
            errs.append(math.sqrt(num / den))
    return errs, mx


@pytest.mark.timeout(300)
def test_self_attention_fullsize():
    """B=3, L=21504, H=12: every head within rel-L2 1e-2 of fp32 (includes the bf16 rounding of the
    prescaled q*scale*log2(e) the kernel feeds the MFMA and the bf16 P of the PV product)."""
    from stableavatar_amd import ops
    g = torch.Generator(device=dev).manual_seed(1)
    qkv = torch.randn(M, 3 * H * D, device=dev, generator=g).bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(M, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * L, L, b * L, L] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, B, L, H)
    # the 128-row-workgroup schedule (auto-selected for the Ulysses N = 8 shape) is the same per-wave
    # arithmetic: bit-identical, here and on the N = 8 per-rank shape (3 heads, half the queries)
    o4 = torch.empty_like(o)
    ops.attention(q, k, v, o4, segs, B, L, H, kernel=2)
    Lh = L // 2
    segs8 = torch.tensor([[b * L, Lh, b * L, L] for b in range(B)], dtype=torch.int32, device=dev)
    o8a, o8b = torch.zeros_like(o), torch.zeros_like(o)
    ops.attention(q[:, :3 * D], k[:, :3 * D], v[:, :3 * D], o8a[:, :3 * D], segs8, B, Lh, 3, kernel=1)
    ops.attention(q[:, :3 * D], k[:, :3 * D], v[:, :3 * D], o8b[:, :3 * D], segs8, B, Lh, 3)
    torch.cuda.synchronize()
    assert torch.equal(o4, o) and torch.equal(o8a, o8b)
    errs, mx = _attn_errors(q, k, v, o, range(B), range(H))
    print(f"attention L={L}: rel-L2 max {max(errs):.2e} mean {sum(errs) / len(errs):.2e}, max|d| {mx:.2e}")
    assert max(errs) < 1e-2, max(errs)


@pytest.mark.timeout(300)
def test_self_attention_fullsize_peaked_scores():
    """Same launch with q scaled x4 (score std ~4: peaked softmax rows, the running max grows across
    many of the 336 key blocks, so the deferred-rescale branch fires): rel-L2 1e-2 on batch row 1."""
    from stableavatar_amd import ops
    g = torch.Generator(device=dev).manual_seed(2)
    qkv = torch.randn(M, 3 * H * D, device=dev, generator=g)
    qkv[:, :H * D] *= 4.0
    qkv = qkv.bfloat16()
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(M, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * L, L, b * L, L] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, B, L, H)
    torch.cuda.synchronize()
    errs, mx = _attn_errors(q, k, v, o, [1], range(H))
    print(f"attention peaked: rel-L2 max {max(errs):.2e}, max|d| {mx:.2e}")
    assert max(errs) < 1e-2, max(errs)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,N,K,epi", [("qkv", 4608, 1536, "bf16"), ("o_proj", 1536, 1536, "res"),
                                          ("ffn_up", 8960, 1536, "gelu"), ("ffn_down", 1536, 8960, "res")])
def test_dit_gemm_fullsize(name, N, K, epi):
    """M = 64 512 through the persistent kernel (auto): 252 x N/256 tiles walked by 256 workgroups."""
    from stableavatar_amd import ops
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev, generator=g) * 0.1
    ref = x.float() @ w.float().t() + b
    if epi == "bf16":
        y = ops.linear(x, w, b, ops.EPI_BF16)
        tol = 1e-2
    elif epi == "gelu":
        y = ops.linear(x, w, b, ops.EPI_GELU_TANH_BF16)
        ref = torch.nn.functional.gelu(ref.bfloat16().float(), approximate="tanh")
        tol = 1e-2
    else:
        gate = torch.randn(B, N, device=dev, generator=g)
        res = torch.randn(M, N, device=dev, generator=g)
        y = res.clone()
        ops.linear(x, w, b, ops.EPI_RES_F32, out=y, residual=y, gate=gate, rows_per_batch=L)
        ref = res + ref.bfloat16().float() * gate.repeat_interleave(L, 0)
        tol = 2e-3
    torch.cuda.synchronize()
    e = rel(y, ref)
    print(f"gemm {name} M={M} N={N} K={K}: rel-L2 {e:.2e}")
    assert e < tol, e
    # the 192-row persistent tiles (picked by auto for the sequence-parallel per-rank shapes) accumulate every
    # output in the same K order: bit-identical, here at M = 64 512, at the N = 8 per-rank M = 8 064, and at M
    # with a partial last tile of either height (12 285 = the per-rank M at 480x832, N = 8; 1 000)
    # and the three-barrier K schedule (GEMM_S9*, auto's default) computes the same products in the same order
    kerns = [ops.GEMM_PERSISTENT192, ops.GEMM_S9, ops.GEMM_S9_192]
    for Mx in (M, 3 * 2688, 3 * 4095, 1000):
        y2 = torch.empty(Mx, N, device=dev, dtype=y.dtype)
        outs = [torch.empty_like(y2) for _ in kerns]
        for yy, kern in [(y2, ops.GEMM_PERSISTENT)] + list(zip(outs, kerns)):
            if epi == "bf16":
                ops.linear(x[:Mx], w, b, ops.EPI_BF16, out=yy, kernel=kern)
            elif epi == "gelu":
                ops.linear(x[:Mx], w, b, ops.EPI_GELU_TANH_BF16, out=yy, kernel=kern)
            else:
                yy.copy_(res[:Mx])
                ops.linear(x[:Mx], w, b, ops.EPI_RES_F32, out=yy, residual=yy, gate=gate, rows_per_batch=L, kernel=kern)
        torch.cuda.synchronize()
        for i, y3 in enumerate(outs):
            assert torch.equal(y2, y3), (name, Mx, kerns[i])


@pytest.mark.timeout(600)
def test_dit_block_fullsize_vs_oracle():
    """A full-width 1-layer DiT at the config-2 shape (21 latent frames at 64x64, L = 21 504, B = 3):
    patch embedding, time / text / image embeddings, vocal projector over all 21 504 tokens, one
    WanAttentionBlock (self-attention at L = 21 504, cross-attention, FFN) and the head, vs the CPU
    oracle: rel-L2 <= 2e-2 and cosine >= 0.9995 (the §8(d) per-forward contract)."""
    from oracle import dit as odit
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    cfg = dict(DIT_FULL, num_layers=1)
    P = synthetic.fill_state_dict(param_shapes(cfg), 51)
    m = WanTransformer3DFantasyModel(**cfg)
    m.load_state_dict(P)
    m = m.to(dev)
    lat = synthetic.seeded_normal((1, 16, 21, 64, 64), 501)
    x = torch.cat([lat] * 3)
    y = synthetic.seeded_normal((3, 20, 21, 64, 64), 502)
    ctx = [synthetic.seeded_normal((24, 4096), 503)] * 2 + [synthetic.seeded_normal((31, 4096), 504)]
    clip = synthetic.seeded_normal((1, 257, 1280), 505).expand(3, -1, -1).contiguous()
    a = synthetic.seeded_normal((1, 167, 768), 506)
    voc = torch.cat([torch.zeros_like(a), a, a])
    t = torch.full((3,), 937.5)
    with torch.no_grad():
        out = m(x=x.to(dev).bfloat16(), t=t.to(dev), context=[c.to(dev) for c in ctx], seq_len=L,
                clip_fea=clip.to(dev), y=y.to(dev).bfloat16(), vocal_embeddings=voc.to(dev),
                video_sample_n_frames=81).float().cpu()
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        ref = odit.forward(P, cfg, x, t, ctx, L, clip, y, voc, 81)
    e = rel(out, ref)
    cos = torch.nn.functional.cosine_similarity(out.flatten().double(), ref.flatten().double(), dim=0).item()
    print(f"DiT block L={L}: rel-L2 {e:.2e}, cosine {cos:.6f}")
    assert e < 2e-2 and cos > 0.9995, (e, cos)


@pytest.mark.timeout(300)
def test_dit_vt_attention_matches_row_v(monkeypatch):
    """the single-GPU self-attention reading V^T from the QKV GEMM's transposed (P-order) epilogue == the V-rows
    path at the config-2 shape (1 full-width layer, L = 21 504, B = 3): the GEMM products and the attention
    arithmetic are the same, so the forward must agree to bf16 rounding of the V projection at most"""
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
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
    outs = {}
    for vt in ("1", "0"):
        monkeypatch.setenv("SA_ATTN_VT", vt)
        with torch.no_grad():
            outs[vt] = m(x=x, t=t, context=ctx, seq_len=L, clip_fea=clip, y=y, vocal_embeddings=voc,
                         video_sample_n_frames=81).float()
    assert next(iter(m._ws.values())).vt is not None  # the V^T path ran
    e = rel(outs["1"], outs["0"])
    print(f"DiT layer V^T vs V rows: rel-L2 {e:.2e}, bit-identical {torch.equal(outs['1'], outs['0'])}")
    assert torch.equal(outs["1"], outs["0"]), e


@pytest.mark.timeout(600)
def test_dit_ragged_nonsquare_vs_oracle():
    """A non-square size whose token counts align with nothing: 240x416 video (30x52 latent, 15x26 = 390
    tokens per frame, L = 8 190 over 21 frames): partial last query / key blocks in self-attention, the
    3-launch cross-attention (frames are not 256-token aligned) with per-frame vocal segments of 390
    query rows, 1 full-width layer, vs the CPU oracle"""
    from oracle import dit as odit
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    cfg = dict(DIT_FULL, num_layers=1)
    P = synthetic.fill_state_dict(param_shapes(cfg), 52)
    m = WanTransformer3DFantasyModel(**cfg)
    m.load_state_dict(P)
    m = m.to(dev)
    lat = synthetic.seeded_normal((1, 16, 21, 30, 52), 511)
    x = torch.cat([lat] * 3)
    y = synthetic.seeded_normal((3, 20, 21, 30, 52), 512)
    ctx = [synthetic.seeded_normal((24, 4096), 513)] * 2 + [synthetic.seeded_normal((31, 4096), 514)]
    clip = synthetic.seeded_normal((1, 257, 1280), 515).expand(3, -1, -1).contiguous()
    a = synthetic.seeded_normal((1, 161, 768), 516)
    voc = torch.cat([torch.zeros_like(a), a, a])
    t = torch.full((3,), 512.0)
    Lr = 21 * 15 * 26
    with torch.no_grad():
        out = m(x=x.to(dev).bfloat16(), t=t.to(dev), context=[c.to(dev) for c in ctx], seq_len=Lr,
                clip_fea=clip.to(dev), y=y.to(dev).bfloat16(), vocal_embeddings=voc.to(dev),
                video_sample_n_frames=81).float().cpu()
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        ref = odit.forward(P, cfg, x, t, ctx, Lr, clip, y, voc, 81)
    e = rel(out, ref)
    cos = torch.nn.functional.cosine_similarity(out.flatten().double(), ref.flatten().double(), dim=0).item()
    print(f"DiT 240x416 (L={Lr}): rel-L2 {e:.2e}, cosine {cos:.6f}")
    assert out.shape == ref.shape and e < 2e-2 and cos > 0.9995, (e, cos)


def _drop_in_pipeline(P):
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes
    from stableavatar_amd.vae import param_shapes as vae_shapes
    dcfg = {k: v for k, v in P["dit"].items() if k != "seed"}
    dit = WanTransformer3DFantasyModel(**dcfg)
    dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), P["dit"]["seed"]))
    vdim = P["vae"]["dim"]
    vae = AutoencoderKLWan(dim=vdim)
    vae.load_state_dict(synthetic.fill_state_dict(dict(vae_shapes(dim=vdim), **encoder_param_shapes(dim=vdim)),
                                                  P["vae"]["seed"]))
    fx = pipe_fixed_inputs(P)
    pipe = WanI2VTalkingInferenceLongPipeline(vae=vae, transformer=dit,
                                              scheduler=FlowMatchEulerDiscreteScheduler(1000, shift=5.0),
                                              **fake_encoders(P, fx))
    return pipe.to(dev), fx


@pytest.mark.timeout(600)
@pytest.mark.parametrize("case", ["small", "config1", "s05", "s10", "s50"])
def test_pipeline_call_vs_reference(case):
    """The drop-in __call__ with the reference's arguments (gen_golden.py): prompt -> fake T5, reference
    image -> fake CLIP + HIP VAE encode -> y, audio -> fake wav2vec per window, 2 windows x N steps,
    HIP VAE decode.  The SURVEY.md §8(d) contract for every case (config 1: 30 layers x 10 forwards of bf16
    drift; measured 7.9e-3 / 49 dB): y rel-L2 < 3e-2, latents rel-L2 <= 3e-2, video PSNR >= 30 dB on [0, 1].
    s05 / s10 / s50: the reference's loop over 5 / 10 / 50 steps of its own schedule (2-layer DiT, 2 windows per
    step; 50 steps = the reference's default, wan_inference_long_pipeline.py:703-792), the drift's growth with
    the step count; each case's numbers are appended to gpurun_out/pipeline_steps_drift.jsonl."""
    from golden_cases import PIPE_STEPS
    P, name = {"small": (PIPE, "pipeline_small.npz"), "config1": (PIPE_C1, "pipeline_c1.npz"),
               "s05": (PIPE_STEPS[5], "pipeline_s05.npz"), "s10": (PIPE_STEPS[10], "pipeline_s10.npz"),
               "s50": (PIPE_STEPS[50], "pipeline_s50.npz")}[case]
    g = np.load(os.path.join(HERE, "golden", name))
    pipe, fx = _drop_in_pipeline(P)
    path = ref_image()
    kw = dict(num_frames=P["clip_length"], height=P["height"], width=P["width"], guidance_scale=6.0,
              num_inference_steps=P["steps"], latents=fx["latents"], text_guide_scale=P["text_guide"],
              audio_guide_scale=P["audio_guide"], vocal_input_values=fx["audio"].numpy(), fps=25, sr=16000,
              cond_file_path=path, overlap_window_length=P["overlap"], clip_length=P["clip_length"])
    with torch.no_grad():
        _, yy = pipe._conditioning(path, P["height"], P["width"], P["clip_length"], torch.float32)
        lat = pipe("pos prompt", negative_prompt="", output_type="latent", **kw).videos
        video = pipe("pos prompt", negative_prompt="", **kw).videos
    torch.cuda.synchronize()
    ey = rel(yy[:1].float().cpu(), g["y"][:1])
    el = rel(lat.float().cpu(), g["latents"])
    gv = g["video"].astype(np.float32)
    frames = list(g["video_frames"]) if "video_frames" in g else list(range(gv.shape[2]))
    pv = psnr(video[:, :, frames].float(), gv, 1.0)
    print(f"pipeline {case}: y rel {ey:.2e}, latents rel {el:.2e}, video PSNR {pv:.1f} dB")
    if case in ("s05", "s10", "s50"):
        os.makedirs("gpurun_out", exist_ok=True)
        with open("gpurun_out/pipeline_steps_drift.jsonl", "a") as f:
            f.write(json.dumps({"steps": P["steps"], "forwards": 2 * P["steps"], "y_rel": ey, "latents_rel": el,
                                "video_psnr_db": pv}) + "\n")
    assert tuple(video.shape) == (1, 3, 1 + 4 * (g["latents"].shape[2] - 1), P["height"], P["width"])
    assert ey < 3e-2, ey
    assert el <= 3e-2, el
    assert pv >= 30.0, pv
