"""DiT forward on the HIP path vs (a) the reference's own output (goldens) and (b) the CPU oracle at
full 1.3B layer dims.  bf16 tolerance: rel-L2 <= 2e-2, cosine >= 0.9995."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import DIT_SMALL, dit_inputs  # noqa: E402

from stableavatar_amd import synthetic  # noqa: E402
from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm()).item()


def cos(a, b):
    a = torch.as_tensor(a).double().cpu().flatten()
    b = torch.as_tensor(b).double().cpu().flatten()
    return (a @ b / (a.norm() * b.norm())).item()


def make_model(cfg, sd=None):
    m = WanTransformer3DFantasyModel(**{k: v for k, v in cfg.items() if k != "seed"})
    if sd is None:
        sd = synthetic.fill_state_dict(param_shapes(cfg), cfg["seed"])
    m.load_state_dict(sd)
    return m.cuda()


def run(m, inp):
    dev = "cuda"
    with torch.no_grad():
        out = m(x=inp["x"].to(dev).bfloat16(), t=inp["t"].to(dev), context=[c.to(dev) for c in inp["context"]],
                seq_len=inp["seq_len"], clip_fea=inp["clip_fea"].to(dev), y=inp["y"].to(dev).bfloat16(),
                vocal_embeddings=inp["vocal"].to(dev), video_sample_n_frames=inp["n_frames"])
    torch.cuda.synchronize()
    return out.float().cpu()


@pytest.mark.parametrize("case", ["full", "short", "wide"])
def test_dit_vs_reference_golden(case):
    m = make_model(DIT_SMALL)
    out = run(m, dit_inputs(DIT_SMALL, case))
    g = np.load(os.path.join(HERE, "golden", "dit_small.npz"))[f"{case}_out"]
    assert out.shape == g.shape
    assert rel(out, g) < 2e-2 and cos(out, g) > 0.9995, (rel(out, g), cos(out, g))


def test_dit_full_dims_vs_oracle():
    """30 layers, ffn 8960, text_dim 4096, text_len 512 at a tiny grid: HIP path vs CPU oracle."""
    from oracle import dit as odit
    cfg = dict(odit.CONFIG_1_3B, seed=5)
    P = synthetic.fill_state_dict(odit.param_shapes(cfg), cfg["seed"])
    m = make_model(cfg, P)
    inp = dit_inputs(dict(cfg, text_dim=4096), "full")
    out = run(m, inp)
    with torch.no_grad():
        ref = odit.forward(P, cfg, inp["x"], inp["t"], inp["context"], inp["seq_len"], inp["clip_fea"], inp["y"],
                           inp["vocal"], inp["n_frames"])
    assert rel(out, ref) < 2e-2 and cos(out, ref) > 0.9995, (rel(out, ref), cos(out, ref))


def test_dit_fused_cross_attention_matches_unfused(monkeypatch):
    """256 tokens per latent frame enables the one-launch text+image+vocal cross-attention; it must
    agree with the three-launch path (both bf16, rel-L2 <= 1e-2)."""
    from stableavatar_amd import synthetic as syn
    m = make_model(DIT_SMALL)
    B, Fw, H, W = 3, 2, 32, 32
    lat = syn.seeded_normal((1, 16, Fw, H, W), 111)
    inp = dict(x=torch.cat([lat] * 3), y=syn.seeded_normal((B, 20, Fw, H, W), 112),
               context=[syn.seeded_normal((20, 64), 113)] * 2 + [syn.seeded_normal((25, 64), 114)],
               clip_fea=syn.seeded_normal((1, 257, 1280), 115).expand(3, -1, -1).contiguous(),
               vocal=torch.cat([torch.zeros(1, 15, 768), syn.seeded_normal((1, 15, 768), 116).repeat(2, 1, 1)]),
               t=torch.full((3,), 500.0), seq_len=Fw * (H // 2) * (W // 2), n_frames=5)
    monkeypatch.setenv("SA_CROSS3", "1")
    fused = run(m, inp)
    monkeypatch.setenv("SA_CROSS3", "0")
    ref = run(m, inp)
    assert rel(fused, ref) < 1e-2 and cos(fused, ref) > 0.9999, (rel(fused, ref), cos(fused, ref))


def test_dit_qfloat8_weights():
    """GPU_memory_mode 'model_cpu_offload_and_qfloat8' (inference.py:517-518): every parameter except
    'modulation' stored as float8_e4m3fn (fp8_optimization.py:29-43).  The HIP path packs the fp8
    parameters exactly; vs the CPU oracle on the same fp8-rounded weights."""
    from oracle import dit as odit
    P = synthetic.fill_state_dict(param_shapes(DIT_SMALL), DIT_SMALL["seed"])
    m = make_model(DIT_SMALL, P)
    for name, p in m.named_parameters():  # convert_model_weight_to_float8(..., exclude=["modulation"])
        if "modulation" not in name:
            p.data = p.data.to(torch.float8_e4m3fn)
    Pq = {k: (v if "modulation" in k else v.to(torch.float8_e4m3fn).float()) for k, v in P.items()}
    inp = dit_inputs(DIT_SMALL, "full")
    out = run(m, inp)
    with torch.no_grad():
        ref = odit.forward(Pq, DIT_SMALL, inp["x"], inp["t"], inp["context"], inp["seq_len"], inp["clip_fea"],
                           inp["y"], inp["vocal"], inp["n_frames"])
    assert rel(out, ref) < 2e-2 and cos(out, ref) > 0.9995, (rel(out, ref), cos(out, ref))


def test_dit_riflex_vs_reference_golden():
    """enable_riflex() (1B:890-905) after the weights are packed swaps the frame RoPE table in place."""
    g = np.load(os.path.join(HERE, "golden", "dit_small.npz"))
    m = make_model(DIT_SMALL)
    inp = dit_inputs(DIT_SMALL, "full")
    base = run(m, inp)
    m.enable_riflex(k=6, L_test=66, L_test_scale=4.886)
    out = run(m, inp)
    ref = g["full_riflex_out"]
    assert rel(out, ref) < 2e-2 and cos(out, ref) > 0.9995, (rel(out, ref), cos(out, ref))
    m.disable_riflex()
    assert torch.equal(run(m, inp), base)


@pytest.mark.parametrize("wh", [(8, 8), (32, 32)], ids=["v_rows_80tok", "vt_1280tok"])
def test_dit_shared_cfg_rows_first_block_once(wh):
    """forward_window(shared_rows=True): the CFG rows' inputs are equal (the pipeline's tripled latents, y and t,
    wan_inference_long_pipeline.py:693-700,730,733), so the first block's self-attention half runs for one row and
    is copied -- the output equals the full computation bit for bit (V rows at 80 tokens, the V^T kernel at 1 280)"""
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    m = make_model(DIT_SMALL)
    H, W = wh
    dev = "cuda"
    lat = synthetic.seeded_normal((1, 16, 5, H, W), 301).to(dev).bfloat16()
    y = WanI2VTalkingInferenceLongPipeline.mask_latents(synthetic.seeded_normal((1, 16, 5, H, W), 302).to(dev),
                                                        17).bfloat16()
    ctx = [synthetic.seeded_normal((20, 64), 303).to(dev)] * 2 + [synthetic.seeded_normal((25, 64), 304).to(dev)]
    clip = synthetic.seeded_normal((1, 257, 1280), 305).expand(3, -1, -1).contiguous().to(dev)
    a = synthetic.seeded_normal((1, 39, 768), 306).to(dev)
    voc = torch.cat([torch.zeros_like(a), a, a])
    t = torch.tensor([937.5], device=dev)
    S = 5 * (H // 2) * (W // 2)
    outs = []
    with torch.no_grad():
        for shared in (False, True):
            outs.append(m.forward_window(lat, 0, True, 3, t, ctx, S, clip, y, voc, 17, shared_rows=shared).clone())
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
