"""VAE decode and the full sliding-window pipeline on the HIP path vs the reference's own outputs
(goldens).  bf16 activations vs the fp32 reference: tolerances stated per test."""
import math
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import PIPE, VAE_ENC_SMALL, VAE_SMALL, pipe_fixed_inputs, vae_latent, vae_video  # noqa: E402

from stableavatar_amd import synthetic  # noqa: E402

pytestmark = pytest.mark.gpu
G = lambda n: np.load(os.path.join(HERE, "golden", n))  # noqa: E731


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm()).item()


def psnr(a, b, peak):
    mse = ((torch.as_tensor(a).double().cpu() - torch.as_tensor(b).double().cpu()) ** 2).mean().item()
    return 10 * math.log10(peak * peak / max(mse, 1e-30))


def make_vae(dim, seed):
    from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes, param_shapes
    v = AutoencoderKLWan(dim=dim)
    shapes = dict(param_shapes(dim=dim), **encoder_param_shapes(dim=dim))
    v.load_state_dict(synthetic.fill_state_dict(shapes, seed), strict=True)
    return v.cuda()


@pytest.mark.parametrize("name", list(VAE_SMALL))
def test_vae_decode_vs_reference(name):
    cfg = VAE_SMALL[name]
    v = make_vae(cfg["dim"], cfg["seed"])
    with torch.no_grad():
        out = v.decode(vae_latent(cfg).cuda()).sample
    torch.cuda.synchronize()
    g = G("vae_small.npz")[name]
    assert tuple(out.shape) == g.shape
    # outputs live in [-1, 1]: PSNR over a peak-to-peak range of 2
    assert psnr(out, g, 2.0) > 40.0 and rel(out, g) < 3e-2, (psnr(out, g, 2.0), rel(out, g))


@pytest.mark.parametrize("chunk", [1, 2, 3])
def test_vae_chunked_decode_equals_whole_clip(chunk):
    """Long-clip decode (config 5) in chunks of latent frames with the causal cache carried between
    chunks == the whole-clip decode, bit for bit (chunk 1 is the reference's own frame-by-frame
    schedule, wan_vae.py:549-574)."""
    v = make_vae(32, 24)
    z = synthetic.seeded_normal((16, 7, 8, 8), 424).cuda()
    with torch.no_grad():
        whole = v.decode_clip(z, chunk=7)
        part = v.decode_clip(z, chunk=chunk)
    torch.cuda.synchronize()
    assert tuple(part.shape) == (3, 25, 64, 64)
    assert torch.equal(whole, part), (whole - part).abs().max().item()


@pytest.mark.parametrize("name", list(VAE_ENC_SMALL))
def test_vae_encode_vs_reference(name):
    """HIP encoder (whole clip, bf16 activations) vs the reference's chunked fp32 encode: the
    posterior parameters cat(mu, log_var) within rel-L2 3e-2 and .mode() == mu."""
    cfg = VAE_ENC_SMALL[name]
    v = make_vae(cfg["dim"], cfg["seed"])
    with torch.no_grad():
        post = v.encode(vae_video(cfg).cuda())[0]
        h = post.parameters
        mode = post.mode()
    torch.cuda.synchronize()
    g = G("vae_enc_small.npz")[name]
    assert tuple(h.shape) == g.shape
    assert torch.equal(mode, h[:, :16])
    assert rel(h, g) < 3e-2, rel(h, g)


def test_vae_encode_full_frame_shape_and_causality():
    """512x512-class property at a GPU-sized clip (dim 96, 33 frames at 128x128): output shape, and
    causality - frames after t change no latent frame before their chunk (encode of a prefix == the
    same prefix of the full encode, up to bf16 reordering noise)."""
    v = make_vae(96, 23)
    x = (0.5 * synthetic.seeded_normal((1, 3, 33, 128, 128), 333)).clamp(-1, 1).cuda()
    with torch.no_grad():
        full = v.encode(x)[0].parameters
        pre = v.encode(x[:, :, :17])[0].parameters
    torch.cuda.synchronize()
    assert tuple(full.shape) == (1, 32, 9, 16, 16) and torch.isfinite(full).all()
    assert rel(pre, full[:, :, :5]) < 1e-6, rel(pre, full[:, :, :5])


def test_pipeline_vs_reference():
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, audio_window, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    g = G("pipeline_small.npz")
    P = PIPE
    dcfg = P["dit"]
    dit = WanTransformer3DFantasyModel(**{k: v for k, v in dcfg.items() if k != "seed"})
    dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), dcfg["seed"]))
    dit = dit.cuda()
    vae = make_vae(P["vae"]["dim"], P["vae"]["seed"])
    fx = pipe_fixed_inputs(P)
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    pipe = WanI2VTalkingInferenceLongPipeline(vae=vae, transformer=dit, scheduler=sched)
    sched.set_timesteps(P["steps"], device="cuda")
    T = fx["latents"].shape[2]
    fpb = (P["clip_length"] - 1) // 4 + 1
    feats = {}
    for (s, e, _) in window_schedule(T, fpb, P["overlap"]):
        sub = fx["audio"][audio_window(s, e, T, 640, fx["audio"].shape[0])]
        a = synthetic.fake_wav2vec_features(sub[None]).cuda()
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a])
    ctx = [fx["neg_embeds"].cuda(), fx["neg_embeds"].cuda(), fx["pos_embeds"].cuda()]
    seq_len = math.ceil(P["width"] // 8 * P["height"] // 8 / 4 * fpb)
    with torch.no_grad():
        lat = pipe.denoise(fx["latents"].cuda(), torch.from_numpy(g["y"]).cuda(), ctx,
                           torch.cat([fx["clip"]] * 3).cuda(), feats, sched.timesteps, sched.sigmas,
                           clip_length=P["clip_length"], seq_len=seq_len, overlap=P["overlap"],
                           text_guide_scale=P["text_guide"], audio_guide_scale=P["audio_guide"])
        video = vae.decode_clip(lat[0].float(), post=True)[None]
    torch.cuda.synchronize()
    assert rel(lat.float(), g["latents"]) < 3e-2, rel(lat.float(), g["latents"])
    assert psnr(video, g["video"], 1.0) > 30.0, psnr(video, g["video"], 1.0)
