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


@pytest.mark.timeout(300)
def test_vae_decode_fullsize_first_frames_vs_oracle():
    """The config-2 decode at full size: the 81 x 512^2 clip's latents [16, 21, 64, 64] decoded by the HIP path
    (full width dim 96, one 21-frame chunk as in the bench) -- its first 21 output frames (latent frames 0-5: the
    first frame's "Rep" path and 5 steady-state frames behind it) vs the fp32 CPU oracle (oracle/vae.py, pinned to
    wan_vae.py:549-574 by the goldens) on those 6 latent frames: the decoder is causal, so they depend on nothing
    later.  The other 60 frames are checked finite here and against the oracle at every frame in
    test_vae_decode_all_frames_vs_oracle (same width and depth, 128^2).  PSNR >= 40 dB over [-1, 1]."""
    from oracle import vae as ovae
    from stableavatar_amd.vae import encoder_param_shapes, param_shapes
    P = synthetic.fill_state_dict(dict(param_shapes(dim=96), **encoder_param_shapes(dim=96)), 61)
    from stableavatar_amd.vae import AutoencoderKLWan
    v = AutoencoderKLWan(dim=96)
    v.load_state_dict(P, strict=True)
    v = v.cuda()
    z = synthetic.seeded_normal((16, 21, 64, 64), 611)
    with torch.no_grad():
        video = v.decode_clip(z.cuda())  # [3, 81, 512, 512]
    torch.cuda.synchronize()
    assert tuple(video.shape) == (3, 81, 512, 512) and torch.isfinite(video).all()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with torch.no_grad():
        ref = ovae.decode(P, z[None, :, :6])[0]  # [3, 21, 512, 512]
    got = video[:, :21].float().cpu()
    p, r = psnr(got, ref, 2.0), rel(got, ref)
    pl = psnr(got[:, 9:], ref[:, 9:], 2.0)
    print(f"VAE decode 81x512^2, frames 0-20 vs fp32 oracle: PSNR {p:.2f} dB (frames 9-20: {pl:.2f}), rel-L2 {r:.2e}")
    assert p >= 40.0 and pl >= 40.0, (p, pl, r)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("chunk", [None, 8])
def test_vae_decode_all_frames_vs_oracle(chunk):
    """Every one of the 81 output frames of a 21-latent-frame decode at the full VAE width (dim 96) on a 128^2 frame
    vs the fp32 oracle's whole-sequence decode: the steady-state frames a 512^2 oracle run cannot reach in a test's
    time.  chunk 8: the long-clip path (config 5) with the causal caches carried across two chunk seams (latent
    frames 8 and 16), as the reference's frame-by-frame loop carries them (wan_vae.py:549-574).  PSNR >= 40 dB."""
    from oracle import vae as ovae
    from stableavatar_amd.vae import encoder_param_shapes, param_shapes
    P = synthetic.fill_state_dict(dict(param_shapes(dim=96), **encoder_param_shapes(dim=96)), 62)
    from stableavatar_amd.vae import AutoencoderKLWan
    v = AutoencoderKLWan(dim=96)
    v.load_state_dict(P, strict=True)
    v = v.cuda()
    z = synthetic.seeded_normal((16, 21, 16, 16), 612)
    with torch.no_grad():
        video = (v.decode_clip(z.cuda()) if chunk is None else v.decode_clip(z.cuda(), chunk=chunk)).float().cpu()
    torch.cuda.synchronize()
    assert tuple(video.shape) == (3, 81, 128, 128)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    with torch.no_grad():
        ref = ovae.decode(P, z[None])[0]
    worst = min(psnr(video[:, f], ref[:, f], 2.0) for f in range(81))
    p = psnr(video, ref, 2.0)
    print(f"VAE decode 81x128^2 chunk {chunk}: PSNR {p:.2f} dB, worst frame {worst:.2f} dB")
    assert p >= 40.0 and worst >= 38.0, (p, worst)


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


@pytest.mark.parametrize("scheme", ["uniform", "log"])
def test_pipeline_vs_reference(scheme):
    """the denoise loop + decode vs the reference's __call__; "log": overlapping_weight_scheme="log"
    (pipeline:761-766) at overlap 3 (golden_cases.PIPE_LOG)"""
    from golden_cases import PIPE_LOG
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, audio_window, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    g = G("pipeline_small.npz" if scheme == "uniform" else "pipeline_log.npz")
    P = PIPE if scheme == "uniform" else PIPE_LOG
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
    noise = fx["latents"].cuda().bfloat16()  # bf16 already: denoise must still leave the caller's tensor alone
    keep = noise.clone()
    with torch.no_grad():
        lat = pipe.denoise(noise, torch.from_numpy(g["y"]).cuda(), ctx,
                           torch.cat([fx["clip"]] * 3).cuda(), feats, sched.timesteps, sched.sigmas,
                           clip_length=P["clip_length"], seq_len=seq_len, overlap=P["overlap"],
                           text_guide_scale=P["text_guide"], audio_guide_scale=P["audio_guide"], scheme=scheme)
        video = vae.decode_clip(lat[0].float(), post=True)[None]
    torch.cuda.synchronize()
    assert torch.equal(noise, keep), "denoise overwrote its input latents"
    assert rel(lat.float(), g["latents"]) < 3e-2, rel(lat.float(), g["latents"])
    assert psnr(video, g["video"], 1.0) > 30.0, psnr(video, g["video"], 1.0)


def _pipe_small():
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    dcfg = PIPE["dit"]
    dit = WanTransformer3DFantasyModel(**{k: v for k, v in dcfg.items() if k != "seed"})
    dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), dcfg["seed"]))
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(2, device="cuda")
    return WanI2VTalkingInferenceLongPipeline(transformer=dit.cuda(), scheduler=sched), sched


def _denoise_with(pipe, sched, seed):
    """one denoise call whose prompt embeddings and CLIP context are built (and freed) inside this call, so the
    caching allocator can hand the next call's same-shape tensors the same addresses"""
    from stableavatar_amd.pipeline import window_schedule
    g = torch.Generator().manual_seed(seed)
    T, fpb = 6, 5
    lat = torch.randn(1, 16, T, 8, 8, generator=torch.Generator().manual_seed(7)).cuda()
    y = torch.randn(3, 20, fpb, 8, 8, generator=torch.Generator().manual_seed(8)).cuda()
    ctx = [torch.randn(12, 64, generator=g).cuda(), None, torch.randn(9, 64, generator=g).cuda()]
    ctx[1] = ctx[0]
    clip = torch.randn(1, 257, 1280, generator=g).expand(3, -1, -1).contiguous().cuda()
    feats = {}
    for (s, e, _) in window_schedule(T, fpb, 2):
        a = synthetic.fake_wav2vec_features(torch.randn(1, 20 * 640, generator=torch.Generator().manual_seed(9)))
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a]).cuda()
    with torch.no_grad():
        out = pipe.denoise(lat, y, ctx, clip, feats, sched.timesteps, sched.sigmas, clip_length=17, seq_len=80,
                           overlap=2, text_guide_scale=3.0, audio_guide_scale=5.0)
    torch.cuda.synchronize()
    return out.cpu()


def test_context_cache_second_call_matches_fresh_model():
    """The text / image K/V cache (transformer._context) must not serve a later call's new prompt or reference
    image from the previous call's K/V: a second call with different same-shape embeddings and CLIP context
    equals a fresh model's output bit for bit (the reference recomputes the context every forward, 1B:993-1002)."""
    pipe, sched = _pipe_small()
    first = _denoise_with(pipe, sched, 1)
    second = _denoise_with(pipe, sched, 2)
    fresh_pipe, fresh_sched = _pipe_small()
    fresh = _denoise_with(fresh_pipe, fresh_sched, 2)
    assert not torch.equal(first, second)
    assert torch.equal(second, fresh), (second.float() - fresh.float()).abs().max().item()
    # the direct forward path (no pipeline invalidation): a new context of the same shape is not a cache hit
    m = pipe.transformer
    x = torch.randn(3, 16, 5, 8, 8, generator=torch.Generator().manual_seed(3)).cuda().bfloat16()
    yv = torch.randn(3, 20, 5, 8, 8, generator=torch.Generator().manual_seed(4)).cuda().bfloat16()
    voc = torch.randn(3, 39, 768, generator=torch.Generator().manual_seed(5)).cuda()

    def fwd(model, seed):
        g = torch.Generator().manual_seed(seed)
        c = [torch.randn(12, 64, generator=g).cuda() for _ in range(3)]
        cl = torch.randn(3, 257, 1280, generator=g).cuda()
        with torch.no_grad():
            o = model(x=x, t=torch.full((3,), 500.0, device="cuda"), context=c, seq_len=80, clip_fea=cl, y=yv,
                      vocal_embeddings=voc, video_sample_n_frames=17)
        torch.cuda.synchronize()
        return o.cpu()

    fwd(m, 11)
    b = fwd(m, 12)
    assert torch.equal(b, fwd(fresh_pipe.transformer, 12))
