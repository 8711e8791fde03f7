"""The 14B family on the HIP path (BASELINE config 4's model): WanTransformer3DFantasy14BModel at its full
width (dim 5120, 40 heads of 128; vocal projector 5120 wide with 8 heads of 640 on every CFG row) and one
layer, vs the reference module's own output (tests/golden/dit14_small.npz, gen_golden.py gen_dit14), and a
wider token grid vs the CPU oracle (oracle/dit.py, pinned to that golden)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import DIT14_SMALL, dit14_inputs  # noqa: E402

from stableavatar_amd import synthetic  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = torch.as_tensor(a).double().cpu(), torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm()).item()


def cos(a, b):
    a, b = torch.as_tensor(a).double().cpu().flatten(), torch.as_tensor(b).double().cpu().flatten()
    return torch.nn.functional.cosine_similarity(a, b, dim=0).item()


@pytest.fixture(scope="module")
def model14():
    from stableavatar_amd.transformer import WanTransformer3DFantasy14BModel, param_shapes
    cfg = dict(DIT14_SMALL, vocal="14B")
    m = WanTransformer3DFantasy14BModel(**{k: v for k, v in cfg.items() if k not in ("seed", "vocal")})
    P = synthetic.fill_state_dict(param_shapes(cfg), cfg["seed"])  # the oracle reads the same dict
    m.load_state_dict(P)
    return m.cuda(), cfg, P


def _run(m, inp):
    with torch.no_grad():
        y = m(x=inp["x"].cuda(), t=inp["t"].cuda(), context=[c.cuda() for c in inp["context"]],
              seq_len=inp["seq_len"], clip_fea=inp["clip_fea"].cuda(), y=inp["y"].cuda(),
              vocal_embeddings=inp["vocal"].cuda())
    torch.cuda.synchronize()
    return y.float().cpu()


def test_dit14_vs_reference_golden(model14):
    m, cfg, _ = model14
    y = _run(m, dit14_inputs(cfg))
    g = np.load(os.path.join(HERE, "golden", "dit14_small.npz"))["out"]
    e, c = rel(y, g), cos(y, g)
    print(f"14B DiT (dim 5120, 1 layer) vs reference: rel-L2 {e:.2e}, cosine {c:.6f}")
    assert y.shape == g.shape and e < 2e-2 and c > 0.9995


def test_dit14_wider_grid_vs_oracle(model14):
    """21 latent frames at 16x16 (64 tokens per frame, 1 344 tokens): several 64-key blocks per vocal frame"""
    from oracle import dit as odit
    m, cfg, P = model14
    inp = dit14_inputs(cfg)
    inp["x"] = synthetic.seeded_normal((1, 16, 21, 16, 16), 121).expand(3, -1, -1, -1, -1).contiguous()
    inp["y"] = synthetic.seeded_normal((3, 20, 21, 16, 16), 122)
    inp["seq_len"] = 21 * 8 * 8
    y = _run(m, inp)
    with torch.no_grad():
        ref = odit.forward(P, cfg, inp["x"], inp["t"], inp["context"], inp["seq_len"], inp["clip_fea"], inp["y"],
                           inp["vocal"], 81)
    e, c = rel(y, ref), cos(y, ref)
    print(f"14B DiT 1 344 tokens vs oracle: rel-L2 {e:.2e}, cosine {c:.6f}")
    assert e < 2e-2 and c > 0.9995


def test_dit14_requires_81_frame_windows(model14):
    m, cfg, _ = model14
    inp = dit14_inputs(cfg)
    with pytest.raises(ValueError):
        m(x=inp["x"].cuda(), t=inp["t"].cuda(), context=[c.cuda() for c in inp["context"]], seq_len=inp["seq_len"],
          clip_fea=inp["clip_fea"].cuda(), y=inp["y"].cuda(), vocal_embeddings=inp["vocal"].cuda(),
          video_sample_n_frames=17)


def test_pipeline_denoise_drives_14b(model14):
    """WanI2VTalkingInferenceLongPipeline.denoise on the 14B model (the reference's pipeline cannot call it,
    SURVEY.md App. A.9): 22 latent frames -> windows (0, 21), (6, 22) at overlap 15 (the second one shorter
    and padded), 2 steps (the blend runs at step 1), vs the oracle loop (oracle/pipeline.py) on the oracle
    14B forward"""
    import math

    from oracle import dit as odit
    from oracle import pipeline as opipe
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, audio_window, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    m, cfg, P = model14
    T, H, W, steps, overlap, clip_length = 22, 4, 4, 2, 15, 81
    lat0 = synthetic.seeded_normal((1, 16, T, H, W), 131).bfloat16()
    y = synthetic.seeded_normal((3, 20, 21, H, W), 132)  # the window conditioning (clip_length frames)
    audio = synthetic.seeded_normal((((T - 1) * 4 + 1) * 640,), 133, 0.1)
    inp = dit14_inputs(cfg)
    ctx = inp["context"]
    clip = inp["clip_fea"]
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(steps, device="cuda")
    pipe = WanI2VTalkingInferenceLongPipeline(transformer=m, scheduler=sched)
    fpb = (clip_length - 1) // 4 + 1
    feats = {}
    for (s, e, _) in window_schedule(T, fpb, overlap):
        a = synthetic.fake_wav2vec_features(audio[audio_window(s, e, T, 640, audio.shape[0])][None]).cuda()
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a])
    seq_len = math.ceil(W * H / 4 * fpb)
    with torch.no_grad():
        out = pipe.denoise(lat0.cuda(), y.cuda().bfloat16(), [c.cuda() for c in ctx], clip.cuda(), feats,
                           sched.timesteps, sched.sigmas, clip_length=clip_length, seq_len=seq_len, overlap=overlap,
                           text_guide_scale=3.0, audio_guide_scale=5.0)
    torch.cuda.synchronize()

    def dit(x, t, context, sl, yy, clip_fea, vocal, n):
        return odit.forward(P, cfg, x.float(), t, context, sl, clip_fea, yy.float(), vocal, n)

    with torch.no_grad():
        ref = opipe.denoise(dit, lat0.float(), y.bfloat16(), ctx, clip, audio,
                            lambda smp: synthetic.fake_wav2vec_features(smp[None]), num_inference_steps=steps,
                            clip_length=clip_length, num_frames=clip_length, height=H * 8, width=W * 8,
                            overlap=overlap, text_guide_scale=3.0, audio_guide_scale=5.0)
    e = rel(out.float(), ref)
    print(f"14B pipeline denoise (2 windows x 2 steps) vs oracle loop: rel-L2 {e:.2e}")
    assert e < 3e-2, e
