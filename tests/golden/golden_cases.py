"""Shared definitions of the golden cases: configs + seeded input builders.  Used by
gen_golden.py (with the reference, here only) and by the tests (oracle / HIP path)."""
import math
import types

import numpy as np
import torch

from stableavatar_amd import synthetic

# dim must be 1536: the vocal projector hard-codes audio_proj_dim=1536 (1B:872)
DIT_SMALL = dict(model_type="i2v", dim=1536, ffn_dim=256, freq_dim=256, text_dim=64, in_dim=36, out_dim=16,
                 num_heads=12, num_layers=2, text_len=32, eps=1e-6, seed=11)


def dit_inputs(cfg, case="full"):
    """CFG batch of 3 at 64x64 video -> 8x8 latent, clip 17 (5 latent frames, seq_len 80).
    'short' is the last-window case: 3 latent frames padded to the 5-frame seq_len; 'wide' a
    non-square 64x96 video (8x12 latent, 24 tokens per frame, seq_len 120)."""
    B, H, W = 3, 8, (12 if case == "wide" else 8)
    Fw = 3 if case == "short" else 5
    n_frames = 17
    seq_len = ((n_frames - 1) // 4 + 1) * (H // 2) * (W // 2)
    lat = synthetic.seeded_normal((1, 16, Fw, H, W), 101)
    x = torch.cat([lat] * 3)
    y = synthetic.seeded_normal((B, 20, 5, H, W), 102)[:, :, :Fw].contiguous()
    neg = synthetic.seeded_normal((20, cfg["text_dim"]), 103)
    pos = synthetic.seeded_normal((25, cfg["text_dim"]), 104)
    clip = synthetic.seeded_normal((1, 257, 1280), 105).expand(3, -1, -1).contiguous()
    a = synthetic.seeded_normal((1, 39, 768), 106)
    vocal = torch.cat([torch.zeros_like(a), a, a])
    t = torch.full((3,), 937.5)
    return dict(x=x, y=y, context=[neg, neg, pos], clip_fea=clip, vocal=vocal, t=t, seq_len=seq_len,
                n_frames=n_frames)


# the 14B DiT at full width (dim 5120, 40 heads of 128; vocal projector 5120 wide, 8 heads of 640) with one
# layer, ffn 256 and text_dim 64 to keep the golden small; its vocal path hard-codes 21 latent frames
DIT14_SMALL = dict(model_type="i2v", dim=5120, ffn_dim=256, freq_dim=256, text_dim=64, in_dim=36, out_dim=16,
                   num_heads=40, num_layers=1, text_len=32, eps=1e-6, seed=13)


def dit14_inputs(cfg):
    """CFG batch of 3 on one 81-frame window: 21 latent frames at 4x4 (2x2 tokens per frame, seq_len 84),
    161 wav2vec tokens (81 frames of 16 kHz audio); the 14B projector runs on all three audio rows."""
    B, F, H, W = 3, 21, 4, 4
    lat = synthetic.seeded_normal((1, 16, F, H, W), 111)
    a = synthetic.seeded_normal((1, 161, 768), 116)
    return dict(x=torch.cat([lat] * 3), y=synthetic.seeded_normal((B, 20, F, H, W), 112),
                context=[synthetic.seeded_normal((20, cfg["text_dim"]), 113)] * 2
                + [synthetic.seeded_normal((25, cfg["text_dim"]), 114)],
                clip_fea=synthetic.seeded_normal((1, 257, 1280), 115).expand(3, -1, -1).contiguous(),
                vocal=torch.cat([torch.zeros_like(a), a, a]), t=torch.full((3,), 937.5), seq_len=F * (H // 2) * (W // 2))


VAE_SMALL = {"dim32_T3_8x8": dict(dim=32, seed=21, T=3, h=8, w=8),
             "dim96_T2_4x4": dict(dim=96, seed=22, T=2, h=4, w=4),
             "dim32_T1_6x4": dict(dim=32, seed=26, T=1, h=6, w=4)}  # one latent frame, non-square


VAE_ENC_SMALL = {"dim32_T9_32x32": dict(dim=32, seed=21, T=9, H=32, W=32),
                 "dim96_T5_16x16": dict(dim=96, seed=22, T=5, H=16, W=16),
                 "dim32_T1_24x16": dict(dim=32, seed=25, T=1, H=24, W=16)}  # a single image, non-square


def vae_video(cfg):
    """Encoder input: [1, 3, T, H, W] video, N(0, 0.5^2) clamped to [-1, 1] like pixel values."""
    return (0.5 * synthetic.seeded_normal((1, 3, cfg["T"], cfg["H"], cfg["W"]), 300 + cfg["seed"])).clamp(-1, 1)


def vae_latent(cfg):
    return synthetic.seeded_normal((1, 16, cfg["T"], cfg["h"], cfg["w"]), 200 + cfg["seed"])


PIPE = dict(dit=dict(DIT_SMALL, num_layers=1, seed=31), vae=dict(dim=32, seed=32), height=64, width=64,
            clip_length=17, steps=3, overlap=2, text_guide=3.0, audio_guide=5.0, neg_len=12, pos_len=9,
            audio_frames=24)


# the "log" overlap blend (pipeline:761-766) needs overlap >= 3 to differ from the uniform ramp
PIPE_LOG = dict(PIPE, overlap=3)

# SURVEY.md §8(d)'s end-to-end contract at the reference's real step count: the reference __call__
# (wan_inference_long_pipeline.py:540-806) over 5 / 10 / 50 sampling steps of its own schedule, 2-layer
# dim-1536 DiT, 2 windows per step, injected noise -> the bf16 drift's growth with the step count
PIPE_STEPS = {n: dict(PIPE, dit=dict(DIT_SMALL, seed=71), vae=dict(dim=32, seed=72), steps=n) for n in (5, 10, 50)}


# BASELINE config 1: the full Wan-1.3B StableAvatar DiT (30 layers, dim 1536, ffn 8960,
# text_dim 4096) and the full-width VAE (dim 96) at 256x256, clip 17 (5 latent frames), 5 sampling steps,
# overlap 2, 24 video frames of audio -> T_lat 6 -> windows (0,5),(3,6) per step
DIT_FULL = dict(model_type="i2v", dim=1536, ffn_dim=8960, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
                num_heads=12, num_layers=30, text_len=512, eps=1e-6)
PIPE_C1 = dict(dit=dict(DIT_FULL, seed=41), vae=dict(dim=96, seed=42), height=256, width=256, clip_length=17,
               steps=5, overlap=2, text_guide=3.0, audio_guide=5.0, neg_len=24, pos_len=31, audio_frames=24)
PIPE_C1_VIDEO_FRAMES = (0, 4, 9, 16, 20)  # decoded frames stored in the golden (fp16)


def pipe_fixed_inputs(P):
    """Seeded inputs of the pipeline golden: 24 video frames of audio @16 kHz -> T_lat 6 -> two
    windows (0,5),(3,6) per step (avoids the reference's single-window hang, App. A.1)."""
    n = P["audio_frames"] * 640
    T = (P["audio_frames"] - 1) // 4 + 1
    return dict(audio=synthetic.seeded_normal((n,), 300, 0.1),
                latents=synthetic.seeded_normal((1, 16, T, P["height"] // 8, P["width"] // 8), 301),
                neg_embeds=synthetic.seeded_normal((P["neg_len"], P["dit"]["text_dim"]), 302),
                pos_embeds=synthetic.seeded_normal((P["pos_len"], P["dit"]["text_dim"]), 303),
                clip=synthetic.seeded_normal((1, 257, 1280), 304))


# TeaCache (wan/models/cache_utils.py, 1B:1021-1103): 10 forwards of DIT_SMALL's "full" inputs over a
# 10-step flow schedule; (coefficients, rel_l1_thresh) per case, num_skip_start_steps 2, no offload
TEACACHE = {"identity_thr1.0": ([1.0, 0.0], 1.0), "identity_thr2.5": ([1.0, 0.0], 2.5),
            "wan13b_thr0.1": (None, 0.1)}
TEACACHE_STEPS = 10


# ---- stand-ins for the once-per-call encoders the pipeline's __call__ drives (tokenizer, umT5, CLIP,
# wav2vec2 processor + model): seeded tensors of the right shapes, shared by gen_golden.py (reference
# pipeline) and the GPU __call__ tests (drop-in pipeline), so both see identical encoder outputs
def fake_encoders(P, fx):
    class Tok:
        def __call__(self, prompt, padding=None, max_length=None, truncation=None, add_special_tokens=None,
                     return_tensors=None):
            n = max_length or 8
            lens = [P["neg_len"] if p == "" else P["pos_len"] for p in prompt]
            ids = torch.ones(len(prompt), n, dtype=torch.long)
            mask = torch.zeros(len(prompt), n, dtype=torch.long)
            for i, ln in enumerate(lens):
                mask[i, :ln] = 1
            return types.SimpleNamespace(input_ids=ids, attention_mask=mask)

        def batch_decode(self, *a, **k):
            return []

    class T5(torch.nn.Module):
        dtype = torch.float32

        def forward(self, ids, attention_mask=None):
            ln = int(attention_mask.sum())
            e = fx["pos_embeds"] if ln == P["pos_len"] else fx["neg_embeds"]
            full = torch.zeros(1, ids.shape[1], e.shape[1], device=ids.device)
            full[0, :ln] = e.to(ids.device)
            return (full,)

    class Clip(torch.nn.Module):
        def forward(self, imgs):
            return fx["clip"].clone().to(imgs[0].device)

    class Proc:
        def __call__(self, samples, sampling_rate=None, return_tensors=None):
            return types.SimpleNamespace(input_values=torch.as_tensor(np.asarray(samples), dtype=torch.float32)[None])

    class W2V(torch.nn.Module):
        def forward(self, x):
            return types.SimpleNamespace(last_hidden_state=synthetic.fake_wav2vec_features(x))

    return dict(tokenizer=Tok(), text_encoder=T5(), clip_image_encoder=Clip(), wav2vec_processor=Proc(),
                wav2vec=W2V())


def ref_image(path="/tmp/_sa_golden_ref.png"):
    """the reference frame of the pipeline goldens (48x40 RGB noise, resized by the pipeline)"""
    from PIL import Image
    img = Image.fromarray((np.random.default_rng(1).random((48, 40, 3)) * 255).astype(np.uint8))
    img.save(path)
    return path


# once-per-call encoders, reduced sizes for the reference goldens: umT5 with its
# per-block relative position embedding (shared_pos False as wan_civitai.yaml:14-26) and 64-wide heads; the
# CLIP ViT visual tower with 80-wide heads (ViT-H/14: 1280 / 16) on a 224 image (257 tokens)
T5_SMALL = dict(vocab=1000, dim=512, dim_attn=512, dim_ffn=1024, num_heads=8, num_layers=2, num_buckets=32,
                shared_pos=False, seed=61, text_len=512, valid=37)
T5_FULL_WIDTH = dict(T5_SMALL, dim=4096, dim_attn=4096, dim_ffn=10240, num_heads=64, seed=62, valid=53)
CLIP_SMALL = dict(dim=320, num_heads=4, num_layers=3, patch=14, image_size=224, seed=63, img_hw=(512, 448))
CLIP_FULL_WIDTH = dict(CLIP_SMALL, dim=1280, num_heads=16, seed=64)


def t5_inputs(cfg):
    ids = torch.from_numpy(np.random.default_rng(cfg["seed"]).integers(2, cfg["vocab"], size=(1, cfg["text_len"])))
    mask = torch.zeros(1, cfg["text_len"], dtype=torch.long)
    mask[:, :cfg["valid"]] = 1
    return ids.masked_fill(mask == 0, 0), mask


def clip_image(cfg):
    """the reference frame as the pipeline hands it to CLIP: [C, 1, H, W] in [-1, 1]"""
    H, W = cfg["img_hw"]
    return synthetic.seeded_normal((3, 1, H, W), 700 + cfg["seed"], 0.5).clamp(-1, 1)


# The examples/case-1 windowed shape at full size (BASELINE config 2's long-clip form): 512x512,
# T_lat 42 (165 video frames), 81-frame windows (21 latent frames) at overlap 15 -> 5 windows per step, with a
# 1-layer full-width DiT, 2 sampling steps of the 50-step schedule (the blend and the scatter run at full size in
# step 2).  The expected latents come from oracle/pipeline.py's loop on the CPU (gen_case1_fullsize.py).
CASE1_FULL = dict(dit=dict(DIT_FULL, num_layers=1, seed=61), T=42, clip_length=81, overlap=15, size=512,
                  steps=50, run_steps=2, text_guide=3.0, audio_guide=5.0)


def case1_fullsize_inputs(C=CASE1_FULL):
    T, h = C["T"], C["size"] // 8
    fpb = (C["clip_length"] - 1) // 4 + 1
    return dict(latents=synthetic.seeded_normal((1, 16, T, h, h), 601),
                y=synthetic.seeded_normal((3, 20, fpb, h, h), 602),
                context=[synthetic.seeded_normal((24, 4096), 603)] * 2 + [synthetic.seeded_normal((31, 4096), 604)],
                clip=synthetic.seeded_normal((1, 257, 1280), 605).expand(3, -1, -1).contiguous(),
                audio=synthetic.seeded_normal(((1 + 4 * (T - 1)) * 640 + 320,), 606, 0.1))
