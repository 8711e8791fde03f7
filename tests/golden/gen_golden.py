"""Generate golden vectors by running the REFERENCE implementation (/root/reference, imported with
the diffusers stand-ins of _refstub.py) on CPU in fp32.  Run here only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

Inputs are regenerated from seeds (stableavatar_amd.synthetic) by the tests; the .npz files hold
outputs (and the few pipeline-internal inputs that need the reference's VAE encoder).  Weights come
from the name-keyed rule of stableavatar_amd.synthetic, so no weights are stored.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import _refstub  # noqa: E402

_refstub.install()

from stableavatar_amd import synthetic  # noqa: E402
from golden_cases import (DIT_SMALL, dit_inputs, VAE_SMALL, vae_latent, VAE_ENC_SMALL, vae_video, PIPE,  # noqa: E402
                          pipe_fixed_inputs)

torch.set_grad_enabled(False)


def load_synthetic(module, seed):
    sd = module.state_dict()
    shapes = {k: tuple(v.shape) for k, v in sd.items()}
    vals = synthetic.fill_state_dict(shapes, seed)
    module.load_state_dict(vals, strict=True)
    return module


def build_ref_dit(cfg):
    from wan.models.wan_fantasy_transformer3d_1B import WanTransformer3DFantasyModel
    m = WanTransformer3DFantasyModel(model_type="i2v", patch_size=(1, 2, 2), text_len=cfg["text_len"],
                                     in_dim=cfg["in_dim"], dim=cfg["dim"], ffn_dim=cfg["ffn_dim"],
                                     freq_dim=cfg["freq_dim"], text_dim=cfg["text_dim"], out_dim=cfg["out_dim"],
                                     num_heads=cfg["num_heads"], num_layers=cfg["num_layers"], qk_norm=True,
                                     cross_attn_norm=True, eps=1e-6)
    return load_synthetic(m.eval(), cfg["seed"])


def gen_dit():
    m = build_ref_dit(DIT_SMALL)
    out = {}
    for case in ("full", "short", "wide"):
        inp = dit_inputs(DIT_SMALL, case)
        y = m(x=inp["x"], t=inp["t"], context=inp["context"], seq_len=inp["seq_len"], clip_fea=inp["clip_fea"],
              y=inp["y"], vocal_embeddings=inp["vocal"], is_clip_level_modeling=False,
              video_sample_n_frames=inp["n_frames"])
        out[f"{case}_out"] = y.numpy()
        print(case, tuple(y.shape), float(y.abs().mean()))
    m.enable_riflex(k=6, L_test=66, L_test_scale=4.886)  # 1B:890-905
    inp = dit_inputs(DIT_SMALL, "full")
    y = m(x=inp["x"], t=inp["t"], context=inp["context"], seq_len=inp["seq_len"], clip_fea=inp["clip_fea"],
          y=inp["y"], vocal_embeddings=inp["vocal"], is_clip_level_modeling=False,
          video_sample_n_frames=inp["n_frames"])
    out["full_riflex_out"] = y.numpy()
    m.disable_riflex()
    # sub-module pins: vocal projector output for the full case
    inp = dit_inputs(DIT_SMALL, "full")
    np.savez_compressed(os.path.join(HERE, "dit_small.npz"), **out)


def build_ref_dit14(cfg):
    from wan.models.wan_fantasy_transformer3d_14B import WanTransformer3DFantasy14BModel
    m = WanTransformer3DFantasy14BModel(model_type="i2v", patch_size=(1, 2, 2), text_len=cfg["text_len"],
                                        in_dim=cfg["in_dim"], dim=cfg["dim"], ffn_dim=cfg["ffn_dim"],
                                        freq_dim=cfg["freq_dim"], text_dim=cfg["text_dim"], out_dim=cfg["out_dim"],
                                        num_heads=cfg["num_heads"], num_layers=cfg["num_layers"], qk_norm=True,
                                        cross_attn_norm=True, eps=1e-6)
    return load_synthetic(m.eval(), cfg["seed"])


def gen_dit14():
    """the 14B DiT at its full width (5120, 40 heads; vocal projector 5120 wide, 8 heads of 640) with
    DIT14_SMALL's reduced depth / ffn / text width, on the 21-latent-frame window its vocal path
    hard-codes (14B forward signature: no video_sample_n_frames)"""
    from golden_cases import DIT14_SMALL, dit14_inputs
    m = build_ref_dit14(DIT14_SMALL)
    inp = dit14_inputs(DIT14_SMALL)
    y = m(x=inp["x"], t=inp["t"], context=inp["context"], seq_len=inp["seq_len"], clip_fea=inp["clip_fea"],
          y=inp["y"], vocal_embeddings=inp["vocal"], is_clip_level_modeling=False)
    print("dit14", tuple(y.shape), float(y.abs().mean()))
    np.savez_compressed(os.path.join(HERE, "dit14_small.npz"), out=y.numpy())


def build_ref_vae(cfg):
    from wan.models.wan_vae import AutoencoderKLWan, _video_vae
    v = AutoencoderKLWan()
    v.model = _video_vae(z_dim=16, dim=cfg["dim"])
    return load_synthetic(v.eval(), cfg["seed"])


def gen_vae():
    out = {}
    for name, cfg in VAE_SMALL.items():
        v = build_ref_vae(cfg)
        z = vae_latent(cfg)
        y = v.decode(z).sample
        out[name] = y.numpy()
        print("vae", name, tuple(y.shape), float(y.abs().mean()))
    np.savez_compressed(os.path.join(HERE, "vae_small.npz"), **out)


def gen_vae_enc():
    """AutoencoderKLWan._encode (wan_vae.py:643-648): chunked 1, 4, 4.. encode with the feature cache;
    stored: cat(normalised mu, log_var) [1, 32, 1+(T-1)/4, H/8, W/8]."""
    out = {}
    for name, cfg in VAE_ENC_SMALL.items():
        v = build_ref_vae(cfg)
        x = vae_video(cfg)
        h = v._encode(x)
        mode = v.encode(x)[0].mode()
        assert torch.equal(mode, h[:, :16])
        out[name] = h.numpy()
        print("vae_enc", name, tuple(h.shape), float(h.abs().mean()))
    np.savez_compressed(os.path.join(HERE, "vae_enc_small.npz"), **out)


def gen_teacache():
    """Reference TeaCache over 10 forwards (t from the 10-step shift-5 schedule): outputs + pattern."""
    from golden_cases import TEACACHE, TEACACHE_STEPS
    from wan.models.cache_utils import get_teacache_coefficients
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    m = build_ref_dit(DIT_SMALL)
    sch = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sch.set_timesteps(TEACACHE_STEPS)
    ts = [float(t) for t in sch.timesteps]
    inp = dit_inputs(DIT_SMALL, "full")
    out = {"timesteps": np.array(ts, dtype=np.float32)}
    for name, (coef, thr) in TEACACHE.items():
        m.enable_teacache(coef if coef is not None else get_teacache_coefficients("wan2.1-fun-1.3b"),
                          TEACACHE_STEPS, thr, num_skip_start_steps=2, offload=False)
        outs, pat = [], []
        for t in ts:
            y = m(x=inp["x"], t=torch.full((3,), t), context=inp["context"], seq_len=inp["seq_len"],
                  clip_fea=inp["clip_fea"], y=inp["y"], vocal_embeddings=inp["vocal"], is_clip_level_modeling=False,
                  video_sample_n_frames=inp["n_frames"])
            outs.append(y.numpy())
            pat.append(int(m.teacache.should_calc))
        m.disable_teacache()
        out[name + "_out"] = np.stack(outs)
        out[name + "_calc"] = np.array(pat, dtype=np.int32)
        print("teacache", name, pat)
    np.savez_compressed(os.path.join(HERE, "teacache_small.npz"), **out)


class _Obj(types.SimpleNamespace):
    def __getitem__(self, i):
        return [self.last][i]


def gen_pipeline(P=PIPE, name="pipeline_small", scheme="uniform"):
    import time
    from wan.pipeline.wan_inference_long_pipeline import WanI2VTalkingInferenceLongPipeline
    from _refstub import FlowMatchEulerDiscreteScheduler

    t_start = time.time()
    dit = build_ref_dit(P["dit"])
    vae = build_ref_vae(P["vae"])
    fx = pipe_fixed_inputs(P)

    from golden_cases import fake_encoders, ref_image
    enc = fake_encoders(P, fx)

    calls = []
    orig = dit.forward

    def traced(**kw):
        calls.append({"F": kw["x"].shape[2], "t": float(kw["t"][0]), "seq_len": kw["seq_len"],
                      "n_audio": kw["vocal_embeddings"].shape[1]})
        if len(calls) == 1:
            calls[0]["y"] = kw["y"].clone()
        return orig(**kw)

    dit.forward = traced
    decoded = {}
    vdec = vae.decode

    def tdec(z, return_dict=True):
        decoded["latents"] = z.clone()
        return vdec(z, return_dict)

    vae.decode = tdec
    path = ref_image()
    pipe = WanI2VTalkingInferenceLongPipeline(vae=vae, transformer=dit,
                                              scheduler=FlowMatchEulerDiscreteScheduler(1000, shift=5.0), **enc)
    video = pipe("pos prompt", negative_prompt="", num_frames=P["clip_length"], height=P["height"],
                 width=P["width"], guidance_scale=6.0, num_inference_steps=P["steps"], latents=fx["latents"],
                 text_guide_scale=P["text_guide"], audio_guide_scale=P["audio_guide"],
                 vocal_input_values=fx["audio"].numpy(), fps=25, sr=16000, cond_file_path=path,
                 overlap_window_length=P["overlap"], clip_length=P["clip_length"],
                 overlapping_weight_scheme=scheme).videos
    out = {"video": video.numpy(), "latents": decoded["latents"].numpy(), "y": calls[0]["y"].numpy(),
           "win_F": np.array([c["F"] for c in calls]), "win_t": np.array([c["t"] for c in calls]),
           "win_seq_len": np.array([c["seq_len"] for c in calls]),
           "win_n_audio": np.array([c["n_audio"] for c in calls])}
    if name == "pipeline_c1":  # big video: keep a few decoded frames in fp16
        from golden_cases import PIPE_C1_VIDEO_FRAMES
        out["video"] = out["video"][:, :, list(PIPE_C1_VIDEO_FRAMES)].astype(np.float16)
        out["video_frames"] = np.array(PIPE_C1_VIDEO_FRAMES)
        out["y"] = out["y"][:1]  # the 3 CFG rows are identical (pipeline:700)
        out["ref_cpu_seconds"] = np.array(time.time() - t_start)
        out["ref_cpu_threads"] = np.array(torch.get_num_threads())
    print(name, "windows", [(c["F"], round(c["t"], 2), c["n_audio"]) for c in calls], tuple(video.shape),
          f"{time.time() - t_start:.1f}s")
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def gen_pipeline_c1():
    """BASELINE config 1 through the reference's own __call__: full 30-layer 1.3B DiT + full VAE at
    256x256, clip 17, 5 steps, 2 windows per step (golden_cases.PIPE_C1)."""
    from golden_cases import PIPE_C1
    gen_pipeline(PIPE_C1, "pipeline_c1")


def gen_pipeline_log():
    """overlapping_weight_scheme="log" (pipeline:761-766) through the reference's __call__: PIPE with overlap 3
    (at overlap 2 the log and uniform ramps are both [0, 1]), windows (0,5),(2,6) per step"""
    from golden_cases import PIPE_LOG
    gen_pipeline(PIPE_LOG, "pipeline_log", scheme="log")


def gen_pipeline_steps():
    """the reference __call__ over 5 / 10 / 50 steps (golden_cases.PIPE_STEPS): pipeline_s05/s10/s50.npz"""
    from golden_cases import PIPE_STEPS
    for n, P in PIPE_STEPS.items():
        gen_pipeline(P, f"pipeline_s{n:02d}")


def gen_keys():
    """state_dict key -> shape of the reference modules the checkpoint loaders fill: the 1.3B DiT
    (WanTransformer3DFantasyModel at the wan_civitai.yaml / Wan2.1-1.3B dims), the full VAE
    (AutoencoderKLWan, keys as in Wan2.1_VAE.pth, i.e. without the "model." prefix its loader adds)."""
    import json
    from golden_cases import DIT_FULL
    from wan.models.wan_fantasy_transformer3d_1B import WanTransformer3DFantasyModel
    from wan.models.wan_vae import AutoencoderKLWan
    cfg = DIT_FULL
    with torch.device("meta"):
        m = WanTransformer3DFantasyModel(model_type="i2v", patch_size=(1, 2, 2), text_len=cfg["text_len"],
                                         in_dim=cfg["in_dim"], dim=cfg["dim"], ffn_dim=cfg["ffn_dim"],
                                         freq_dim=cfg["freq_dim"], text_dim=cfg["text_dim"], out_dim=cfg["out_dim"],
                                         num_heads=cfg["num_heads"], num_layers=cfg["num_layers"], qk_norm=True,
                                         cross_attn_norm=True, eps=1e-6)
        v = AutoencoderKLWan()
    from golden_cases import CLIP_SMALL, T5_SMALL
    from wan.models.wan_text_encoder import WanT5EncoderModel
    with torch.device("meta"):
        t5 = WanT5EncoderModel(vocab=256384, dim=4096, dim_attn=4096, dim_ffn=10240, num_heads=64, num_layers=24,
                               num_buckets=32, shared_pos=False, dropout=0.0)  # wan_civitai.yaml:14-26
    clip = build_ref_clip_visual(dict(CLIP_SMALL, dim=1280, num_heads=16, num_layers=32))  # ViT-H/14
    from wan.models.wan_fantasy_transformer3d_14B import WanTransformer3DFantasy14BModel
    with torch.device("meta"):  # wan_civitai 14B widths (dim 5120, 40 heads, 40 layers, ffn 13824)
        m14 = WanTransformer3DFantasy14BModel(model_type="i2v", patch_size=(1, 2, 2), text_len=512, in_dim=36,
                                              dim=5120, ffn_dim=13824, freq_dim=256, text_dim=4096, out_dim=16,
                                              num_heads=40, num_layers=40, qk_norm=True, cross_attn_norm=True,
                                              eps=1e-6)
    out = {"dit_1_3b": {k: list(t.shape) for k, t in m.state_dict().items()},
           "dit_14b": {k: list(t.shape) for k, t in m14.state_dict().items()},
           "vae": {k[len("model."):]: list(t.shape) for k, t in v.state_dict().items()},
           "umt5_xxl": {k: list(t.shape) for k, t in t5.state_dict().items()},
           "clip_visual_vit_h14": {"model.visual." + k: list(t.shape) for k, t in clip.state_dict().items()}}
    with open(os.path.join(HERE, "ref_keys.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("keys", len(out["dit_1_3b"]), len(out["vae"]))


def build_ref_t5(cfg):
    from wan.models.wan_text_encoder import WanT5EncoderModel
    m = WanT5EncoderModel(vocab=cfg["vocab"], dim=cfg["dim"], dim_attn=cfg["dim_attn"], dim_ffn=cfg["dim_ffn"],
                          num_heads=cfg["num_heads"], num_layers=cfg["num_layers"], num_buckets=cfg["num_buckets"],
                          shared_pos=cfg["shared_pos"], dropout=0.0)
    return load_synthetic(m.eval(), cfg["seed"])


def build_ref_clip_visual(cfg):
    from wan.models.wan_image_encoder import VisionTransformer
    v = VisionTransformer(image_size=cfg["image_size"], patch_size=cfg["patch"], dim=cfg["dim"], mlp_ratio=4,
                          out_dim=1024, num_heads=cfg["num_heads"], num_layers=cfg["num_layers"], pool_type="token",
                          pre_norm=True, post_norm=False, activation="gelu")
    wrap = torch.nn.Module()
    wrap.model = torch.nn.Module()
    wrap.model.visual = v  # CLIPModel's key prefix: model.visual.*
    load_synthetic(wrap.eval(), cfg["seed"])
    return v


def gen_encoders():
    """umT5 (WanT5EncoderModel.forward) and the CLIP visual tower as CLIPModel.forward runs it
    (F.interpolate bicubic to 224, *0.5+0.5, Normalize(mean, std) -- the torchvision Normalize is written
    out here because torchvision is stubbed -- then visual(x, use_31_block=True)), at reduced sizes."""
    import torch.nn.functional as F
    from golden_cases import CLIP_SMALL, T5_SMALL, clip_image, t5_inputs
    from golden_cases import T5_FULL_WIDTH
    out = {}
    m = build_ref_t5(T5_SMALL)
    ids, mask = t5_inputs(T5_SMALL)
    out["t5_out"] = m(ids, attention_mask=mask)[0].numpy()
    # the reference loads umT5 with torch_dtype=bf16 (inference.py:464-469): its bf16 run is the deployed
    # semantics (unscaled T5 logits rounded to bf16 move the output by several %); both are stored
    out["t5_out_bf16"] = m.to(torch.bfloat16)(ids, attention_mask=mask)[0].float().numpy()
    for L, valid in ((512, T5_FULL_WIDTH["valid"]), (100, 100)):
        c = dict(T5_FULL_WIDTH, text_len=L, valid=valid)
        mf = build_ref_t5(c)
        ids, mask = t5_inputs(c)
        out[f"t5_full_L{L}"] = mf(ids, attention_mask=mask)[0][:, :valid].numpy().astype(np.float16)
        out[f"t5_full_L{L}_bf16"] = mf.to(torch.bfloat16)(ids, attention_mask=mask)[0][:, :valid].float().numpy().astype(np.float16)
        del mf
    v = build_ref_clip_visual(CLIP_SMALL)
    img = clip_image(CLIP_SMALL)
    x = F.interpolate(img.transpose(0, 1), size=(224, 224), mode="bicubic", align_corners=False)
    x = x.mul_(0.5).add_(0.5)
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073]).view(1, 3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711]).view(1, 3, 1, 1)
    out["clip_pre"] = ((x - mean) / std).numpy()
    out["clip_out"] = v((x - mean) / std, use_31_block=True).numpy()
    print("encoders", out["t5_out"].shape, out["clip_out"].shape)
    np.savez_compressed(os.path.join(HERE, "encoders_small.npz"), **out)


def gen_tables():
    from wan.models.vocal_projector_fantasy import split_audio_sequence, split_tensor_with_padding
    from _refstub import FlowMatchEulerDiscreteScheduler
    out = {}
    for L, nf in ((167, 81), (161, 81), (39, 17), (23, 17), (100, 33), (400, 81)):
        r = split_audio_sequence(L, num_frames=nf)
        x = torch.arange(L, dtype=torch.float32).view(1, L, 1) + 1.0
        sub, lens = split_tensor_with_padding(x, r, expand_length=4)
        out[f"split_{L}_{nf}_ranges"] = np.array(r)
        out[f"split_{L}_{nf}_rows"] = (sub[0, :, :, 0].numpy() - 1.0).astype(np.int64)  # -1 marks zero rows
        out[f"split_{L}_{nf}_lens"] = lens.numpy()
    from wan.models.wan_fantasy_transformer3d_1B import get_1d_rotary_pos_embed_riflex
    fr = get_1d_rotary_pos_embed_riflex(1024, 128 - 4 * (128 // 6), use_real=False, k=6, L_test=66,
                                        L_test_scale=4.886)
    out["riflex_frame_cos"] = fr.real.float().numpy()
    out["riflex_frame_sin"] = fr.imag.float().numpy()
    s = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    s.set_timesteps(50)
    out["sched50_timesteps"] = s.timesteps.numpy()
    out["sched50_sigmas"] = s.sigmas.numpy()
    np.savez_compressed(os.path.join(HERE, "tables.npz"), **out)


if __name__ == "__main__":
    which = sys.argv[1:] or ["tables", "dit", "vae", "vae_enc", "teacache", "pipeline"]
    for w in which:
        globals()["gen_" + w]()
