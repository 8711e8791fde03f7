"""The reference's command line (inference.py flags :238-409, main :412-578) end to end on the HIP modules,
with a tiny synthetic model tree written in the layout the reference reads: wan_civitai.yaml-style config,
DiT config.json + safetensors at the root (transformer_subpath ./), the StableAvatar transformer3d-square.pt
overlay ({"state_dict": ...}), Wan2.1_VAE.pth, umT5 .pth, the open-CLIP .pth (visual + a text-tower key that
is ignored), a tokenizer directory and a wav2vec2 directory (transformers save_pretrained), a reference PNG
and a 16 kHz WAV.  Checks that the command line reaches the pipeline with the reference's call arguments
(inference.py:544-568), that the written video is that call's output, and that the call is deterministic (the same
pipeline re-run with the captured arguments gives the same bytes)."""
import json
import os

import numpy as np
import pytest
import torch

from stableavatar_amd import synthetic

pytestmark = pytest.mark.gpu

T5 = dict(vocab=300, dim=512, dim_attn=512, dim_ffn=1024, num_heads=8, num_layers=2, num_buckets=32, shared_pos=False)
DIT = dict(model_type="i2v", dim=1536, ffn_dim=256, freq_dim=256, text_dim=512, in_dim=36, out_dim=16, num_heads=12,
           num_layers=2, text_len=64, eps=1e-6)


def _write_tree(root):
    import yaml
    from safetensors.torch import save_file
    from scipy.io import wavfile
    from tokenizers import Tokenizer, models, pre_tokenizers, processors
    from transformers import (PreTrainedTokenizerFast, Wav2Vec2Config, Wav2Vec2CTCTokenizer,
                              Wav2Vec2FeatureExtractor, Wav2Vec2Model, Wav2Vec2Processor)

    from stableavatar_amd.encoders import clip_param_shapes, t5_param_shapes
    from stableavatar_amd.transformer import param_shapes
    from stableavatar_amd.vae import encoder_param_shapes
    from stableavatar_amd.vae import param_shapes as vae_shapes
    cfg = {"format": "civitai", "pipeline": "Wan",
           "transformer_additional_kwargs": {"transformer_subpath": "./",
                                             "dict_mapping": {"in_dim": "in_channels", "dim": "hidden_size"}},
           "vae_kwargs": {"vae_subpath": "Wan2.1_VAE.pth", "temporal_compression_ratio": 4,
                          "spatial_compression_ratio": 8, "dim": 32},
           "text_encoder_kwargs": dict(T5, text_encoder_subpath="t5.pth", tokenizer_subpath="tokenizer",
                                       text_length=512, dropout=0.0),
           "scheduler_kwargs": {"scheduler_subpath": None, "num_train_timesteps": 1000, "shift": 5.0,
                                "use_dynamic_shifting": False, "base_shift": 0.5, "max_shift": 1.15,
                                "base_image_seq_len": 256, "max_image_seq_len": 4096},
           "image_encoder_kwargs": {"image_encoder_subpath": "clip.pth", "num_layers": 2}}
    with open(os.path.join(root, "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    # DiT: config.json + safetensors at the root, then the StableAvatar overlay
    with open(os.path.join(root, "config.json"), "w") as f:
        json.dump({k: v for k, v in DIT.items()}, f)
    sd = synthetic.fill_state_dict(param_shapes(DIT), 81)
    save_file(sd, os.path.join(root, "diffusion_pytorch_model.safetensors"))
    overlay = synthetic.fill_state_dict({k: v for k, v in param_shapes(DIT).items() if "vocal" in k}, 82)
    torch.save({"state_dict": overlay}, os.path.join(root, "transformer3d-square.pt"))
    vsd = synthetic.fill_state_dict(dict(vae_shapes(dim=32), **encoder_param_shapes(dim=32)), 83)
    torch.save({k[len("model."):]: v for k, v in vsd.items()}, os.path.join(root, "Wan2.1_VAE.pth"))
    torch.save(synthetic.fill_state_dict(t5_param_shapes(**T5), 84), os.path.join(root, "t5.pth"))
    csd = synthetic.fill_state_dict(clip_param_shapes(num_layers=2), 85)
    csd = {k[len("model."):]: v for k, v in csd.items()}
    csd["textual.token_embedding.weight"] = torch.zeros(4, 8)  # text tower: ignored by the visual path
    torch.save(csd, os.path.join(root, "clip.pth"))
    # tokenizer: word-level over a small vocabulary, </s> appended (umT5 adds eos)
    words = ["<pad>", "</s>", "<unk>"] + [f"w{i}" for i in range(200)] + ["a", "woman", "is", "singing"]
    tok = Tokenizer(models.WordLevel({w: i for i, w in enumerate(words)}, unk_token="<unk>"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.post_processor = processors.TemplateProcessing(single="$A </s>", special_tokens=[("</s>", 1)])
    tdir = os.path.join(root, "tokenizer")
    PreTrainedTokenizerFast(tokenizer_object=tok, pad_token="<pad>", eos_token="</s>", unk_token="<unk>",
                            model_max_length=512).save_pretrained(tdir)
    # wav2vec2: 768-wide features (the vocal projector's input), one transformer layer
    wdir = os.path.join(root, "wav2vec")
    torch.manual_seed(0)
    Wav2Vec2Model(Wav2Vec2Config(hidden_size=768, num_hidden_layers=1, num_attention_heads=12,
                                 intermediate_size=256)).save_pretrained(wdir)
    with open(os.path.join(root, "vocab.json"), "w") as f:
        json.dump({"<pad>": 0, "<s>": 1, "</s>": 2, "<unk>": 3, "|": 4, "A": 5}, f)
    Wav2Vec2Processor(feature_extractor=Wav2Vec2FeatureExtractor(), tokenizer=Wav2Vec2CTCTokenizer(
        os.path.join(root, "vocab.json"))).save_pretrained(wdir)
    # inputs: 24 video frames of 16 kHz audio (T_lat 6 -> two windows of clip 17), a reference image
    wavfile.write(os.path.join(root, "audio.wav"), 16000,
                  (0.1 * np.random.default_rng(0).standard_normal(24 * 640)).astype(np.float32))
    from PIL import Image
    Image.fromarray((np.random.default_rng(1).random((80, 72, 3)) * 255).astype(np.uint8)).save(
        os.path.join(root, "reference.png"))


@pytest.mark.timeout(600)
def test_inference_cli_end_to_end(tmp_path, monkeypatch):
    from stableavatar_amd import inference
    from stableavatar_amd.inference import main
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    root = str(tmp_path)
    _write_tree(root)
    out_dir = os.path.join(root, "output")
    calls = []
    orig = WanI2VTalkingInferenceLongPipeline.__call__

    def spy(self, *a, **kw):
        out = orig(self, *a, **kw)
        calls.append((self, a, kw, out.videos.detach().float().cpu().clone()))
        return out

    monkeypatch.setattr(WanI2VTalkingInferenceLongPipeline, "__call__", spy)
    main(["--config_path", os.path.join(root, "config.yaml"), "--pretrained_model_name_or_path", root,
          "--transformer_path", os.path.join(root, "transformer3d-square.pt"),
          "--pretrained_wav2vec_path", os.path.join(root, "wav2vec"),
          "--validation_reference_path", os.path.join(root, "reference.png"),
          "--validation_driven_audio_path", os.path.join(root, "audio.wav"), "--output_dir", out_dir,
          "--validation_prompts", "a woman is singing", "--seed", "42", "--ulysses_degree", "1", "--ring_degree", "1",
          "--motion_frame", "25", "--sample_steps", "2", "--width", "64", "--height", "64",
          "--overlap_window_length", "2", "--clip_sample_n_frames", "17", "--GPU_memory_mode", "model_full_load",
          "--sample_text_guide_scale", "3.0", "--sample_audio_guide_scale", "5.0"])
    # the reference's call (inference.py:544-568): the CLI's flags mapped to the pipeline arguments
    assert len(calls) == 1
    pipe, a, kw, video = calls[0]
    assert a[0] == "a woman is singing"
    assert kw["negative_prompt"] == inference.NEGATIVE_PROMPT
    want = dict(num_frames=17, height=64, width=64, guidance_scale=6.0, num_inference_steps=2, text_guide_scale=3.0,
                audio_guide_scale=5.0, motion_frame=25, fps=25, sr=16000, seed=42, overlap_window_length=2,
                clip_length=17, cond_file_path=os.path.join(root, "reference.png"))
    for k_, v_ in want.items():
        assert kw[k_] == v_, (k_, kw[k_], v_)
    assert kw["vocal_input_values"].shape == (24 * 640,)  # 16 kHz audio as written (no resampling needed)
    if os.path.exists(os.path.join(out_dir, "video.npy")):
        v = np.load(os.path.join(out_dir, "video.npy"))
        assert v.shape == (1, 3, 21, 64, 64) and np.isfinite(v).all() and v.min() >= 0 and v.max() <= 1
        assert len(os.listdir(os.path.join(out_dir, "animated_images"))) == 21
        assert np.array_equal(v, video.numpy()), "the saved video is the pipeline call's output"
    else:
        assert os.path.exists(os.path.join(out_dir, "video_without_audio.mp4"))
    # deterministic: the same pipeline, the captured arguments and a fresh generator at the same seed
    kw2 = dict(kw, generator=torch.Generator(device=kw["generator"].device).manual_seed(42))
    with torch.no_grad():
        again = orig(pipe, *a, **kw2).videos.float().cpu()
    assert torch.equal(again, video)
