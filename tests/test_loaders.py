"""Checkpoint loaders of the drop-in modules (CPU): the same files and keys the reference reads.

* WanTransformer3DFantasyModel.from_pretrained (wan_fantasy_transformer3d_1B.py:1210-1339): config.json +
  diffusion_pytorch_model.safetensors / sharded *.safetensors / .bin, `dict_mapping`, forced patch / norms,
  patch_embedding widening (zero-filled extra input channels), shape-mismatched keys skipped;
* the StableAvatar weights on top (inference.py:485-490): torch.load of transformer3d-square.pt, a flat
  or {"state_dict": ...} nested dict, load_state_dict(strict=False);
* AutoencoderKLWan.from_pretrained (wan_vae.py:683-704): a Wan2.1_VAE.pth / .safetensors whose keys get
  the "model." prefix.
Key names and shapes are pinned to the reference modules' own state_dicts (tests/golden/ref_keys.json,
written by gen_golden.py from /root/reference)."""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from stableavatar_amd import synthetic
from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes
from stableavatar_amd.vae import param_shapes as vae_param_shapes

HERE = os.path.dirname(os.path.abspath(__file__))
SMALL = dict(model_type="i2v", dim=1536, ffn_dim=256, freq_dim=256, text_dim=64, in_dim=36, out_dim=16,
             num_heads=12, num_layers=2, text_len=32, eps=1e-6)
# the yaml's transformer_additional_kwargs (deepspeed_config/wan2.1/wan_civitai.yaml:5-7)
ADD_KW = {"transformer_subpath": "./", "dict_mapping": {"in_dim": "in_channels", "dim": "hidden_size"}}


def _ref_keys():
    with open(os.path.join(HERE, "golden", "ref_keys.json")) as f:
        return json.load(f)


def test_dit_keys_match_reference_1_3b():
    """param_shapes(1.3B) == the reference module's state_dict keys and shapes (1 143 keys, App. C)."""
    ref = _ref_keys()["dit_1_3b"]
    cfg = dict(SMALL, ffn_dim=8960, text_dim=4096, num_layers=30, text_len=512)
    ours = {k: list(v) for k, v in param_shapes(cfg).items()}
    assert len(ours) == len(ref) == 1143
    assert ours == ref


def test_vae_keys_match_reference():
    ref = _ref_keys()["vae"]
    ours = {k[len("model."):]: list(v) for k, v in dict(vae_param_shapes(), **encoder_param_shapes()).items()}
    assert ours == ref


def _config_json(path, cfg):
    conf = {"_class_name": "WanModel", "_diffusers_version": "0.30.0", "dim": cfg["dim"], "eps": cfg["eps"],
            "ffn_dim": cfg["ffn_dim"], "freq_dim": cfg["freq_dim"], "in_dim": cfg["in_dim"],
            "model_type": cfg["model_type"], "num_heads": cfg["num_heads"], "num_layers": cfg["num_layers"],
            "out_dim": cfg["out_dim"], "text_len": cfg["text_len"], "text_dim": cfg["text_dim"]}
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(conf, f)


def _same(model, sd):
    own = model.state_dict()
    for k, v in sd.items():
        assert torch.equal(own[k].float(), v.float()), k


@pytest.mark.parametrize("layout", ["single", "sharded", "bin"])
def test_dit_from_pretrained(tmp_path, layout):
    sd = synthetic.fill_state_dict(param_shapes(SMALL), 5)
    _config_json(tmp_path, SMALL)
    if layout == "single":
        save_file(sd, str(tmp_path / "diffusion_pytorch_model.safetensors"))
    elif layout == "sharded":
        keys = sorted(sd)
        save_file({k: sd[k] for k in keys[::2]}, str(tmp_path / "diffusion_pytorch_model-00001-of-00002.safetensors"))
        save_file({k: sd[k] for k in keys[1::2]}, str(tmp_path / "diffusion_pytorch_model-00002-of-00002.safetensors"))
    else:
        torch.save(sd, str(tmp_path / "diffusion_pytorch_model.bin"))
    m = WanTransformer3DFantasyModel.from_pretrained(str(tmp_path), transformer_additional_kwargs=dict(ADD_KW),
                                                     torch_dtype=torch.float32)
    assert m.num_layers == 2 and m.dim == 1536 and m.in_dim == 36
    _same(m, sd)
    mb = WanTransformer3DFantasyModel.from_pretrained(str(tmp_path), transformer_additional_kwargs=dict(ADD_KW))
    assert all(p.dtype == torch.bfloat16 for p in mb.parameters())  # torch_dtype default (1B:1338)


def test_dit_from_pretrained_subfolder_and_widening(tmp_path):
    """A 16-channel base checkpoint loaded into the 36-channel i2v model: the extra patch-embedding input
    channels are zero-filled (1B:1311-1315); keys of another shape are skipped (1B:1317-1324)."""
    sub = tmp_path / "transformer"
    sub.mkdir()
    _config_json(sub, SMALL)
    base = dict(SMALL, in_dim=16)
    sd = synthetic.fill_state_dict(param_shapes(base), 6)
    sd["head.head.bias"] = torch.zeros(7)  # shape mismatch -> skipped
    save_file(sd, str(sub / "diffusion_pytorch_model.safetensors"))
    m = WanTransformer3DFantasyModel.from_pretrained(str(tmp_path), subfolder="transformer",
                                                     transformer_additional_kwargs=dict(ADD_KW),
                                                     torch_dtype=torch.float32)
    w = m.state_dict()["patch_embedding.weight"]
    assert w.shape[1] == 36
    assert torch.equal(w[:, :16], sd["patch_embedding.weight"]) and not w[:, 16:].any()
    assert m.state_dict()["head.head.bias"].shape == (64,)


def test_dit_missing_config_raises(tmp_path):
    with pytest.raises(RuntimeError):
        WanTransformer3DFantasyModel.from_pretrained(str(tmp_path))


@pytest.mark.parametrize("nested", [False, True])
def test_stableavatar_checkpoint_on_top(tmp_path, nested):
    """inference.py:485-490: torch.load(transformer3d-square.pt) -> ["state_dict"] when nested ->
    load_state_dict(strict=False) over the from_pretrained model."""
    m = WanTransformer3DFantasyModel(**SMALL)
    m.load_state_dict(synthetic.fill_state_dict(param_shapes(SMALL), 7))
    sa = synthetic.fill_state_dict({k: v for k, v in param_shapes(SMALL).items()
                                    if k.startswith(("vocal_projector.", "blocks.1.cross_attn."))}, 8)
    path = str(tmp_path / "transformer3d-square.pt")
    torch.save({"state_dict": sa, "global_step": 1} if nested else sa, path)
    state_dict = torch.load(path, map_location="cpu", weights_only=True)
    state_dict = state_dict["state_dict"] if "state_dict" in state_dict else state_dict
    missing, unexpected = m.load_state_dict(state_dict, strict=False)
    assert not unexpected and len(missing) == len(param_shapes(SMALL)) - len(sa)
    _same(m, sa)
    assert m._packed is None  # repacked on the next forward


@pytest.mark.parametrize("fmt", ["pth", "safetensors"])
def test_vae_from_pretrained(tmp_path, fmt):
    shapes = dict(vae_param_shapes(dim=32), **encoder_param_shapes(dim=32))
    sd = synthetic.fill_state_dict(shapes, 9)
    raw = {k[len("model."):]: v for k, v in sd.items()}  # Wan2.1_VAE.pth keys carry no prefix
    path = str(tmp_path / f"Wan2.1_VAE.{fmt}")
    if fmt == "pth":
        torch.save(raw, path)
    else:
        save_file(raw, path)
    v = AutoencoderKLWan.from_pretrained(path, additional_kwargs={"dim": 32, "vae_subpath": "x", "unused": 1})
    _same(v, sd)


def test_wav2vec2_keys_match_transformers():
    """the HIP wav2vec2 (stableavatar_amd/wav2vec.py) takes transformers' Wav2Vec2Model state_dict as is, the
    Wav2Vec2ForCTC prefix / head and the legacy weight-norm names (wav2vec2-base-960h) included, and its
    feature-encoder length formula matches transformers'"""
    import torch
    from transformers import Wav2Vec2Config, Wav2Vec2Model as HF

    from stableavatar_amd.wav2vec import Wav2Vec2Model
    hf = HF(Wav2Vec2Config(num_hidden_layers=2))
    ours = Wav2Vec2Model(hf.config)
    assert set(ours.state_dict()) == set(hf.state_dict()) - {"masked_spec_embed"}
    ours.load_state_dict(hf.state_dict())
    legacy = {"wav2vec2." + k.replace("parametrizations.weight.original0", "weight_g")
              .replace("parametrizations.weight.original1", "weight_v"): v for k, v in hf.state_dict().items()}
    legacy["lm_head.weight"] = torch.zeros(4, 768)
    ours.load_state_dict(legacy)
    sd = ours.state_dict()
    assert all(torch.equal(sd[k], v) for k, v in hf.state_dict().items() if k in sd)
    with pytest.raises(KeyError):
        ours.load_state_dict({k: v for k, v in hf.state_dict().items() if "layers.1." not in k})
    for n in (400, 8000, 16123, 51840):
        assert ours.frames(n) == int(hf._get_feat_extract_output_lengths(torch.tensor(n)))
