"""wav2vec2 on the HIP path vs the reference's own audio encoder: transformers'
Wav2Vec2Model (what inference.py:475-476 loads and wan_inference_long_pipeline.py:727-729 calls per window),
run in fp32 on the host as the reference does, with the wav2vec2-base geometry (7-layer conv feature encoder,
768 wide, 12 heads, ffn 3072) and seeded random weights.

Contract: our output (bf16 GEMM operands, fp32 hidden states) is no further from the fp32 reference than
1.5x the reference model's own bf16-vs-fp32 drift, and at most 3e-2 rel-L2 in any case."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _models(layers):
    from transformers import Wav2Vec2Config, Wav2Vec2Model as HF

    from stableavatar_amd.wav2vec import Wav2Vec2Model
    torch.manual_seed(0)
    hf = HF(Wav2Vec2Config(num_hidden_layers=layers)).eval()
    ours = Wav2Vec2Model(hf.config)
    ours.load_state_dict(hf.state_dict())
    return hf, ours.cuda()


def _audio(n, seed):
    a = np.random.default_rng(seed).standard_normal(n).astype(np.float32) * 0.1
    a = (a - a.mean()) / np.sqrt(a.var() + 1e-7)  # Wav2Vec2FeatureExtractor do_normalize
    return torch.from_numpy(a)[None]


@pytest.mark.parametrize("n_samples", [16000 + 123, 51840])  # ~1 s, and one 81-frame window at 25 fps
def test_wav2vec2_vs_transformers(n_samples):
    hf, ours = _models(12)
    x = _audio(n_samples, n_samples)
    with torch.no_grad():
        ref = hf(x).last_hidden_state
        ref_bf = hf.to(torch.bfloat16)(x.bfloat16()).last_hidden_state.float()
        out = ours(x.cuda()).last_hidden_state
    torch.cuda.synchronize()
    assert out.shape == ref.shape and out.dtype == torch.float32
    assert out.shape[1] == ours.frames(n_samples)
    e, drift = rel(out, ref), rel(ref_bf, ref)
    cos = torch.nn.functional.cosine_similarity(out.double().cpu().flatten(), ref.double().flatten(), dim=0).item()
    print(f"wav2vec2 {n_samples} samples (T={out.shape[1]}): rel-L2 {e:.2e}, cosine {cos:.6f}; "
          f"reference bf16 drift {drift:.2e}")
    assert e < min(3e-2, max(1.5 * drift, 1e-2)), (e, drift)


def test_wav2vec2_from_pretrained_legacy_and_ctc_layouts(tmp_path):
    """transformers' save_pretrained directory, and the same weights as a Wav2Vec2ForCTC checkpoint with the
    legacy weight_g / weight_v names (wav2vec2-base-960h's layout)"""
    from safetensors.torch import save_file

    from stableavatar_amd.wav2vec import Wav2Vec2Model
    hf, ours = _models(2)
    hf.save_pretrained(str(tmp_path / "w2v"))
    a = Wav2Vec2Model.from_pretrained(str(tmp_path / "w2v")).cuda()
    sd = {}
    for k, v in hf.state_dict().items():
        k = k.replace("parametrizations.weight.original0", "weight_g").replace("parametrizations.weight.original1",
                                                                              "weight_v")
        sd["wav2vec2." + k] = v.contiguous()
    sd["lm_head.weight"] = torch.zeros(32, 768)
    (tmp_path / "ctc").mkdir()
    save_file(sd, str(tmp_path / "ctc" / "model.safetensors"))
    (tmp_path / "ctc" / "config.json").write_text((tmp_path / "w2v" / "config.json").read_text())
    b = Wav2Vec2Model.from_pretrained(str(tmp_path / "ctc")).cuda()
    x = _audio(8000, 1).cuda()
    with torch.no_grad():
        o0, oa, ob = (m(x).last_hidden_state for m in (ours, a, b))
    assert torch.equal(o0, oa) and torch.equal(o0, ob)
