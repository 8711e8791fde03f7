"""The once-per-call encoders on the HIP path: umT5 (WanT5EncoderModel) and the
CLIP ViT-H/14 visual tower (CLIPModel), vs the reference's own outputs at reduced size (goldens) and vs
the CPU oracle (oracle/encoders.py, pinned to those goldens) at the real widths (umT5-XXL: dim 4096,
64 heads of 64, ffn 10240; ViT-H/14: dim 1280, 16 heads of 80) with 2 layers.  bf16 GEMM operands vs
the fp32 reference: rel-L2 <= 2e-2."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

from golden_cases import CLIP_FULL_WIDTH, CLIP_SMALL, T5_FULL_WIDTH, T5_SMALL, clip_image, t5_inputs  # noqa: E402

from stableavatar_amd import synthetic  # noqa: E402

pytestmark = pytest.mark.gpu
G = lambda n: np.load(os.path.join(HERE, "golden", n))  # noqa: E731


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).norm() / b.norm()).item()


def _t5(c):
    from stableavatar_amd.encoders import WanT5EncoderModel, t5_param_shapes
    kw = {k: c[k] for k in ("vocab", "dim", "dim_attn", "dim_ffn", "num_heads", "num_layers", "num_buckets",
                            "shared_pos")}
    P = synthetic.fill_state_dict(t5_param_shapes(**kw), c["seed"])
    m = WanT5EncoderModel(**kw)
    m.load_state_dict(P)
    return m.cuda(), P, kw


def _clip(c):
    from stableavatar_amd.encoders import CLIPModel, clip_param_shapes
    P = synthetic.fill_state_dict(clip_param_shapes(c["dim"], c["num_layers"], c["patch"], c["image_size"]),
                                  c["seed"])
    m = CLIPModel(dim=c["dim"], num_heads=c["num_heads"], num_layers=c["num_layers"], patch_size=c["patch"],
                  image_size=c["image_size"])
    m.load_state_dict(P)
    return m.cuda(), P


def test_t5_vs_reference_golden():
    """The reference runs umT5 in bf16 (inference.py:464-469); T5's unscaled logits rounded to bf16 move its
    output several % from its own fp32 run.  Contract: no further from the reference's bf16 output, nor from
    its fp32 output, than 1.5x the reference's own bf16-vs-fp32 drift."""
    m, _, _ = _t5(T5_SMALL)
    ids, mask = t5_inputs(T5_SMALL)
    with torch.no_grad():
        out = m(ids.cuda(), attention_mask=mask.cuda())[0]
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16 and tuple(out.shape) == (1, 512, T5_SMALL["dim"])
    g = G("encoders_small.npz")
    e_bf, e_32, drift = rel(out, g["t5_out_bf16"]), rel(out, g["t5_out"]), rel(g["t5_out_bf16"], g["t5_out"])
    print(f"t5 small: vs reference bf16 {e_bf:.2e}, vs reference fp32 {e_32:.2e} (reference bf16 drift {drift:.2e})")
    assert e_bf < 1.5 * drift and e_32 < 1.5 * drift, (e_bf, e_32, drift)


@pytest.mark.parametrize("L,valid", [(512, 53), (100, 100)])
def test_t5_full_width_vs_reference(L, valid):
    """umT5-XXL widths (2 layers, small vocabulary), the reference's bf16 and fp32 outputs on the valid
    rows; L = 100 is padded to 128 keys inside (masked) and trimmed back."""
    c = dict(T5_FULL_WIDTH, text_len=L, valid=valid)
    m, _, _ = _t5(c)
    ids, mask = t5_inputs(c)
    with torch.no_grad():
        out = m(ids.cuda(), attention_mask=mask.cuda())[0]
    torch.cuda.synchronize()
    assert tuple(out.shape) == (1, L, 4096)
    g = G("encoders_small.npz")
    rb, r32 = g[f"t5_full_L{L}_bf16"].astype(np.float32), g[f"t5_full_L{L}"].astype(np.float32)
    o = out[:, :valid].float()
    e_bf, e_32, drift = rel(o, rb), rel(o, r32), rel(rb, r32)
    print(f"t5 full width L={L}: vs reference bf16 {e_bf:.2e}, vs fp32 {e_32:.2e} (reference drift {drift:.2e})")
    assert e_bf < 1.5 * drift and e_32 < 1.5 * drift, (e_bf, e_32, drift)


def test_clip_vs_reference_golden():
    m, _ = _clip(CLIP_SMALL)
    with torch.no_grad():
        out = m([clip_image(CLIP_SMALL).cuda()])
    torch.cuda.synchronize()
    assert tuple(out.shape) == (1, 257, CLIP_SMALL["dim"]) and out.dtype == torch.float32
    e = rel(out, G("encoders_small.npz")["clip_out"])
    print(f"clip small vs reference: rel-L2 {e:.2e}")
    assert e < 2e-2, e


def test_clip_full_width_vs_oracle():
    from oracle import encoders as oenc
    c = CLIP_FULL_WIDTH
    m, P = _clip(c)
    img = clip_image(c)
    with torch.no_grad():
        out = m([img.cuda()])
        ref = oenc.clip_visual(P, oenc.clip_preprocess(img, c["image_size"]), c["num_heads"], c["num_layers"],
                               c["patch"])
    e = rel(out, ref)
    print(f"clip full width: rel-L2 {e:.2e}")
    assert e < 2e-2, e
