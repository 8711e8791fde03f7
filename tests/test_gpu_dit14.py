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
