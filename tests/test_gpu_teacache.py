"""TeaCache (optional, wan/models/cache_utils.py + 1B:1021-1103) on the HIP path vs the reference's own
10-forward runs (goldens): the compute/skip pattern must match exactly and every output (computed or
residual-reused) within the bf16 tolerance of SURVEY.md §8(d)."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, HERE)

from golden_cases import DIT_SMALL, TEACACHE, TEACACHE_STEPS, dit_inputs  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(TEACACHE))
def test_teacache_vs_reference(name):
    from test_gpu_dit import make_model, rel, run
    from stableavatar_amd.teacache import get_teacache_coefficients
    g = np.load(os.path.join(HERE, "golden", "teacache_small.npz"))
    coef, thr = TEACACHE[name]
    m = make_model(DIT_SMALL)
    m.enable_teacache(coef if coef is not None else get_teacache_coefficients("wan2.1-fun-1.3b"), TEACACHE_STEPS,
                      thr, num_skip_start_steps=2, offload=False)
    inp = dit_inputs(DIT_SMALL, "full")
    pat = []
    for k, t in enumerate(g["timesteps"]):
        out = run(m, dict(inp, t=torch.full((3,), float(t))))
        pat.append(int(m.teacache.should_calc))
        err = rel(out, g[name + "_out"][k])
        assert err < 2e-2, (k, err)
    assert pat == g[name + "_calc"].tolist(), (pat, g[name + "_calc"].tolist())
    assert m.teacache.cnt == 0  # reset after num_steps forwards (cache_utils.py reset)
