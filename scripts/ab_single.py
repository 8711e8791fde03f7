"""Single-GPU DiT forward on the golden cases, printing rel-L2 vs the reference golden and a checksum, for
A/B of two builds of the library (SA_LIB=<path>).  usage: python scripts/ab_single.py <out.pt>"""
import os
import sys

import numpy as np
import torch

HERE = os.path.join(os.getcwd(), "tests")
sys.path.insert(0, os.getcwd())
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))
from test_gpu_dit import make_model, run  # noqa: E402
from golden_cases import DIT_SMALL, dit_inputs  # noqa: E402

m = make_model(DIT_SMALL)
g = np.load(os.path.join(HERE, "golden", "dit_small.npz"))
outs = {}
for c in ("full", "short", "wide"):
    o = run(m, dit_inputs(DIT_SMALL, c))
    ref = torch.as_tensor(g[f"{c}_out"]).double()
    print(c, f"{((o.double() - ref).norm() / ref.norm()).item():.4e}", f"{o.double().abs().sum().item():.6f}")
    outs[c] = o
torch.save(outs, sys.argv[1])
