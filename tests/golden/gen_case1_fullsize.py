"""Expected latents of the case-1 full-size windowed loop (golden_cases.CASE1_FULL) from the CPU oracle
(oracle/pipeline.py's restatement of wan_inference_long_pipeline.py:703-790 with oracle/dit.py, both pinned to the
reference's own goldens by tests/test_oracle_golden.py).  Writes tests/golden/case1_fullsize.npz: the bf16 latents
after 2 of the 50 sampling steps, stored as their raw 16-bit patterns.  CPU only (~10 full-width forwards)."""
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from golden_cases import CASE1_FULL, case1_fullsize_inputs  # noqa: E402

from oracle import dit as odit  # noqa: E402
from oracle import pipeline as opipe  # noqa: E402
from stableavatar_amd import synthetic  # noqa: E402


def main():
    C = CASE1_FULL
    cfg = {k: v for k, v in C["dit"].items() if k != "seed"}
    P = synthetic.fill_state_dict(odit.param_shapes(cfg), C["dit"]["seed"])
    inp = case1_fullsize_inputs(C)
    n = [0]

    def dit(x, t, context, seq_len, yy, clip_fea, vocal, nfr):
        n[0] += 1
        t0 = time.time()
        out = odit.forward(P, cfg, x.to(torch.bfloat16).float(), t, context, seq_len, clip_fea,
                           yy.to(torch.bfloat16).float(), vocal, nfr)
        print(f"forward {n[0]}: {time.time() - t0:.1f}s", flush=True)
        return out

    enc = lambda s: synthetic.fake_wav2vec_features(torch.as_tensor(s)[None])  # noqa: E731
    with torch.no_grad():
        lat = opipe.denoise(dit, inp["latents"].to(torch.bfloat16).float(), inp["y"], inp["context"], inp["clip"],
                            inp["audio"], enc, num_inference_steps=C["steps"], clip_length=C["clip_length"],
                            num_frames=C["clip_length"], height=C["size"], width=C["size"], overlap=C["overlap"],
                            text_guide_scale=C["text_guide"], audio_guide_scale=C["audio_guide"],
                            max_steps=C["run_steps"])
    bits = lat.to(torch.bfloat16).view(torch.int16).numpy()
    np.savez_compressed(os.path.join(HERE, "case1_fullsize.npz"), latents_bf16=bits, forwards=n[0])
    print("forwards", n[0], "latents", tuple(lat.shape))


if __name__ == "__main__":
    main()
