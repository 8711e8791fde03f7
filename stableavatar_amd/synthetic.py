"""Synthetic, seeded stand-ins for what the offline environment lacks: checkpoint weights and the
once-per-call encoders (T5, CLIP, wav2vec2).  The same name-keyed rule feeds the reference modules
(golden generation, in the survey container), the CPU oracle and the HIP path, so all three see
bit-identical parameters without shipping any weights.

Rule per parameter (numpy PCG64 keyed by [seed, crc32(name)]):
  1-D '*weight' / 'gamma'  -> 1 + 0.1 N(0,1)       (norm scales)
  '*bias'                  -> 0.05 N(0,1)
  '*modulation'            -> N(0,1) / sqrt(last dim)   (as the reference init, 1B:648)
  other                    -> N(0,1) / sqrt(fan_in), fan_in = prod(shape[1:])
Zero-initialised reference params (k_vocal/v_vocal 1B:526-531, VAE AttentionBlock.proj wan_vae.py:241)
are re-randomised so those paths are exercised.
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch


def _std_for(name: str, shape) -> tuple[float, float]:
    """(mean, std) of the rule above."""
    leaf = name.rsplit(".", 1)[-1]
    if "modulation" in name:
        return 0.0, 1.0 / math.sqrt(shape[-1])
    if leaf == "bias":
        return 0.0, 0.05
    if len(shape) == 1 and (leaf in ("weight", "gamma")):
        return 1.0, 0.1
    if leaf == "gamma":
        return 1.0, 0.1
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
    return 0.0, 1.0 / math.sqrt(max(fan_in, 1))


def param_tensor(name: str, shape, seed: int = 0, backend: str = "numpy", device="cpu") -> torch.Tensor:
    mean, std = _std_for(name, tuple(shape))
    key = zlib.crc32(name.encode())
    if backend == "numpy":
        rng = np.random.Generator(np.random.PCG64([seed, key]))
        a = rng.standard_normal(size=tuple(shape), dtype=np.float32) * np.float32(std) + np.float32(mean)
        return torch.from_numpy(a).to(device)
    g = torch.Generator(device=device)
    g.manual_seed((seed << 32) ^ key)
    return torch.randn(tuple(shape), generator=g, device=device, dtype=torch.float32) * std + mean


def fill_state_dict(shapes: dict, seed: int = 0, backend: str = "numpy", device="cpu") -> dict:
    """{name: shape} -> {name: fp32 tensor} following the rule above."""
    return {n: param_tensor(n, s, seed, backend, device) for n, s in shapes.items()}


def timing_state_dict(shapes: dict, seed: int = 0) -> dict:
    """{name: shape} -> fp32 tensors with the rule's mean / std per name, but tiled from ONE seeded block of 2^20
    normals instead of a generator per tensor: for runs that only time the arithmetic (bench.py's CPU baseline),
    where filling 1.7 G parameters one generator at a time would take longer than the measured work.  The values
    are normal floats of the same scale (no denormals), so the timing is that of real weights."""
    base = torch.from_numpy(np.random.Generator(np.random.PCG64(seed)).standard_normal(1 << 20, dtype=np.float32))
    out = {}
    for n, shp in shapes.items():
        mean, std = _std_for(n, tuple(shp))
        cnt = int(np.prod(shp)) if len(shp) else 1
        nb = base.numel()
        reps = -(-cnt // nb)
        src = base[:min(cnt, nb)] * std + mean
        t = torch.empty(reps * src.numel())
        t.view(reps, src.numel()).copy_(src.expand(reps, -1))  # one (threaded) write pass
        out[n] = t[:cnt].view(tuple(shp))
    return out


def seeded_normal(shape, seed: int, scale: float = 1.0) -> torch.Tensor:
    rng = np.random.Generator(np.random.PCG64(seed))
    return torch.from_numpy(rng.standard_normal(size=tuple(shape), dtype=np.float32) * np.float32(scale))


# ---- encoder stand-ins (the real T5 / CLIP / wav2vec2 weights are not available offline) ----

def fake_wav2vec_features(samples: torch.Tensor, seed: int = 7, dim: int = 768) -> torch.Tensor:
    """Deterministic stand-in for Wav2Vec2Model(...).last_hidden_state: frames the 16 kHz signal like
    wav2vec2 (receptive field 400, stride 320 -> (n-400)//320+1 tokens) and projects each frame
    with a fixed seeded matrix + tanh.  samples: [B, n] float32 -> [B, tokens, dim]."""
    x = samples.float()
    if x.dim() == 1:
        x = x[None]
    n = x.shape[-1]
    tokens = (n - 400) // 320 + 1
    frames = x.unfold(-1, 400, 320)[:, :tokens]  # [B, tokens, 400]
    proj = seeded_normal((400, dim), seed, scale=1.0 / math.sqrt(400.0)).to(x.device)
    return torch.tanh(frames @ proj * 8.0)
