"""FlowMatchEulerDiscreteScheduler as used by the reference pipeline (diffusers 0.30.1, constructed
at inference.py:491-496 with wan_civitai.yaml shift 5.0 / 1000 train steps).  Host-side bookkeeping
only: the step arithmetic itself runs fused in the sa_flow_step kernel.  diffusers is not installed
offline, so this restates its published algorithm (parity of the sigma table: see DESIGN.md)."""
from __future__ import annotations

import numpy as np
import torch


class FlowMatchEulerDiscreteScheduler:
    order = 1

    def __init__(self, num_train_timesteps=1000, shift=1.0, use_dynamic_shifting=False, base_shift=0.5,
                 max_shift=1.15, base_image_seq_len=256, max_image_seq_len=4096, **_):
        if use_dynamic_shifting:
            raise NotImplementedError("dynamic shifting is not used by the StableAvatar configs")
        N = num_train_timesteps
        s = torch.from_numpy(np.linspace(1, N, N, dtype=np.float32)[::-1].copy() / N)
        s = shift * s / (1 + (shift - 1) * s)
        self.num_train_timesteps, self.shift = N, shift
        self.timesteps = s * N
        self.sigmas = s
        self.sigma_min, self.sigma_max = s[-1].item(), s[0].item()
        self._step_index = None
        self.config = type("cfg", (), dict(num_train_timesteps=N, shift=shift, use_dynamic_shifting=False))()

    def set_timesteps(self, num_inference_steps=None, device=None, sigmas=None, mu=None, **_):
        if sigmas is None:
            t = np.linspace(self.sigma_max * self.num_train_timesteps, self.sigma_min * self.num_train_timesteps,
                            num_inference_steps)
            sigmas = t / self.num_train_timesteps
        sigmas = self.shift * np.asarray(sigmas) / (1 + (self.shift - 1) * np.asarray(sigmas))
        s = torch.from_numpy(sigmas).to(dtype=torch.float32, device=device)
        self.timesteps = s * self.num_train_timesteps
        self.sigmas = torch.cat([s, torch.zeros(1, device=s.device)])
        self.num_inference_steps = len(s)
        self._step_index = None

    def step(self, model_output, timestep, sample, return_dict=False, **_):
        """Reference semantics (for callers that step manually); the pipeline uses sa_flow_step."""
        if self._step_index is None:
            idx = (self.timesteps == timestep).nonzero()
            self._step_index = idx[1 if len(idx) > 1 else 0].item()
        out = sample.float() + (self.sigmas[self._step_index + 1] - self.sigmas[self._step_index]) * model_output
        self._step_index += 1
        return (out.to(model_output.dtype),)
