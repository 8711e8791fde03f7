"""TeaCache for the DiT (reference: wan/models/cache_utils.py:1-80, used at
wan_fantasy_transformer3d_1B.py:874-888 and :1021-1103; enabled by inference.py:526-535 with
--enable_teacache / --teacache_threshold / --num_skip_start_steps / --teacache_offload).

Decision logic and state are the reference's: the modulated input is e0 (the time projection,
[B, 6, dim] fp32), the distance is mean|cur - prev| / mean|prev| rescaled by a degree-4
polynomial and accumulated; a forward whose accumulated distance stays under the threshold skips
all 30 blocks and adds the residual (x_after_blocks - x_before_blocks) of the last computed forward
instead.  The first forward, the last of `num_steps` and the first `num_skip_start_steps` always
compute; the counter resets every `num_steps` forwards (so with several sliding windows per step
the reference's counter runs per forward call, not per sampling step -- kept as is).
This is an optional mode that changes numerics."""
from __future__ import annotations

import numpy as np
import torch


def get_teacache_coefficients(model_name):
    """cache_utils.py:5-16.  The reference's first test is `"wan2.1-t2v-1.3b" or ...`, a non-empty
    string, so every name gets the 1.3B coefficients; reproduced as is."""
    del model_name
    return [-5.21862437e+04, 9.23041404e+03, -5.28275948e+02, 1.36987616e+01, -4.99875664e-02]


class TeaCache:
    """cache_utils.py:19-80 (same constructor arguments and checks)."""

    def __init__(self, coefficients, num_steps: int, rel_l1_thresh: float = 0.0, num_skip_start_steps: int = 0,
                 offload: bool = True):
        if num_steps < 1:
            raise ValueError(f"`num_steps` must be greater than 0 but is {num_steps}.")
        if rel_l1_thresh < 0:
            raise ValueError(f"`rel_l1_thresh` must be greater than or equal to 0 but is {rel_l1_thresh}.")
        if num_skip_start_steps < 0 or num_skip_start_steps > num_steps:
            raise ValueError(f"`num_skip_start_steps` must be in [0, num_steps={num_steps}], got "
                             f"{num_skip_start_steps}.")
        self.coefficients = coefficients
        self.num_steps = num_steps
        self.rel_l1_thresh = rel_l1_thresh
        self.num_skip_start_steps = num_skip_start_steps
        self.offload = offload
        self.rescale_func = np.poly1d(coefficients)
        self.reset()

    @staticmethod
    def compute_rel_l1_distance(prev: torch.Tensor, cur: torch.Tensor) -> float:
        return ((cur - prev).abs().mean() / prev.abs().mean()).cpu().item()

    def reset(self):
        self.cnt = 0
        self.should_calc = True
        self.accumulated_rel_l1_distance = 0
        self.previous_modulated_input = None
        self.previous_residual = None
        self.previous_residual_cond = None
        self.previous_residual_uncond = None

    def decide(self, modulated_inp: torch.Tensor, cond_flag: bool) -> bool:
        """1B:1022-1044: whether this forward runs the blocks."""
        if not cond_flag:
            return self.should_calc
        skip_flag = self.cnt < self.num_skip_start_steps
        if self.cnt == 0 or self.cnt == self.num_steps - 1 or skip_flag:
            should_calc = True
            self.accumulated_rel_l1_distance = 0
        else:
            d = self.compute_rel_l1_distance(self.previous_modulated_input, modulated_inp)
            self.accumulated_rel_l1_distance += self.rescale_func(d)
            if self.accumulated_rel_l1_distance < self.rel_l1_thresh:
                should_calc = False
            else:
                should_calc = True
                self.accumulated_rel_l1_distance = 0
        self.previous_modulated_input = modulated_inp
        self.cnt += 1
        if self.cnt == self.num_steps:
            self.reset()
        self.should_calc = should_calc
        return should_calc

    def store(self, residual: torch.Tensor, cond_flag: bool):
        r = residual.cpu() if self.offload else residual
        if cond_flag:
            self.previous_residual_cond = r
        else:
            self.previous_residual_uncond = r

    def residual(self, cond_flag: bool, device) -> torch.Tensor:
        r = self.previous_residual_cond if cond_flag else self.previous_residual_uncond
        return r.to(device)
