"""Drop-in WanTransformer3DFantasyModel (reference: wan/models/wan_fantasy_transformer3d_1B.py)."""
from __future__ import annotations

import torch


def rope_params(max_seq_len: int, dim: int, theta: float = 10000.0) -> torch.Tensor:
    """Angles of rope_params (1B:223-231) in fp64: [max_seq_len, dim/2]."""
    return torch.outer(torch.arange(max_seq_len, dtype=torch.float64),
                       1.0 / torch.pow(theta, torch.arange(0, dim, 2, dtype=torch.float64).div(dim)))


def rope_table(head_dim: int = 128, max_seq_len: int = 1024) -> torch.Tensor:
    """fp32 (cos, sin) table [max_seq_len, head_dim/2, 2] of the concatenated frame/height/width
    frequencies of self.freqs (1B:855-862), computed in fp64 like the reference."""
    d = head_dim
    ang = torch.cat([rope_params(max_seq_len, d - 4 * (d // 6)), rope_params(max_seq_len, 2 * (d // 6)),
                     rope_params(max_seq_len, 2 * (d // 6))], dim=1)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()
