"""Drop-in for the reference's only kernel-dispatch seam, ``attention(q, k, v, ...)``
(wan/models/wan_fantasy_transformer3d_1B.py:158-207), on the HIP kernels.

The reference runs its SDPA branch (flash-attn is forced off at 1B:45-46): q/k/v [B, L, N, D] are
transposed to heads-first, ``F.scaled_dot_product_attention(q, k, v, attn_mask=None, is_causal=causal,
dropout_p=dropout_p)`` is called, so the scale is always 1/sqrt(D) (``softmax_scale`` / ``q_scale`` /
``window_size`` / ``dtype`` / ``deterministic`` / ``fa_version`` are not used on that branch) and
``q_lens`` / ``k_lens`` only raise a warning (1B:190-193).  This function keeps that contract:

* head_dim 128 -> ``sa_attn_fwd`` (flash attention, bf16 in, fp32 softmax/accumulate, bf16 out);
* other head dims (<= 256, multiple of 8) -> ``sa_attn_small`` (fp32 online softmax);
* causal masks and dropout are not part of the inference path: they raise instead of silently differing.
Returns [B, Lq, N, D] in the dtype of q (bf16 on the reference's autocast path).
"""
from __future__ import annotations

import warnings

import torch

from . import ops


def attention(q, k, v, q_lens=None, k_lens=None, dropout_p=0., softmax_scale=None, q_scale=None, causal=False,
              window_size=(-1, -1), deterministic=False, dtype=torch.bfloat16, fa_version=None):
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4:
        raise ValueError("attention expects q, k, v of shape [B, L, N, D]")
    B, Lq, N, D = q.shape
    if k.shape[0] != B or v.shape[0] != B or k.shape[2] != N or v.shape[2] != N or k.shape[1] != v.shape[1] \
            or k.shape[3] != D or v.shape[3] != D:
        raise ValueError(f"shape mismatch q {tuple(q.shape)} k {tuple(k.shape)} v {tuple(v.shape)}")
    if not (q.is_cuda and k.is_cuda and v.is_cuda):
        raise RuntimeError("attention runs on the MI355X HIP kernels: q, k, v must be GPU tensors")
    if causal:
        raise NotImplementedError("causal attention is not on the StableAvatar inference path")
    if dropout_p:
        raise NotImplementedError("attention dropout is a training feature (dropout_p must be 0)")
    if q_lens is not None or k_lens is not None:
        warnings.warn('Padding mask is disabled when using scaled_dot_product_attention. It can have a significant '
                      'impact on performance.')
    Lk = k.shape[1]
    out_dtype = q.dtype
    if Lk == 0 or Lq == 0:  # SDPA over no keys returns zeros
        return torch.zeros(B, Lq, N, D, device=q.device, dtype=out_dtype)
    qb, kb, vb = (t.to(torch.bfloat16).contiguous().view(-1, N * D) for t in (q, k, v))
    o = torch.empty(B * Lq, N * D, device=q.device, dtype=torch.bfloat16)
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32).to(q.device)
    if D == 128:
        ops.attention(qb, kb, vb, o, segs, B, Lq, N)
    else:
        if D > 256 or D % 8:
            raise NotImplementedError(f"head_dim {D}: the small-attention kernel takes D <= 256 (multiple of 8)")
        ops.attention_small(qb, kb, vb, o, segs, B, Lq, Lk, N, D)
    return o.view(B, Lq, N, D).to(out_dtype)
