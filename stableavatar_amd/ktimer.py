"""Per-kernel-class time inside a timed region, from HIP events (bench.py's `kernels` record).

While a KernelTimer is installed (`with KernelTimer() as kt:`), every C-ABI launch that goes through
`_lib.call` is followed by one HIP event on the launching stream (the current torch stream: every ops.* wrapper
launches there).  The interval from the previous event on that stream to this one is charged to the launch's
kernel class, so each class's time includes the kernel boundary in front of it (and any torch work queued on
the stream between two library launches), and the classes of one stream sum to that stream's busy span.
Classes follow the DiT block (wan_fantasy_transformer3d_1B.py:650-695): the GEMMs by role (their epilogue and
shape), self- / cross- / vocal-projector attention, LayerNorm, q/k RMSNorm + RoPE, the sampler step, the VAE.
"""
from __future__ import annotations

from collections import defaultdict

import torch

from . import _lib

# sa_gemm_bf16_panels / sa_gemm_bf16_ex argument positions (include/stableavatar_hip.h)
_G_M, _G_N, _G_K, _G_EPI = 10, 11, 12, 14


def classify(name: str, args) -> str:
    if name in ("sa_gemm_bf16_panels", "sa_gemm_bf16_ex"):
        m, n, k, epi = args[_G_M], args[_G_N], args[_G_K], args[_G_EPI]
        if epi == 3:  # fp32 gated residual: O-projection / cross-O (K = dim) or FFN-down (K = ffn_dim)
            return "gemm_residual_ffn_down" if k > n else "gemm_residual_o_proj"
        if epi == 1:
            return "gemm_gelu_ffn_up"
        if epi in (6, 7):  # the self-attention's V projection stored as V^T
            return "gemm_bf16_v_transposed"
        if epi == 0 and m >= 4096:  # token-row GEMMs (the context / vocal K|V ones have a few thousand rows)
            return {3 * k: "gemm_bf16_qkv", 2 * k: "gemm_bf16_qk", k: "gemm_bf16_cross_q"}.get(n, "gemm_other")
        return "gemm_other"
    if name in ("sa_attn_fwd_map", "sa_attn_fwd_ex", "sa_attn_fwd"):
        return "self_attention"
    if name == "sa_attn_cross3":
        return "cross_attention"
    if name == "sa_attn_small":
        return "vocal_projector_attention"
    if name == "sa_layernorm_mod":
        return "layernorm_modulate"
    if name in ("sa_qk_rmsnorm_rope", "sa_qkv_pack"):
        return "qk_rmsnorm_rope"
    if name in ("sa_conv3d_cl", "sa_conv3d_cl_down"):
        return "vae_conv"
    if name.startswith("sa_vae_") or name in ("sa_softmax_rows", "sa_transpose_bf16"):
        return "vae_other"
    if name == "sa_flow_step":
        return "flow_step"
    return "other"


class KernelTimer:
    def __init__(self):
        self.last = {}      # stream handle -> last event on it
        self.spans = []     # (class, ev0, ev1)
        self._prev = None

    def __enter__(self):
        self._prev, _lib._timer = _lib._timer, self
        return self

    def __exit__(self, *exc):
        _lib._timer = self._prev
        return False

    def before(self, name, args):
        s = torch.cuda.current_stream()
        if s.cuda_stream not in self.last:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(s)
            self.last[s.cuda_stream] = ev

    def after(self, name, args):
        s = torch.cuda.current_stream()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(s)
        self.spans.append((classify(name, args), self.last[s.cuda_stream], ev))
        self.last[s.cuda_stream] = ev

    def summary(self, clips: int) -> dict:
        """ms per clip and launches per clip by class (call after the region's closing synchronize)"""
        ms, n = defaultdict(float), defaultdict(int)
        for c, e0, e1 in self.spans:
            ms[c] += e0.elapsed_time(e1)
            n[c] += 1
        order = sorted(ms, key=lambda c: -ms[c])
        return {"ms_per_clip": {c: round(ms[c] / clips, 1) for c in order},
                "launches_per_clip": {c: n[c] // clips for c in order},
                "us_per_launch": {c: round(1e3 * ms[c] / n[c], 1) for c in order},
                "sum_ms_per_clip": round(sum(ms.values()) / clips, 1),
                "streams": len(self.last)}
