"""wav2vec2 audio encoder on the HIP kernels.

Drop-in for the ``transformers.Wav2Vec2Model`` the reference loads at inference.py:475-476 and calls once
per sliding window at wan_inference_long_pipeline.py:727-729 (``self.wav2vec(input_values).last_hidden_state``).
Same constructor config, ``from_pretrained(dir)`` over a transformers model directory (config.json +
model.safetensors / pytorch_model.bin; the ``wav2vec2.`` prefix of a ``Wav2Vec2ForCTC`` checkpoint such as
wav2vec2-base-960h is stripped, as transformers does), same call and output attribute.

Architecture (transformers ``modeling_wav2vec2``, the ``feat_extract_norm="group"`` / post-LN variant that
wav2vec2-base uses):
  feature encoder  conv0 (1 -> 512, k 10, s 5) + GroupNorm(512 groups) + GELU, convs 1-6 (k 3,3,3,3,2,2,
                   s 2, no bias) + GELU                         -> sa_w2v_conv0_gn_gelu, sa_conv1d_im2col + GEMM
  projection       LayerNorm(512) -> Linear(512, 768)            -> sa_layernorm_mod + GEMM (fp32 hidden)
  positional conv  Conv1d(768, 768, k 128, pad 64, 16 groups), weight norm over dim 2, last frame dropped,
                   GELU, added; LayerNorm                        -> im2col + 16 group GEMMs, sa_add_f32_bf16
  12 layers        h = LN(h + O(attn(QKV(h)))); h = LN(h + W2(GELU(W1(h))))   (post-LN)
Hidden states stay fp32 between layers (the reference runs the whole model in fp32 on the host); GEMM
operands are bf16 and every Linear output is rounded to bf16 before its residual add, like the DiT's
epilogues.  Contract vs transformers' fp32 model: tests/test_gpu_wav2vec.py.
"""
from __future__ import annotations

import json
import os
from types import SimpleNamespace

import torch
from torch import nn

from . import ops
from ._lib import call
from .encoders import _register

_DEFAULTS = dict(conv_dim=(512,) * 7, conv_kernel=(10, 3, 3, 3, 3, 2, 2), conv_stride=(5, 2, 2, 2, 2, 2, 2),
                 conv_bias=False, feat_extract_norm="group", feat_extract_activation="gelu",
                 num_conv_pos_embeddings=128, num_conv_pos_embedding_groups=16, hidden_size=768,
                 num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072, hidden_act="gelu",
                 layer_norm_eps=1e-5, do_stable_layer_norm=False)


def _load_state_dict(path):
    for name in ("model.safetensors", "pytorch_model.bin"):
        f = os.path.join(path, name)
        if os.path.exists(f):
            if name.endswith(".safetensors"):
                from safetensors.torch import load_file
                return load_file(f)
            return torch.load(f, map_location="cpu", weights_only=True)
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin under {path}")


def wav2vec2_param_shapes(cfg) -> dict:
    """{state_dict key: shape} of transformers' Wav2Vec2Model (group-norm feature encoder, post-LN layers;
    the positional conv's weight norm in the parametrizations layout, original0 = g, original1 = v)."""
    C = cfg["conv_dim"][0]
    S = {"feature_extractor.conv_layers.0.conv.weight": (C, 1, cfg["conv_kernel"][0]),
         "feature_extractor.conv_layers.0.layer_norm.weight": (C,),
         "feature_extractor.conv_layers.0.layer_norm.bias": (C,)}
    for i in range(1, len(cfg["conv_dim"])):
        S[f"feature_extractor.conv_layers.{i}.conv.weight"] = (C, C, cfg["conv_kernel"][i])
    H, F = cfg["hidden_size"], cfg["intermediate_size"]
    k, G = cfg["num_conv_pos_embeddings"], cfg["num_conv_pos_embedding_groups"]
    S.update({"feature_projection.layer_norm.weight": (C,), "feature_projection.layer_norm.bias": (C,),
              "feature_projection.projection.weight": (H, C), "feature_projection.projection.bias": (H,),
              "encoder.pos_conv_embed.conv.bias": (H,),
              "encoder.pos_conv_embed.conv.parametrizations.weight.original0": (1, 1, k),
              "encoder.pos_conv_embed.conv.parametrizations.weight.original1": (H, H // G, k),
              "encoder.layer_norm.weight": (H,), "encoder.layer_norm.bias": (H,)})
    for i in range(cfg["num_hidden_layers"]):
        p = f"encoder.layers.{i}."
        for n in ("q", "k", "v", "out"):
            S[p + f"attention.{n}_proj.weight"] = (H, H)
            S[p + f"attention.{n}_proj.bias"] = (H,)
        for n in ("layer_norm", "final_layer_norm"):
            S[p + f"{n}.weight"] = (H,)
            S[p + f"{n}.bias"] = (H,)
        S[p + "feed_forward.intermediate_dense.weight"] = (F, H)
        S[p + "feed_forward.intermediate_dense.bias"] = (F,)
        S[p + "feed_forward.output_dense.weight"] = (H, F)
        S[p + "feed_forward.output_dense.bias"] = (H,)
    return S


def _canonical_keys(sd):
    """a transformers checkpoint -> this module's keys: drop the Wav2Vec2ForCTC prefix and head, pretraining-
    only tensors, and map the legacy weight_g / weight_v names of the positional conv's weight norm"""
    out = {}
    for k, v in sd.items():
        if k.startswith("wav2vec2."):
            k = k[len("wav2vec2."):]
        if k.startswith(("lm_head.", "masked_spec_embed", "quantizer.", "project_", "dropout_features")):
            continue
        k = k.replace("pos_conv_embed.conv.weight_g", "pos_conv_embed.conv.parametrizations.weight.original0")
        k = k.replace("pos_conv_embed.conv.weight_v", "pos_conv_embed.conv.parametrizations.weight.original1")
        out[k] = v
    return out


class Wav2Vec2Model(nn.Module):
    """``transformers.Wav2Vec2Model`` forward (inference) on the HIP kernels: same state_dict keys,
    ``__call__(input_values)`` returns an object with ``last_hidden_state`` [B, T, hidden] fp32."""

    def __init__(self, config=None, **kw):
        super().__init__()
        cfg = dict(_DEFAULTS)
        if config is not None:
            src = config if isinstance(config, dict) else config.to_dict()
            cfg.update({k: src[k] for k in _DEFAULTS if k in src})
        cfg.update(kw)
        for k in ("conv_dim", "conv_kernel", "conv_stride"):
            cfg[k] = tuple(cfg[k])
        if cfg["feat_extract_norm"] != "group" or cfg["do_stable_layer_norm"]:
            raise NotImplementedError("only the feat_extract_norm='group', post-LN wav2vec2 variant (wav2vec2-base, "
                                      "as used by the reference) is implemented")
        if cfg["conv_bias"]:
            raise NotImplementedError("conv_bias=True feature encoders are not implemented")
        for a in ("hidden_act", "feat_extract_activation"):
            if cfg[a] != "gelu":
                raise NotImplementedError(f"{a}={cfg[a]!r}: only exact GELU is implemented")
        if len(set(cfg["conv_dim"])) != 1 or cfg["conv_dim"][0] % 8 or cfg["conv_kernel"][0] > 64:
            raise NotImplementedError("feature-encoder widths must be equal and a multiple of 8, conv0 kernel <= 64")
        if cfg["hidden_size"] % cfg["num_conv_pos_embedding_groups"] or \
                (cfg["hidden_size"] // cfg["num_conv_pos_embedding_groups"]) % 8:
            raise NotImplementedError("positional-conv groups must be a multiple of 8 channels wide")
        self.config = SimpleNamespace(**cfg)
        _register(self, wav2vec2_param_shapes(cfg))
        self._packed = None

    @classmethod
    def from_pretrained(cls, path, **kw):
        with open(os.path.join(path, "config.json")) as f:
            cfg = json.load(f)
        m = cls(cfg, **kw)
        m.load_state_dict(_load_state_dict(path), strict=True)
        return m

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._packed = None
        sd = _canonical_keys(state_dict)
        own = set(self.state_dict())
        if strict:
            missing = own - set(sd)
            if missing:
                raise KeyError(f"Wav2Vec2Model: missing keys {sorted(missing)[:8]}")
        return super().load_state_dict({k: v for k, v in sd.items() if k in own}, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):
        self._packed = None
        return super()._apply(fn, recurse)

    def _pack(self):
        if self._packed is not None:
            return self._packed
        c = self.config
        P_ = dict(self.named_parameters())
        dev = P_["encoder.layer_norm.weight"].device
        if dev.type != "cuda":
            raise RuntimeError("Wav2Vec2Model runs on the MI355X HIP kernels: move it to 'cuda'")
        f32 = lambda k: P_[k].detach().float().contiguous()  # noqa: E731
        bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
        C, H, G = c.conv_dim[0], c.hidden_size, c.num_conv_pos_embedding_groups
        P = SimpleNamespace(device=dev)
        P.conv0 = f32("feature_extractor.conv_layers.0.conv.weight").reshape(C, -1).contiguous()
        P.gn_w = f32("feature_extractor.conv_layers.0.layer_norm.weight")
        P.gn_b = f32("feature_extractor.conv_layers.0.layer_norm.bias")
        # conv l: [out, in, k] -> [out, k*in] with column j*in + c (the im2col order)
        P.convs = [bf(f32(f"feature_extractor.conv_layers.{i}.conv.weight").permute(0, 2, 1).reshape(C, -1))
                   for i in range(1, len(c.conv_dim))]
        P.fp_ln_w, P.fp_ln_b = f32("feature_projection.layer_norm.weight"), f32("feature_projection.layer_norm.bias")
        P.fp_w, P.fp_b = bf(f32("feature_projection.projection.weight")), f32("feature_projection.projection.bias")
        pre = "encoder.pos_conv_embed.conv."
        g, v = f32(pre + "parametrizations.weight.original0"), f32(pre + "parametrizations.weight.original1")
        # torch weight_norm(dim=2): w = g * v / ||v|| with the norm over every dim but 2 (one per tap)
        w = v * (g / v.pow(2).sum(dim=(0, 1), keepdim=True).sqrt())
        P.pos_w = bf(w.permute(0, 2, 1).reshape(H, -1))  # [H, k*cg], row o belongs to group o // cg
        P.pos_b = f32(pre + "bias")
        P.enc_ln_w, P.enc_ln_b = f32("encoder.layer_norm.weight"), f32("encoder.layer_norm.bias")
        P.layers = []
        for i in range(c.num_hidden_layers):
            p = f"encoder.layers.{i}."
            a = p + "attention."
            P.layers.append(SimpleNamespace(
                w_qkv=bf(torch.cat([f32(a + f"{n}_proj.weight") for n in "qkv"])),
                b_qkv=torch.cat([f32(a + f"{n}_proj.bias") for n in "qkv"]).contiguous(),
                w_o=bf(f32(a + "out_proj.weight")), b_o=f32(a + "out_proj.bias"),
                ln_w=f32(p + "layer_norm.weight"), ln_b=f32(p + "layer_norm.bias"),
                w1=bf(f32(p + "feed_forward.intermediate_dense.weight")),
                b1=f32(p + "feed_forward.intermediate_dense.bias"),
                w2=bf(f32(p + "feed_forward.output_dense.weight")), b2=f32(p + "feed_forward.output_dense.bias"),
                fln_w=f32(p + "final_layer_norm.weight"), fln_b=f32(p + "final_layer_norm.bias")))
        self._packed = P
        return P

    def frames(self, n_samples):
        """output length of the feature encoder for n_samples input samples"""
        T = n_samples
        for k, s in zip(self.config.conv_kernel, self.config.conv_stride):
            T = (T - k) // s + 1
        return T

    @torch.no_grad()
    def forward(self, input_values, attention_mask=None, **kw):
        if attention_mask is not None:
            raise NotImplementedError("attention_mask: the reference calls wav2vec2 without one")
        P = self._pack()
        x = input_values.to(P.device, torch.float32)
        if x.dim() == 1:
            x = x[None]
        outs = [self._forward_one(P, x[b].contiguous()) for b in range(x.shape[0])]
        return SimpleNamespace(last_hidden_state=torch.stack(outs), extract_features=None, hidden_states=None,
                               attentions=None)

    def _forward_one(self, P, audio):
        c = self.config
        dev = audio.device
        C = c.conv_dim[0]
        T = (audio.shape[0] - c.conv_kernel[0]) // c.conv_stride[0] + 1
        if T <= 0:
            raise ValueError(f"wav2vec2: {audio.shape[0]} samples is shorter than one conv0 window")
        h = torch.empty(T, C, device=dev, dtype=torch.bfloat16)
        call("sa_w2v_conv0_gn_gelu", audio.data_ptr(), audio.shape[0], P.conv0.data_ptr(), C, c.conv_kernel[0],
             c.conv_stride[0], P.gn_w.data_ptr(), P.gn_b.data_ptr(), 1e-5, h.data_ptr(), T, ops._stream())
        for w, k, s in zip(P.convs, c.conv_kernel[1:], c.conv_stride[1:]):
            To = (T - k) // s + 1
            if To <= 0:
                raise ValueError("wav2vec2: input too short for the feature encoder")
            cols = torch.empty(To, k * C, device=dev, dtype=torch.bfloat16)
            call("sa_conv1d_im2col", h.data_ptr(), h.stride(0), T, 0, 1, C, k, s, 0, cols.data_ptr(), To, k * C,
                 ops._stream())
            h = ops.linear(cols, w, None, ops.EPI_GELU_ERF_BF16)
            T = To
        eps = c.layer_norm_eps
        hn = ops.layernorm_mod(h, torch.empty_like(h), eps, weight=P.fp_ln_w, bias=P.fp_ln_b)
        H, G = c.hidden_size, c.num_conv_pos_embedding_groups
        x = ops.linear(hn, P.fp_w, P.fp_b, ops.EPI_F32)  # [T, H] fp32 hidden states
        xb = ops.cast_bf16(x, torch.empty(T, H, device=dev, dtype=torch.bfloat16))
        # positional conv: 16 groups of cg channels, k taps, padding k//2, the (T+1)-th output dropped
        k, cg = c.num_conv_pos_embeddings, H // G
        cols = torch.empty(G, T, k * cg, device=dev, dtype=torch.bfloat16)
        call("sa_conv1d_im2col", xb.data_ptr(), xb.stride(0), T, 0, G, cg, k, 1, k // 2, cols.data_ptr(), T, k * cg,
             ops._stream())
        pos = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
        for g in range(G):
            sl = slice(g * cg, (g + 1) * cg)
            ops.linear(cols[g], P.pos_w[sl], P.pos_b[sl], ops.EPI_GELU_ERF_BF16, out=pos[:, sl])
        call("sa_add_f32_bf16", x.data_ptr(), x.stride(0), pos.data_ptr(), pos.stride(0), T, H, ops._stream())
        ops.layernorm_mod(x, x, eps, weight=P.enc_ln_w, bias=P.enc_ln_b)
        nh = c.num_attention_heads
        hd = H // nh
        segs = torch.tensor([[0, T, 0, T]], dtype=torch.int32, device=dev)
        att = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
        for L in P.layers:
            ops.cast_bf16(x, xb)
            qkv = ops.linear(xb, L.w_qkv, L.b_qkv, ops.EPI_BF16)
            ops.attention_small(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], att, segs, 1, T, T, nh, hd)
            ops.linear(att, L.w_o, L.b_o, ops.EPI_RES_F32, out=x, residual=x)
            ops.layernorm_mod(x, x, eps, weight=L.ln_w, bias=L.ln_b)
            ops.cast_bf16(x, xb)
            f = ops.linear(xb, L.w1, L.b1, ops.EPI_GELU_ERF_BF16)
            ops.linear(f, L.w2, L.b2, ops.EPI_RES_F32, out=x, residual=x)
            ops.layernorm_mod(x, x, eps, weight=L.fln_w, bias=L.fln_b)
        return x
