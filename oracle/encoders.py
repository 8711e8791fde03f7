"""ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

CPU fp32 restatement of the once-per-call encoders the pipeline drives:
* umT5 text encoder: WanT5EncoderModel (wan/models/wan_text_encoder.py: T5LayerNorm, T5Attention
  (no 1/sqrt(d) scaling, relative-position bias, key padding mask), T5FeedForward (fc1 * GELU_tanh(gate)),
  T5SelfAttention, T5RelativeEmbedding._relative_position_bucket, WanT5EncoderModel.forward);
* open-CLIP XLM-R ViT-H/14 visual tower as CLIPModel.forward runs it (wan/models/wan_image_encoder.py:
  bicubic resize to image_size, *0.5+0.5, Normalize, VisionTransformer.forward with use_31_block:
  patch Conv2d, class token, positional embedding, pre-norm, all blocks but the last).
Parameters are plain {state_dict key: tensor} dicts with the reference's key names.  Pinned to
reference goldens by tests/test_oracle_golden.py (gen_golden.py t5 / clip).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)  # wan_image_encoder.py:459-460
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


# ---------------------------------------------------------------------------------------------- umT5

def t5_param_shapes(vocab, dim, dim_attn, dim_ffn, num_heads, num_layers, num_buckets, shared_pos=True):
    S = {"token_embedding.weight": (vocab, dim), "norm.weight": (dim,)}
    if shared_pos:
        S["pos_embedding.embedding.weight"] = (num_buckets, num_heads)
    for i in range(num_layers):
        p = f"blocks.{i}."
        S[p + "norm1.weight"] = (dim,)
        for n in ("q", "k", "v"):
            S[p + f"attn.{n}.weight"] = (dim_attn, dim)
        S[p + "attn.o.weight"] = (dim, dim_attn)
        S[p + "norm2.weight"] = (dim,)
        S[p + "ffn.gate.0.weight"] = (dim_ffn, dim)
        S[p + "ffn.fc1.weight"] = (dim_ffn, dim)
        S[p + "ffn.fc2.weight"] = (dim, dim_ffn)
        if not shared_pos:
            S[p + "pos_embedding.embedding.weight"] = (num_buckets, num_heads)
    return S


def t5_relative_bucket(lq, lk, num_buckets, bidirectional=True, max_dist=128):
    """T5RelativeEmbedding._relative_position_bucket of rel_pos = j - i, [lq, lk] int64."""
    rel_pos = torch.arange(lk).unsqueeze(0) - torch.arange(lq).unsqueeze(1)
    if bidirectional:
        num_buckets //= 2
        rel_buckets = (rel_pos > 0).long() * num_buckets
        rel_pos = torch.abs(rel_pos)
    else:
        rel_buckets = 0
        rel_pos = -torch.min(rel_pos, torch.zeros_like(rel_pos))
    max_exact = num_buckets // 2
    rel_pos_large = max_exact + (torch.log(rel_pos.float() / max_exact) / math.log(max_dist / max_exact) *
                                 (num_buckets - max_exact)).long()
    rel_pos_large = torch.min(rel_pos_large, torch.full_like(rel_pos_large, num_buckets - 1))
    return rel_buckets + torch.where(rel_pos < max_exact, rel_pos, rel_pos_large)


def _t5_norm(x, w, eps=1e-6):
    return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))


def _t5_gelu(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def t5_forward(P, input_ids, attention_mask, num_heads, num_layers, num_buckets, shared_pos=True):
    """WanT5EncoderModel.forward in fp32: input_ids [B, L] long, attention_mask [B, L] -> [B, L, dim]."""
    x = P["token_embedding.weight"][input_ids].float()
    b, L, dim = x.shape
    bucket = t5_relative_bucket(L, L, num_buckets)

    def pos_bias(key):  # [1, N, L, L]
        return P[key].float()[bucket].permute(2, 0, 1).unsqueeze(0)

    shared = pos_bias("pos_embedding.embedding.weight") if shared_pos else None
    mask = attention_mask.view(b, 1, 1, -1)
    for i in range(num_layers):
        p = f"blocks.{i}."
        e = shared if shared_pos else pos_bias(p + "pos_embedding.embedding.weight")
        h = _t5_norm(x, P[p + "norm1.weight"].float())
        q = (h @ P[p + "attn.q.weight"].float().t()).view(b, L, num_heads, -1)
        k = (h @ P[p + "attn.k.weight"].float().t()).view(b, L, num_heads, -1)
        v = (h @ P[p + "attn.v.weight"].float().t()).view(b, L, num_heads, -1)
        bias = torch.zeros(b, num_heads, L, L) + e
        bias = bias.masked_fill(mask == 0, torch.finfo(torch.float32).min)
        a = torch.einsum("binc,bjnc->bnij", q, k) + bias
        a = F.softmax(a, dim=-1)
        o = torch.einsum("bnij,bjnc->binc", a, v).reshape(b, L, -1)
        x = x + o @ P[p + "attn.o.weight"].float().t()
        h = _t5_norm(x, P[p + "norm2.weight"].float())
        f = (h @ P[p + "ffn.fc1.weight"].float().t()) * _t5_gelu(h @ P[p + "ffn.gate.0.weight"].float().t())
        x = x + f @ P[p + "ffn.fc2.weight"].float().t()
    return _t5_norm(x, P["norm.weight"].float())


# ---------------------------------------------------------------------------------------------- CLIP

def clip_param_shapes(dim=1280, num_layers=32, patch=14, image_size=224, mlp_ratio=4, prefix="model.visual."):
    n_pos = (image_size // patch) ** 2 + 1
    S = {prefix + "patch_embedding.weight": (dim, 3, patch, patch), prefix + "cls_embedding": (1, 1, dim),
         prefix + "pos_embedding": (1, n_pos, dim), prefix + "pre_norm.weight": (dim,),
         prefix + "pre_norm.bias": (dim,), prefix + "post_norm.weight": (dim,), prefix + "post_norm.bias": (dim,),
         prefix + "head": (dim, 1024)}
    mid = int(dim * mlp_ratio)
    for i in range(num_layers):
        p = f"{prefix}transformer.{i}."
        S.update({p + "norm1.weight": (dim,), p + "norm1.bias": (dim,), p + "attn.to_qkv.weight": (3 * dim, dim),
                  p + "attn.to_qkv.bias": (3 * dim,), p + "attn.proj.weight": (dim, dim), p + "attn.proj.bias": (dim,),
                  p + "norm2.weight": (dim,), p + "norm2.bias": (dim,), p + "mlp.0.weight": (mid, dim),
                  p + "mlp.0.bias": (mid,), p + "mlp.2.weight": (dim, mid), p + "mlp.2.bias": (dim,)})
    return S


def clip_preprocess(img, image_size=224):
    """CLIPModel.forward preprocessing of one image [C, 1, H, W] in [-1, 1] -> [1, C, S, S]."""
    x = F.interpolate(img.transpose(0, 1).float(), size=(image_size, image_size), mode="bicubic",
                      align_corners=False)
    x = x * 0.5 + 0.5
    mean = torch.tensor(CLIP_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(CLIP_STD).view(1, 3, 1, 1)
    return (x - mean) / std


def clip_visual(P, x, num_heads, num_layers, patch=14, prefix="model.visual.", eps=1e-5):
    """VisionTransformer.forward(x, use_31_block=True): [B, 3, S, S] -> [B, 1 + (S/patch)^2, dim] after all
    blocks but the last (activation nn.GELU, pre-norm, no post-norm on this path)."""
    g = lambda n: P[prefix + n].float()  # noqa: E731
    x = F.conv2d(x, g("patch_embedding.weight"), stride=patch).flatten(2).permute(0, 2, 1)
    b = x.shape[0]
    x = torch.cat([g("cls_embedding").expand(b, -1, -1), x], dim=1) + g("pos_embedding")
    dim = x.shape[-1]
    x = F.layer_norm(x, (dim,), g("pre_norm.weight"), g("pre_norm.bias"), eps)
    d = dim // num_heads
    for i in range(num_layers - 1):
        p = f"transformer.{i}."
        h = F.layer_norm(x, (dim,), g(p + "norm1.weight"), g(p + "norm1.bias"), eps)
        qkv = (h @ g(p + "attn.to_qkv.weight").t() + g(p + "attn.to_qkv.bias")).view(b, -1, 3, num_heads, d)
        q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, -1, dim)
        x = x + o @ g(p + "attn.proj.weight").t() + g(p + "attn.proj.bias")
        h = F.layer_norm(x, (dim,), g(p + "norm2.weight"), g(p + "norm2.bias"), eps)
        h = F.gelu(h @ g(p + "mlp.0.weight").t() + g(p + "mlp.0.bias"))
        x = x + h @ g(p + "mlp.2.weight").t() + g(p + "mlp.2.bias")
    return x
