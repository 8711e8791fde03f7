"""ORACLE — test infrastructure only (imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product path).

CPU fp32 restatement of the StableAvatar Wan-2.1 1.3B DiT forward
(wan/models/wan_fantasy_transformer3d_1B.py, wan/models/vocal_projector_fantasy_1B.py,
wan/models/vocal_projector_fantasy.py).  Functional form over a state dict `P` whose keys are the
reference's own parameter names.  Pinned against goldens produced by the reference itself
(tests/golden/gen_golden.py -> tests/golden/*.npz, checked by tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# ---------------------------------------------------------------- primitives


def sinusoidal_embedding_1d(dim, position):
    """1B:210-220 (fp64)."""
    half = dim // 2
    pos = position.to(torch.float64)
    sinus = torch.outer(pos, torch.pow(10000, -torch.arange(half, dtype=torch.float64).div(half)))
    return torch.cat([torch.cos(sinus), torch.sin(sinus)], dim=1)


def rope_params(max_seq_len, dim, theta=10000):
    """1B:223-231: complex128 polar table."""
    fr = torch.outer(torch.arange(max_seq_len, dtype=torch.float64),
                     1.0 / torch.pow(theta, torch.arange(0, dim, 2, dtype=torch.float64).div(dim)))
    return torch.polar(torch.ones_like(fr), fr)


def model_freqs(d):
    """self.freqs of 1B:855-862."""
    return torch.cat([rope_params(1024, d - 4 * (d // 6)), rope_params(1024, 2 * (d // 6)),
                      rope_params(1024, 2 * (d // 6))], dim=1)


def rope_apply(x, grid_sizes, freqs):
    """1B:295-323.  x [B, L, n, d]; tokens past f*h*w stay unrotated."""
    n, c = x.size(2), x.size(3) // 2
    fr = freqs.split([c - 2 * (c // 3), c // 3, c // 3], dim=1)
    out = []
    for i, (f, h, w) in enumerate(grid_sizes):
        s = f * h * w
        xi = torch.view_as_complex(x[i, :s].to(torch.float32).reshape(s, n, -1, 2))
        fi = torch.cat([fr[0][:f].view(f, 1, 1, -1).expand(f, h, w, -1),
                        fr[1][:h].view(1, h, 1, -1).expand(f, h, w, -1),
                        fr[2][:w].view(1, 1, w, -1).expand(f, h, w, -1)], dim=-1).reshape(s, 1, -1)
        xi = torch.view_as_real(xi * fi).flatten(2)
        out.append(torch.cat([xi, x[i, s:]]))
    return torch.stack(out).float()


def rms_norm(x, w, eps):
    """WanRMSNorm 1B:326-342."""
    x = x.float()
    return x * torch.rsqrt(x.pow(2).mean(dim=-1, keepdim=True) + eps) * w


def layer_norm(x, eps, w=None, b=None):
    return F.layer_norm(x.float(), (x.shape[-1],), w, b, eps)


def linear(P, name, x):
    return F.linear(x, P[name + ".weight"], P.get(name + ".bias"))


def attention(q, k, v):
    """SDPA path of attention(), 1B:158-207 (no mask).  q [B, Lq, N, D]."""
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
    return o.transpose(1, 2).contiguous()


# ---------------------------------------------------------------- DiT blocks


def self_attn(P, pre, x, grid_sizes, freqs, heads, eps=1e-6):
    """WanSelfAttention.forward 1B:383-413."""
    b, s, dim = x.shape
    d = dim // heads
    q = rms_norm(linear(P, pre + ".q", x), P[pre + ".norm_q.weight"], eps).view(b, s, heads, d)
    k = rms_norm(linear(P, pre + ".k", x), P[pre + ".norm_k.weight"], eps).view(b, s, heads, d)
    v = linear(P, pre + ".v", x).view(b, s, heads, d)
    o = attention(rope_apply(q, grid_sizes, freqs), rope_apply(k, grid_sizes, freqs), v)
    return linear(P, pre + ".o", o.flatten(2))


def cross_attn(P, pre, x, context, vocal_context, latents_num_frames, heads, eps=1e-6):
    """WanI2VTalkingCrossAttention.forward 1B:534-605 (4-D vocal context path)."""
    ctx_img, ctx = context[:, :257], context[:, 257:]
    b, dim = x.size(0), x.size(2)
    n, d = heads, dim // heads
    q = rms_norm(linear(P, pre + ".q", x), P[pre + ".norm_q.weight"], eps).view(b, -1, n, d)
    k = rms_norm(linear(P, pre + ".k", ctx), P[pre + ".norm_k.weight"], eps).view(b, -1, n, d)
    v = linear(P, pre + ".v", ctx).view(b, -1, n, d)
    k_img = rms_norm(linear(P, pre + ".k_img", ctx_img), P[pre + ".norm_k_img.weight"], eps).view(b, -1, n, d)
    v_img = linear(P, pre + ".v_img", ctx_img).view(b, -1, n, d)
    img_x = attention(q, k_img, v_img)
    txt_x = attention(q, k, v)
    F_ = latents_num_frames
    vq = q.view(b * F_, -1, n, d)
    vk = linear(P, pre + ".k_vocal", vocal_context).view(b * F_, -1, n, d)
    vv = linear(P, pre + ".v_vocal", vocal_context).view(b * F_, -1, n, d)
    voc_x = attention(vq, vk, vv).view(b, q.size(1), n, d).flatten(2)
    return linear(P, pre + ".o", txt_x.flatten(2) + img_x.flatten(2) + voc_x)


def block(P, pre, x, e0, grid_sizes, freqs, context, vocal_context, latents_num_frames, heads, eps=1e-6):
    """WanAttentionBlock.forward 1B:650-695 (cross_attn_norm=True: norm3 affine)."""
    e = (P[pre + ".modulation"] + e0).chunk(6, dim=1)
    y = self_attn(P, pre + ".self_attn", layer_norm(x, eps) * (1 + e[1]) + e[0], grid_sizes, freqs, heads, eps)
    x = x + y * e[2]
    x = x + cross_attn(P, pre + ".cross_attn",
                       layer_norm(x, eps, P[pre + ".norm3.weight"], P[pre + ".norm3.bias"]),
                       context, vocal_context, latents_num_frames, heads, eps)
    h = layer_norm(x, eps) * (1 + e[4]) + e[3]
    h = linear(P, pre + ".ffn.2", F.gelu(linear(P, pre + ".ffn.0", h), approximate="tanh"))
    return x + h * e[5]


# ---------------------------------------------------------------- vocal projector


def split_audio_sequence(audio_proj_length, num_frames=81):
    """vocal_projector_fantasy.py:39-78."""
    tokens_per_frame = audio_proj_length / num_frames
    half = int(tokens_per_frame * 4 / 2)
    pos = []
    for i in range(int((num_frames - 1) / 4) + 1):
        if i == 0:
            pos.append(0)
        else:
            st = tokens_per_frame * ((i - 1) * 4 + 1)
            en = tokens_per_frame * (i * 4 + 1)
            pos.append(int((st + en) / 2) - 1)
    ranges = [[p - half, p + half] for p in pos]
    ranges[0] = [-(half * 2 - ranges[1][0]), ranges[1][0]]
    return ranges


def split_index_table(audio_len, num_frames, expand_length=4):
    """Row-gather form of split_tensor_with_padding (vocal_projector_fantasy.py:81-131): for each
    latent frame the list of source token indices, -1 for the zero rows appended at the END
    (front and back padding are both appended after the valid part, :120-125)."""
    rows, lens = [], []
    for s, e in split_audio_sequence(audio_len, num_frames):
        s, e = s - expand_length, e + expand_length
        mx = audio_len - 1
        pad = max(-s, 0) + max(e - mx, 0)
        vs, ve = max(s, 0), min(e, mx)
        valid = list(range(vs, ve + 1)) if vs <= ve else []
        rows.append(valid + [-1] * pad)
        lens.append(len(valid))
    return rows, lens


def vocal_projector(P, pre, vocal_embeddings, video_sample_n_frames, latents, e0, e, heads=8, eps=1e-6):
    """FantasyTalkingVocalCondition1BModel.forward (vocal_projector_fantasy_1B.py:433-450); with the
    14B model's two-layer VocalProjModel (vocal_projector_fantasy_14B.py:385-398) when its keys are present."""
    if pre + ".proj_model.proj_1.weight" in P:
        feat = F.linear(vocal_embeddings, P[pre + ".proj_model.proj_1.weight"])
        feat = layer_norm(feat, 1e-5, P[pre + ".proj_model.norm_1.weight"], P[pre + ".proj_model.norm_1.bias"])
        feat = F.linear(feat, P[pre + ".proj_model.proj_2.weight"])
        feat = layer_norm(feat, 1e-5, P[pre + ".proj_model.norm_2.weight"], P[pre + ".proj_model.norm_2.bias"])
    else:
        feat = F.linear(vocal_embeddings, P[pre + ".proj_model.proj.weight"])
        feat = layer_norm(feat, 1e-5, P[pre + ".proj_model.norm.weight"], P[pre + ".proj_model.norm.bias"])
    rows, _ = split_index_table(feat.size(1), video_sample_n_frames)
    Fn = len(rows)
    zero = feat.new_zeros(feat.size(0), 1, feat.size(2))
    padded = torch.cat([feat, zero], 1)
    idx = torch.tensor([[r if r >= 0 else feat.size(1) for r in row] for row in rows])
    x = padded[:, idx.flatten()]  # [b, F*n, C]
    b, C = x.size(0), x.size(2)
    d = C // heads
    for i in range(2):
        bp = f"{pre}.blocks.{i}"
        em = (P[bp + ".modulation"] + e0).chunk(6, dim=1)
        x = x + (layer_norm(x, eps) * (1 + em[1]) + em[0]) * em[2]
        hq = layer_norm(x, eps, P[bp + ".norm3.weight"], P[bp + ".norm3.bias"])
        cp = bp + ".cross_attn"
        q = rms_norm(linear(P, cp + ".q", hq), P[cp + ".norm_q.weight"], eps).view(b * Fn, -1, heads, d)
        k = rms_norm(linear(P, cp + ".k", latents), P[cp + ".norm_k.weight"], eps).view(b * Fn, -1, heads, d)
        v = linear(P, cp + ".v", latents).view(b * Fn, -1, heads, d)
        o = attention(q, k, v).view(b, -1, heads, d).flatten(2)
        x = x + linear(P, cp + ".o", o)
        h = layer_norm(x, eps) * (1 + em[4]) + em[3]
        x = x + linear(P, bp + ".ffn.2", F.gelu(linear(P, bp + ".ffn.0", h), approximate="tanh")) * em[5]
    ef = (P[pre + ".final_head.modulation"] + e.unsqueeze(1)).chunk(2, dim=1)
    x = linear(P, pre + ".final_head.final_proj", layer_norm(x, eps) * (1 + ef[1]) + ef[0])
    return x.view(b, Fn, -1, C)


# ---------------------------------------------------------------- full forward


def forward(P, cfg, x, t, context, seq_len, clip_fea, y, vocal_embeddings, video_sample_n_frames=81):
    """WanTransformer3DFantasyModel.forward 1B:928-1159 for the inference call of
    wan_inference_long_pipeline.py:740-750 (is_clip_level_modeling=False, SP off, TeaCache off); with
    cfg["vocal"] == "14B" WanTransformer3DFantasy14BModel.forward (14B:922-1152: 81-frame vocal path on
    every CFG row).
    x, y: [B, C, F, H, W]; context: list of [L_i, text_dim]; returns [B, out_dim, F, H, W]."""
    dim, heads, eps = cfg["dim"], cfg["num_heads"], cfg.get("eps", 1e-6)
    text_len, freq_dim, out_dim = cfg["text_len"], cfg["freq_dim"], cfg["out_dim"]
    d = dim // heads
    freqs = model_freqs(d)
    xin = torch.cat([x, y], dim=1).float()
    xe = F.conv3d(xin, P["patch_embedding.weight"], P["patch_embedding.bias"], stride=(1, 2, 2))
    B = xe.size(0)
    grid = [tuple(xe.shape[2:])] * B
    xe = xe.flatten(2).transpose(1, 2)
    assert xe.size(1) <= seq_len
    xe = torch.cat([xe, xe.new_zeros(B, seq_len - xe.size(1), dim)], dim=1)
    e = linear(P, "time_embedding.2", F.silu(linear(P, "time_embedding.0",
                                                   sinusoidal_embedding_1d(freq_dim, t).float())))
    e0 = linear(P, "time_projection.1", F.silu(e)).unflatten(1, (6, dim))
    ctx = torch.stack([torch.cat([u.float(), u.new_zeros(text_len - u.size(0), u.size(1)).float()])
                       for u in context])
    ctx = linear(P, "text_embedding.2", F.gelu(linear(P, "text_embedding.0", ctx), approximate="tanh"))
    ci = layer_norm(clip_fea.float(), 1e-5, P["img_emb.proj.0.weight"], P["img_emb.proj.0.bias"])
    ci = linear(P, "img_emb.proj.3", F.gelu(linear(P, "img_emb.proj.1", ci)))
    ci = layer_norm(ci, 1e-5, P["img_emb.proj.4.weight"], P["img_emb.proj.4.bias"])
    ctx = torch.cat([ci, ctx], dim=1)
    if cfg.get("vocal", "1B") == "14B":  # every row through the projector (14B:1008)
        vocal_ctx = vocal_projector(P, "vocal_projector", vocal_embeddings.float(), 81, xe, e0, e)
    elif vocal_embeddings.size(0) > 1:
        v = vocal_projector(P, "vocal_projector", vocal_embeddings[-1:].float(), video_sample_n_frames,
                            xe[-1:], e0[-1:], e[-1:])
        vocal_ctx = torch.cat([torch.zeros_like(v), v, v])
    else:
        vocal_ctx = vocal_projector(P, "vocal_projector", vocal_embeddings.float(), video_sample_n_frames, xe, e0, e)
    Fl = (video_sample_n_frames - 1) // 4 + 1
    h = xe
    for i in range(cfg["num_layers"]):
        h = block(P, f"blocks.{i}", h, e0, grid, freqs, ctx, vocal_ctx, Fl, heads, eps)
    eh = (P["head.modulation"] + e.unsqueeze(1)).chunk(2, dim=1)
    h = linear(P, "head.head", layer_norm(h, eps) * (1 + eh[1]) + eh[0])
    out = []
    for u, (f, hh, ww) in zip(h, grid):
        u = u[:f * hh * ww].view(f, hh, ww, 1, 2, 2, out_dim)
        u = torch.einsum("fhwpqrc->cfphqwr", u).reshape(out_dim, f, hh * 2, ww * 2)
        out.append(u)
    return torch.stack(out)


def param_shapes(cfg):
    """{name: shape} of the reference module for config `cfg` (same keys as its state_dict); the 14B
    module's with cfg["vocal"] == "14B"."""
    if cfg.get("vocal", "1B") == "14B":
        return _param_shapes_14b(cfg)
    dim, ffn, L = cfg["dim"], cfg["ffn_dim"], cfg["num_layers"]
    S = {"patch_embedding.weight": (dim, cfg["in_dim"], 1, 2, 2), "patch_embedding.bias": (dim,),
         "text_embedding.0.weight": (dim, cfg["text_dim"]), "text_embedding.0.bias": (dim,),
         "text_embedding.2.weight": (dim, dim), "text_embedding.2.bias": (dim,),
         "time_embedding.0.weight": (dim, cfg["freq_dim"]), "time_embedding.0.bias": (dim,),
         "time_embedding.2.weight": (dim, dim), "time_embedding.2.bias": (dim,),
         "time_projection.1.weight": (6 * dim, dim), "time_projection.1.bias": (6 * dim,)}
    for i in range(L):
        p = f"blocks.{i}"
        S[p + ".modulation"] = (1, 6, dim)
        for n in ("q", "k", "v", "o"):
            S[f"{p}.self_attn.{n}.weight"] = (dim, dim)
            S[f"{p}.self_attn.{n}.bias"] = (dim,)
        S[p + ".self_attn.norm_q.weight"] = (dim,)
        S[p + ".self_attn.norm_k.weight"] = (dim,)
        S[p + ".norm3.weight"] = (dim,)
        S[p + ".norm3.bias"] = (dim,)
        for n in ("q", "k", "v", "o", "k_img", "v_img", "k_vocal", "v_vocal"):
            S[f"{p}.cross_attn.{n}.weight"] = (dim, dim)
            S[f"{p}.cross_attn.{n}.bias"] = (dim,)
        for n in ("norm_q", "norm_k", "norm_k_img"):
            S[f"{p}.cross_attn.{n}.weight"] = (dim,)
        S[p + ".ffn.0.weight"] = (ffn, dim)
        S[p + ".ffn.0.bias"] = (ffn,)
        S[p + ".ffn.2.weight"] = (dim, ffn)
        S[p + ".ffn.2.bias"] = (dim,)
    S["head.modulation"] = (1, 2, dim)
    S["head.head.weight"] = (cfg["out_dim"] * 4, dim)
    S["head.head.bias"] = (cfg["out_dim"] * 4,)
    S.update({"img_emb.proj.0.weight": (1280,), "img_emb.proj.0.bias": (1280,),
              "img_emb.proj.1.weight": (1280, 1280), "img_emb.proj.1.bias": (1280,),
              "img_emb.proj.3.weight": (dim, 1280), "img_emb.proj.3.bias": (dim,),
              "img_emb.proj.4.weight": (dim,), "img_emb.proj.4.bias": (dim,)})
    vp = "vocal_projector"
    S[vp + ".proj_model.proj.weight"] = (1536, 768)
    S[vp + ".proj_model.norm.weight"] = (1536,)
    S[vp + ".proj_model.norm.bias"] = (1536,)
    for i in range(2):
        bp = f"{vp}.blocks.{i}"
        S[bp + ".modulation"] = (1, 6, 1536)
        S[bp + ".norm3.weight"] = (1536,)
        S[bp + ".norm3.bias"] = (1536,)
        for n in ("q", "o"):
            S[f"{bp}.cross_attn.{n}.weight"] = (1536, 1536)
            S[f"{bp}.cross_attn.{n}.bias"] = (1536,)
        for n in ("k", "v"):
            S[f"{bp}.cross_attn.{n}.weight"] = (1536, dim)
            S[f"{bp}.cross_attn.{n}.bias"] = (1536,)
        S[bp + ".cross_attn.norm_q.weight"] = (1536,)
        S[bp + ".cross_attn.norm_k.weight"] = (1536,)
        S[bp + ".ffn.0.weight"] = (3072, 1536)
        S[bp + ".ffn.0.bias"] = (3072,)
        S[bp + ".ffn.2.weight"] = (1536, 3072)
        S[bp + ".ffn.2.bias"] = (1536,)
    S[vp + ".final_head.modulation"] = (1, 2, 1536)
    S[vp + ".final_head.final_proj.weight"] = (1536, 1536)
    S[vp + ".final_head.final_proj.bias"] = (1536,)
    return S


def _param_shapes_14b(cfg):
    """WanTransformer3DFantasy14BModel (14B:823-866): the 1.3B layout at the model's width, plus the 14B
    vocal projector (vocal_projector_fantasy_14B.py:385-425): 768 -> 2048 -> dim projection, width dim."""
    S = {k: v for k, v in param_shapes(dict(cfg, vocal="1B")).items() if not k.startswith("vocal_projector")}
    dim, vp = cfg["dim"], "vocal_projector"
    S.update({vp + ".proj_model.proj_1.weight": (2048, 768), vp + ".proj_model.norm_1.weight": (2048,),
              vp + ".proj_model.norm_1.bias": (2048,), vp + ".proj_model.proj_2.weight": (dim, 2048),
              vp + ".proj_model.norm_2.weight": (dim,), vp + ".proj_model.norm_2.bias": (dim,)})
    for i in range(2):
        bp = f"{vp}.blocks.{i}"
        S[bp + ".modulation"] = (1, 6, dim)
        for n in ("norm3.weight", "norm3.bias", "cross_attn.norm_q.weight", "cross_attn.norm_k.weight",
                  "cross_attn.q.bias", "cross_attn.k.bias", "cross_attn.v.bias", "cross_attn.o.bias", "ffn.2.bias"):
            S[f"{bp}.{n}"] = (dim,)
        for n in ("q", "k", "v", "o"):
            S[f"{bp}.cross_attn.{n}.weight"] = (dim, dim)
        S[bp + ".ffn.0.weight"] = (2 * dim, dim)
        S[bp + ".ffn.0.bias"] = (2 * dim,)
        S[bp + ".ffn.2.weight"] = (dim, 2 * dim)
    S[vp + ".final_head.modulation"] = (1, 2, dim)
    S[vp + ".final_head.final_proj.weight"] = (dim, dim)
    S[vp + ".final_head.final_proj.bias"] = (dim,)
    return S


CONFIG_1_3B = dict(model_type="i2v", dim=1536, ffn_dim=8960, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
                   num_heads=12, num_layers=30, text_len=512, eps=1e-6)


def flops_forward(cfg, B, L, text_len=512, n_img=257, n_voc=17, F_=21):
    """Analytic matmul FLOPs (2/MAC) of one forward (used by bench/roofline)."""
    dim, ffn, nl = cfg["dim"], cfg["ffn_dim"], cfg["num_layers"]
    per_layer = (2 * B * L * dim * dim * 4            # q k v o
                 + 4 * B * L * L * dim                # QK^T + PV
                 + 2 * B * L * dim * dim * 2          # cross q, o
                 + 2 * B * (text_len + n_img) * dim * dim * 2 + 2 * B * F_ * n_voc * dim * dim * 2
                 + 4 * B * L * (text_len + n_img + n_voc) * dim
                 + 2 * B * L * dim * ffn * 2)
    return nl * per_layer + 2 * B * L * dim * cfg["in_dim"] * 4 + 2 * B * L * dim * 64
