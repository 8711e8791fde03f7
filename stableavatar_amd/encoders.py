"""Drop-in umT5 text encoder and CLIP image encoder on the HIP kernels.

* ``WanT5EncoderModel`` (reference: wan/models/wan_text_encoder.py): same constructor arguments,
  state_dict keys (``token_embedding``, ``blocks.N.{norm1,attn.{q,k,v,o},norm2,ffn.{gate.0,fc1,fc2},
  pos_embedding.embedding}``, ``norm``), ``from_pretrained(path, additional_kwargs, low_cpu_mem_usage,
  torch_dtype)`` and ``forward(input_ids, attention_mask) -> (x,)`` as the pipeline calls it
  (wan_inference_long_pipeline.py:270).  Per block: T5LayerNorm (sa_t5_rmsnorm) -> fused q|k|v GEMM ->
  per-head scores by a head-batched GEMM (no 1/sqrt(d) scaling, T5Attention.forward) -> relative-position
  bias + key mask + softmax (sa_t5_softmax_bias) -> P.V by a head-batched GEMM -> o GEMM with the residual
  add -> T5LayerNorm -> fused gate|fc1 GEMM -> fc1 * GELU_tanh(gate) (sa_t5_geglu) -> fc2 GEMM + residual.
  Residual stream fp32 (the reference keeps it bf16: a stated difference, within the test tolerance).
* ``CLIPModel`` (reference: wan/models/wan_image_encoder.py CLIPModel): the open-CLIP XLM-R ViT-H/14 visual
  tower as ``CLIPModel.forward`` runs it: bicubic resize + Normalize (sa_clip_preprocess), patch Conv2d as a
  GEMM whose residual input is the positional embedding (+ class token), pre-norm, then all blocks but the
  last (use_31_block): LN -> q|k|v GEMM -> attention (head dim 80, sa_attn_small) -> proj GEMM + residual,
  LN -> fc1 GEMM + GELU(erf) -> fc2 GEMM + residual.  Keys ``model.visual.*``; the checkpoint's text-tower
  keys (XLM-R) are not used by the pipeline and are ignored.  The reference runs CLIP in fp32; here GEMM
  operands are bf16 (fp32 accumulate, fp32 residual stream).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import ops
from ._lib import call

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)  # wan_image_encoder.py:459-460
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def _register(root: nn.Module, shapes: dict):
    for name, shp in shapes.items():
        *path, leaf = name.split(".")
        mod = root
        for p in path:
            if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                mod.add_module(p, nn.Module())
            mod = getattr(mod, p)
        mod.register_parameter(leaf, nn.Parameter(torch.empty(shp), requires_grad=False))


def _load_file(path):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def _filter_kwargs(cls, kw):
    import inspect
    sig = set(inspect.signature(cls.__init__).parameters) - {"self", "cls"}
    return {k: v for k, v in kw.items() if k in sig}


# ================================================================================================ umT5

def t5_param_shapes(vocab, dim, dim_attn, dim_ffn, num_heads, num_layers, num_buckets, shared_pos=True):
    """{state_dict key: shape} of the reference WanT5EncoderModel."""
    S = {"token_embedding.weight": (vocab, dim)}
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
    S["norm.weight"] = (dim,)
    return S


def relative_position_bucket(lq, lk, num_buckets, bidirectional=True, max_dist=128):
    """T5RelativeEmbedding._relative_position_bucket (wan_text_encoder.py) of rel_pos = j - i, computed
    with the same float32 ops on the host: int32 [lq, lk]."""
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
    return (rel_buckets + torch.where(rel_pos < max_exact, rel_pos, rel_pos_large)).to(torch.int32)


class WanT5EncoderModel(nn.Module):
    def __init__(self, vocab, dim, dim_attn, dim_ffn, num_heads, num_layers, num_buckets, shared_pos=True,
                 dropout=0.1):
        super().__init__()
        assert dim_attn % num_heads == 0
        self.vocab, self.dim, self.dim_attn, self.dim_ffn = vocab, dim, dim_attn, dim_ffn
        self.num_heads, self.num_layers, self.num_buckets, self.shared_pos = num_heads, num_layers, num_buckets, shared_pos
        self.head_dim = dim_attn // num_heads
        _register(self, t5_param_shapes(vocab, dim, dim_attn, dim_ffn, num_heads, num_layers, num_buckets, shared_pos))
        self._packed = None
        self._buckets = {}

    @property
    def dtype(self):
        return torch.bfloat16  # the pipeline reads text_encoder.dtype (pipeline:245)

    @classmethod
    def from_pretrained(cls, pretrained_model_path, additional_kwargs={}, low_cpu_mem_usage=False,
                        torch_dtype=torch.bfloat16):
        """wan_text_encoder.py WanT5EncoderModel.from_pretrained: a .pth / .safetensors state_dict with the
        module's own keys; constructor arguments filtered from additional_kwargs (the yaml's
        text_encoder_kwargs)."""
        model = cls(**_filter_kwargs(cls, additional_kwargs))
        sd = _load_file(pretrained_model_path)
        missing = set(model.state_dict()) - set(sd)
        if missing:
            raise ValueError(f"{pretrained_model_path} misses {len(missing)} keys, e.g. {sorted(missing)[:3]}")
        model.load_state_dict({k: v for k, v in sd.items() if k in model.state_dict()}, strict=True)
        return model.to(torch_dtype)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._packed = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):
        self._packed = None
        self._buckets = {}
        return super()._apply(fn, recurse)

    def _pack(self):
        if self._packed is not None:
            return self._packed
        dev = self.token_embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("WanT5EncoderModel runs on the MI355X HIP kernels: move it to 'cuda'")
        P = dict(self.named_parameters())
        bf = lambda n: P[n].detach().to(torch.bfloat16).contiguous()  # noqa: E731
        f32 = lambda n: P[n].detach().float().contiguous()  # noqa: E731
        pk = SimpleNamespace(emb=bf("token_embedding.weight"), norm=f32("norm.weight"), layers=[])
        shared = bf("pos_embedding.embedding.weight") if self.shared_pos else None
        for i in range(self.num_layers):
            p = f"blocks.{i}."
            L = SimpleNamespace()
            L.n1, L.n2 = f32(p + "norm1.weight"), f32(p + "norm2.weight")
            L.w_qkv = torch.cat([P[p + f"attn.{n}.weight"].detach() for n in "qkv"]).to(torch.bfloat16).contiguous()
            L.w_o = bf(p + "attn.o.weight")
            L.w_gf = torch.cat([P[p + "ffn.gate.0.weight"].detach(), P[p + "ffn.fc1.weight"].detach()]).to(
                torch.bfloat16).contiguous()
            L.w_fc2 = bf(p + "ffn.fc2.weight")
            L.pos = shared if self.shared_pos else bf(p + "pos_embedding.embedding.weight")
            pk.layers.append(L)
        self._packed = pk
        return pk

    def _bucket(self, L, dev):
        t = self._buckets.get(L)
        if t is None:
            t = relative_position_bucket(L, L, self.num_buckets).to(dev).contiguous()
            self._buckets[L] = t
        return t

    def forward(self, input_ids=None, attention_mask=None):
        pk = self._pack()
        dev = pk.emb.device
        ids = input_ids.to(dev)
        B, L0 = ids.shape
        mask = torch.ones(B, L0, dtype=torch.int32, device=dev) if attention_mask is None else \
            attention_mask.to(device=dev, dtype=torch.int32)
        L = -(-L0 // 64) * 64  # the P.V GEMM takes K = L in steps of 64: pad keys, masked out
        if L != L0:
            ids = torch.cat([ids, ids.new_zeros(B, L - L0)], 1)
            mask = torch.cat([mask, mask.new_zeros(B, L - L0)], 1)
        mask = mask.contiguous()
        H, hd, da, dim, dff = self.num_heads, self.head_dim, self.dim_attn, self.dim, self.dim_ffn
        M = B * L
        xb = torch.empty(M, dim, device=dev, dtype=torch.bfloat16)
        ops.gather_rows(pk.emb, ids.reshape(-1).to(torch.int32).contiguous(), xb)
        x = torch.empty(M, dim, device=dev, dtype=torch.float32)
        call("sa_cast_bf16_f32", xb.data_ptr(), x.data_ptr(), x.numel(), ops._stream())
        bucket = self._bucket(L, dev)
        h = torch.empty(M, dim, device=dev, dtype=torch.bfloat16)
        o = torch.empty(M, da, device=dev, dtype=torch.bfloat16)
        S = torch.empty(H, L, L, device=dev, dtype=torch.float32)
        Pm = torch.empty(H, L, L, device=dev, dtype=torch.bfloat16)
        Vt = torch.empty(H, hd, L, device=dev, dtype=torch.bfloat16)
        g = torch.empty(M, dff, device=dev, dtype=torch.bfloat16)
        st = ops._stream()
        for Ly in pk.layers:
            call("sa_t5_rmsnorm", x.data_ptr(), dim, 1, h.data_ptr(), dim, Ly.n1.data_ptr(), M, dim, 1e-6, st)
            qkv = ops.linear(h, Ly.w_qkv, None, ops.EPI_BF16)  # [M, 3 da] = q | k | v
            for b in range(B):
                base = qkv.data_ptr() + b * L * 3 * da * 2
                # S[h] = Q_h K_h^T (T5 does not scale the scores), heads as the GEMM batch
                call("sa_gemm_bf16_ex", base, 3 * da, hd, base + da * 2, 3 * da, hd, 0, S.data_ptr(), L, L * L, L, L,
                     hd, H, ops.EPI_F32, 0, 0, 0, 0, 0, 0, 0, 0, st)
                call("sa_t5_softmax_bias", S.data_ptr(), L, Pm.data_ptr(), L, 1, H, L, L, bucket.data_ptr(),
                     Ly.pos.data_ptr(), mask[b].data_ptr(), st)
                call("sa_transpose_bf16", base + 2 * da * 2, 3 * da, hd, Vt.data_ptr(), L, hd * L, L, hd, H, st)
                call("sa_gemm_bf16_ex", Pm.data_ptr(), L, L * L, Vt.data_ptr(), L, hd * L, 0,
                     o.data_ptr() + b * L * da * 2, da, hd, L, hd, L, H, ops.EPI_BF16, 0, 0, 0, 0, 0, 0, 0, 0, st)
            ops.linear(o, Ly.w_o, None, ops.EPI_RES_F32, out=x, residual=x)
            call("sa_t5_rmsnorm", x.data_ptr(), dim, 1, h.data_ptr(), dim, Ly.n2.data_ptr(), M, dim, 1e-6, st)
            gf = ops.linear(h, Ly.w_gf, None, ops.EPI_BF16)  # [M, 2 dff] = gate | fc1
            call("sa_t5_geglu", gf.data_ptr(), 2 * dff, g.data_ptr(), dff, M, dff, st)
            ops.linear(g, Ly.w_fc2, None, ops.EPI_RES_F32, out=x, residual=x)
        out = torch.empty(M, dim, device=dev, dtype=torch.bfloat16)
        call("sa_t5_rmsnorm", x.data_ptr(), dim, 1, out.data_ptr(), dim, pk.norm.data_ptr(), M, dim, 1e-6, st)
        return (out.view(B, L, dim)[:, :L0],)


# ================================================================================================ CLIP

def clip_param_shapes(dim=1280, num_layers=32, patch=14, image_size=224, mlp_ratio=4, out_dim=1024,
                      prefix="model.visual."):
    """{key: shape} of the visual tower of the reference CLIPModel (VisionTransformer, pool 'token',
    pre-norm: patch Conv2d without bias)."""
    n_pos = (image_size // patch) ** 2 + 1
    S = {prefix + "patch_embedding.weight": (dim, 3, patch, patch), prefix + "cls_embedding": (1, 1, dim),
         prefix + "pos_embedding": (1, n_pos, dim), prefix + "pre_norm.weight": (dim,),
         prefix + "pre_norm.bias": (dim,)}
    mid = int(dim * mlp_ratio)
    for i in range(num_layers):
        p = f"{prefix}transformer.{i}."
        S.update({p + "norm1.weight": (dim,), p + "norm1.bias": (dim,), p + "attn.to_qkv.weight": (3 * dim, dim),
                  p + "attn.to_qkv.bias": (3 * dim,), p + "attn.proj.weight": (dim, dim), p + "attn.proj.bias": (dim,),
                  p + "norm2.weight": (dim,), p + "norm2.bias": (dim,), p + "mlp.0.weight": (mid, dim),
                  p + "mlp.0.bias": (mid,), p + "mlp.2.weight": (dim, mid), p + "mlp.2.bias": (dim,)})
    S.update({prefix + "post_norm.weight": (dim,), prefix + "post_norm.bias": (dim,), prefix + "head": (dim, out_dim)})
    return S


class CLIPModel(nn.Module):
    """CLIPModel (wan_image_encoder.py) visual path; defaults = open-CLIP XLM-R ViT-H/14."""

    def __init__(self, dim=1280, num_heads=16, num_layers=32, patch_size=14, image_size=224, mlp_ratio=4):
        super().__init__()
        self.dim, self.num_heads, self.num_layers = dim, num_heads, num_layers
        self.patch, self.image_size, self.mlp_ratio = patch_size, image_size, mlp_ratio
        _register(self, clip_param_shapes(dim, num_layers, patch_size, image_size, mlp_ratio))
        self._packed = None

    @property
    def dtype(self):
        return torch.float32

    @classmethod
    def from_pretrained(cls, pretrained_model_path, transformer_additional_kwargs={}):
        """wan_image_encoder.py CLIPModel.from_pretrained: keys get the "model." prefix; the text tower's
        keys of the open-CLIP checkpoint are ignored (only the visual tower is on the pipeline's path)."""
        model = cls(**_filter_kwargs(cls, transformer_additional_kwargs))
        sd = {"model." + k: v for k, v in _load_file(pretrained_model_path).items()}
        own = model.state_dict()
        missing = set(own) - set(sd)
        if missing:
            raise ValueError(f"{pretrained_model_path} misses {len(missing)} visual keys, e.g. {sorted(missing)[:3]}")
        model.load_state_dict({k: v for k, v in sd.items() if k in own}, strict=True)
        return model

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._packed = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):
        self._packed = None
        return super()._apply(fn, recurse)

    def _pack(self):
        if self._packed is not None:
            return self._packed
        v = self.model.visual
        dev = v.pos_embedding.device
        if dev.type != "cuda":
            raise RuntimeError("CLIPModel runs on the MI355X HIP kernels: move it to 'cuda'")
        P = {k: t.detach() for k, t in v.named_parameters()}
        bf = lambda n: P[n].to(torch.bfloat16).contiguous()  # noqa: E731
        f32 = lambda n: P[n].float().contiguous()  # noqa: E731
        dim = self.dim
        kin = 3 * self.patch * self.patch
        kpad = -(-kin // 64) * 64
        wpe = torch.zeros(dim, kpad, device=dev, dtype=torch.bfloat16)
        wpe[:, :kin] = P["patch_embedding.weight"].reshape(dim, kin).to(torch.bfloat16)
        pos = P["pos_embedding"][0].float().clone()
        pos[0] += P["cls_embedding"][0, 0].float()  # class token row: its GEMM row is zero
        pk = SimpleNamespace(w_pe=wpe, kpad=kpad, pos=pos.contiguous(), pre_w=f32("pre_norm.weight"),
                             pre_b=f32("pre_norm.bias"), layers=[],
                             mean=torch.tensor(CLIP_MEAN, device=dev), std=torch.tensor(CLIP_STD, device=dev))
        for i in range(self.num_layers - 1):  # use_31_block: the last block is never run
            p = f"transformer.{i}."
            pk.layers.append(SimpleNamespace(
                n1w=f32(p + "norm1.weight"), n1b=f32(p + "norm1.bias"), w_qkv=bf(p + "attn.to_qkv.weight"),
                b_qkv=f32(p + "attn.to_qkv.bias"), w_o=bf(p + "attn.proj.weight"), b_o=f32(p + "attn.proj.bias"),
                n2w=f32(p + "norm2.weight"), n2b=f32(p + "norm2.bias"), w_f1=bf(p + "mlp.0.weight"),
                b_f1=f32(p + "mlp.0.bias"), w_f2=bf(p + "mlp.2.weight"), b_f2=f32(p + "mlp.2.bias")))
        self._packed = pk
        return pk

    def _encode_image(self, pk, img):
        """img fp32 [3, H, W] in [-1, 1] -> fp32 [tokens, dim]"""
        dev = pk.w_pe.device
        S, Pz, dim, Hn = self.image_size, self.patch, self.dim, self.num_heads
        st = ops._stream()
        pre = torch.empty(3, S, S, device=dev, dtype=torch.float32)
        call("sa_clip_preprocess", img.data_ptr(), 3, img.shape[1], img.shape[2], pre.data_ptr(), S,
             pk.mean.data_ptr(), pk.std.data_ptr(), st)
        n = (S // Pz) ** 2 + 1
        cols = torch.empty(n, pk.kpad, device=dev, dtype=torch.bfloat16)
        call("sa_clip_patch_im2col", pre.data_ptr(), 3, S, Pz, cols.data_ptr(), pk.kpad, st)
        x = torch.empty(n, dim, device=dev, dtype=torch.float32)
        ops.linear(cols, pk.w_pe, None, ops.EPI_RES_F32, out=x, residual=pk.pos)  # + class token + positions
        ops.layernorm_mod(x, x, 1e-5, weight=pk.pre_w, bias=pk.pre_b)
        h = torch.empty(n, dim, device=dev, dtype=torch.bfloat16)
        o = torch.empty(n, dim, device=dev, dtype=torch.bfloat16)
        segs = torch.tensor([[0, n, 0, n]], dtype=torch.int32).to(dev)
        d = dim // Hn
        for Ly in pk.layers:
            ops.layernorm_mod(x, h, 1e-5, weight=Ly.n1w, bias=Ly.n1b)
            qkv = ops.linear(h, Ly.w_qkv, Ly.b_qkv, ops.EPI_BF16)
            ops.attention_small(qkv[:, :dim], qkv[:, dim:2 * dim], qkv[:, 2 * dim:], o, segs, 1, n, n, Hn, d)
            ops.linear(o, Ly.w_o, Ly.b_o, ops.EPI_RES_F32, out=x, residual=x)
            ops.layernorm_mod(x, h, 1e-5, weight=Ly.n2w, bias=Ly.n2b)
            m = ops.linear(h, Ly.w_f1, Ly.b_f1, ops.EPI_GELU_ERF_BF16)
            ops.linear(m, Ly.w_f2, Ly.b_f2, ops.EPI_RES_F32, out=x, residual=x)
        return x

    def forward(self, videos):
        """videos: list of [C, F, H, W] in [-1, 1] (the pipeline passes one [3, 1, H, W] reference frame,
        pipeline:665-678) -> [sum F, 1 + (224/14)^2, dim] fp32 (visual(x, use_31_block=True))."""
        pk = self._pack()
        dev = pk.w_pe.device
        outs = []
        for u in videos:
            for f in range(u.shape[1]):
                img = u[:, f].to(device=dev, dtype=torch.float32).contiguous()
                outs.append(self._encode_image(pk, img))
        return torch.stack(outs)
