"""Drop-in WanTransformer3DFantasyModel for MI355X (reference:
wan/models/wan_fantasy_transformer3d_1B.py + wan/models/vocal_projector_fantasy_1B.py).

Same constructor arguments, state_dict keys, `from_pretrained(...)` and
`forward(x, t, context, seq_len, clip_fea, y, cond_flag, vocal_embeddings, is_clip_level_modeling,
video_sample_n_frames)` as the reference; every op of the forward runs as a HIP kernel from
libstableavatar_hip.so (there is no eager/CPU fallback).

Residual stream is kept in fp32 ([B*L, dim], rows = batch-major tokens), GEMM operands in bf16,
norms/softmax/RoPE in fp32.  Weights are re-packed once per load into fused layouts:
self-attn QKV [3*dim, dim]; cross-attn text/img/vocal K|V [2*dim, dim]; patch embedding as a
[dim, 192] GEMM (K padded from 144).  Step-invariant cross-attention K/V of the text and image
context are cached across forwards (they depend only on the prompt and reference image).
"""
from __future__ import annotations

import glob
import json
import math
import os
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import ops, sp


def rope_params(max_seq_len: int, dim: int, theta: float = 10000.0) -> torch.Tensor:
    """Angles of rope_params (1B:223-231) in fp64: [max_seq_len, dim/2]."""
    return torch.outer(torch.arange(max_seq_len, dtype=torch.float64),
                       1.0 / torch.pow(theta, torch.arange(0, dim, 2, dtype=torch.float64).div(dim)))


def riflex_params(max_seq_len: int, dim: int, k: int, L_test: int, L_test_scale=None,
                  theta: float = 10000.0) -> torch.Tensor:
    """Angles of get_1d_rotary_pos_embed_riflex (1B:236-291) in fp64: rope_params with the k-th
    intrinsic frequency replaced by 0.9 * 2 pi / L_test (then divided by L_test_scale)."""
    freqs = 1.0 / torch.pow(theta, torch.arange(0, dim, 2, dtype=torch.float64).div(dim))
    freqs[k - 1] = 0.9 * 2 * math.pi / L_test
    if L_test_scale is not None:
        freqs[k - 1] = freqs[k - 1] / L_test_scale
    return torch.outer(torch.arange(max_seq_len, dtype=torch.float64), freqs)


def rope_table(head_dim: int = 128, max_seq_len: int = 1024, riflex=None) -> torch.Tensor:
    """fp32 (cos, sin) table [max_seq_len, head_dim/2, 2] of the concatenated frame/height/width
    frequencies of self.freqs (1B:855-862), computed in fp64 like the reference.  riflex = (k, L_test,
    L_test_scale) swaps the frame axis for RIFLEx's frequencies (enable_riflex, 1B:890-905)."""
    d = head_dim
    df = d - 4 * (d // 6)
    frame = rope_params(max_seq_len, df) if riflex is None else riflex_params(max_seq_len, df, *riflex)
    ang = torch.cat([frame, rope_params(max_seq_len, 2 * (d // 6)), rope_params(max_seq_len, 2 * (d // 6))], dim=1)
    return torch.stack([torch.cos(ang), torch.sin(ang)], -1).float().contiguous()


def split_audio_sequence(audio_proj_length, num_frames=81):
    """vocal_projector_fantasy.py:39-78 (same integer arithmetic)."""
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


def split_rows(audio_len, num_frames, expand_length=4):
    """Gather table of split_tensor_with_padding (vocal_projector_fantasy.py:81-131): per latent
    frame the source token rows, then -1 (zero rows) for front AND back padding, both appended."""
    rows = []
    for s, e in split_audio_sequence(audio_len, num_frames):
        s, e = s - expand_length, e + expand_length
        mx = audio_len - 1
        pad = max(-s, 0) + max(e - mx, 0)
        vs, ve = max(s, 0), min(e, mx)
        rows.append((list(range(vs, ve + 1)) if vs <= ve else []) + [-1] * pad)
    return rows


def vocal_dim(cfg: dict) -> int:
    """width of the vocal projector: 1536 for the 1.3B model (1B:872), the DiT width for 14B (14B:866)"""
    return cfg["dim"] if cfg.get("vocal", "1B") == "14B" else 1536


def param_shapes(cfg: dict) -> dict:
    """{state_dict key: shape} of the reference WanTransformer3DFantasyModel (1B:829-872), or of
    WanTransformer3DFantasy14BModel (14B:823-866) with cfg["vocal"] = "14B"."""
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
    if cfg.get("model_type", "i2v") == "i2v":
        S.update({"img_emb.proj.0.weight": (1280,), "img_emb.proj.0.bias": (1280,),
                  "img_emb.proj.1.weight": (1280, 1280), "img_emb.proj.1.bias": (1280,),
                  "img_emb.proj.3.weight": (dim, 1280), "img_emb.proj.3.bias": (dim,),
                  "img_emb.proj.4.weight": (dim,), "img_emb.proj.4.bias": (dim,)})
    vp = "vocal_projector"
    # 1.3B: FantasyTalkingVocalCondition1BModel(audio_proj_dim=1536) (1B:872, vocal_projector_fantasy_1B.py:
    # 389-431); 14B: audio_proj_dim = dim and a two-layer audio projection 768 -> 2048 -> dim (14B:866,
    # vocal_projector_fantasy_14B.py:385-425); both: 2 blocks of 8 heads, ffn 2 x width, final head
    vd = vocal_dim(cfg)
    if cfg.get("vocal", "1B") == "14B":
        S[vp + ".proj_model.proj_1.weight"] = (2048, 768)
        S[vp + ".proj_model.norm_1.weight"] = (2048,)
        S[vp + ".proj_model.norm_1.bias"] = (2048,)
        S[vp + ".proj_model.proj_2.weight"] = (vd, 2048)
        S[vp + ".proj_model.norm_2.weight"] = (vd,)
        S[vp + ".proj_model.norm_2.bias"] = (vd,)
    else:
        S[vp + ".proj_model.proj.weight"] = (vd, 768)
        S[vp + ".proj_model.norm.weight"] = (vd,)
        S[vp + ".proj_model.norm.bias"] = (vd,)
    for i in range(2):
        bp = f"{vp}.blocks.{i}"
        S[bp + ".modulation"] = (1, 6, vd)
        S[bp + ".norm3.weight"] = (vd,)
        S[bp + ".norm3.bias"] = (vd,)
        for n in ("q", "o"):
            S[f"{bp}.cross_attn.{n}.weight"] = (vd, vd)
            S[f"{bp}.cross_attn.{n}.bias"] = (vd,)
        for n in ("k", "v"):
            S[f"{bp}.cross_attn.{n}.weight"] = (vd, dim)
            S[f"{bp}.cross_attn.{n}.bias"] = (vd,)
        S[bp + ".cross_attn.norm_q.weight"] = (vd,)
        S[bp + ".cross_attn.norm_k.weight"] = (vd,)
        S[bp + ".ffn.0.weight"] = (2 * vd, vd)
        S[bp + ".ffn.0.bias"] = (2 * vd,)
        S[bp + ".ffn.2.weight"] = (vd, 2 * vd)
        S[bp + ".ffn.2.bias"] = (vd,)
    S[vp + ".final_head.modulation"] = (1, 2, vd)
    S[vp + ".final_head.final_proj.weight"] = (vd, vd)
    S[vp + ".final_head.final_proj.bias"] = (vd,)
    return S


def _register_tree(root: nn.Module, shapes: dict, dtype):
    for name, shp in shapes.items():
        *path, leaf = name.split(".")
        mod = root
        for p in path:
            if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                mod.add_module(p, nn.Module())
            mod = getattr(mod, p)
        mod.register_parameter(leaf, nn.Parameter(torch.empty(shp, dtype=dtype), requires_grad=False))


class _Seg:
    """Cache of device segment tables {q_row0, q_len, kv_row0, kv_len} for sa_attn_fwd."""

    def __init__(self):
        self._c = {}

    def get(self, key, rows, device):
        t = self._c.get(key)
        if t is None or t.device != device:
            t = torch.tensor(rows, dtype=torch.int32).reshape(-1, 4).to(device)
            self._c[key] = t
        return t


class WanTransformer3DFantasyModel(nn.Module):
    """Audio-driven Wan-2.1 DiT (1B:741-1184) on HIP kernels."""

    VOCAL = "1B"  # vocal projector family (param_shapes)

    def __init__(self, model_type="i2v", patch_size=(1, 2, 2), text_len=512, in_dim=16, dim=2048, ffn_dim=8192,
                 freq_dim=256, text_dim=4096, out_dim=16, num_heads=16, num_layers=32, window_size=(-1, -1),
                 qk_norm=True, cross_attn_norm=True, eps=1e-6, in_channels=16, hidden_size=2048, **_):
        super().__init__()
        assert model_type in ("t2v", "i2v")
        if tuple(patch_size) != (1, 2, 2) or not qk_norm or not cross_attn_norm:
            raise ValueError("the StableAvatar path uses patch (1,2,2), qk_norm and cross_attn_norm (1B:1234-1237)")
        if tuple(window_size) != (-1, -1):
            raise ValueError("windowed attention is not part of the inference path")
        assert dim % num_heads == 0 and dim // num_heads == 128, "HIP attention kernel is built for head_dim 128"
        self.model_type = model_type
        self.patch_size = tuple(patch_size)
        self.text_len, self.in_dim, self.dim, self.ffn_dim = text_len, in_dim, dim, ffn_dim
        self.freq_dim, self.text_dim, self.out_dim = freq_dim, text_dim, out_dim
        self.num_heads, self.num_layers, self.eps = num_heads, num_layers, eps
        self.d = dim // num_heads
        self.config = SimpleNamespace(model_type=model_type, patch_size=self.patch_size, text_len=text_len,
                                      in_dim=in_dim, dim=dim, ffn_dim=ffn_dim, freq_dim=freq_dim, text_dim=text_dim,
                                      out_dim=out_dim, num_heads=num_heads, num_layers=num_layers,
                                      window_size=window_size, qk_norm=qk_norm, cross_attn_norm=cross_attn_norm,
                                      eps=eps, in_channels=in_channels, hidden_size=hidden_size)
        self._cfg = dict(model_type=model_type, dim=dim, ffn_dim=ffn_dim, freq_dim=freq_dim, text_dim=text_dim,
                         in_dim=in_dim, out_dim=out_dim, num_heads=num_heads, num_layers=num_layers,
                         text_len=text_len, vocal=self.VOCAL)
        self.vd = vocal_dim(self._cfg)
        _register_tree(self, param_shapes(self._cfg), torch.float32)
        self.sp_world_size, self.sp_world_rank, self.sp_group = 1, 0, None
        self.teacache = None  # enable_teacache() (1B:867)
        self._riflex = None  # enable_riflex() (1B:890-905)
        self.attn_kernel = 0  # self-attention schedule (sa_attn_fwd_ex; 0 = auto), for in-situ A/B
        self._packed = None
        self._ws = {}
        self._ctx_cache = None
        self._segs = _Seg()
        self._sp_ex = None
        self._split_cache = {}
        self._events = None  # optional list to record (start, end) events around self-attention
        self._sp_enabled = False
        self._sp_loopback = False

    # ------------------------------------------------------------------ loading

    @classmethod
    def from_config(cls, config, **kw):
        import inspect
        p = set(inspect.signature(cls.__init__).parameters) - {"self"}
        return cls(**{k: v for k, v in {**config, **kw}.items() if k in p})

    @classmethod
    def from_pretrained(cls, pretrained_model_path, subfolder=None, transformer_additional_kwargs={},
                        low_cpu_mem_usage=False, torch_dtype=torch.bfloat16):
        """Same directory contract as 1B:1210-1339: config.json + diffusion_pytorch_model
        .bin/.safetensors or sharded *.safetensors; dict_mapping; forced patch/qk/cross norms;
        size-mismatched keys skipped; patch_embedding in_dim widening zero-filled."""
        if subfolder is not None:
            pretrained_model_path = os.path.join(pretrained_model_path, subfolder)
        cfg_file = os.path.join(pretrained_model_path, "config.json")
        if not os.path.isfile(cfg_file):
            raise RuntimeError(f"{cfg_file} does not exist")
        with open(cfg_file) as f:
            config = json.load(f)
        kw = dict(transformer_additional_kwargs)
        for key, target in kw.pop("dict_mapping", {}).items():
            kw[target] = config[key]
        kw.update(patch_size=(1, 2, 2), qk_norm=True, window_size=(-1, -1), cross_attn_norm=True)
        model = cls.from_config(config, **kw)
        bin_file = os.path.join(pretrained_model_path, "diffusion_pytorch_model.bin")
        st_file = bin_file.replace(".bin", ".safetensors")
        if os.path.exists(bin_file):
            sd = torch.load(bin_file, map_location="cpu", weights_only=True)
        else:
            from safetensors.torch import load_file
            files = [st_file] if os.path.exists(st_file) else sorted(
                glob.glob(os.path.join(pretrained_model_path, "*.safetensors")))
            sd = {}
            for fn in files:
                sd.update(load_file(fn))
        own = model.state_dict()
        pe = "patch_embedding.weight"
        if pe in sd and sd[pe].shape != own[pe].shape and sd[pe].shape[1] < own[pe].shape[1]:
            w = torch.zeros(own[pe].shape, dtype=sd[pe].dtype)
            w[:, :sd[pe].shape[1]] = sd[pe]
            sd[pe] = w
        sd = {k: v for k, v in sd.items() if k in own and own[k].shape == v.shape}
        model.load_state_dict(sd, strict=False)
        return model.to(torch_dtype)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._packed = None
        self._ctx_cache = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):
        self._packed = None
        self._ctx_cache = None
        self._ws = {}
        return super()._apply(fn, recurse)

    def enable_riflex(self, k=6, L_test=66, L_test_scale=4.886):
        """1B:890-905: RIFLEx frame frequencies for length extrapolation."""
        self._riflex = (k, L_test, L_test_scale)
        self._set_rope()

    def disable_riflex(self):
        """1B:907-916."""
        self._riflex = None
        self._set_rope()

    def _set_rope(self):
        if self._packed is not None:
            self._packed.rope = rope_table(self.d, riflex=self._riflex).to(self._packed.rope.device)

    def enable_teacache(self, coefficients, num_steps: int, rel_l1_thresh: float, num_skip_start_steps: int = 0,
                        offload: bool = True):
        """1B:874-885 (inference.py:526-535)."""
        from .teacache import TeaCache
        self.teacache = TeaCache(coefficients, num_steps, rel_l1_thresh=rel_l1_thresh,
                                 num_skip_start_steps=num_skip_start_steps, offload=offload)

    def disable_teacache(self):
        self.teacache = None

    def enable_multi_gpus_inference(self, group=None, loopback=None):
        """Ulysses sequence parallelism over torch.distributed (RCCL); replaces the xfuser path
        installed at 1B:918-923 with single-GPU semantics.  loopback=True (default: env
        SA_SP_LOOPBACK=1) also sends this rank's own token chunk through the point-to-point transport (a transfer
        to itself), so at degree 1 every exchange of the layer runs on RCCL; the output is unchanged."""
        import torch.distributed as dist
        self.sp_group = group
        self.sp_world_size = dist.get_world_size(group)
        self.sp_world_rank = dist.get_rank(group)
        self._sp_enabled = True  # the exchange path runs even at degree 1 (pack + row-mapped attention + panels)
        self._sp_loopback = (os.environ.get("SA_SP_LOOPBACK", "0") == "1") if loopback is None else bool(loopback)

    def disable_multi_gpus_inference(self):
        """back to single-GPU forwards (every rank its own clip)"""
        self.sp_group, self.sp_world_size, self.sp_world_rank = None, 1, 0
        self._sp_enabled = False

    # ------------------------------------------------------------------ packing

    def _pack(self):
        if self._packed is not None:
            return self._packed
        dev = self.patch_embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("WanTransformer3DFantasyModel runs on the MI355X HIP kernels: move it to 'cuda'")
        # parameters stored as float8_e4m3fn by the reference's qfloat8 memory mode
        # (wan/utils/fp8_optimization.py:29-43, inference.py:517-518) are upcast exactly before packing
        fp8 = (torch.float8_e4m3fn, torch.float8_e5m2)
        P = {k: (v.detach().float() if v.dtype in fp8 else v) for k, v in self.named_parameters()}
        bf = lambda n: P[n].detach().to(torch.bfloat16).contiguous()  # noqa: E731
        f32 = lambda n: P[n].detach().float().contiguous()  # noqa: E731
        cat_bf = lambda *ns: torch.cat([P[n].detach() for n in ns], 0).to(torch.bfloat16).contiguous()  # noqa: E731
        cat_f = lambda *ns: torch.cat([P[n].detach() for n in ns], 0).float().contiguous()  # noqa: E731
        dim = self.dim
        pk = SimpleNamespace()
        kin = self.in_dim * 4
        pk.kpad = ((kin + 63) // 64) * 64
        wpe = torch.zeros(dim, pk.kpad, device=dev, dtype=torch.bfloat16)
        wpe[:, :kin] = P["patch_embedding.weight"].detach().reshape(dim, kin).to(torch.bfloat16)
        pk.w_pe, pk.b_pe = wpe, f32("patch_embedding.bias")
        tkpad = ((self.text_dim + 63) // 64) * 64
        pk.text_kpad = tkpad
        w0 = torch.zeros(dim, tkpad, device=dev, dtype=torch.bfloat16)
        w0[:, :self.text_dim] = P["text_embedding.0.weight"].detach().to(torch.bfloat16)
        pk.w_t0, pk.b_t0 = w0, f32("text_embedding.0.bias")
        pk.w_t2, pk.b_t2 = bf("text_embedding.2.weight"), f32("text_embedding.2.bias")
        pk.w_te0, pk.b_te0 = bf("time_embedding.0.weight"), f32("time_embedding.0.bias")
        pk.w_te2, pk.b_te2 = bf("time_embedding.2.weight"), f32("time_embedding.2.bias")
        pk.w_tp, pk.b_tp = bf("time_projection.1.weight"), f32("time_projection.1.bias")
        pk.mod = torch.cat([P[f"blocks.{i}.modulation"].detach() for i in range(self.num_layers)], 0).float().contiguous()
        pk.layers = []
        # per-frame vocal K|V weights of every block stacked [layers * 2 * dim, vd]: the vocal context is the same for
        # all blocks of a forward, so one GEMM forms every block's vocal keys and values (L.w_kv_v are views)
        pk.w_kv_v_all = torch.cat([P[f"blocks.{i}.cross_attn.{n}_vocal.weight"].detach() for i in range(self.num_layers)
                                   for n in ("k", "v")], 0).to(torch.bfloat16).contiguous()
        pk.b_kv_v_all = torch.cat([P[f"blocks.{i}.cross_attn.{n}_vocal.bias"].detach() for i in range(self.num_layers)
                                   for n in ("k", "v")], 0).float().contiguous()
        for i in range(self.num_layers):
            p = f"blocks.{i}."
            L = SimpleNamespace()
            L.w_qkv = cat_bf(p + "self_attn.q.weight", p + "self_attn.k.weight", p + "self_attn.v.weight")
            L.b_qkv = cat_f(p + "self_attn.q.bias", p + "self_attn.k.bias", p + "self_attn.v.bias")
            # views for the single-GPU V^T path: q|k rows into the QKV rows, v into V^T (EPI_BF16_TP32)
            L.w_qk, L.b_qk = L.w_qkv[:2 * self.dim], L.b_qkv[:2 * self.dim]
            L.w_v, L.b_v = L.w_qkv[2 * self.dim:], L.b_qkv[2 * self.dim:]
            L.nq, L.nk = f32(p + "self_attn.norm_q.weight"), f32(p + "self_attn.norm_k.weight")
            L.w_o, L.b_o = bf(p + "self_attn.o.weight"), f32(p + "self_attn.o.bias")
            L.n3w, L.n3b = f32(p + "norm3.weight"), f32(p + "norm3.bias")
            c = p + "cross_attn."
            L.w_cq, L.b_cq = bf(c + "q.weight"), f32(c + "q.bias")
            L.cnq, L.cnk, L.cnki = f32(c + "norm_q.weight"), f32(c + "norm_k.weight"), f32(c + "norm_k_img.weight")
            L.w_kv_t, L.b_kv_t = cat_bf(c + "k.weight", c + "v.weight"), cat_f(c + "k.bias", c + "v.bias")
            L.w_kv_i, L.b_kv_i = cat_bf(c + "k_img.weight", c + "v_img.weight"), cat_f(c + "k_img.bias", c + "v_img.bias")
            L.w_kv_v, L.b_kv_v = pk.w_kv_v_all[2 * dim * i:2 * dim * (i + 1)], pk.b_kv_v_all[2 * dim * i:2 * dim * (i + 1)]
            L.w_co, L.b_co = bf(c + "o.weight"), f32(c + "o.bias")
            L.w_f0, L.b_f0 = bf(p + "ffn.0.weight"), f32(p + "ffn.0.bias")
            L.w_f2, L.b_f2 = bf(p + "ffn.2.weight"), f32(p + "ffn.2.bias")
            pk.layers.append(L)
        pk.head_mod = f32("head.modulation").reshape(1, 2, dim)
        pk.w_head, pk.b_head = bf("head.head.weight"), f32("head.head.bias")
        if self.model_type == "i2v":
            pk.ie0w, pk.ie0b = f32("img_emb.proj.0.weight"), f32("img_emb.proj.0.bias")
            pk.w_ie1, pk.b_ie1 = bf("img_emb.proj.1.weight"), f32("img_emb.proj.1.bias")
            pk.w_ie3, pk.b_ie3 = bf("img_emb.proj.3.weight"), f32("img_emb.proj.3.bias")
            pk.ie4w, pk.ie4b = f32("img_emb.proj.4.weight"), f32("img_emb.proj.4.bias")
        vp = "vocal_projector."
        V = SimpleNamespace()
        if self.VOCAL == "14B":  # two-layer audio projection (vocal_projector_fantasy_14B.py:385-398)
            V.proj = [(bf(vp + "proj_model.proj_1.weight"), f32(vp + "proj_model.norm_1.weight"),
                       f32(vp + "proj_model.norm_1.bias")),
                      (bf(vp + "proj_model.proj_2.weight"), f32(vp + "proj_model.norm_2.weight"),
                       f32(vp + "proj_model.norm_2.bias"))]
        else:
            V.proj = [(bf(vp + "proj_model.proj.weight"), f32(vp + "proj_model.norm.weight"),
                       f32(vp + "proj_model.norm.bias"))]
        V.mod = torch.cat([P[f"{vp}blocks.{i}.modulation"].detach() for i in range(2)], 0).float().contiguous()
        V.blocks = []
        for i in range(2):
            b = f"{vp}blocks.{i}."
            B_ = SimpleNamespace()
            B_.n3w, B_.n3b = f32(b + "norm3.weight"), f32(b + "norm3.bias")
            B_.w_q, B_.b_q = bf(b + "cross_attn.q.weight"), f32(b + "cross_attn.q.bias")
            B_.w_kv = cat_bf(b + "cross_attn.k.weight", b + "cross_attn.v.weight")
            B_.b_kv = cat_f(b + "cross_attn.k.bias", b + "cross_attn.v.bias")
            B_.nq, B_.nk = f32(b + "cross_attn.norm_q.weight"), f32(b + "cross_attn.norm_k.weight")
            B_.w_o, B_.b_o = bf(b + "cross_attn.o.weight"), f32(b + "cross_attn.o.bias")
            B_.w_f0, B_.b_f0 = bf(b + "ffn.0.weight"), f32(b + "ffn.0.bias")
            B_.w_f2, B_.b_f2 = bf(b + "ffn.2.weight"), f32(b + "ffn.2.bias")
            V.blocks.append(B_)
        V.fmod = f32(vp + "final_head.modulation").reshape(1, 2, self.vd)
        V.w_fp, V.b_fp = bf(vp + "final_head.final_proj.weight"), f32(vp + "final_head.final_proj.bias")
        pk.vocal = V
        pk.rope = rope_table(self.d, riflex=self._riflex).to(dev)
        self._packed = pk
        return pk

    # ------------------------------------------------------------------ workspace

    def _workspace(self, M, dev):
        key = (M, dev)
        ws = self._ws.get(key)
        if ws is None:
            dim = self.dim
            ws = SimpleNamespace(
                x=torch.empty(M, dim, device=dev, dtype=torch.float32),
                mod=torch.empty(M, dim, device=dev, dtype=torch.bfloat16),
                qkv=torch.empty(M, 3 * dim, device=dev, dtype=torch.bfloat16),
                att=torch.empty(M, dim, device=dev, dtype=torch.bfloat16),
                ffn=torch.empty(M, self.ffn_dim, device=dev, dtype=torch.bfloat16),
                vt=None,  # V^T [dim, M rounded up to 64] of the single-GPU self-attention, allocated on first use
            )
            self._ws = {key: ws}  # keep one shape at a time
        return ws

    def _vt_attention(self, Lp, dev) -> bool:
        """the single-GPU self-attention reads V as V^T written by the QKV GEMM's transposed epilogue (attention
        kernel 3: 6.20 vs 6.41 ms per config-2 launch, bit-identical, profiles/r05/attn_ab_v6_v6t_v12_r5b.jsonl)
        when the batch rows start on 32-key boundaries; SA_ATTN_VT=0 or an explicit attn_kernel keeps V in rows"""
        return (dev.type == "cuda" and self.attn_kernel == 0 and Lp % 32 == 0
                and os.environ.get("SA_ATTN_VT", "1") != "0")

    # ------------------------------------------------------------------ context (step-invariant)

    def invalidate_context(self):
        """drop the cached text / image K/V (the pipeline calls this at the start of every denoise)"""
        self._ctx_cache = None

    def _sp_exchange(self, plan, B, Lc, dev):
        """the sequence-parallel exchange buffers (attention inputs, send slabs, output / panel buffer, pack
        table, output row map) for this shape, kept across layers, steps and calls (one shape at a time)"""
        key = (plan, B, Lc, self.d, str(dev), id(self.sp_group), self._sp_loopback)
        ex = self._sp_ex
        if ex is None or ex[0] != key:
            self._sp_ex = None  # free the previous shape's buffers first
            ex = self._sp_ex = (key, sp.UlyssesExchange(plan, B, Lc, self.d, dev, self.sp_group,
                                                        loopback=self._sp_loopback))
        return ex[1]

    @staticmethod
    def _ctx_key(context, clip_fea):
        """(tensor, version) of every context input.  The cache holds the tensors themselves and matches
        by identity, so a hit cannot come from a new tensor the caching allocator placed at a freed
        address (an address key could return the previous call's prompt / image K/V)."""
        return tuple((c, c._version) for c in context) + (((clip_fea, clip_fea._version),)
                                                          if clip_fea is not None else ())

    def _context(self, pk, context, clip_fea, B, dev):
        key = self._ctx_key(context, clip_fea)
        if self._ctx_cache is not None:
            old = self._ctx_cache[0]
            if len(old) == len(key) and all(a is c and va == vc for (a, va), (c, vc) in zip(old, key)):
                return self._ctx_cache[1]
            self._ctx_cache = None  # release the previous call's tensors and K/V before building new ones
        dim, tl = self.dim, self.text_len
        # text: pad each prompt to text_len with zeros (the pads are attended, 1B:993-999)
        tin = torch.zeros(B, tl, pk.text_kpad, device=dev, dtype=torch.bfloat16)
        for b, c in enumerate(context):
            tin[b, :c.shape[0], :c.shape[1]] = c.to(device=dev, dtype=torch.bfloat16)
        h = ops.linear(tin.view(B * tl, pk.text_kpad), pk.w_t0, pk.b_t0, ops.EPI_GELU_TANH_BF16)
        ctx_t = ops.linear(h, pk.w_t2, pk.b_t2, ops.EPI_BF16)
        # image: MLPProj (1B:726-738): LN(1280) -> Linear -> GELU(erf) -> Linear -> LN(dim)
        ni = 0
        if self.model_type == "i2v":
            ni = clip_fea.shape[1]
            cf = clip_fea.to(device=dev, dtype=torch.float32).reshape(B * ni, -1).contiguous()
            cn = torch.empty(B * ni, cf.shape[1], device=dev, dtype=torch.bfloat16)
            ops.layernorm_mod(cf, cn, 1e-5, weight=pk.ie0w, bias=pk.ie0b)
            h1 = ops.linear(cn, pk.w_ie1, pk.b_ie1, ops.EPI_GELU_ERF_BF16)
            h3 = ops.linear(h1, pk.w_ie3, pk.b_ie3, ops.EPI_F32)
            ctx_i = torch.empty(B * ni, dim, device=dev, dtype=torch.bfloat16)
            ops.layernorm_mod(h3, ctx_i, 1e-5, weight=pk.ie4w, bias=pk.ie4b)
        kv = []
        for L in pk.layers:
            kvt = ops.linear(ctx_t, L.w_kv_t, L.b_kv_t, ops.EPI_BF16)      # [B*tl, 2dim] = k | v
            ops.qk_rmsnorm_rope(kvt, 0, -1, L.cnk, None, dim, self.eps)
            kvi = None
            if ni:
                kvi = ops.linear(ctx_i, L.w_kv_i, L.b_kv_i, ops.EPI_BF16)
                ops.qk_rmsnorm_rope(kvi, 0, -1, L.cnki, None, dim, self.eps)
            kv.append((kvt, kvi))
        out = SimpleNamespace(kv=kv, text_len=tl, img_len=ni)
        self._ctx_cache = (key, out)
        return out

    # ------------------------------------------------------------------ vocal projector

    def _vocal(self, pk, vocal_embeddings, n_frames, lat_bf16, Lq, e0_row, e_row, dev, frames=None):
        """FantasyTalkingVocalCondition{1B,14B}Model.forward (vocal_projector_fantasy_1B.py:433-450,
        _14B.py:431-449) for one audio row; lat_bf16 = patch-embedded tokens of that row [Lq, dim].
        Returns [F*n, vd] bf16 (vd = 1536 for 1.3B, the DiT width for 14B).
        frames = (f0, nf): latent frames f0 .. f0+nf-1 only (lat_bf16 then holds just their tokens, and the result is
        [nf*n, vd]).  Every op of the projector is per row except the attention, whose queries of frame f attend only
        to frame f's tokens (:259-270), so these rows equal those of the whole projector bit for bit: a
        sequence-parallel rank computes the frames its token chunk covers."""
        V, vd = pk.vocal, self.vd
        hdv = vd // 8  # 8 heads: D = 192 (1.3B) or 640 (14B)
        feat = vocal_embeddings.to(device=dev, dtype=torch.bfloat16).contiguous()
        Na = feat.shape[0]
        for j, (w, nw, nb) in enumerate(V.proj):  # Linear (no bias) + LayerNorm, once or twice
            f = ops.linear(feat, w, None, ops.EPI_F32)
            last = j == len(V.proj) - 1
            feat = ops.layernorm_mod(f, f if last else torch.empty(Na, f.shape[1], device=dev, dtype=torch.bfloat16),
                                     1e-5, weight=nw, bias=nb)
        key = (Na, n_frames)
        rows = self._split_cache.get(key)
        if rows is None:
            r = split_rows(Na, n_frames)
            rows = (torch.tensor([i for row in r for i in row], dtype=torch.int32, device=dev), len(r), len(r[0]))
            self._split_cache[key] = rows
        idx, Fn, nper = rows
        f0, nf = (0, Fn) if frames is None else frames
        Mv = nf * nper
        x = torch.empty(Mv, vd, device=dev, dtype=torch.float32)
        ops.gather_rows(feat, idx[f0 * nper:(f0 + nf) * nper], x)
        em = torch.empty(2, 1, 6, vd, device=dev, dtype=torch.float32)
        ops.mod_add(V.mod, e0_row, em)
        hb = torch.empty(Mv, vd, device=dev, dtype=torch.bfloat16)
        G = Lq // Fn
        assert lat_bf16.shape[0] == nf * G
        segs = self._segs.get(("vp", nf, nper, G), [[f * nper, nper, f * G, G] for f in range(nf)], dev)
        for i, B_ in enumerate(V.blocks):
            e = em[i, 0]
            # "self-attention" branch is x + modulate(LN(x))*e2 (vocal_projector_fantasy_1B.py:345-347)
            ops.layernorm_mod(x, x, 1e-6, shift=e[0:1], scale=e[1:2], gate=e[2:3], rows_per_batch=Mv)
            ops.layernorm_mod(x, hb, 1e-6, weight=B_.n3w, bias=B_.n3b)
            q = ops.linear(hb, B_.w_q, B_.b_q, ops.EPI_BF16)
            ops.qk_rmsnorm_rope(q, 0, -1, B_.nq, None, vd, 1e-6)
            kv = ops.linear(lat_bf16, B_.w_kv, B_.b_kv, ops.EPI_BF16)
            ops.qk_rmsnorm_rope(kv, 0, -1, B_.nk, None, vd, 1e-6)
            o = torch.empty(Mv, vd, device=dev, dtype=torch.bfloat16)
            ops.attention_small(q, kv[:, :vd], kv[:, vd:], o, segs, nf, nper, G, 8, hdv)
            ops.linear(o, B_.w_o, B_.b_o, ops.EPI_RES_F32, out=x, residual=x)
            ops.layernorm_mod(x, hb, 1e-6, shift=e[3:4], scale=e[4:5], rows_per_batch=Mv)
            h = ops.linear(hb, B_.w_f0, B_.b_f0, ops.EPI_GELU_TANH_BF16)
            ops.linear(h, B_.w_f2, B_.b_f2, ops.EPI_RES_F32, out=x, residual=x, gate=e[5:6], rows_per_batch=Mv)
        ef = torch.empty(1, 1, 2, vd, device=dev, dtype=torch.float32)
        ops.mod_add(V.fmod, e_row, ef, e_jstride=0)
        ops.layernorm_mod(x, hb, 1e-6, shift=ef[0, 0, 0:1], scale=ef[0, 0, 1:2], rows_per_batch=Mv)
        return ops.linear(hb, V.w_fp, V.b_fp, ops.EPI_BF16), Fn, nper

    # ------------------------------------------------------------------ sequence parallel, one stream per CFG row

    def _row_streams(self, B, dev):
        """B HIP streams (one per CFG row) for the SP_OVERLAP=4 layer schedule, kept per device"""
        st = getattr(self, "_rstreams", None)
        if st is None or len(st) < B or st[0].device != dev:
            st = self._rstreams = [torch.cuda.Stream(dev) for _ in range(B)]
        return st[:B]

    def _row_cross_segs(self, B, Lc, ctx, voc_list, dev):
        """per-row cross-attention segment tables (query rows relative to the row's chunk, key rows absolute in the
        shared text / image / vocal K|V buffers) for the three-launch path"""
        out = []
        for b in range(B):
            txt = self._segs.get(("rtxt", b, Lc, ctx.text_len), [[0, Lc, b * ctx.text_len, ctx.text_len]], dev)
            img = self._segs.get(("rimg", b, Lc, ctx.img_len), [[0, Lc, b * ctx.img_len, ctx.img_len]], dev)
            vl = [[q0 - b * Lc, ql, k0, kl] for q0, ql, k0, kl in voc_list if b * Lc <= q0 < (b + 1) * Lc]
            voc = self._segs.get(("rvoc", b, Lc, tuple(map(tuple, vl))), vl, dev)
            out.append((txt, img, voc, len(vl), max(s_[1] for s_ in vl)))
        return out

    def _sp_layer_rows(self, pk, L, li, x, ws, em, ex, pack_kw, rank, Lc, Lq, hg, hgd, grid, segs_rows, row_segs,
                       ctx, kvv, nper, Gf, n_fr, use_cross3, rstreams, sa=True):
        """One DiT block (1B:650-695) with Ulysses sequence parallelism, each CFG row on its own stream
        (SA_SP_OVERLAP=4): row b's Q/K/V exchange (wan_xfuser.py:102-107) travels while the other rows compute
        (their QKV GEMMs, attention, O-projection, cross-attention and FFN), and its head-output exchange travels
        under the other rows' attention and FFN.  The host issues the phases of the three rows interleaved
        (QKV+pack+send for every row, then attention+send back for every row, then the rest of the block), so the
        transport sees the same order of transfers on every rank.  Per-row kernels are the batched ones applied to
        row slices: the output is bit-identical to the batched schedule.  sa=False: the self-attention half already
        ran (_sp_self_attention_row0), the block starts at its cross-attention."""
        dim, H_, eps = self.dim, self.num_heads, self.eps
        B = len(rstreams)
        rope_kw = dict(rope=pk.rope, rows_per_batch=Lc, tok_offset=rank * Lc, grid=grid, head_dim=self.d,
                       n_frame_pairs=self.d // 2 - 2 * (self.d // 6), n_height_pairs=self.d // 6)
        tl, ni = ctx.text_len, ctx.img_len
        kvt, kvi = ctx.kv[li]
        nv = n_fr * nper
        pend, back = [], []
        # the rows' attention launches run concurrently: the tiles past their last full round over the CUs (in the
        # last row's launch) run as key halves (ops.attn_tail_split), all rows on the 8-wave kernel then
        n_row = hg * -(-Lq // 256)
        splits = [ops.attn_tail_split(b * n_row, n_row, x.device) if self.attn_kernel == 0 else 0 for b in range(B)]
        akern = 1 if any(splits) else self.attn_kernel
        for b, st in enumerate(rstreams if sa else []):  # self-attention inputs (1B:675-676) and the Q/K/V exchange
            rs = slice(b * Lc, (b + 1) * Lc)
            with torch.cuda.stream(st):
                ops.layernorm_mod(x[rs], ws.mod[rs], eps, shift=em[b:b + 1, 0], scale=em[b:b + 1, 1],
                                  rows_per_batch=Lc)
                ops.linear(ws.mod[rs], L.w_qkv, L.b_qkv, ops.EPI_BF16, out=ws.qkv[rs])
                ops.qkv_pack(ws.qkv[rs], L.nq, L.nk, dim, eps, b_offset=b, **pack_kw, **rope_kw)
                pend.append(ex.heads([b]))
        for b, st in enumerate(rstreams if sa else []):  # attention over every key, head outputs back to the owners
            with torch.cuda.stream(st):
                pend[b].wait()
                ev0 = self._record_event()
                ops.attention(ex.q, ex.kv[:, :hgd], ex.kv[:, hgd:], ex.obuf, segs_rows[b], 1, Lq, hg,
                              kernel=akern, o_rows=ex.omap, split_tiles=splits[b])
                self._record_span(ev0, rows=1, batch=B)
                back.append(ex.tokens([b]))
        for b, st in enumerate(rstreams):  # O-projection + gated residual, cross-attention, FFN (1B:677-691)
            rs = slice(b * Lc, (b + 1) * Lc)
            xr, mod, att = x[rs], ws.mod[rs], ws.att[rs]
            with torch.cuda.stream(st):
                if sa:
                    back[b].wait()
                    a0, pnl = ex.panels(range(b, b + 1))
                    ops.linear(a0, L.w_o, L.b_o, ops.EPI_RES_F32, out=xr, residual=xr, gate=em[b:b + 1, 2],
                               rows_per_batch=Lc, a_panels=pnl)
                ops.layernorm_mod(xr, mod, eps, weight=L.n3w, bias=L.n3b)
                qc = ws.qkv[rs, :dim]
                ops.linear(mod, L.w_cq, L.b_cq, ops.EPI_BF16, out=qc)
                ops.qk_rmsnorm_rope(qc, 0, -1, L.cnq, None, dim, eps)
                kv_b = kvv[b * nv:(b + 1) * nv]
                if use_cross3:
                    kt, ki = kvt[b * tl:(b + 1) * tl], kvi[b * ni:(b + 1) * ni]
                    ops.attention_cross3(qc, kt[:, :dim], kt[:, dim:], tl, ki[:, :dim], ki[:, dim:], ni, kv_b[:, :dim],
                                         kv_b[:, dim:], nper, Gf, n_fr, att, 1, Lc, H_, tok_offset=rank * Lc)
                else:
                    s_txt, s_img, s_voc, n_voc, q_voc = row_segs[b]
                    ops.attention(qc, kvt[:, :dim], kvt[:, dim:], att, s_txt, 1, Lc, H_)
                    if kvi is not None:
                        ops.attention(qc, kvi[:, :dim], kvi[:, dim:], att, s_img, 1, Lc, H_, accumulate=True)
                    ops.attention(qc, kvv[:, :dim], kvv[:, dim:], att, s_voc, n_voc, q_voc, H_, accumulate=True)
                ops.linear(att, L.w_co, L.b_co, ops.EPI_RES_F32, out=xr, residual=xr)
                ops.layernorm_mod(xr, mod, eps, shift=em[b:b + 1, 3], scale=em[b:b + 1, 4], rows_per_batch=Lc)
                ops.linear(mod, L.w_f0, L.b_f0, ops.EPI_GELU_TANH_BF16, out=ws.ffn[rs])
                ops.linear(ws.ffn[rs], L.w_f2, L.b_f2, ops.EPI_RES_F32, out=xr, residual=xr, gate=em[b:b + 1, 5],
                           rows_per_batch=Lc)

    # ------------------------------------------------------------------ timing hooks (bench.py)

    def _sp_self_attention_row0(self, L, x, ws, em, ex, pack_kw, rope_kw, Lc, Lq, hg, hgd, seg0, B):
        """The first block's self-attention half (1B:675-679) for CFG row 0 through the Ulysses exchange (its Q/K/V
        and head outputs only), on the current stream, the residual stream then copied to rows 1..B-1: the CFG rows
        enter the block identical (forward_window shared_rows), and every rank takes this path together"""
        dim, eps = self.dim, self.eps
        rs = slice(0, Lc)
        ops.layernorm_mod(x[rs], ws.mod[rs], eps, shift=em[0:1, 0], scale=em[0:1, 1], rows_per_batch=Lc)
        ops.linear(ws.mod[rs], L.w_qkv, L.b_qkv, ops.EPI_BF16, out=ws.qkv[rs])
        ops.qkv_pack(ws.qkv[rs], L.nq, L.nk, dim, eps, b_offset=0, **pack_kw, **rope_kw)
        ex.heads([0]).wait()
        ev0 = self._record_event()
        ops.attention(ex.q, ex.kv[:, :hgd], ex.kv[:, hgd:], ex.obuf, seg0, 1, Lq, hg, kernel=self.attn_kernel,
                      o_rows=ex.omap)
        self._record_span(ev0, rows=1, batch=B)
        ex.tokens([0]).wait()
        a0, pnl = ex.panels(range(0, 1))
        ops.linear(a0, L.w_o, L.b_o, ops.EPI_RES_F32, out=x[rs], residual=x[rs], gate=em[0:1, 2], rows_per_batch=Lc,
                   a_panels=pnl)
        for b in range(1, B):
            x[b * Lc:(b + 1) * Lc].copy_(x[rs])

    def _self_attention_rows(self, pk, L, x, ws, em, nb, Lc, Lp, use_vt, rope_kw, dev, batch, normed=False):
        """The self-attention half of a block (1B:675-679) on the first nb CFG rows of the single-GPU layout: LN +
        modulate (unless `normed`), q|k (+ v as V^T for kernel 3, or q|k|v rows), RMSNorm + RoPE, attention,
        O-projection + gated residual into x"""
        dim, H_ = self.dim, self.num_heads
        r = slice(0, nb * Lc)
        xr, mod, qkv, att = x[r], ws.mod[r], ws.qkv[r], ws.att[r]
        if not normed:
            ops.layernorm_mod(xr, mod, self.eps, shift=em[:nb, 0], scale=em[:nb, 1], rows_per_batch=Lc)
        segs = self._segs.get(("self", nb, Lp), [[b * Lp, Lp, b * Lp, Lp] for b in range(nb)], dev)
        if use_vt:
            # q|k into the QKV rows, v straight into V^T (keys in P's order per 32) for attention kernel 3
            ops.linear(mod, L.w_qk, L.b_qk, ops.EPI_BF16, out=qkv[:, :2 * dim])
            ops.linear(mod, L.w_v, L.b_v, ops.EPI_BF16_TP32, out=ws.vt)
            ops.qk_rmsnorm_rope(qkv, 0, dim, L.nq, L.nk, dim, self.eps, **rope_kw)
            ev0 = self._record_event()
            ops.attention(qkv[:, :dim], qkv[:, dim:2 * dim], ws.vt, att, segs, nb, Lp, H_, kernel=ops.ATTN_VT_P32)
        else:
            ops.linear(mod, L.w_qkv, L.b_qkv, ops.EPI_BF16, out=qkv)
            ops.qk_rmsnorm_rope(qkv, 0, dim, L.nq, L.nk, dim, self.eps, **rope_kw)
            ev0 = self._record_event()
            ops.attention(qkv[:, :dim], qkv[:, dim:2 * dim], qkv[:, 2 * dim:], att, segs, nb, Lp, H_,
                          kernel=self.attn_kernel)
        self._record_span(ev0, rows=nb, batch=batch)
        ops.linear(att, L.w_o, L.b_o, ops.EPI_RES_F32, out=xr, residual=xr, gate=em[:nb, 2], rows_per_batch=Lc)

    def _record_event(self):
        """HIP event on the current stream (the one the attention kernel is launched on), or None."""
        if self._events is None:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _record_span(self, ev0, rows, batch):
        """close a self-attention span opened by _record_event; `rows` of the `batch` CFG rows ran in it"""
        if ev0 is None:
            return
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self._events.append((ev0, ev1, rows / batch))

    # ------------------------------------------------------------------ forward

    def forward(self, x, t, context, seq_len, clip_fea=None, y=None, cond_flag=True, vocal_embeddings=None,
                is_clip_level_modeling=False, video_sample_n_frames=81):
        """1B:928-1159.  x, y: [B, C, F, H, W] tensors (or lists of [C, F, H, W]); context: list of
        [L_i, text_dim]; t: [B]; vocal_embeddings: [B, N_audio, 768].  Returns [B, out_dim, F, H, W]
        (bf16)."""
        if isinstance(x, (list, tuple)):
            x = torch.stack(list(x))
        if isinstance(y, (list, tuple)):
            y = torch.stack(list(y))
        return self.forward_window(x, 0, False, x.shape[0], t, context, seq_len, clip_fea, y, vocal_embeddings,
                                   video_sample_n_frames, is_clip_level_modeling, cond_flag=cond_flag)

    def forward_window(self, lat, frame_offset, broadcast, B, t, context, seq_len, clip_fea, y, vocal_embeddings,
                       video_sample_n_frames=81, is_clip_level_modeling=False, out=None, cond_flag=True,
                       shared_rows=False):
        """Forward on frames [frame_offset, frame_offset + Fw) of `lat` ([B|1, C, T, H, W]); with
        broadcast=True one latent row feeds all B CFG rows (the pipeline's torch.cat([latents]*3)).
        shared_rows=True (with broadcast): the caller guarantees the B rows of y are equal too, as the pipeline's
        CFG batch has them (y tripled at wan_inference_long_pipeline.py:693-700, x at :730, t expanded at :733) --
        then every row's input to the first block's self-attention half (patch embedding, time modulation) is the
        same, and that half (1B:675-679) runs for one row and is copied to the others: bit-identical output."""
        if is_clip_level_modeling:
            raise NotImplementedError("clip-level audio modeling is a training mode (1B:1011-1015)")
        if self.model_type == "i2v":
            assert clip_fea is not None and y is not None
        # the patch-embedding Conv3d runs under the pipeline's bf16 autocast (pipeline:738): bf16 operands
        if lat.dtype != torch.bfloat16:
            lat = lat.to(torch.bfloat16)
        if y is not None and y.dtype != torch.bfloat16:
            y = y.to(torch.bfloat16)
        pk = self._pack()
        dev = pk.w_pe.device
        dim, H_ = self.dim, self.num_heads
        Fw = y.shape[2] if y is not None else lat.shape[2] - frame_offset
        Hh, Ww = lat.shape[3], lat.shape[4]
        hp, wp = Hh // 2, Ww // 2
        real = Fw * hp * wp
        NS, rank = self.sp_world_size, self.sp_world_rank
        SP = self._sp_enabled  # sequence-parallel path (NS ranks; at NS = 1 no transfer, the same kernels)
        S = int(seq_len)  # the single-GPU sequence (1B:983): these keys are attended, SP's extra pads are not
        Lp = sp.padded_len(S, NS)
        assert real <= S, "seq_len smaller than the token count"
        Lc = Lp // NS  # tokens of each CFG row held by this rank (all of them without SP)
        ws = self._workspace(B * Lc, dev)

        # patch embedding (1B:972-983): im2col + GEMM, padding rows zero; with SP every rank embeds
        # the whole sequence (the vocal projector reads it, 1B:1004-1009) and keeps its chunk (1B:1019)
        cols = torch.empty(B, Lp, pk.kpad, device=dev, dtype=torch.bfloat16)
        ops.patch_im2col(lat, y, B, Fw, Hh, Ww, cols, pk.kpad, Lp, x_frame_offset=frame_offset,
                         x_batch_broadcast=broadcast)
        xfull = ws.x if not SP else torch.empty(B * Lp, dim, device=dev, dtype=torch.float32)
        call_gemm_batched(cols, pk.w_pe, pk.b_pe, xfull, B, real, Lp, dim, pk.kpad)
        if real < Lp:
            for b in range(B):
                ops.fill_(xfull[b * Lp + real:(b + 1) * Lp], 0.0)
        if SP:
            ws.x.view(B, Lc, dim).copy_(xfull.view(B, Lp, dim)[:, rank * Lc:(rank + 1) * Lc])

        # time embedding (fp32, 1B:986-990)
        tt = t.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        if tt.numel() == 1:
            tt = tt.expand(B).contiguous()
        sin = torch.empty(B, self.freq_dim, device=dev, dtype=torch.float32)
        ops.timestep_embed(tt, self.freq_dim, sin)
        h1 = torch.empty(B, dim, device=dev, dtype=torch.float32)
        ops.small_linear_f32(sin, pk.w_te0, pk.b_te0, h1, act_out=1)
        e = torch.empty(B, dim, device=dev, dtype=torch.float32)
        ops.small_linear_f32(h1, pk.w_te2, pk.b_te2, e)
        e0 = torch.empty(B, 6 * dim, device=dev, dtype=torch.float32)
        ops.small_linear_f32(e, pk.w_tp, pk.b_tp, e0, act_in=1)
        e0 = e0.view(B, 6, dim)
        emod = torch.empty(self.num_layers, B, 6, dim, device=dev, dtype=torch.float32)
        ops.mod_add(pk.mod, e0, emod)
        hmod = torch.empty(1, B, 2, dim, device=dev, dtype=torch.float32)
        ops.mod_add(pk.head_mod, e, hmod, e_jstride=0)

        ctx = self._context(pk, context, clip_fea, B, dev)

        # TeaCache (1B:1021-1044): optional, decided on e0 before any block work
        tc = self.teacache
        x = ws.x
        should_calc = True if tc is None else tc.decide(e0, cond_flag)
        if not should_calc:  # 1B:1048-1050: reuse the last computed residual
            ws.x.add_(tc.residual(cond_flag, dev))
        else:
            x_in = ws.x.clone() if tc is not None else None
            # vocal context (1B:1004-1009): projector on the last (full-condition) row only
            n_fr = (video_sample_n_frames - 1) // 4 + 1
            if S % n_fr:
                raise ValueError("seq_len must split evenly into latent frames for the per-frame audio attention")
            G = S // n_fr
            # the latent frames this rank's tokens belong to (SP pads past S join the last frame): the only vocal
            # context rows its cross-attention reads (sp.vocal_segments); without SP every frame
            if SP:
                t0, t1 = rank * Lc, min((rank + 1) * Lc, S)
                vf0 = min(t0 // G, n_fr - 1)
                vnf = min(max(t1 - 1, t0) // G, n_fr - 1) - vf0 + 1
            else:
                vf0, vnf = 0, n_fr
            lat_row = torch.empty(vnf * G, dim, device=dev, dtype=torch.bfloat16)
            if vocal_embeddings.shape[0] == 1 and B != 1:
                raise ValueError("a single audio row drives a batch of 1 (1B:1008-1009); CFG batches pass 3 rows")
            # 1.3B: the projector runs on the last (full-condition) row only, the unconditional row gets
            # zeros (1B:1004-1009); 14B: every row through the projector with its own audio (14B:1008)
            rows_v = B if (self.VOCAL == "14B" or vocal_embeddings.shape[0] == 1) else 1
            voc_rows = []
            for r in range(rows_v):
                src = B - 1 if rows_v == 1 else r
                ops.cast_bf16(xfull[src * Lp + vf0 * G:src * Lp + (vf0 + vnf) * G], lat_row)
                vv, Fn, nper = self._vocal(pk, vocal_embeddings[src], video_sample_n_frames, lat_row, S,
                                           e0[src:src + 1], e[src:src + 1], dev, frames=(vf0, vnf))
                if self.vd != dim:
                    raise ValueError("vocal context width must equal the DiT width")
                voc_rows.append(vv)
            assert Fn == n_fr
            vr = slice(vf0 * nper, (vf0 + vnf) * nper)  # the computed frames' rows of each CFG row's context
            if rows_v == 1 and vnf == n_fr:
                vctx = torch.zeros(B, Fn * nper, dim, device=dev, dtype=torch.bfloat16)
                for b in range(1, B):
                    vctx[b].copy_(voc_rows[0])
            elif vnf == n_fr:
                vctx = torch.stack(voc_rows)
            else:
                vctx = torch.zeros(B, Fn * nper, dim, device=dev, dtype=torch.bfloat16)
                for b in range(B):
                    if rows_v == B or b >= 1:
                        vctx[b, vr].copy_(voc_rows[b if rows_v == B else 0])
            vctx = vctx.view(B * Fn * nper, dim)

            if SP:
                plan = sp.make_plan(NS, rank, H_)
                ex = self._sp_exchange(plan, B, Lc, dev)
                Lq, hg, hgd = plan.G * Lc, plan.hg, plan.hg * self.d
                pack_kw = dict(table=ex.table, G=plan.G, R=plan.R, my_part=plan.part)
                # keys: the S tokens of the single-GPU sequence (the SP pads past S are queries only, their
                # outputs are never read), so any degree reproduces the single-GPU forward
                segs_self = self._segs.get(("self_sp", B, Lp, Lq, S), [[b * Lq, Lq, b * Lp, S] for b in range(B)],
                                           dev)
                # exchange schedule (SA_SP_OVERLAP: 0 one synchronous batched exchange per direction; 2 per-row
                # exchanges and per-row attention; 3 per-row Q/K/V exchanges, batched attention; 1 = auto:
                # 2 when per-row attention launches add no waves over the CUs -- a row's launch has ceil(Lq /
                # 256) x hg workgroups and B serial launches must not need more rounds than the batched one --
                # else 3 (N = 8: 63 workgroups per row would leave most CUs idle, but the Q/K/V exchange of
                # row b can still travel under the QKV GEMMs of rows b+1..; per-row GEMMs there take as many
                # rounds over the CUs as the batched one)
                n_cu = torch.cuda.get_device_properties(dev).multi_processor_count if dev.type == "cuda" else 256
                wg_row = -(-Lq // 256) * hg
                ov = os.environ.get("SA_SP_OVERLAP", "1")
                if ov == "1" and B > 1 and dev.type == "cuda":
                    # one stream per CFG row through the whole block: its compute alone matches the best of the
                    # other schedules at every degree (per-rank forward with the transfers stubbed out, N = 2 / 4 / 8:
                    # 197.2 / 103.3 / 59.3 ms vs 198.5 / 103.8 / 59.0 ms, profiles/r04/sp_rank_compute_r4s.jsonl)
                    # and every transfer travels under the other rows' work
                    ov = "4"
                elif ov == "1":
                    ov = "2" if B * -(-wg_row // n_cu) <= -(-(B * wg_row) // n_cu) else "3"
                sp_rows, sp_rows_x = ov == "2", ov == "3" and B > 1
                sp_streams = ov == "4" and B > 1 and dev.type == "cuda"
                if sp_rows or sp_streams:
                    segs_rows = [self._segs.get(("self_sp_row", b, Lp, Lq, S), [[b * Lq, Lq, b * Lp, S]], dev)
                                 for b in range(B)]
            else:
                sp_rows = sp_rows_x = sp_streams = False
                segs_self = self._segs.get(("self", B, Lp), [[b * Lp, Lp, b * Lp, Lp] for b in range(B)], dev)
            segs_txt = self._segs.get(("txt", B, Lc, ctx.text_len), sp.local_segments(B, Lc, ctx.text_len), dev)
            segs_img = self._segs.get(("img", B, Lc, ctx.img_len), sp.local_segments(B, Lc, ctx.img_len), dev)
            voc_list = sp.vocal_segments(B, S, Lc, rank, n_fr, nper)
            segs_voc = self._segs.get(("voc", B, S, Lc, rank, n_fr, nper), voc_list, dev)
            voc_n, voc_q = len(voc_list), max(s_[1] for s_ in voc_list)
            use_cross3 = (ctx.img_len > 0 and G % 256 == 0 and (rank * Lc) % 256 == 0 and (rank + 1) * Lc <= S
                          and os.environ.get("SA_CROSS3", "1") != "0")
            x = ws.x
            use_vt = not SP and self._vt_attention(Lp, dev)
            # shared_rows: the first block's self-attention half once (single-GPU layout, or the one-stream and
            # per-row-stream Ulysses schedules)
            dedup = shared_rows and broadcast and B > 1 and (not SP or sp_streams or not (sp_rows or sp_rows_x))
            if use_vt and ws.vt is None:
                # zero-filled once: the pad columns past B * Lp are read (as P = 0 keys) by a partial last block, which
                # stages a whole 64-key block: up to (B-1)*Lp + ceil64(Lp) <= ceil64(M) + 64 columns
                ws.vt = torch.zeros(dim, (ws.x.shape[0] + 63) // 64 * 64 + 64, device=dev, dtype=torch.bfloat16)
            # per-frame vocal K|V of every block in one GEMM [B * n_fr * nper, layers * 2 * dim] (1B:575-578: the
            # block's k_vocal / v_vocal of the shared vocal context); under SP only the rows of the frames this rank's
            # queries read (the others are never read)
            kvv_all = torch.empty(B * n_fr * nper, pk.w_kv_v_all.shape[0], device=dev, dtype=torch.bfloat16)
            if vnf == n_fr:
                ops.linear(vctx, pk.w_kv_v_all, pk.b_kv_v_all, ops.EPI_BF16, out=kvv_all)
            else:
                for b in range(B):
                    r0 = b * n_fr * nper + vf0 * nper
                    ops.linear(vctx[r0:r0 + vnf * nper], pk.w_kv_v_all, pk.b_kv_v_all, ops.EPI_BF16,
                               out=kvv_all[r0:r0 + vnf * nper])
            grid = (Fw, hp, wp)
            if sp_streams:
                # every CFG row through the whole layer on its own HIP stream (_sp_layer_rows); rows are independent
                rstreams = self._row_streams(B, dev)
                main = torch.cuda.current_stream(dev)
                for rs_ in rstreams:
                    rs_.wait_stream(main)
                row_segs = self._row_cross_segs(B, Lc, ctx, voc_list, dev)
            for li, L in enumerate(pk.layers):
                kvv = kvv_all[:, 2 * dim * li:2 * dim * (li + 1)]
                em = emod[li]  # [B, 6, dim]
                rope_kw = dict(rope=pk.rope, rows_per_batch=Lc, tok_offset=rank * Lc, grid=grid, head_dim=self.d,
                               n_frame_pairs=self.d // 2 - 2 * (self.d // 6), n_height_pairs=self.d // 6)
                first_shared = li == 0 and dedup
                if first_shared:
                    # the CFG rows enter the first block identical (shared_rows): its self-attention half for
                    # row 0 only, then the residual stream copied to the other rows
                    if SP:
                        seg0 = self._segs.get(("self_sp_row", 0, Lp, Lq, S), [[0, Lq, 0, S]], dev)
                        self._sp_self_attention_row0(L, x, ws, em, ex, pack_kw, rope_kw, Lc, Lq, hg, hgd, seg0, B)
                        if sp_streams:
                            for rs_ in rstreams:
                                rs_.wait_stream(main)
                    else:
                        self._self_attention_rows(pk, L, x, ws, em, 1, Lc, Lp, use_vt, rope_kw, dev, batch=B)
                        for b in range(1, B):
                            x[b * Lc:(b + 1) * Lc].copy_(x[:Lc])
                if sp_streams:
                    self._sp_layer_rows(pk, L, li, x, ws, em, ex, pack_kw, rank, Lc, Lq, hg, hgd, grid,
                                        segs_rows, row_segs, ctx, kvv, nper, G, n_fr, use_cross3, rstreams,
                                        sa=not first_shared)
                    continue
                if not first_shared:  # self-attention (1B:675-679)
                    ops.layernorm_mod(x, ws.mod, self.eps, shift=em[:, 0], scale=em[:, 1], rows_per_batch=Lc)
                    if SP and sp_rows:
                        # Ulysses pipelined over the CFG rows: row b's Q/K/V exchange is issued right after its
                        # QKV GEMM + pack (so it travels under rows b+1..'s GEMMs), row b's attention waits
                        # only on it, and row b's output exchange travels under the next rows' attention and
                        # the earlier rows' O-projections
                        pend = []
                        for b in range(B):
                            rs = slice(b * Lc, (b + 1) * Lc)
                            ops.linear(ws.mod[rs], L.w_qkv, L.b_qkv, ops.EPI_BF16, out=ws.qkv[rs])
                            ops.qkv_pack(ws.qkv[rs], L.nq, L.nk, dim, self.eps, b_offset=b, **pack_kw, **rope_kw)
                            pend.append(ex.heads([b]))
                        back = []
                        for b in range(B):
                            pend[b].wait()
                            ev0 = self._record_event()
                            ops.attention(ex.q, ex.kv[:, :hgd], ex.kv[:, hgd:], ex.obuf, segs_rows[b], 1, Lq, hg,
                                          kernel=self.attn_kernel, o_rows=ex.omap)
                            self._record_span(ev0, rows=1, batch=B)
                            back.append(ex.tokens([b]))
                        for b in range(B):
                            rs = slice(b * Lc, (b + 1) * Lc)
                            back[b].wait()
                            a0, pnl = ex.panels(range(b, b + 1))
                            ops.linear(a0, L.w_o, L.b_o, ops.EPI_RES_F32, out=x[rs], residual=x[rs],
                                       gate=em[b:b + 1, 2], rows_per_batch=Lc, a_panels=pnl)
                    elif SP:
                        if sp_rows_x:
                            # per-row Q/K/V exchanges issued as each row's QKV GEMM + pack lands (they travel
                            # under the later rows' GEMMs), one batched attention once all have arrived
                            pend = []
                            for b in range(B):
                                rs = slice(b * Lc, (b + 1) * Lc)
                                ops.linear(ws.mod[rs], L.w_qkv, L.b_qkv, ops.EPI_BF16, out=ws.qkv[rs])
                                ops.qkv_pack(ws.qkv[rs], L.nq, L.nk, dim, self.eps, b_offset=b, **pack_kw, **rope_kw)
                                pend.append(ex.heads([b]))
                            for p_ in pend:
                                p_.wait()
                        else:  # one exchange per direction for all rows
                            ops.linear(ws.mod, L.w_qkv, L.b_qkv, ops.EPI_BF16, out=ws.qkv)
                            ops.qkv_pack(ws.qkv, L.nq, L.nk, dim, self.eps, **pack_kw, **rope_kw)
                            ex.heads(range(B)).wait()
                        # Ulysses: full-sequence attention of this rank's (query part, head group), outputs written
                        # to the owners' send slabs / this rank's own O-projection panel, then heads -> tokens
                        ev0 = self._record_event()
                        split = ops.attn_tail_split(0, B * hg * -(-Lq // 256), dev) if self.attn_kernel == 0 else 0
                        ops.attention(ex.q, ex.kv[:, :hgd], ex.kv[:, hgd:], ex.obuf, segs_self, B, Lq, hg,
                                      kernel=self.attn_kernel, o_rows=ex.omap, split_tiles=split)
                        self._record_span(ev0, rows=B, batch=B)
                        ex.tokens(range(B)).wait()
                        a0, pnl = ex.panels()
                        ops.linear(a0, L.w_o, L.b_o, ops.EPI_RES_F32, out=x, residual=x, gate=em[:, 2],
                                   rows_per_batch=Lc, a_panels=pnl)
                    else:
                        self._self_attention_rows(pk, L, x, ws, em, B, Lc, Lp, use_vt, rope_kw, dev, batch=B,
                                                  normed=True)
                # cross-attention: text + image + per-frame vocal (1B:534-605, 684)
                ops.layernorm_mod(x, ws.mod, self.eps, weight=L.n3w, bias=L.n3b)
                qc = ws.qkv[:, :dim]
                ops.linear(ws.mod, L.w_cq, L.b_cq, ops.EPI_BF16, out=qc)
                ops.qk_rmsnorm_rope(qc, 0, -1, L.cnq, None, dim, self.eps)
                kvt, kvi = ctx.kv[li]
                if use_cross3:  # text + image + vocal in one launch, bf16 sum as 1B:602
                    ops.attention_cross3(qc, kvt[:, :dim], kvt[:, dim:], ctx.text_len, kvi[:, :dim], kvi[:, dim:],
                                         ctx.img_len, kvv[:, :dim], kvv[:, dim:], nper, G, n_fr, ws.att, B, Lc, H_,
                                         tok_offset=rank * Lc)
                else:
                    ops.attention(qc, kvt[:, :dim], kvt[:, dim:], ws.att, segs_txt, B, Lc, H_)
                    if kvi is not None:
                        ops.attention(qc, kvi[:, :dim], kvi[:, dim:], ws.att, segs_img, B, Lc, H_, accumulate=True)
                    ops.attention(qc, kvv[:, :dim], kvv[:, dim:], ws.att, segs_voc, voc_n, voc_q, H_, accumulate=True)
                ops.linear(ws.att, L.w_co, L.b_co, ops.EPI_RES_F32, out=x, residual=x)
                # FFN (1B:687-691)
                ops.layernorm_mod(x, ws.mod, self.eps, shift=em[:, 3], scale=em[:, 4], rows_per_batch=Lc)
                ops.linear(ws.mod, L.w_f0, L.b_f0, ops.EPI_GELU_TANH_BF16, out=ws.ffn)
                ops.linear(ws.ffn, L.w_f2, L.b_f2, ops.EPI_RES_F32, out=x, residual=x, gate=em[:, 5], rows_per_batch=Lc)
            if sp_streams:
                for rs_ in rstreams:
                    main.wait_stream(rs_)
            if tc is not None:  # 1B:1096-1099
                tc.store(ws.x - x_in, cond_flag)
                del x_in

        # head (1B:715-723) + unpatchify (1B:1161-1184)
        hm = hmod[0]
        ops.layernorm_mod(x, ws.mod, self.eps, shift=hm[:, 0], scale=hm[:, 1], rows_per_batch=Lc)
        ho = ops.linear(ws.mod, pk.w_head, pk.b_head, ops.EPI_BF16)
        if SP:  # every rank gets the whole prediction (1B:1150-1152)
            ho = sp.gather_tokens(ho, B, Lc, NS, self.sp_group)
        if out is None:
            out = torch.empty(B, self.out_dim, Fw, Hh, Ww, device=dev, dtype=torch.bfloat16)
        ops.unpatchify(ho, Lp, B, self.out_dim, Fw, Hh, Ww, out)
        return out


class WanTransformer3DFantasy14BModel(WanTransformer3DFantasyModel):
    """WanTransformer3DFantasy14BModel (wan_fantasy_transformer3d_14B.py:735-1178): the same DiT at the 14B
    widths (wan_civitai 14B: dim 5120, 40 heads, 40 layers, ffn 13824) with the 14B vocal projector
    (two-layer audio projection, width = dim, 8 heads of 640, run on every CFG row with its own audio,
    14B:1008).  The reference's forward has no video_sample_n_frames (its vocal path hard-codes 81 video /
    21 latent frames, 14B:1008-1010, vocal_projector_fantasy_14B.py:254), which is why its long pipeline
    cannot drive it; here forward also accepts the 1.3B keyword and requires 81."""

    VOCAL = "14B"

    def forward_window(self, lat, frame_offset, broadcast, B, t, context, seq_len, clip_fea, y, vocal_embeddings,
                       video_sample_n_frames=81, is_clip_level_modeling=False, out=None, cond_flag=True,
                       shared_rows=False):
        if video_sample_n_frames != 81:
            raise ValueError("the 14B vocal path is built for 81-frame windows (21 latent frames, 14B:1008-1010)")
        return super().forward_window(lat, frame_offset, broadcast, B, t, context, seq_len, clip_fea, y,
                                      vocal_embeddings, 81, is_clip_level_modeling, out=out, cond_flag=cond_flag,
                                      shared_rows=shared_rows)


def call_gemm_batched(cols, w, bias, xout, B, real, Lp, dim, kpad):
    """patch-embedding GEMM per batch row over its real tokens only (pads stay zero, 1B:983)."""
    from ._lib import call
    call("sa_gemm_bf16", cols.data_ptr(), kpad, Lp * kpad, w.data_ptr(), kpad, 0, bias.data_ptr(), xout.data_ptr(),
         dim, Lp * dim, real, dim, kpad, B, ops.EPI_F32, 0, 0, 0, 0, 0, 0, ops._stream())
