"""Drop-in AutoencoderKLWan for MI355X (reference: wan/models/wan_vae.py).

Same state_dict keys ('model.conv1/conv2.*', 'model.encoder.*', 'model.decoder.*'),
`from_pretrained(path, additional_kwargs)`, `decode(z, return_dict=True) -> DecoderOutput(sample=...)`
and `encode(x, return_dict=True) -> AutoencoderKLOutput(latent_dist=...)` (`encode(x)[0].mode()` as the
pipeline calls it, wan_inference_long_pipeline.py:414-415) as the reference.  Decoder and encoder run
over the whole clip at once (equivalent to the reference's chunked causal feature cache, see
oracle/vae.py) with channels-last bf16 activations and every conv as an MFMA implicit GEMM.  The
encoder (reference frame + zeros, once per call) is SURVEY.md §8(f) row 1.
"""
from __future__ import annotations

from types import SimpleNamespace

import torch
import torch.nn as nn

from . import ops
from ._lib import call

MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
        0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
       3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


def decoder_layout(dim=96, z_dim=16, dim_mult=(1, 2, 4, 4), num_res_blocks=2, temperal_upsample=(True, True, False)):
    """Module list of Decoder3d (wan_vae.py:372-424): (kind, name, in, out)."""
    dims = [dim * u for u in [dim_mult[-1]] + list(dim_mult[::-1])]
    L = [("conv", "conv1", z_dim, dims[0]),
         ("res", "middle.0", dims[0], dims[0]), ("attn", "middle.1", dims[0], dims[0]),
         ("res", "middle.2", dims[0], dims[0])]
    k = 0
    for i, (din, dout) in enumerate(zip(dims[:-1], dims[1:])):
        if i in (1, 2, 3):
            din = din // 2
        for _ in range(num_res_blocks + 1):
            L.append(("res", f"upsamples.{k}", din, dout))
            k += 1
            din = dout
        if i != len(dim_mult) - 1:
            L.append(("up3d" if temperal_upsample[i] else "up2d", f"upsamples.{k}", dout, dout // 2))
            k += 1
    L.append(("head", "head", dims[-1], 3))
    return L


def param_shapes(dim=96, z_dim=16):
    """{key: shape} of the decode half of AutoencoderKLWan ('model.' prefix, wan_vae.py:683-704)."""
    S = {"model.conv2.weight": (z_dim, z_dim, 1, 1, 1), "model.conv2.bias": (z_dim,)}
    p = "model.decoder."
    for kind, name, cin, cout in decoder_layout(dim, z_dim):
        q = p + name
        if kind == "conv":
            S[q + ".weight"] = (cout, cin, 3, 3, 3)
            S[q + ".bias"] = (cout,)
        elif kind == "res":
            S[q + ".residual.0.gamma"] = (cin, 1, 1, 1)
            S[q + ".residual.2.weight"] = (cout, cin, 3, 3, 3)
            S[q + ".residual.2.bias"] = (cout,)
            S[q + ".residual.3.gamma"] = (cout, 1, 1, 1)
            S[q + ".residual.6.weight"] = (cout, cout, 3, 3, 3)
            S[q + ".residual.6.bias"] = (cout,)
            if cin != cout:
                S[q + ".shortcut.weight"] = (cout, cin, 1, 1, 1)
                S[q + ".shortcut.bias"] = (cout,)
        elif kind == "attn":
            S[q + ".norm.gamma"] = (cin, 1, 1)
            S[q + ".to_qkv.weight"] = (cin * 3, cin, 1, 1)
            S[q + ".to_qkv.bias"] = (cin * 3,)
            S[q + ".proj.weight"] = (cin, cin, 1, 1)
            S[q + ".proj.bias"] = (cin,)
        elif kind in ("up3d", "up2d"):
            S[q + ".resample.1.weight"] = (cout, cin, 3, 3)
            S[q + ".resample.1.bias"] = (cout,)
            if kind == "up3d":
                S[q + ".time_conv.weight"] = (cin * 2, cin, 3, 1, 1)
                S[q + ".time_conv.bias"] = (cin * 2,)
        elif kind == "head":
            S[q + ".0.gamma"] = (cin, 1, 1, 1)
            S[q + ".2.weight"] = (cout, cin, 3, 3, 3)
            S[q + ".2.bias"] = (cout,)
    return S


def encoder_layout(dim=96, dim_mult=(1, 2, 4, 4), num_res_blocks=2, temperal_downsample=(False, True, True)):
    """Module list of Encoder3d (wan_vae.py:268-319): (kind, name, in, out)."""
    dims = [dim * u for u in [1] + list(dim_mult)]
    L = [("conv", "conv1", 3, dims[0])]
    k = 0
    for i, (din, dout) in enumerate(zip(dims[:-1], dims[1:])):
        for _ in range(num_res_blocks):
            L.append(("res", f"downsamples.{k}", din, dout))
            k += 1
            din = dout
        if i != len(dim_mult) - 1:
            L.append(("down3d" if temperal_downsample[i] else "down2d", f"downsamples.{k}", dout, dout))
            k += 1
    L += [("res", "middle.0", dims[-1], dims[-1]), ("attn", "middle.1", dims[-1], dims[-1]),
          ("res", "middle.2", dims[-1], dims[-1]), ("head", "head", dims[-1], None)]
    return L


def encoder_param_shapes(dim=96, z_dim=16):
    """{key: shape} of the encode half of AutoencoderKLWan ('model.conv1', 'model.encoder.*')."""
    S = {"model.conv1.weight": (2 * z_dim, 2 * z_dim, 1, 1, 1), "model.conv1.bias": (2 * z_dim,)}
    for kind, name, cin, cout in encoder_layout(dim):
        q = "model.encoder." + name
        if kind == "conv":
            S[q + ".weight"] = (cout, cin, 3, 3, 3)
            S[q + ".bias"] = (cout,)
        elif kind == "res":
            S[q + ".residual.0.gamma"] = (cin, 1, 1, 1)
            S[q + ".residual.2.weight"] = (cout, cin, 3, 3, 3)
            S[q + ".residual.2.bias"] = (cout,)
            S[q + ".residual.3.gamma"] = (cout, 1, 1, 1)
            S[q + ".residual.6.weight"] = (cout, cout, 3, 3, 3)
            S[q + ".residual.6.bias"] = (cout,)
            if cin != cout:
                S[q + ".shortcut.weight"] = (cout, cin, 1, 1, 1)
                S[q + ".shortcut.bias"] = (cout,)
        elif kind == "attn":
            S[q + ".norm.gamma"] = (cin, 1, 1)
            S[q + ".to_qkv.weight"] = (cin * 3, cin, 1, 1)
            S[q + ".to_qkv.bias"] = (cin * 3,)
            S[q + ".proj.weight"] = (cin, cin, 1, 1)
            S[q + ".proj.bias"] = (cin,)
        elif kind in ("down2d", "down3d"):
            S[q + ".resample.1.weight"] = (cout, cin, 3, 3)
            S[q + ".resample.1.bias"] = (cout,)
            if kind == "down3d":
                S[q + ".time_conv.weight"] = (cout, cout, 3, 1, 1)
                S[q + ".time_conv.bias"] = (cout,)
        elif kind == "head":
            S[q + ".0.gamma"] = (cin, 1, 1, 1)
            S[q + ".2.weight"] = (2 * z_dim, cin, 3, 3, 3)
            S[q + ".2.bias"] = (2 * z_dim,)
    return S


def _cout_pad(cout):
    if cout > 96:
        return ((cout + 191) // 192) * 192
    if cout > 16:
        return ((cout + 95) // 96) * 96
    return 16


def _pack_conv(w, b, cin_pad=None, cout_store=None):
    """torch conv weight [Cout, Cin, (kt,) kh, kw] -> bf16 [Cout_pad][kt][kh][kw][Cin_pad] + fp32 bias."""
    w = w.detach().float()
    if w.dim() == 4:
        w = w.unsqueeze(2)
    cout, cin, kt, kh, kw = w.shape
    cin_p = cin_pad or cin
    cout_s = cout_store or cout
    cp = _cout_pad(cout_s)
    out = torch.zeros(cp, kt, kh, kw, cin_p, device=w.device, dtype=torch.float32)
    out[:cout, :, :, :, :cin] = w.permute(0, 2, 3, 4, 1)
    bias = torch.zeros(cp, device=w.device, dtype=torch.float32)
    bias[:cout] = b.detach().float()
    return SimpleNamespace(w=out.to(torch.bfloat16).contiguous(), b=bias, cin=cin_p, cout=cout_s, cout_pad=cp,
                           kt=kt, kh=kh, kw=kw)


class _SeqState:
    """causal caches of a chunk-by-chunk decode in one process"""

    def __init__(self):
        self.d = {}

    def get(self, key, like):
        return self.d.get(key)

    def put(self, key, val):
        self.d[key] = val

    def skip(self, key, like):
        pass


def _world(group):
    import torch.distributed as dist
    return dist.get_world_size(group)


def _gloo(group):
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


class _ChainState:
    """causal caches of the multi-rank decode: rank r's chunk takes every cache from rank r-1 and passes its
    updated cache to rank r+1, in the (identical) order of the cache points.  RCCL: async P2P on the
    collective stream (the receiver's stream waits, no host sync); gloo (ranks sharing one GPU in tests):
    host-staged."""

    def __init__(self, group, rank, n):
        import torch.distributed as dist
        self.group, self.rank, self.n = group, rank, n
        self.prev_g = dist.get_global_rank(group, rank - 1) if rank > 0 else None
        self.next_g = dist.get_global_rank(group, rank + 1) if rank + 1 < n else None
        self.sends = []
        self.local = {}
        self.first_sub, self.last_sub = True, True

    def begin(self, first_sub, last_sub):
        """a rank decodes its run in sub-chunks: only the first takes its caches from rank r-1 and only the
        last hands them to rank r+1; in between they stay local"""
        self.first_sub, self.last_sub = first_sub, last_sub

    def get(self, key, like):
        import torch.distributed as dist
        if not self.first_sub:
            return self.local.get(key)
        if self.prev_g is None:
            return None
        shape = (2,) + tuple(like.shape[1:])
        if _gloo(self.group) and like.is_cuda:
            h = torch.empty(shape, dtype=like.dtype)
            dist.recv(h, self.prev_g, group=self.group)
            return h.to(like.device)
        # RCCL: a one-op batch_isend_irecv group on the process group's communicator -- the primitive the sequence-
        # parallel exchange and the degree-1 loopback test run (a bare irecv would set up a separate per-pair
        # communicator lazily); the caller's stream waits for it, the host does not
        t = torch.empty(shape, dtype=like.dtype, device=like.device)
        for w in dist.batch_isend_irecv([dist.P2POp(dist.irecv, t, group=self.group, group_peer=self.rank - 1)]):
            w.wait()
        return t

    def put(self, key, val):
        import torch.distributed as dist
        if not self.last_sub:
            self.local[key] = val
            return
        if self.next_g is None:
            return
        if _gloo(self.group) and val.is_cuda:
            h = val.cpu()
            self.sends.append((dist.isend(h, self.next_g, group=self.group), h))
        elif _gloo(self.group):
            self.sends.append((dist.isend(val, self.next_g, group=self.group), val))
        else:
            # keep every Work batch_isend_irecv returns: finish() waits on all of them
            ws = dist.batch_isend_irecv([dist.P2POp(dist.isend, val, group=self.group, group_peer=self.rank + 1)])
            self.sends.append((list(ws or []), val))

    def skip(self, key, like):
        prev = self.get(key, like)
        if prev is None:
            prev = torch.zeros((2,) + tuple(like.shape[1:]), device=like.device, dtype=like.dtype)
        self.put(key, prev)

    def finish(self):
        for w, _ in self.sends:
            for x in (w if isinstance(w, list) else [w]):
                x.wait()
        self.sends = []


class _LoopbackChain(_ChainState):
    """Virtual rank v of n decoded in turn on ONE rank (degree-1 RCCL test of the wavefront): every cache hand-off is a
    point-to-point send to this rank itself with its matching receive in one coalesced group (sp._p2p), the
    received copy queued for virtual rank v + 1."""

    def __init__(self, group, v, n, fifo):
        import torch.distributed as dist
        self.group, self.rank, self.n, self.fifo = group, v, n, fifo
        self.me = dist.get_rank(group)
        self.sends, self.local = [], {}
        self.first_sub, self.last_sub = True, True

    def get(self, key, like):
        if not self.first_sub:
            return self.local.get(key)
        if self.rank == 0:
            return None
        pend, t = self.fifo.popleft()
        pend.wait()
        return t

    def put(self, key, val):
        from . import sp
        if not self.last_sub:
            self.local[key] = val
            return
        if self.rank + 1 >= self.n:
            return
        t = torch.empty_like(val)
        self.fifo.append((sp._p2p([(val, self.me)], [(t, self.me)], self.group), t))

    def finish(self):
        pass


def _all_gather(buf, N, group):
    """[N, *buf.shape]: every rank's buf (gathered as the concatenation along dim 0)"""
    import torch.distributed as dist
    shape = (N * buf.shape[0],) + tuple(buf.shape[1:])
    if _gloo(group) and buf.is_cuda:
        out = torch.empty(shape, dtype=buf.dtype)
        dist.all_gather_into_tensor(out, buf.cpu(), group=group)
        out = out.to(buf.device)
    else:
        out = torch.empty(shape, dtype=buf.dtype, device=buf.device)
        dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    return out.view((N,) + tuple(buf.shape))


class DecoderOutput:
    def __init__(self, sample):
        self.sample = sample


class DiagonalGaussianDistribution:
    """diffusers' posterior over h = cat(mean, logvar) (wan_vae.py:656); the pipeline uses .mode()."""

    def __init__(self, parameters):
        self.parameters = parameters
        self.mean, self.logvar = torch.chunk(parameters, 2, dim=1)
        self.logvar = torch.clamp(self.logvar, -30.0, 20.0)
        self.std = torch.exp(0.5 * self.logvar)
        self.var = torch.exp(self.logvar)

    def mode(self):
        return self.mean

    def sample(self, generator=None):
        noise = torch.randn(self.mean.shape, generator=generator, dtype=self.mean.dtype).to(self.mean.device)
        return self.mean + self.std * noise


class AutoencoderKLOutput:
    def __init__(self, latent_dist):
        self.latent_dist = latent_dist

    def __getitem__(self, i):
        return (self.latent_dist,)[i]


class AutoencoderKLWan(nn.Module):
    """wan_vae.py:619-704, decode path on HIP kernels."""

    def __init__(self, latent_channels=16, temporal_compression_ratio=4, spacial_compression_ratio=8, dim=96):
        super().__init__()
        self.config = SimpleNamespace(latent_channels=latent_channels,
                                      temporal_compression_ratio=temporal_compression_ratio,
                                      spacial_compression_ratio=spacial_compression_ratio)
        self.z_dim, self.dim = latent_channels, dim
        self.mean = torch.tensor(MEAN, dtype=torch.float32)
        self.std = torch.tensor(STD, dtype=torch.float32)
        shapes = dict(param_shapes(dim, latent_channels), **encoder_param_shapes(dim, latent_channels))
        for name, shp in shapes.items():
            *path, leaf = name.split(".")
            mod = self
            for p in path:
                if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                    mod.add_module(p, nn.Module())
                mod = getattr(mod, p)
            mod.register_parameter(leaf, nn.Parameter(torch.empty(shp), requires_grad=False))
        self._packed = None
        self._packed_enc = None
        self.decode_group = None  # enable_multi_gpus_inference(): decode over several ranks

    @property
    def dtype(self):
        return torch.float32

    @classmethod
    def from_pretrained(cls, pretrained_model_path, additional_kwargs={}):
        import inspect
        sig = set(inspect.signature(cls.__init__).parameters) - {"self"}
        model = cls(**{k: v for k, v in additional_kwargs.items() if k in sig})
        if pretrained_model_path.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(pretrained_model_path)
        else:
            sd = torch.load(pretrained_model_path, map_location="cpu", weights_only=True)
        sd = {"model." + k: v for k, v in sd.items()}
        model.load_state_dict(sd, strict=False)
        return model

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._packed = self._packed_enc = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _apply(self, fn, recurse=True):
        self._packed = self._packed_enc = None
        return super()._apply(fn, recurse)

    # ------------------------------------------------------------------ packing

    def _pack(self):
        if self._packed is not None:
            return self._packed
        dev = self.model.conv2.weight.device
        if dev.type != "cuda":
            raise RuntimeError("AutoencoderKLWan.decode runs on the MI355X HIP kernels: move it to 'cuda'")
        P = dict(self.named_parameters())
        zp = ((self.z_dim + 31) // 32) * 32
        pk = SimpleNamespace(zp=zp, layers=[])
        pk.conv2 = _pack_conv(P["model.conv2.weight"], P["model.conv2.bias"], cin_pad=zp, cout_store=zp)
        pk.mean, pk.std = self.mean.to(dev), self.std.to(dev)
        g = lambda n: P[n].detach().float().reshape(-1).contiguous()  # noqa: E731
        for kind, name, cin, cout in decoder_layout(self.dim, self.z_dim):
            q = "model.decoder." + name
            e = SimpleNamespace(kind=kind, cin=cin, cout=cout)
            if kind == "conv":
                e.conv = _pack_conv(P[q + ".weight"], P[q + ".bias"], cin_pad=zp)
            elif kind == "res":
                e.g0, e.g3 = g(q + ".residual.0.gamma"), g(q + ".residual.3.gamma")
                e.c1 = _pack_conv(P[q + ".residual.2.weight"], P[q + ".residual.2.bias"])
                e.c2 = _pack_conv(P[q + ".residual.6.weight"], P[q + ".residual.6.bias"])
                e.sc = (_pack_conv(P[q + ".shortcut.weight"], P[q + ".shortcut.bias"])
                        if q + ".shortcut.weight" in P else None)
            elif kind == "attn":
                e.g = g(q + ".norm.gamma")
                e.qkv = _pack_conv(P[q + ".to_qkv.weight"], P[q + ".to_qkv.bias"])
                e.proj = _pack_conv(P[q + ".proj.weight"], P[q + ".proj.bias"])
            elif kind in ("up3d", "up2d"):
                e.rs = _pack_conv(P[q + ".resample.1.weight"], P[q + ".resample.1.bias"])
                if kind == "up3d":
                    e.tc = _pack_conv(P[q + ".time_conv.weight"], P[q + ".time_conv.bias"])
            elif kind == "head":
                e.g = g(q + ".0.gamma")
                e.conv = _pack_conv(P[q + ".2.weight"], P[q + ".2.bias"], cout_store=4)
            pk.layers.append(e)
        self._packed = pk
        return pk

    def _pack_enc(self):
        if self._packed_enc is not None:
            return self._packed_enc
        dev = self.model.conv1.weight.device
        if dev.type != "cuda":
            raise RuntimeError("AutoencoderKLWan.encode runs on the MI355X HIP kernels: move it to 'cuda'")
        P = dict(self.named_parameters())
        g = lambda n: P[n].detach().float().reshape(-1).contiguous()  # noqa: E731
        z2 = 2 * self.z_dim
        pk = SimpleNamespace(layers=[], mean=self.mean.to(dev), std=self.std.to(dev),
                             zero3=torch.zeros(3, device=dev), one3=torch.ones(3, device=dev))
        pk.conv1 = _pack_conv(P["model.conv1.weight"], P["model.conv1.bias"])
        for kind, name, cin, cout in encoder_layout(self.dim):
            q = "model.encoder." + name
            e = SimpleNamespace(kind=kind, cin=cin, cout=cout)
            if kind == "conv":  # 3 input channels, zero-padded to the 32-deep K step
                e.conv = _pack_conv(P[q + ".weight"], P[q + ".bias"], cin_pad=32)
            elif kind == "res":
                e.g0, e.g3 = g(q + ".residual.0.gamma"), g(q + ".residual.3.gamma")
                e.c1 = _pack_conv(P[q + ".residual.2.weight"], P[q + ".residual.2.bias"])
                e.c2 = _pack_conv(P[q + ".residual.6.weight"], P[q + ".residual.6.bias"])
                e.sc = (_pack_conv(P[q + ".shortcut.weight"], P[q + ".shortcut.bias"])
                        if q + ".shortcut.weight" in P else None)
            elif kind == "attn":
                e.g = g(q + ".norm.gamma")
                e.qkv = _pack_conv(P[q + ".to_qkv.weight"], P[q + ".to_qkv.bias"])
                e.proj = _pack_conv(P[q + ".proj.weight"], P[q + ".proj.bias"])
            elif kind in ("down2d", "down3d"):
                e.rs = _pack_conv(P[q + ".resample.1.weight"], P[q + ".resample.1.bias"])
                if kind == "down3d":
                    e.tc = _pack_conv(P[q + ".time_conv.weight"], P[q + ".time_conv.bias"])
            elif kind == "head":
                e.g = g(q + ".0.gamma")
                e.conv = _pack_conv(P[q + ".2.weight"], P[q + ".2.bias"])
                assert e.conv.cout == z2
            pk.layers.append(e)
        self._packed_enc = pk
        return pk

    # ------------------------------------------------------------------ kernels

    @staticmethod
    def _conv(x, T, H, W, c, residual=None, upsample=False, out=None, out_f32=False, interleave=0, prev=None):
        if out is None:
            if interleave:
                out = torch.empty(2 * T, H, W, interleave, device=x.device, dtype=torch.bfloat16)
            else:
                out = torch.empty(T, H, W, c.cout, device=x.device,
                                  dtype=torch.float32 if out_f32 else torch.bfloat16)
        call("sa_conv3d_cl", x.data_ptr(), T, H, W, c.cin, int(upsample), c.w.data_ptr(), c.b.data_ptr(), c.cout,
             c.cout_pad, c.kt, c.kh, c.kw, 0 if residual is None else residual.data_ptr(), out.data_ptr(),
             int(out_f32), interleave, 0 if prev is None else prev.data_ptr(), ops._stream())
        return out

    @staticmethod
    def _cache(state, key, x):
        """Chunked decode: (the causal cache for this chunk's conv input, update) -- CausalConv3d's
        cache_x (wan_vae.py:27-36): the last 2 input frames seen so far, zeros before the clip."""
        if state is None:
            return None
        prev = state.get(key, x)
        if prev is None:
            prev = torch.zeros((2,) + tuple(x.shape[1:]), device=x.device, dtype=x.dtype)
        state.put(key, torch.cat([prev, x])[-2:].clone() if x.shape[0] < 2 else x[-2:].clone())
        return prev

    @staticmethod
    def _cache_skip(state, key, x):
        """a cache point this chunk does not reach (the first chunk's up3d time_conv with one frame): the
        cache stays as it was (zeros before the clip)"""
        if state is not None:
            state.skip(key, x)

    @staticmethod
    def _rms(x, gamma, silu):
        y = torch.empty_like(x)
        C = x.shape[-1]
        call("sa_vae_rmsnorm_silu", x.data_ptr(), y.data_ptr(), gamma.data_ptr(), x.numel() // C, C, int(silu),
             ops._stream())
        return y

    def _res(self, e, x, T, H, W, state=None):
        h = self._conv(x, T, H, W, e.sc) if e.sc is not None else x
        y = self._rms(x, e.g0, True)
        y = self._conv(y, T, H, W, e.c1, prev=self._cache(state, (id(e), 1), y))
        y = self._rms(y, e.g3, True)
        return self._conv(y, T, H, W, e.c2, residual=h, prev=self._cache(state, (id(e), 2), y))

    def _attn(self, e, x, T, H, W):
        """AttentionBlock (wan_vae.py:243-265): per-frame single-head attention over H*W tokens."""
        C = x.shape[-1]
        HW = H * W
        y = self._rms(x, e.g, False)
        qkv = self._conv(y, T, H, W, e.qkv).view(T, HW, 3 * C)
        q, k, v = qkv[:, :, :C], qkv[:, :, C:2 * C], qkv[:, :, 2 * C:]
        o = torch.empty(T, HW, C, device=x.device, dtype=torch.bfloat16)
        HWp = ((HW + 63) // 64) * 64  # the P·V GEMM contracts over keys: pad them to the 64-deep K tile
        alloc = torch.empty if HWp == HW else torch.zeros
        vt = alloc(T, C, HWp, device=x.device, dtype=torch.bfloat16)
        call("sa_transpose_bf16", v.data_ptr(), v.stride(1), v.stride(0), vt.data_ptr(), HWp, C * HWp, HW, C, T,
             ops._stream())
        chunk = max(1, min(T, (1 << 30) // (HW * HW * 6)))  # bound the fp32 score buffer
        s = torch.empty(chunk, HW, HW, device=x.device, dtype=torch.float32)
        p = alloc(chunk, HW, HWp, device=x.device, dtype=torch.bfloat16)
        for t0 in range(0, T, chunk):
            n = min(chunk, T - t0)
            ops.bmm_nt(q[t0:t0 + n], k[t0:t0 + n], s[:n])
            call("sa_softmax_rows", s.data_ptr(), HW, p.data_ptr(), HWp, n * HW, HW, float(C) ** -0.5, ops._stream())
            ops.bmm_nt(p[:n], vt[t0:t0 + n], o[t0:t0 + n], epilogue=ops.EPI_BF16)
        return self._conv(o.view(T, H, W, C), T, H, W, e.proj, residual=x)

    def _up(self, e, x, T, H, W, state=None, first=True):
        C = x.shape[-1]
        if e.kind == "up3d" and not first:  # a later chunk: every frame goes through time_conv
            u = torch.empty(2 * T, H, W, C, device=x.device, dtype=torch.bfloat16)
            self._conv(x, T, H, W, e.tc, out=u, interleave=C, prev=self._cache(state, id(e), x))
            x, T = u, 2 * T
        elif e.kind == "up3d" and T > 1:
            u = torch.empty(1 + 2 * (T - 1), H, W, C, device=x.device, dtype=torch.bfloat16)
            u[0].copy_(x[0])
            self._conv(x[1:], T - 1, H, W, e.tc, out=u[1:], interleave=C, prev=self._cache(state, id(e), x[1:]))
            x, T = u, 1 + 2 * (T - 1)
        elif e.kind == "up3d":
            self._cache_skip(state, id(e), x)
        return self._conv(x, T, 2 * H, 2 * W, e.rs, upsample=True), T, 2 * H, 2 * W

    @staticmethod
    def _down(e, x, T, H, W):
        """Resample downsample2d/3d (wan_vae.py:91-100, :142-157) in whole-clip form: stride-2 3x3
        conv with right/bottom zero padding per frame; 3d: frame 0 kept, frames 1.. = stride-2
        time_conv over frames (2j-2, 2j-1, 2j)."""
        C = x.shape[-1]
        y = torch.empty(T, H // 2, W // 2, e.rs.cout, device=x.device, dtype=torch.bfloat16)
        call("sa_conv3d_cl_down", x.data_ptr(), T, H, W, C, 1, e.rs.w.data_ptr(), e.rs.b.data_ptr(), e.rs.cout,
             e.rs.cout_pad, y.data_ptr(), ops._stream())
        H, W = H // 2, W // 2
        if e.kind == "down3d" and T > 1:
            To = 1 + (T - 1) // 2
            z = torch.empty(To, H, W, e.tc.cout, device=x.device, dtype=torch.bfloat16)
            z[0].copy_(y[0])
            call("sa_conv3d_cl_down", y.data_ptr(), To - 1, H, W, e.rs.cout, 2, e.tc.w.data_ptr(), e.tc.b.data_ptr(),
                 e.tc.cout, e.tc.cout_pad, z[1:].data_ptr(), ops._stream())
            y, T = z, To
        return y, T, H, W

    def encode_clip(self, v):
        """v [3, T, H, W] (T = 1 + 4k, H, W multiples of 8) -> [32, 1 + k, H/8, W/8] fp32 =
        cat((mu - mean) / std, log_var) (AutoencoderKLWan_.encode, wan_vae.py:519-547)."""
        pk = self._pack_enc()
        dev = pk.mean.device
        C3, T, H, W = v.shape
        if C3 != 3 or (T - 1) % 4 or H % 8 or W % 8:
            raise ValueError(f"encode expects [3, 1+4k, 8h, 8w] frames, got {tuple(v.shape)}")
        vc = v.to(device=dev, dtype=torch.float32).contiguous()
        x = torch.empty(T, H, W, 32, device=dev, dtype=torch.bfloat16)
        call("sa_vae_input", vc.data_ptr(), 3, T * H * W, pk.zero3.data_ptr(), pk.one3.data_ptr(), x.data_ptr(), 32,
             ops._stream())
        for e in pk.layers:
            if e.kind == "conv":
                x = self._conv(x, T, H, W, e.conv)
            elif e.kind == "res":
                x = self._res(e, x, T, H, W)
            elif e.kind == "attn":
                x = self._attn(e, x, T, H, W)
            elif e.kind in ("down2d", "down3d"):
                x, T, H, W = self._down(e, x, T, H, W)
            elif e.kind == "head":
                y = self._rms(x, e.g, True)
                x = self._conv(y, T, H, W, e.conv)
        h = self._conv(x, T, H, W, pk.conv1, out_f32=True)
        out = torch.empty(2 * self.z_dim, T, H, W, device=dev, dtype=torch.float32)
        call("sa_vae_latent_out", h.data_ptr(), h.shape[-1], self.z_dim, T * H * W, pk.mean.data_ptr(),
             pk.std.data_ptr(), out.data_ptr(), ops._stream())
        return out

    def encode(self, x, return_dict=True):
        """wan_vae.py:650-660: [B, 3, 1+4k, H, W] -> AutoencoderKLOutput(latent_dist=posterior over
        cat(mu, log_var) [B, 32, 1+k, H/8, W/8]); the pipeline takes encode(x)[0].mode()."""
        h = torch.stack([self.encode_clip(u) for u in x])
        post = DiagonalGaussianDistribution(h)
        if not return_dict:
            return (post,)
        return AutoencoderKLOutput(latent_dist=post)

    decode_chunk = 24  # latent frames per chunk of a long clip (bounds the activations to ~100 frames)

    def decode_clip(self, z, post=False, chunk=None):
        """z [16, T, h, w] fp32 (one batch item) -> [3, 1+4(T-1), 8h, 8w] fp32 in [-1,1]
        (post=True: decode_latents' [0,1] mapping, pipeline:425-430).  Clips longer than `chunk`
        latent frames are decoded chunk by chunk with the reference's causal cache carried between
        chunks (every kt=3 conv gets the last 2 input frames of the previous chunk), so memory stays
        bounded for arbitrarily long (config 5, 1000+ frame) clips and the result equals the
        whole-clip decode."""
        pk = self._pack()
        dev = pk.mean.device
        Cz, T, H, W = z.shape
        chunk = chunk or self.decode_chunk
        if self.decode_group is not None and (_world(self.decode_group) > 1 or self.decode_loopback > 1):
            return self._decode_parallel(pk, z, post, chunk)
        if T <= chunk:
            return self._decode_chunk(pk, z, True, None, post)
        out = torch.empty(3, 1 + 4 * (T - 1), 8 * H, 8 * W, device=dev, dtype=torch.float32)
        state = _SeqState()
        for c0 in range(0, T, chunk):
            c1 = min(c0 + chunk, T)
            y = self._decode_chunk(pk, z[:, c0:c1], c0 == 0, state, post)
            o0 = 0 if c0 == 0 else 1 + 4 * (c0 - 1)
            out[:, o0:o0 + y.shape[1]].copy_(y)
        return out

    def enable_multi_gpus_inference(self, group=None, loopback_ranks=0):
        """Decode over the ranks of `group` (default: the torch.distributed world): rank r decodes the r-th
        contiguous run of latent frames, taking each causal conv's 2-frame cache from rank r-1 and handing
        its own to rank r+1 (P2P, one send per cache point: a wavefront over the ranks), then one gather.
        Bit-identical to the single-GPU decode (the chunked decode == whole-clip decode).
        loopback_ranks = n > 1 on a group of ONE rank: that rank decodes the n runs in turn and every hand-off
        between them is a transfer to itself through the group's transport (the degree-1 RCCL test)."""
        import torch.distributed as dist
        self.decode_group = group if group is not None else dist.group.WORLD
        self.decode_loopback = int(loopback_ranks) if _world(self.decode_group) == 1 else 0
        return self

    decode_loopback = 0

    def disable_multi_gpus_inference(self):
        self.decode_group = None
        self.decode_loopback = 0
        return self

    def _decode_parallel(self, pk, z, post, chunk):
        import torch.distributed as dist
        import collections
        grp = self.decode_group
        N, r = _world(grp), dist.get_rank(grp)
        virt = self.decode_loopback if N == 1 else 0  # virtual ranks decoded in turn on this one rank
        dev = pk.mean.device
        Cz, T, H, W = z.shape
        n = min(max(N, virt), T)
        bounds = [round(i * T / n) for i in range(n + 1)]  # contiguous runs of latent frames
        frames = lambda i: (1 + 4 * (bounds[1] - 1)) if i == 0 else 4 * (bounds[i + 1] - bounds[i])  # noqa: E731
        fmax = max(frames(i) for i in range(n))
        buf = torch.zeros(max(1, virt), fmax, 3, 8 * H, 8 * W, device=dev, dtype=torch.float32)
        fifo = collections.deque()
        for v in (range(n) if virt else [r]):
            if v >= n:
                continue
            state = _LoopbackChain(grp, v, n, fifo) if virt else _ChainState(grp, v, n)
            bv = buf[v if virt else 0]
            o = 0
            subs = list(range(bounds[v], bounds[v + 1], chunk))
            for j, c0 in enumerate(subs):  # sub-chunks of <= `chunk` latent frames bound the activations
                c1 = min(c0 + chunk, bounds[v + 1])
                state.begin(j == 0, j == len(subs) - 1)
                y = self._decode_chunk(pk, z[:, c0:c1], c0 == 0, state, post)  # [3, F, 8H, 8W]
                bv[o:o + y.shape[1]].copy_(y.transpose(0, 1))
                o += y.shape[1]
            state.finish()
            assert o == frames(v)
        assert not fifo
        allb = _all_gather(buf.view(-1, *buf.shape[2:]) if virt else buf[0], N, grp)
        allb = allb.view(max(N, virt), fmax, *buf.shape[2:])  # [ranks, fmax, 3, 8H, 8W]
        out = torch.cat([allb[i, :frames(i)] for i in range(n)]).transpose(0, 1).contiguous()
        assert out.shape[1] == 1 + 4 * (T - 1)
        return out

    def _decode_chunk(self, pk, z, first, state, post):
        dev = pk.mean.device
        Cz, T, H, W = z.shape
        zc = z.to(device=dev, dtype=torch.float32).contiguous()
        x = torch.empty(T, H, W, pk.zp, device=dev, dtype=torch.bfloat16)
        call("sa_vae_input", zc.data_ptr(), Cz, T * H * W, pk.mean.data_ptr(), pk.std.data_ptr(), x.data_ptr(),
             pk.zp, ops._stream())
        x = self._conv(x, T, H, W, pk.conv2)
        for e in pk.layers:
            if e.kind == "conv":
                x = self._conv(x, T, H, W, e.conv, prev=self._cache(state, id(e), x))
            elif e.kind == "res":
                x = self._res(e, x, T, H, W, state)
            elif e.kind == "attn":
                x = self._attn(e, x, T, H, W)
            elif e.kind in ("up3d", "up2d"):
                x, T, H, W = self._up(e, x, T, H, W, state, first)
            elif e.kind == "head":
                y = self._rms(x, e.g, True)
                x = self._conv(y, T, H, W, e.conv, out_f32=True, prev=self._cache(state, id(e), y))
        out = torch.empty(3, T, H, W, device=dev, dtype=torch.float32)
        call("sa_vae_output", x.data_ptr(), 4, 3, T * H * W, out.data_ptr(), int(post), ops._stream())
        return out

    def decode(self, z, return_dict=True):
        """wan_vae.py:666-681: [B, 16, T, h, w] -> DecoderOutput(sample=[B, 3, 1+4(T-1), 8h, 8w])."""
        dec = torch.stack([self.decode_clip(u) for u in z])
        if not return_dict:
            return (dec,)
        return DecoderOutput(sample=dec)
