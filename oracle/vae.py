"""ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

CPU fp32 restatement of the Wan-2.1 3-D causal VAE decoder and encoder (wan/models/wan_vae.py).
The reference decodes one latent frame at a time with a 2-frame causal feature cache
(wan_vae.py:549-574, CausalConv3d :20-39, Resample :104-163).  That schedule is equivalent to
running every layer over the whole clip at once with:
  * CausalConv3d: 2 zero frames of front padding (the cache supplies the real previous frames);
  * Resample 'upsample3d': frame 0 bypasses time_conv ('Rep', :108-111); frames 1.. go through a
    causal time_conv over the sub-sequence that EXCLUDES frame 0 (the first cached chunk is
    zero-filled, :123-131), then each output frame splits into two (:137-140).
The encoder (wan_vae.py:519-547) runs chunks of 1, 4, 4, ... frames with the same cache; in
whole-clip form:
  * CausalConv3d as above;
  * Resample 'downsample2d' / 'downsample3d': ZeroPad2d((0,1,0,1)) + 3x3 stride-2 conv per frame;
    'downsample3d' then keeps frame 0 (its first chunk is only cached, :145-148) and maps frames
    1.. through time_conv (3,1,1) stride 2 WITHOUT padding over [last frame of the previous chunk,
    chunk] (:150-157), i.e. output j >= 1 = time_conv(frames 2j-2, 2j-1, 2j) of the whole clip.
This module implements the whole-clip forms; tests/test_oracle_golden.py pins them against the
reference's own chunked decode / encode outputs.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

MEAN = [-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
        0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921]
STD = [2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
       3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160]


def decoder_layout(dim=96, z_dim=16, dim_mult=(1, 2, 4, 4), num_res_blocks=2, temperal_upsample=(True, True, False)):
    """Module list of Decoder3d (wan_vae.py:372-424): list of (kind, name, in, out)."""
    dims = [dim * u for u in [dim_mult[-1]] + list(dim_mult[::-1])]
    L = [("conv", "conv1", z_dim, dims[0], 3),
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


def param_shapes(dim=96, z_dim=16, **kw):
    """{name: shape} of the decoder half of AutoencoderKLWan (prefix 'model.')."""
    S = {"model.conv2.weight": (z_dim, z_dim, 1, 1, 1), "model.conv2.bias": (z_dim,)}
    p = "model.decoder."
    for kind, name, cin, cout, *_ in decoder_layout(dim, z_dim, **kw):
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


def causal_conv3d(x, w, b):
    """CausalConv3d (wan_vae.py:20-39) over a whole clip: causal time padding, symmetric space."""
    kt, kh, kw = w.shape[2:]
    x = F.pad(x, ((kw - 1) // 2, (kw - 1) // 2, (kh - 1) // 2, (kh - 1) // 2, kt - 1, 0))
    return F.conv3d(x, w, b)


def rms_norm(x, gamma):
    """RMS_norm (wan_vae.py:42-57): F.normalize over channels * sqrt(C) * gamma."""
    return F.normalize(x, dim=1) * (x.shape[1] ** 0.5) * gamma


def residual_block(P, q, x):
    """ResidualBlock (wan_vae.py:189-223)."""
    h = causal_conv3d(x, P[q + ".shortcut.weight"], P[q + ".shortcut.bias"]) if q + ".shortcut.weight" in P else x
    y = F.silu(rms_norm(x, P[q + ".residual.0.gamma"]))
    y = causal_conv3d(y, P[q + ".residual.2.weight"], P[q + ".residual.2.bias"])
    y = F.silu(rms_norm(y, P[q + ".residual.3.gamma"]))
    y = causal_conv3d(y, P[q + ".residual.6.weight"], P[q + ".residual.6.bias"])
    return y + h


def attention_block(P, q, x):
    """AttentionBlock (wan_vae.py:226-265): single-head spatial attention per frame."""
    b, c, t, h, w = x.shape
    idn = x
    y = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    y = rms_norm(y, P[q + ".norm.gamma"])
    qkv = F.conv2d(y, P[q + ".to_qkv.weight"], P[q + ".to_qkv.bias"])
    qkv = qkv.reshape(b * t, 1, c * 3, -1).permute(0, 1, 3, 2).contiguous()
    qq, kk, vv = qkv.chunk(3, dim=-1)
    o = F.scaled_dot_product_attention(qq, kk, vv)
    o = o.squeeze(1).permute(0, 2, 1).reshape(b * t, c, h, w)
    o = F.conv2d(o, P[q + ".proj.weight"], P[q + ".proj.bias"])
    return o.reshape(b, t, c, h, w).permute(0, 2, 1, 3, 4) + idn


def resample_up(P, q, x, temporal):
    """Resample upsample2d/upsample3d (wan_vae.py:69-163) in whole-clip form."""
    b, c, t, h, w = x.shape
    if temporal and t > 1:
        rest = causal_conv3d(x[:, :, 1:], P[q + ".time_conv.weight"], P[q + ".time_conv.bias"])
        rest = rest.reshape(b, 2, c, t - 1, h, w)
        rest = torch.stack((rest[:, 0], rest[:, 1]), 3).reshape(b, c, (t - 1) * 2, h, w)
        x = torch.cat([x[:, :, :1], rest], 2)
    t = x.shape[2]
    y = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    y = F.interpolate(y, scale_factor=(2.0, 2.0), mode="nearest-exact")
    y = F.conv2d(y, P[q + ".resample.1.weight"], P[q + ".resample.1.bias"], padding=1)
    return y.reshape(b, t, y.shape[1], 2 * h, 2 * w).permute(0, 2, 1, 3, 4)


def decode(P, z, dim=96, z_dim=16, **kw):
    """AutoencoderKLWan.decode(z).sample (wan_vae.py:666-681, :549-574): z [B,16,T,h,w] ->
    [B,3,1+4(T-1),8h,8w] clamped to [-1, 1]."""
    mean = torch.tensor(MEAN, dtype=torch.float32).view(1, z_dim, 1, 1, 1)
    std = torch.tensor(STD, dtype=torch.float32).view(1, z_dim, 1, 1, 1)
    x = z.float() * std + mean   # z / (1/std) + mean
    x = causal_conv3d(x, P["model.conv2.weight"], P["model.conv2.bias"])
    p = "model.decoder."
    for kind, name, cin, cout, *_ in decoder_layout(dim, z_dim, **kw):
        q = p + name
        if kind == "conv":
            x = causal_conv3d(x, P[q + ".weight"], P[q + ".bias"])
        elif kind == "res":
            x = residual_block(P, q, x)
        elif kind == "attn":
            x = attention_block(P, q, x)
        elif kind == "up3d":
            x = resample_up(P, q, x, True)
        elif kind == "up2d":
            x = resample_up(P, q, x, False)
        elif kind == "head":
            x = F.silu(rms_norm(x, P[q + ".0.gamma"]))
            x = causal_conv3d(x, P[q + ".2.weight"], P[q + ".2.bias"])
    return x.clamp(-1, 1)


def flops_decode(T, h, w, dim=96, z_dim=16):
    """Analytic conv/attention FLOPs (2/MAC) of a whole-clip decode."""
    fl = 0
    t, hh, ww = T, h, w
    fl += 2 * t * hh * ww * z_dim * z_dim
    for kind, name, cin, cout, *_ in decoder_layout(dim, z_dim):
        n = t * hh * ww
        if kind == "conv":
            fl += 2 * n * 27 * cin * cout
        elif kind == "res":
            fl += 2 * n * 27 * (cin * cout + cout * cout) + (2 * n * cin * cout if cin != cout else 0)
        elif kind == "attn":
            fl += 2 * n * cin * cin * 4 + 4 * t * (hh * ww) ** 2 * cin
        elif kind in ("up3d", "up2d"):
            if kind == "up3d":
                fl += 2 * (t - 1) * hh * ww * 3 * cin * 2 * cin
                t = 1 + 2 * (t - 1)
            hh, ww = 2 * hh, 2 * ww
            fl += 2 * t * hh * ww * 9 * cin * cout
        elif kind == "head":
            fl += 2 * n * 27 * cin * cout
    return fl


def encoder_layout(dim=96, dim_mult=(1, 2, 4, 4), num_res_blocks=2, temperal_downsample=(False, True, True)):
    """Module list of Encoder3d (wan_vae.py:268-319): list of (kind, name, in, out)."""
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
    """{name: shape} of the encoder half of AutoencoderKLWan (prefix 'model.'); head -> 2*z_dim."""
    S = {"model.conv1.weight": (2 * z_dim, 2 * z_dim, 1, 1, 1), "model.conv1.bias": (2 * z_dim,)}
    p = "model.encoder."
    for kind, name, cin, cout in encoder_layout(dim):
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


def resample_down(P, q, x, temporal):
    """Resample downsample2d/downsample3d (wan_vae.py:91-100, :142-157) in whole-clip form."""
    b, c, t, h, w = x.shape
    y = x.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w)
    y = F.conv2d(F.pad(y, (0, 1, 0, 1)), P[q + ".resample.1.weight"], P[q + ".resample.1.bias"], stride=2)
    x = y.reshape(b, t, c, y.shape[2], y.shape[3]).permute(0, 2, 1, 3, 4)
    if temporal and t > 1:
        rest = F.conv3d(x, P[q + ".time_conv.weight"], P[q + ".time_conv.bias"], stride=(2, 1, 1))
        x = torch.cat([x[:, :, :1], rest], 2)
    return x


def encode(P, x, dim=96, z_dim=16):
    """AutoencoderKLWan._encode(x) (wan_vae.py:519-547, :643-648): video [B,3,1+4k,H,W] in [-1,1] ->
    [B, 2*z_dim, 1+k, H/8, W/8] = cat(normalised mu, log_var) (the posterior's parameters; .mode() is
    the first z_dim channels)."""
    x = x.float()
    if (x.shape[2] - 1) % 4:
        raise ValueError("the chunked encoder consumes 1 + 4k frames")
    p = "model.encoder."
    for kind, name, cin, cout in encoder_layout(dim):
        q = p + name
        if kind == "conv":
            x = causal_conv3d(x, P[q + ".weight"], P[q + ".bias"])
        elif kind == "res":
            x = residual_block(P, q, x)
        elif kind == "attn":
            x = attention_block(P, q, x)
        elif kind in ("down2d", "down3d"):
            x = resample_down(P, q, x, kind == "down3d")
        elif kind == "head":
            x = F.silu(rms_norm(x, P[q + ".0.gamma"]))
            x = causal_conv3d(x, P[q + ".2.weight"], P[q + ".2.bias"])
    x = causal_conv3d(x, P["model.conv1.weight"], P["model.conv1.bias"])
    mu, log_var = x.chunk(2, dim=1)
    mean = torch.tensor(MEAN, dtype=torch.float32).view(1, z_dim, 1, 1, 1)
    std = torch.tensor(STD, dtype=torch.float32).view(1, z_dim, 1, 1, 1)
    return torch.cat([(mu - mean) * (1.0 / std), log_var], 1)


def flops_encode(T, H, W, dim=96, z_dim=16):
    """Analytic conv/attention FLOPs (2/MAC) of a whole-clip encode of T = 1+4k frames at H x W."""
    fl = 0
    t, hh, ww = T, H, W
    for kind, name, cin, cout in encoder_layout(dim):
        n = t * hh * ww
        if kind == "conv":
            fl += 2 * n * 27 * cin * cout
        elif kind == "res":
            fl += 2 * n * 27 * (cin * cout + cout * cout) + (2 * n * cin * cout if cin != cout else 0)
        elif kind == "attn":
            fl += 2 * n * cin * cin * 4 + 4 * t * (hh * ww) ** 2 * cin
        elif kind in ("down2d", "down3d"):
            hh, ww = hh // 2, ww // 2
            fl += 2 * t * hh * ww * 9 * cin * cout
            if kind == "down3d":
                t = 1 + (t - 1) // 2
                fl += 2 * (t - 1) * hh * ww * 3 * cout * cout
        elif kind == "head":
            fl += 2 * n * 27 * cin * 2 * z_dim
    fl += 2 * t * hh * ww * (2 * z_dim) ** 2
    return fl
