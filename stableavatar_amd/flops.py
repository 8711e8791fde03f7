"""Analytic FLOP counts (2 FLOP per MAC, matmul/conv/attention only) used for the roofline
figures in bench.py.  Validated against torch FlopCounterMode in SURVEY.md §6 (427.8 TFLOP per
1.3B forward at B=3, L=21504)."""


def dit_forward_flops(B=3, L=21504, dim=1536, ffn=8960, layers=30, in_dim=36, text_len=512, n_img=257,
                      n_voc=17, n_frames=21, text_dim=4096):
    per_layer = (2 * B * L * dim * dim * 4                  # self q k v o
                 + 4 * B * L * L * dim                      # QK^T + PV
                 + 2 * B * L * dim * dim * 2                # cross q, o
                 + 4 * B * L * (text_len + n_img + n_voc) * dim
                 + 2 * B * L * dim * ffn * 2)               # FFN
    ctx = layers * 2 * B * (text_len + n_img + n_frames * n_voc) * dim * dim * 2
    return layers * per_layer + ctx + 2 * B * L * dim * in_dim * 4 + 2 * B * L * dim * 64 \
        + 2 * B * text_len * (text_dim * dim + dim * dim)


def self_attention_flops(B=3, L=21504, heads=12, head_dim=128):
    """QK^T + PV of one self-attention launch."""
    return 4 * B * heads * L * L * head_dim


def vae_decode_flops(T=21, h=64, w=64, dim=96, z_dim=16):
    dims = [dim * u for u in (4, 4, 4, 2, 1)]
    fl = 2 * T * h * w * z_dim * z_dim
    t, hh, ww = T, h, w
    fl += 2 * t * hh * ww * 27 * z_dim * dims[0]                          # conv1
    n = t * hh * ww
    fl += 2 * (2 * n * 27 * 2 * dims[0] * dims[0])                        # middle res x2
    fl += 2 * n * dims[0] * dims[0] * 4 + 4 * t * (hh * ww) ** 2 * dims[0]  # middle attention
    cin = dims[0]
    for i, (din, dout) in enumerate(zip(dims[:-1], dims[1:])):
        if i in (1, 2, 3):
            din //= 2
        n = t * hh * ww
        for _ in range(3):
            fl += 2 * n * 27 * (din * dout + dout * dout) + (2 * n * din * dout if din != dout else 0)
            din = dout
        if i < 3:
            if i < 2:
                fl += 2 * (t - 1) * hh * ww * 3 * dout * 2 * dout
                t = 1 + 2 * (t - 1)
            hh, ww = 2 * hh, 2 * ww
            fl += 2 * t * hh * ww * 9 * dout * (dout // 2)
        cin = dout
    fl += 2 * t * hh * ww * 27 * cin * 3                                   # head
    return fl


def vae_encode_flops(T=81, H=512, W=512, dim=96, z_dim=16):
    """Conv/attention FLOPs (2/MAC) of a whole-clip VAE encode of T = 1+4k frames (107.2 TFLOP at
    81 x 512 x 512); walks stableavatar_amd.vae.encoder_layout."""
    from .vae import encoder_layout
    fl = 0
    t, hh, ww = T, H, W
    for kind, _name, cin, cout in encoder_layout(dim):
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
    return fl + 2 * t * hh * ww * (2 * z_dim) ** 2
