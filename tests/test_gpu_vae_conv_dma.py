"""The LDS-DMA implicit-GEMM conv (conv3d_dma_kernel, vae.hip) against the register-staged one
(SA_CONV_DMA=0, bit-identical expected: same K order and MFMA sequence) and against an fp32 torch
CausalConv3d (wan_vae.py:20-39: causal time padding 2 frames, spatial padding 1; nearest-exact 2x
upsample of Upsample :60-66; time_conv interleave of Resample 'upsample3d' :137-140)."""
import os

import pytest
import torch
import torch.nn.functional as F

from stableavatar_amd import ops
from stableavatar_amd._lib import call

pytestmark = pytest.mark.gpu
dev = "cuda"


def _conv(x, T, H, W, cin, w, b, cout, cout_pad, k, dma, residual=None, upsample=False, out_f32=False,
          interleave=0, prev=None):
    kt, kh, kw = k
    if interleave:
        out = torch.empty(2 * T, H, W, interleave, device=dev, dtype=torch.bfloat16)
    else:
        out = torch.empty(T, H, W, cout, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
    os.environ["SA_CONV_DMA"] = str(dma)
    try:
        call("sa_conv3d_cl", x.data_ptr(), T, H, W, cin, int(upsample), w.data_ptr(), b.data_ptr(), cout, cout_pad,
             kt, kh, kw, 0 if residual is None else residual.data_ptr(), out.data_ptr(), int(out_f32), interleave,
             0 if prev is None else prev.data_ptr(), ops._stream())
    finally:
        os.environ.pop("SA_CONV_DMA", None)
    torch.cuda.synchronize()
    return out


def _ref(x, T, H, W, cin, w, b, cout, k, residual=None, upsample=False, interleave=0, prev=None):
    """fp32 torch: x channels-last [T, Hin, Win, Cin] -> [T, H, W, Cout]"""
    kt, kh, kw = k
    xc = x.float().permute(3, 0, 1, 2)[None]  # [1, C, T, Hin, Win]
    if upsample:
        xc = xc.repeat_interleave(2, dim=3).repeat_interleave(2, dim=4)
    if kt > 1:
        pad = prev.float().permute(3, 0, 1, 2)[None] if prev is not None else torch.zeros_like(xc[:, :, :kt - 1])
        xc = torch.cat([pad, xc], dim=2)
    wt = w[:cout].float().reshape(cout, kt, kh, kw, cin).permute(0, 4, 1, 2, 3)
    y = F.conv3d(xc, wt, b[:cout].float(), padding=(0, (kh - 1) // 2, (kw - 1) // 2))[0].permute(1, 2, 3, 0)
    if interleave:
        y = y.reshape(T, H, W, 2, interleave).permute(0, 3, 1, 2, 4).reshape(2 * T, H, W, interleave)
    if residual is not None:
        y = y + residual.float()
    return y


CASES = [
    # (T, H, W, cin, cout, k, options)
    (3, 16, 16, 96, 96, (3, 3, 3), {}),
    (2, 16, 8, 96, 96, (3, 3, 3), {"prev": True, "residual": True}),
    (2, 16, 16, 192, 96, (1, 3, 3), {"upsample": True}),
    (3, 16, 16, 64, 192, (3, 3, 3), {"prev": True}),
    (2, 8, 16, 128, 384, (3, 3, 3), {"residual": True}),
    (2, 16, 16, 96, 4, (3, 3, 3), {"out_f32": True}),
    (2, 16, 16, 32, 96, (1, 1, 1), {}),
    (2, 16, 16, 96, 192, (3, 1, 1), {"interleave": 96, "prev": True}),
    # image rows of >= 128 pixels
    (2, 4, 128, 96, 96, (3, 3, 3), {"prev": True, "residual": True}),
    (2, 4, 256, 96, 4, (3, 3, 3), {"out_f32": True}),
    (2, 2, 128, 64, 96, (1, 3, 3), {"upsample": True}),
    (3, 2, 128, 32, 192, (3, 3, 3), {}),
]


@pytest.mark.parametrize("variant", [1, 2], ids=["rows128", "rows256"])
@pytest.mark.parametrize("case", range(len(CASES)))
def test_conv_dma_vs_register_staged_and_torch(case, variant):
    """SA_CONV_DMA: 1 = 128-row tiles; 2 (default) = 256-row tiles where H*W % 256 == 0 (2-stage ring for the
    192-wide convs)"""
    T, H, W, cin, cout, k, o = CASES[case]
    g = torch.Generator(device=dev).manual_seed(case)
    up = o.get("upsample", False)
    Hin, Win = (H // 2, W // 2) if up else (H, W)
    cout_pad = 16 if cout <= 16 else (192 * ((cout + 191) // 192) if cout > 96 else 96)
    kvol = k[0] * k[1] * k[2]
    x = torch.randn(T, Hin, Win, cin, device=dev, generator=g).bfloat16()
    w = (torch.randn(cout_pad, kvol * cin, device=dev, generator=g) / (kvol * cin) ** 0.5).bfloat16()
    b = torch.randn(cout_pad, device=dev, generator=g)
    prev = torch.randn(k[0] - 1, Hin, Win, cin, device=dev, generator=g).bfloat16() if o.get("prev") else None
    il = o.get("interleave", 0)
    res = (torch.randn(T, H, W, cout, device=dev, generator=g).bfloat16() if o.get("residual") else None)
    kw = dict(residual=res, upsample=up, out_f32=o.get("out_f32", False), interleave=il, prev=prev)
    y_dma = _conv(x, T, H, W, cin, w, b, cout, cout_pad, k, variant, **kw)
    y_reg = _conv(x, T, H, W, cin, w, b, cout, cout_pad, k, 0, **kw)
    assert torch.equal(y_dma, y_reg)
    ref = _ref(x, T, H, W, cin, w, b, cout, k, residual=res, upsample=up, interleave=il, prev=prev)
    err = ((y_dma.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("C", [96, 192, 384])
@pytest.mark.parametrize("silu", [0, 1])
def test_rmsnorm3_bit_identical(C, silu):
    """rmsnorm_silu3_kernel (every lane busy for C = 96 / 192 / 384) vs rmsnorm_silu_kernel: same sum order,
    bit-identical; and vs torch RMS_norm (wan_vae.py:42-57: F.normalize * sqrt(C) * gamma) + SiLU"""
    rows = 1000 + 37
    g = torch.Generator(device=dev).manual_seed(C + silu)
    x = (torch.randn(rows, C, device=dev, generator=g) * 3).bfloat16()
    x[5] = 0  # an all-zero row: the 1e-12 clamp
    gamma = torch.rand(C, device=dev, generator=g) + 0.5
    outs = []
    for v in ("1", "0"):
        y = torch.empty_like(x)
        os.environ["SA_RMS3"] = v
        try:
            call("sa_vae_rmsnorm_silu", x.data_ptr(), y.data_ptr(), gamma.data_ptr(), rows, C, silu, ops._stream())
        finally:
            os.environ.pop("SA_RMS3", None)
        torch.cuda.synchronize()
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    ref = F.normalize(x.float(), dim=1) * C ** 0.5 * gamma
    if silu:
        ref = F.silu(ref)
    assert ((outs[0].float() - ref).norm() / ref.norm()).item() < 1e-2
