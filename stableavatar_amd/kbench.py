"""Kernel micro-benchmarks at the config-2 (512x512x81f, CFG batch 3) shapes of the DiT.
python -m stableavatar_amd.kbench  -> one JSON line per kernel with TFLOP/s (random data)."""
from __future__ import annotations

import json
import sys

import torch

from . import ops


def _time(fn, iters=10, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def vt_layout(v, mode, rows_pad=64):
    """V^T in the layout self-attention kernels 3 / 4 read (sa_attn_fwd_map): [H*128, Rv] bf16, row h*128 + d = d of
    head h for every key row (rows padded with zeros to a multiple of rows_pad).  mode 3: the keys of each 32-key
    chunk in P's permuted order (position 8g + j <- key 4g + j for j < 4, 16 + 4g + j - 4 for j >= 4); mode 4: natural
    order.  Built by torch (tests / A-B only; the DiT's QKV GEMM writes it itself)."""
    R, HD = v.shape
    Rv = (R + rows_pad - 1) // rows_pad * rows_pad + 64  # + one 64-key block: a ragged last block stages all 64
    vt = torch.zeros(HD, Rv, device=v.device, dtype=v.dtype)
    vt[:, :R] = v.t()
    if mode == 3:
        p = torch.arange(32, device=v.device)
        perm = torch.where(p % 8 < 4, 4 * (p // 8) + p % 8, 16 + 4 * (p // 8) + p % 8 - 4)
        idx = (torch.arange(Rv, device=v.device) // 32) * 32 + perm[torch.arange(Rv, device=v.device) % 32]
        vt = vt[:, idx].contiguous()
    return vt


def main(which=("gemm", "attn")):
    dev = "cuda"
    torch.manual_seed(0)
    M = 3 * 21504
    res = []
    if "gemmvar" in which:  # A/B of the GEMM kernels in one process (rule: interleaved rounds)
        import os
        # spec "K" or "K:G": K = kernel (0 auto, 1 ping-pong, 2 persistent), G = tile-raster group_m
        gvars = tuple(os.environ.get("SA_KB_GVARS", "1,2").split(","))
        for (Mx, N, K, epi, name) in [(M, 4608, 1536, ops.EPI_BF16, "qkv"), (M, 1536, 1536, ops.EPI_RES_F32, "o_proj"),
                                      (M, 1536, 1536, ops.EPI_BF16, "cross_q"),
                                      (M, 8960, 1536, ops.EPI_GELU_TANH_BF16, "ffn_up"),
                                      (M, 1536, 8960, ops.EPI_RES_F32, "ffn_down"),
                                      (M, 1536, 8960, ops.EPI_BF16, "ffn_down_bf16"),
                                      (M, 1536, 1536, ops.EPI_BF16_TP32, "v_t"),
                                      (8192, 8192, 8192, ops.EPI_BF16, "sq8192")]:
            if os.environ.get("SA_KB_SHAPES") and name not in os.environ["SA_KB_SHAPES"].split(","):
                continue
            x = (torch.rand(Mx, K, device=dev) * 2 - 1).bfloat16()
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
            b = torch.randn(N, device=dev)
            if epi == ops.EPI_BF16_TP32:  # the V^T operand of self-attention: [N, M rounded up to 64]
                out = torch.empty(N, (Mx + 63) // 64 * 64, device=dev, dtype=torch.bfloat16)
            else:
                out = torch.empty(Mx, N, device=dev, dtype=torch.float32 if epi == ops.EPI_RES_F32 else torch.bfloat16)
            gate = torch.randn(3, N, device=dev)
            ref = None
            times = {v: [] for v in gvars}
            same = {}
            for rnd in range(3):
                for v in gvars:
                    vv, _, gm = v.partition(":")
                    kw = dict(kernel=int(vv), group_m=int(gm or 0))
                    if epi == ops.EPI_RES_F32:
                        out.zero_()
                        fn = lambda: ops.linear(x, w, b, epi, out=out, residual=out, gate=gate, rows_per_batch=21504,
                                                **kw)
                    else:
                        fn = lambda: ops.linear(x, w, b, epi, out=out, **kw)
                    times[v].append(_time(fn, iters=5, warmup=1))
                    if epi == ops.EPI_RES_F32:  # one clean launch on a zero residual for the comparison
                        out.zero_()
                        ops.linear(x, w, b, epi, out=out, residual=out, gate=gate, rows_per_batch=21504, **kw)
                    o = out.float()
                    if ref is None:
                        ref = o.clone()
                    if int(vv) >= 8 or os.environ.get("SA_KB_NOCHECK"):  # measurement kernels / builds
                        continue
                    err = ((o - ref).norm() / ref.norm()).item()
                    assert err < 1e-2, (name, v, err)
                    same.setdefault(v, True)
                    same[v] = same[v] and bool(torch.equal(o, ref))
            fl = 2.0 * Mx * N * K
            r = {"kernel": f"gemm_{name}", "M": Mx, "N": N, "K": K}
            ms_ref = _time(lambda: torch.nn.functional.linear(x, w), iters=5, warmup=1)
            r["torch_tflops"] = round(fl / ms_ref / 1e9, 1)
            for v in gvars:
                ms = sorted(times[v])[1]
                r[f"v{v}_ms"] = round(ms, 4)
                r[f"v{v}_tflops"] = round(fl / ms / 1e9, 1)
                r[f"v{v}_bitident"] = same.get(v)
            res.append(r)
            print(json.dumps(r), flush=True)
            del x, w, out
    if "attnvar" in which:
        import os
        L, H, D = 21504, 12, 128
        qkv = torch.randn(3 * L, 3 * H * D, device=dev).bfloat16()
        segs = torch.tensor([[b * L, L, b * L, L] for b in range(3)], dtype=torch.int32, device=dev)
        q, k, v_ = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
        outs = {}
        variants = tuple(int(v) for v in os.environ.get("SA_KB_AVARS", "1").split(","))
        vts = {m: vt_layout(v_, 3) for m in (3,) if m in variants}  # kernel 3 reads V^T
        times = {v: [] for v in variants}
        for rnd in range(3):
            for v in variants:
                o = torch.empty(3 * L, H * D, device=dev, dtype=torch.bfloat16)
                vin = vts.get(v, v_)
                times[v].append(_time(lambda: ops.attention(q, k, vin, o, segs, 3, L, H, kernel=v), iters=3, warmup=1))
                outs[v] = o.float()
        # fp32 reference on a sample of query rows of every head (batch row 2)
        qi = torch.arange(0, L, 997, device=dev)
        ref = torch.empty(len(qi), H * D, device=dev)
        for hh in range(H):
            sl = slice(hh * D, (hh + 1) * D)
            s_ = (q[2 * L + qi, sl].float() @ k[2 * L:, sl].float().t()) * D ** -0.5
            ref[:, sl] = torch.softmax(s_, -1) @ v_[2 * L:, sl].float()
        fl = 4.0 * 3 * H * L * L * D
        r = {"kernel": "attn_self"}
        for v in variants:
            ms = sorted(times[v])[1]
            r[f"err_v{v}_v{variants[0]}"] = ((outs[v] - outs[variants[0]]).norm() / outs[variants[0]].norm()).item()
            r[f"v{v}_bitident"] = bool(torch.equal(outs[v], outs[variants[0]]))
            r[f"err_v{v}_fp32"] = ((outs[v][2 * L + qi] - ref).norm() / ref.norm()).item()
            r[f"v{v}_ms"] = round(ms, 3)
            r[f"v{v}_tflops"] = round(fl / ms / 1e9, 1)
        res.append(r)
        print(json.dumps(r), flush=True)
    if "attnclip" in which:
        res.extend(attn_clip_inputs())
    if "cross3" in which:  # the fused text + image + per-frame vocal cross-attention at config 2
        L, H, D, B, nper, nfr = 21504, 12, 128, 3, 32, 21
        q = torch.randn(B * L, H * D, device=dev).bfloat16()
        kvt = torch.randn(B * 512, 2 * H * D, device=dev).bfloat16()
        kvi = torch.randn(B * 257, 2 * H * D, device=dev).bfloat16()
        kvv = torch.randn(B * nfr * nper, 2 * H * D, device=dev).bfloat16()
        o = torch.empty(B * L, H * D, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.attention_cross3(q, kvt[:, :H * D], kvt[:, H * D:], 512, kvi[:, :H * D], kvi[:, H * D:], 257,
                                          kvv[:, :H * D], kvv[:, H * D:], nper, L // nfr, nfr, o, B, L, H)
        ms = sorted(_time(fn, iters=20, warmup=3) for _ in range(5))[2]
        fl = 4.0 * B * H * L * D * (512 + 257 + nper)
        import hashlib
        r = {"kernel": "attn_cross3", "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
             "out_sum": float(o.float().abs().sum()),
             "out_sha": hashlib.sha256(o.view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:16]}
        res.append(r)
        print(json.dumps(r), flush=True)
    if "gemm" in which:
        for (N, K, epi, name) in [(4608, 1536, ops.EPI_BF16, "qkv"), (1536, 1536, ops.EPI_RES_F32, "o_proj"),
                                  (8960, 1536, ops.EPI_GELU_TANH_BF16, "ffn_up"),
                                  (1536, 8960, ops.EPI_RES_F32, "ffn_down")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
            b = torch.randn(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=torch.float32 if epi == ops.EPI_RES_F32 else torch.bfloat16)
            gate = torch.randn(3, N, device=dev)
            if epi == ops.EPI_RES_F32:
                fn = lambda: ops.linear(x, w, b, epi, out=out, residual=out, gate=gate, rows_per_batch=21504)
            else:
                fn = lambda: ops.linear(x, w, b, epi, out=out)
            ms = _time(fn)
            ms_ref = _time(lambda: torch.nn.functional.linear(x, w))
            fl = 2.0 * M * N * K
            res.append({"kernel": f"gemm_{name}", "M": M, "N": N, "K": K, "ms": round(ms, 4),
                        "tflops": round(fl / ms / 1e9, 1), "torch_ms": round(ms_ref, 4),
                        "torch_tflops": round(fl / ms_ref / 1e9, 1)})
            print(json.dumps(res[-1]), flush=True)
            del x, w, out
    if "attn" in which:
        L, H, D = 21504, 12, 128
        qkv = torch.randn(3 * L, 3 * H * D, device=dev).bfloat16()
        o = torch.empty(3 * L, H * D, device=dev, dtype=torch.bfloat16)
        segs = torch.tensor([[b * L, L, b * L, L] for b in range(3)], dtype=torch.int32, device=dev)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
        fn = lambda: ops.attention(q, k, v, o, segs, 3, L, H)
        ms = _time(fn, iters=5)
        fl = 4.0 * 3 * H * L * L * D
        qh = q.view(3, L, H, D).transpose(1, 2)
        kh = k.view(3, L, H, D).transpose(1, 2)
        vh = v.view(3, L, H, D).transpose(1, 2)
        try:
            ms_ref = _time(lambda: torch.nn.functional.scaled_dot_product_attention(qh, kh, vh), iters=3)
        except Exception:  # noqa: BLE001
            ms_ref = float("nan")
        res.append({"kernel": "attn_self", "L": L, "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1),
                    "torch_sdpa_ms": round(ms_ref, 3), "torch_tflops": round(fl / ms_ref / 1e9, 1)})
        print(json.dumps(res[-1]), flush=True)
    if "gemmsq" in which:  # square shapes of the guide's GEMM template figures (random [-1, 1) operands)
        for n in (4096, 8192):
            x = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16()
            w = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16()
            out = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
            ms = _time(lambda: ops.linear(x, w, None, ops.EPI_BF16, out=out), iters=10, warmup=3)
            ms_ref = _time(lambda: torch.nn.functional.linear(x, w), iters=10, warmup=3)
            fl = 2.0 * n ** 3
            res.append({"kernel": f"gemm_sq{n}", "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
                        "torch_tflops": round(fl / ms_ref / 1e9, 1)})
            print(json.dumps(res[-1]), flush=True)
            del x, w, out
    if "attn1" in which:  # 3 bare self-attention launches (PMC passes: FETCH_SIZE / WRITE_SIZE)
        L, H, D = 21504, 12, 128
        qkv = torch.randn(3 * L, 3 * H * D, device=dev).bfloat16()
        o = torch.empty(3 * L, H * D, device=dev, dtype=torch.bfloat16)
        segs = torch.tensor([[b * L, L, b * L, L] for b in range(3)], dtype=torch.int32, device=dev)
        for _ in range(3):
            ops.attention(qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:], o, segs, 3, L, H)
        torch.cuda.synchronize()
        res.append({"kernel": "attn_self_x3", "algorithmic_bytes_per_launch": 4 * 3 * L * H * D * 2})
        print(json.dumps(res[-1]), flush=True)
    if "gemm1" in which:  # one launch of each DiT GEMM shape (PMC passes)
        for (N, K, epi, name) in [(4608, 1536, ops.EPI_BF16, "qkv"), (1536, 1536, ops.EPI_RES_F32, "o_proj"),
                                  (8960, 1536, ops.EPI_GELU_TANH_BF16, "ffn_up"),
                                  (1536, 8960, ops.EPI_RES_F32, "ffn_down")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
            b = torch.randn(N, device=dev)
            out = torch.zeros(M, N, device=dev, dtype=torch.float32 if epi == ops.EPI_RES_F32 else torch.bfloat16)
            if epi == ops.EPI_RES_F32:
                ops.linear(x, w, b, epi, out=out, residual=out)
            else:
                ops.linear(x, w, b, epi, out=out)
            torch.cuda.synchronize()
            del x, w, out
        res.append({"kernel": "gemm_x4"})
        print(json.dumps(res[-1]), flush=True)
    if "dit" in which:
        res.append(bench_dit())
        print(json.dumps(res[-1]), flush=True)
    if "dit14" in which:
        res.append(bench_dit14())
        print(json.dumps(res[-1]), flush=True)
    if "dit14full" in which:  # BASELINE config 4's model: one whole 40-layer forward at 720p x 81 frames
        res.append(bench_dit14(layer_counts=(40,)))
        print(json.dumps(res[-1]), flush=True)
    if "lnvar" in which:  # LayerNorm: one row per wave vs rows sharing the modulation through LDS (interleaved)
        import os
        x = torch.randn(M, 1536, device=dev)
        em = torch.randn(3, 6, 1536, device=dev)
        w, bb = torch.randn(1536, device=dev), torch.randn(1536, device=dev)
        ob = torch.empty(M, 1536, device=dev, dtype=torch.bfloat16)
        modes = {"adaln": dict(shift=em[:, 0], scale=em[:, 1], rows_per_batch=21504),
                 "affine": dict(weight=w, bias=bb)}
        nws = os.environ.get("SA_KB_LNVARS", "0,8,16").split(",")
        for name, kw in modes.items():
            times = {v: [] for v in nws}
            for rnd in range(3):
                for v in nws:
                    os.environ["SA_LN_SHARED"] = v
                    times[v].append(_time(lambda: ops.layernorm_mod(x, ob, 1e-6, **kw), iters=20, warmup=3))
            os.environ.pop("SA_LN_SHARED", None)
            r = {"kernel": f"layernorm_{name}", "M": M}
            for v in nws:
                ms = sorted(times[v])[1]
                r[f"rows{v}_us"] = round(ms * 1e3, 1)
                r[f"rows{v}_tbs"] = round(M * 1536 * 6 / ms / 1e9, 2)
            res.append(r)
            print(json.dumps(r), flush=True)
    if "ditenv" in which:  # in-situ A/B of an environment switch inside full DiT forwards (SA_KB_ENVVARS)
        import os
        res.append(bench_dit(env_variants=tuple(os.environ.get("SA_KB_ENVVARS", "SA_LN_SHARED=0,SA_LN_SHARED=8")
                                                .split(","))))
        print(json.dumps(res[-1]), flush=True)
    if "ditvar" in which:  # in-situ A/B of attention variants inside full DiT forwards (interleaved)
        import os
        avars = tuple(int(v) for v in os.environ.get("SA_KB_AVARS", "1").split(","))
        res.append(bench_dit(attn_variants=avars))
        print(json.dumps(res[-1]), flush=True)
    return res


def bench_dit14(layer_counts=(1, 2)):
    """BASELINE config 4's model on one GPU: WanTransformer3DFantasy14BModel (dim 5120, 40 heads, ffn 13824)
    at 720x1280 (90x160 latent, 21 latent frames: L = 75 600 tokens, B = 3 CFG rows), forwards with 1 and 2
    layers; the difference is one block's time, the remainder the embeddings + 14B vocal projector + head."""
    from . import synthetic
    from .flops import dit_forward_flops
    from .transformer import WanTransformer3DFantasy14BModel, param_shapes
    cfg = dict(model_type="i2v", dim=5120, ffn_dim=13824, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
               num_heads=40, text_len=512)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    lat = torch.randn(1, 16, 21, 90, 160, device=dev, generator=g).bfloat16()
    y = torch.randn(3, 20, 21, 90, 160, device=dev, generator=g).bfloat16()
    ctx = [torch.randn(n, 4096, device=dev, generator=g) for n in (120, 120, 60)]
    clip = torch.randn(3, 257, 1280, device=dev, generator=g)
    a = torch.randn(1, 161, 768, device=dev, generator=g)
    voc = torch.cat([torch.zeros_like(a), a, a])
    t = torch.tensor([990.0], device=dev)
    L = 21 * 45 * 80
    ms = {}
    for nl in layer_counts:
        m = WanTransformer3DFantasy14BModel(**cfg, num_layers=nl).to(dev)
        m.load_state_dict(synthetic.fill_state_dict(param_shapes(dict(cfg, num_layers=nl, vocal="14B")), 0,
                                                    backend="torch", device=dev))
        print(f"[kbench] dit14: {nl}-layer model loaded, timing", file=sys.stderr, flush=True)
        with torch.no_grad():
            ms[nl] = _time(lambda: m.forward_window(lat, 0, True, 3, t, ctx, L, clip, y, voc, 81), iters=2, warmup=1)
        del m
        torch.cuda.empty_cache()
    if tuple(layer_counts) == (40,):  # the whole 40-layer forward, measured
        fl_fwd = dit_forward_flops(B=3, L=L, dim=5120, ffn=13824, layers=40)
        return {"kernel": "dit14_forward_720p_40_layers", "L": L, "ms_forward": round(ms[40], 0),
                "tflop_per_forward": round(fl_fwd / 1e12, 0), "tflops": round(fl_fwd / ms[40] / 1e9, 1),
                "clip_s_projected_50_steps": round(50 * ms[40] / 1e3, 0)}
    per_layer = ms[2] - ms[1]
    fl_layer = dit_forward_flops(B=3, L=L, dim=5120, ffn=13824, layers=1) - dit_forward_flops(
        B=3, L=L, dim=5120, ffn=13824, layers=0)
    fl_fwd = dit_forward_flops(B=3, L=L, dim=5120, ffn=13824, layers=40)
    fwd40 = ms[1] - per_layer + 40 * per_layer
    return {"kernel": "dit14_forward_720p", "L": L, "ms_1_layer": round(ms[1], 1), "ms_2_layers": round(ms[2], 1),
            "ms_per_layer": round(per_layer, 1), "tflops_per_layer": round(fl_layer / per_layer / 1e9, 1),
            "ms_forward_40_layers_projected": round(fwd40, 0), "tflop_per_forward": round(fl_fwd / 1e12, 0),
            "tflops_forward_projected": round(fl_fwd / fwd40 / 1e9, 1)}


def attn_clip_inputs(layers=(0, 15, 29)):
    """The self-attention launches' operands of one config-2 DiT forward (random-init weights, bench_dit's
    inputs) against random operands of the same shapes: per captured layer, the launch time with q/k and V^T each
    from the forward or from randn (2 x 2), so a difference splits into the scores' side (rescale frequency) and
    the data's side (switching power)."""
    from . import ops as _ops
    captured, calls = [], [0]
    real = _ops.attention

    def spy(q, k, v, o, segs, B, L, H, **kw):
        if kw.get("kernel") == _ops.ATTN_VT_P32:
            if calls[0] in layers:
                captured.append((calls[0], q.clone(), k.clone(), v.clone(), segs.clone(), B, L, H))
            calls[0] += 1
        return real(q, k, v, o, segs, B, L, H, **kw)
    fwd = bench_dit(fwd_only=True)
    _ops.attention = spy
    try:
        with torch.no_grad():
            fwd()
    finally:
        _ops.attention = real
    torch.cuda.synchronize()
    out = []
    for (li, q, k, vt, segs, B, L, H) in captured:
        qr, kr = torch.randn_like(q.float()).bfloat16(), torch.randn_like(k.float()).bfloat16()
        vr = torch.randn_like(vt.float()).bfloat16()
        o = torch.empty(B * L, H * 128, device=q.device, dtype=torch.bfloat16)
        combos = {"qk_clip_v_clip": (q, k, vt), "qk_rand_v_clip": (qr, kr, vt), "qk_clip_v_rand": (q, k, vr),
                  "qk_rand_v_rand": (qr, kr, vr)}
        times = {c: [] for c in combos}
        for _ in range(3):
            for c, (a, b_, v) in combos.items():
                times[c].append(_time(lambda: real(a, b_, v, o, segs, B, L, H, kernel=_ops.ATTN_VT_P32), iters=3,
                                      warmup=1))
        # scaled score statistics on a sample of rows (head 0, batch row 0): spread of the row max, log2 units
        qs = q[:L:997, :128].float()
        sc = qs @ k[:L, :128].float().t() * (128 ** -0.5) * 1.4426950408889634
        r = {"kernel": "attn_clip_inputs", "layer": li, "q_rms": round(q.float().pow(2).mean().sqrt().item(), 3),
             "k_rms": round(k.float().pow(2).mean().sqrt().item(), 3),
             "row_max_log2_mean": round(sc.max(1).values.mean().item(), 2),
             "score_std_log2": round(sc.std().item(), 2)}
        for c in combos:
            r[f"{c}_ms"] = round(sorted(times[c])[1], 3)
        out.append(r)
        print(json.dumps(r), flush=True)
    return out


def bench_dit(iters=3, attn_variants=None, env_variants=None, fwd_only=False):
    """One full 30-layer DiT forward at config 2 (B=3 CFG, 21 latent frames at 64x64, L=21504).
    attn_variants: time the forward under each self-attention schedule, interleaved rounds."""
    from . import synthetic
    from .transformer import WanTransformer3DFantasyModel, param_shapes
    cfg = dict(model_type="i2v", dim=1536, ffn_dim=8960, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
               num_heads=12, num_layers=30, text_len=512)
    dev = "cuda"
    m = WanTransformer3DFantasyModel(**cfg)
    m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), 0, backend="torch", device=dev))
    m = m.to(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    lat = torch.randn(1, 16, 21, 64, 64, device=dev, generator=g).bfloat16()
    y = torch.randn(3, 20, 21, 64, 64, device=dev, generator=g).bfloat16()
    ctx = [torch.randn(n, 4096, device=dev, generator=g) for n in (120, 120, 60)]
    clip = torch.randn(3, 257, 1280, device=dev, generator=g)
    voc = torch.randn(3, 167, 768, device=dev, generator=g)
    t = torch.tensor([990.0], device=dev)

    def fwd():
        return m.forward_window(lat, 0, True, 3, t, ctx, 21504, clip, y, voc, 81)

    if fwd_only:
        return fwd
    from .flops import dit_forward_flops
    fl = dit_forward_flops()
    if env_variants:  # "K=V" settings of one environment switch read per call by the library, interleaved
        import os
        times = {v: [] for v in env_variants}
        with torch.no_grad():
            for _ in range(3):
                for v in env_variants:
                    k, _, val = v.partition("=")
                    os.environ[k] = val
                    times[v].append(_time(fwd, iters=2, warmup=1))
                    os.environ.pop(k, None)
        r = {"kernel": "dit_forward_env_ab", "tflop": round(fl / 1e12, 1)}
        for v in env_variants:
            r[f"{v}_ms"] = round(sorted(times[v])[1], 2)
        return r
    if attn_variants:
        times = {v: [] for v in attn_variants}
        with torch.no_grad():
            for _ in range(3):
                for v in attn_variants:
                    m.attn_kernel = v
                    times[v].append(_time(fwd, iters=2, warmup=1))
        m.attn_kernel = 0
        r = {"kernel": "dit_forward_attn_ab", "tflop": round(fl / 1e12, 1)}
        for v in attn_variants:
            r[f"attn_v{v}_ms"] = round(sorted(times[v])[1], 2)
        return r
    with torch.no_grad():
        ms = _time(fwd, iters=iters, warmup=1)
    return {"kernel": "dit_forward", "ms": round(ms, 2), "tflop": round(fl / 1e12, 1),
            "tflops": round(fl / ms / 1e9, 1)}


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("gemm", "attn"))
