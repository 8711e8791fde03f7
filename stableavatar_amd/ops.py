"""Tensor-level wrappers over the C ABI.  Every function launches HIP kernels from
libstableavatar_hip.so on the current torch stream; there is no CPU / eager fallback.
Tensors must already live on the GPU with the dtype/layout documented per function.
"""
from __future__ import annotations

import os

import torch

from ._lib import call

EPI_BF16, EPI_GELU_TANH_BF16, EPI_F32, EPI_RES_F32, EPI_GELU_ERF_BF16, EPI_SILU_F32, EPI_BF16_T, EPI_BF16_TP32 = range(8)
F32, BF16 = 0, 1


def _p(t):
    return 0 if t is None else t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _dt(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    raise TypeError(f"unsupported dtype {t.dtype}")


_N_CU = {}


def _n_cu(device) -> int:
    """compute units of a device (cached)"""
    i = torch.device(device).index or 0
    if i not in _N_CU:
        _N_CU[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return _N_CU[i]


def _check(t, dtype, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: expected a GPU tensor")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


GEMM_AUTO, GEMM_PINGPONG, GEMM_PERSISTENT, GEMM_PERSISTENT192 = 0, 1, 2, 3
# the persistent kernel on the three-barrier (s9) K schedule: tile rows by auto / 256 / 192
GEMM_S9_AUTO, GEMM_S9, GEMM_S9_192 = 5, 6, 7


def linear(x, weight, bias=None, epilogue=EPI_BF16, out=None, residual=None, gate=None, rows_per_batch=0,
           kernel=GEMM_AUTO, group_m=0, a_panels=None):
    """y = epi(x @ weight^T + bias).  x: bf16 [M, K] (row stride may exceed K), weight: bf16 [N, K].
    EPI_RES_F32: out(f32) = residual + y * gate[row // rows_per_batch] (gate f32 [B, N] view).
    kernel / group_m: per-call GEMM schedule selection (A/B benchmarks and tests; default auto).
    a_panels = (panel_cols, panel_stride): x is the first of K / panel_cols column panels [M, panel_cols],
    panel p starting panel_stride elements after x (sa_gemm_bf16_panels; EPI_RES_F32 only)."""
    _check(x, torch.bfloat16, "linear.x")
    _check(weight, torch.bfloat16, "linear.weight")
    M, K = x.shape
    N = weight.shape[0]
    pc = ps = 0
    if a_panels is not None:
        pc, ps = a_panels
        if K != pc or weight.shape[1] % pc or epilogue != EPI_RES_F32:
            raise ValueError("linear: a_panels needs x = the first [M, panel_cols] panel and EPI_RES_F32")
        K = weight.shape[1]
        base = x.untyped_storage().data_ptr()
        end = x.data_ptr() + ((K // pc - 1) * ps + (M - 1) * x.stride(0) + pc) * 2
        if end > base + x.untyped_storage().nbytes():
            raise ValueError("linear: the column panels run past x's storage")
    assert weight.shape[1] == K and x.stride(1) == 1 and weight.stride(1) == 1
    f32_out = epilogue in (EPI_F32, EPI_RES_F32, EPI_SILU_F32)
    if epilogue in (EPI_BF16_T, EPI_BF16_TP32):  # out = C^T [N, >= M] (row n = column n of the product: V^T)
        if out is None:  # zeroed: attention kernels 3 / 4 read the pad columns as masked keys (must be finite), and
            # 64 columns past ceil64(M) cover the whole 64-key block a segment's ragged last block stages
            out = torch.zeros(N, (M + 63) // 64 * 64 + 64, device=x.device, dtype=torch.bfloat16)
        if out.dtype != torch.bfloat16 or out.stride(1) != 1 or out.shape[0] != N or out.shape[1] < M:
            raise ValueError(f"linear: EPI_BF16_T(P32) needs out bf16 [N, >= M], got {tuple(out.shape)}")
    elif out is None:
        out = torch.empty(M, N, device=x.device, dtype=torch.float32 if f32_out else torch.bfloat16)
    assert out.dtype == (torch.float32 if f32_out else torch.bfloat16) and out.stride(1) == 1
    if epilogue not in (EPI_BF16_T, EPI_BF16_TP32) and tuple(out.shape) != (M, N):
        raise ValueError(f"linear: out shape {tuple(out.shape)} != {(M, N)}")
    if bias is not None:
        _check(bias, torch.float32, "linear.bias")
    ldr = 0
    gstride = 0
    if epilogue == EPI_RES_F32:
        assert residual is not None and residual.dtype == torch.float32
        ldr = residual.stride(0)
        if gate is not None:
            assert gate.dtype == torch.float32 and gate.stride(-1) == 1
            gstride = gate.stride(0)
    call("sa_gemm_bf16_panels", x.data_ptr(), x.stride(0), 0, weight.data_ptr(), weight.stride(0), 0, _p(bias),
         out.data_ptr(), out.stride(0), 0, M, N, K, 1, epilogue, _p(residual), ldr, 0, _p(gate), gstride,
         rows_per_batch, kernel, group_m, pc, ps, _stream())
    return out


def bmm_nt(a, b, out, epilogue=EPI_F32, kernel=GEMM_AUTO):
    """out[z] = a[z] @ b[z]^T for 3-D bf16 a [Z, M, K], b [Z, N, K]."""
    Z, M, K = a.shape
    N = b.shape[1]
    call("sa_gemm_bf16_ex", a.data_ptr(), a.stride(1), a.stride(0), b.data_ptr(), b.stride(1), b.stride(0), 0,
         out.data_ptr(), out.stride(1), out.stride(0), M, N, K, Z, epilogue, 0, 0, 0, 0, 0, 0, kernel, 0, _stream())
    return out


ATTN_AUTO = 0
# kernel id of sa_attn_fwd_ex that reads V as V^T [H*128, Rv]: keys permuted per 32 in P's order (the QKV GEMM's
# EPI_BF16_TP32 output)
ATTN_VT_P32 = 3


def attn_tail_split(n_tiles_before, n_tiles, device):
    """How many of a launch's (segment, head, 256-query block) tiles to run as two key halves (sa_attn_fwd_split):
    the tiles past the last full round over the CUs when that round is at most half full, counting n_tiles_before
    tiles of launches running concurrently ahead of this one (the per-CFG-row streams of the sequence-parallel
    schedule); 0 = no split.  SA_ATTN_SPLIT=0 disables it."""
    if os.environ.get("SA_ATTN_SPLIT", "1") == "0":
        return 0
    ncu = _n_cu(device)
    total = n_tiles_before + n_tiles
    t = total % ncu
    return t if total > ncu and 0 < t <= ncu // 2 and t <= n_tiles else 0


def attention(q, k, v, out, segs, nseg, max_q_len, heads, head_dim=128, scale=None, accumulate=False,
              kernel=ATTN_AUTO, o_rows=None, split_tiles=0):
    """Flash attention over row-segment table `segs` (int32 [nseg,4] on device); kernel = per-call
    schedule selection (sa_attn_fwd_ex; 0 = auto); o_rows = int32 device map query row -> output row of
    `out` (sa_attn_fwd_map); split_tiles > 0: the last split_tiles tiles as two key halves + a merge
    (sa_attn_fwd_split, 8-wave kernel)."""
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (out, "out")):
        _check(t, torch.bfloat16, f"attention.{n}")
        assert t.stride(-1) == 1
    assert segs.dtype == torch.int32 and segs.is_cuda
    if o_rows is not None:
        assert o_rows.dtype == torch.int32 and o_rows.is_cuda and o_rows.is_contiguous()
    if scale is None:
        scale = head_dim ** -0.5
    if split_tiles:
        work = torch.empty(split_tiles * 2 * 256 * (head_dim + 2), device=q.device, dtype=torch.float32)
        call("sa_attn_fwd_split", q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), segs.data_ptr(), nseg,
             max_q_len, heads, head_dim, q.stride(0), k.stride(0), v.stride(0), out.stride(0), float(scale),
             int(accumulate), _p(o_rows), int(split_tiles), work.data_ptr(), work.numel() * 4, _stream())
        return out
    call("sa_attn_fwd_map", q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), segs.data_ptr(), nseg,
         max_q_len, heads, head_dim, q.stride(0), k.stride(0), v.stride(0), out.stride(0), float(scale),
         int(accumulate), kernel, _p(o_rows), _stream())
    return out


def attention_cross3(q, kt, vt, t_len, ki, vi, i_len, kv, vv, nper, tokens_per_frame, n_frames, out, batch, q_len,
                     heads, tok_offset=0, head_dim=128, scale=None):
    """Text + image + per-frame vocal cross-attention summed in bf16 (1B:556-603), one launch."""
    for t, n in ((q, "q"), (kt, "kt"), (vt, "vt"), (ki, "ki"), (vi, "vi"), (kv, "kv"), (vv, "vv"), (out, "out")):
        _check(t, torch.bfloat16, f"attention_cross3.{n}")
        assert t.stride(-1) == 1
    assert kt.stride(0) == vt.stride(0) and ki.stride(0) == vi.stride(0) and kv.stride(0) == vv.stride(0)
    if scale is None:
        scale = head_dim ** -0.5
    call("sa_attn_cross3", q.data_ptr(), q.stride(0), kt.data_ptr(), vt.data_ptr(), kt.stride(0), t_len,
         ki.data_ptr(), vi.data_ptr(), ki.stride(0), i_len, kv.data_ptr(), vv.data_ptr(), kv.stride(0), nper,
         tokens_per_frame, n_frames, tok_offset, out.data_ptr(), out.stride(0), batch, q_len, heads, float(scale),
         _stream())
    return out


def layernorm_mod(x, out, eps, weight=None, bias=None, shift=None, scale=None, gate=None, rows_per_batch=0):
    """Row LayerNorm (+affine) (+y*(1+scale[b])+shift[b]) (+x+y*gate[b]).  x/out 2-D f32|bf16."""
    M, C = x.shape
    mstride = 0
    if scale is not None:
        mstride = scale.stride(0)
        assert shift.stride(0) == mstride
    call("sa_layernorm_mod", x.data_ptr(), x.stride(0), _dt(x), out.data_ptr(), out.stride(0), _dt(out), _p(weight),
         _p(bias), _p(shift), _p(scale), mstride, _p(gate), rows_per_batch, M, C, float(eps), _stream())
    return out


def qk_rmsnorm_rope(x, q_col, k_col, wq, wk, C, eps, rope=None, rows_per_batch=0, tok_offset=0, grid=(1, 1, 1),
                    head_dim=128, n_frame_pairs=0, n_height_pairs=0, M=None):
    M = x.shape[0] if M is None else M
    F, H, W = grid
    call("sa_qk_rmsnorm_rope", x.data_ptr(), x.stride(0), q_col, k_col, wq.data_ptr(), _p(wk), M, C, head_dim,
         float(eps), _p(rope), rows_per_batch, tok_offset, F, H, W, n_frame_pairs, n_height_pairs, _stream())
    return x


def qkv_pack(x, wq, wk, C, eps, table, G, R, my_part, rope=None, rows_per_batch=0, tok_offset=0, grid=(1, 1, 1),
             head_dim=128, n_frame_pairs=0, n_height_pairs=0, b_offset=0):
    """RMSNorm + RoPE of the q / k columns of the [M, 3C] QKV rows x, written with v into the sequence-parallel
    send slabs / attention inputs that the int64 device `table` [G*R, 6] names (sa_qkv_pack)."""
    _check(x, torch.bfloat16, "qkv_pack.x")
    assert x.stride(1) == 1 and x.shape[1] >= 3 * C
    assert table.dtype == torch.int64 and table.is_cuda and tuple(table.shape) == (G * R, 6)
    F, H, W = grid
    call("sa_qkv_pack", x.data_ptr(), x.stride(0), wq.data_ptr(), wk.data_ptr(), x.shape[0], C, head_dim, float(eps),
         _p(rope), rows_per_batch, tok_offset, F, H, W, n_frame_pairs, n_height_pairs, table.data_ptr(), G, R, my_part,
         b_offset, _stream())


def patch_im2col(x, y, B, F, H, W, out, Kpad, Lpad, x_frame_offset=0, x_batch_broadcast=False):
    """x: [Bx, Cx, Tx, H, W] bf16 (frames x_frame_offset.. used), y: [B, Cy, >=F, H, W] bf16."""
    _check(x, torch.bfloat16, "patch_im2col.x")
    if y is not None:
        _check(y, torch.bfloat16, "patch_im2col.y")
    xc = x.stride(1)
    xb = 0 if x_batch_broadcast else x.stride(0)
    xf = x.stride(2)
    xptr = x.data_ptr() + x_frame_offset * xf * x.element_size()
    if y is not None:
        yb, yc, yf, ycn, yptr = y.stride(0), y.stride(1), y.stride(2), y.shape[1], y.data_ptr()
    else:
        yb = yc = yf = ycn = yptr = 0
    call("sa_patch_im2col", xptr, xb, xc, xf, x.shape[1], yptr, yb, yc, yf, ycn, B, F, H, W, out.data_ptr(), Kpad,
         Lpad, _stream())
    return out


def unpatchify(head_out, Lpad, B, C, F, H, W, out):
    call("sa_unpatchify", head_out.data_ptr(), head_out.stride(0), Lpad, B, C, F, H, W, out.data_ptr(), _dt(out),
         _stream())
    return out


def timestep_embed(t, dim, out):
    call("sa_timestep_embed", t.data_ptr(), t.shape[0], dim, out.data_ptr(), _stream())
    return out


def small_linear_f32(x, weight, bias, out, act_in=0, act_out=0):
    M, K = x.shape
    N = weight.shape[0]
    call("sa_small_linear_f32", x.data_ptr(), x.stride(0), M, weight.data_ptr(), weight.stride(0), _p(bias),
         out.data_ptr(), out.stride(0), N, K, act_in, act_out, _stream())
    return out


def mod_add(mod, e, out, e_jstride=None):
    """out[l,b,j,c] = mod[l,j,c] + e[b,j,c]  (e 2-D [B, C] with e_jstride=0 broadcasts over j)."""
    L, J, C = mod.shape
    B = e.shape[0]
    ej = e.stride(1) if e_jstride is None else e_jstride
    call("sa_mod_add", mod.data_ptr(), e.data_ptr(), e.stride(0), ej, out.data_ptr(), L, B, J, C, _stream())
    return out


def attention_small(q, k, v, out, segs, nseg, max_q_len, max_kv_len, heads, head_dim, scale=None, nsplit=None):
    """Attention for head dims sa_attn_fwd does not take.  nsplit = key splits per 32-query chunk (None: auto -- split
    when the launch has at most half as many workgroups as the device has CUs, so each CU takes one split)."""
    if scale is None:
        scale = head_dim ** -0.5
    wgs = nseg * heads * -(-max_q_len // 32)
    if nsplit is None:
        nsplit = 1
        if head_dim <= 256 and q.is_cuda and 2 * wgs <= _n_cu(q.device):
            nsplit = min(-(-max_kv_len // 64), _n_cu(q.device) // wgs)
    if nsplit > 1:
        work = torch.empty(wgs * nsplit * 32 * (head_dim + 2), device=q.device, dtype=torch.float32)
        call("sa_attn_small_split", q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), segs.data_ptr(), nseg,
             max_q_len, max_kv_len, heads, head_dim, q.stride(0), k.stride(0), v.stride(0), out.stride(0),
             float(scale), int(nsplit), work.data_ptr(), work.numel() * 4, _stream())
        return out
    call("sa_attn_small", q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), segs.data_ptr(), nseg, max_q_len,
         max_kv_len, heads, head_dim, q.stride(0), k.stride(0), v.stride(0), out.stride(0), float(scale), _stream())
    return out


def flow_step(latents_all, pred_all, noise, start, dsigma, audio_scale, text_scale, overlap, prev_end, weights,
              blend):
    C, T = latents_all.shape[1], latents_all.shape[2]
    R, Fw = noise.shape[0], noise.shape[2]
    HW = noise.shape[3] * noise.shape[4]
    call("sa_flow_step", latents_all.data_ptr(), pred_all.data_ptr(), noise.data_ptr(), R, C, T, Fw, HW, start,
         float(dsigma), float(audio_scale), float(text_scale), overlap, prev_end, _p(weights), int(blend), _stream())


def gather_rows(inp, idx, out):
    row_bytes = inp.shape[-1] * inp.element_size()
    call("sa_gather_rows", inp.data_ptr(), inp.stride(0) * inp.element_size(), idx.data_ptr(), idx.shape[0],
         out.data_ptr(), out.stride(0) * out.element_size(), row_bytes, _stream())
    return out


def fill_(t, value):
    assert t.dtype == torch.float32 and t.is_contiguous()
    call("sa_fill_f32", t.data_ptr(), t.numel(), float(value), _stream())
    return t


def cast_bf16(x, out):
    assert x.is_contiguous() and out.is_contiguous()
    call("sa_cast_f32_bf16", x.data_ptr(), out.data_ptr(), x.numel(), _stream())
    return out
