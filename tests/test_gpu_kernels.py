"""Per-kernel numerics of libstableavatar_hip.so against plain PyTorch fp32 references of the
same op (floating-point kernels: tolerances stated per test).  Runs on the MI355X only."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("M,N,K", [(300, 520, 192), (512, 256, 64), (64512 // 16, 1536, 1536)])
def test_gemm_epilogues(M, N, K):
    from stableavatar_amd import ops
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev)
    ref = x.float() @ w.float().t() + b
    y = ops.linear(x, w, b, ops.EPI_BF16)
    assert rel(y, ref) < 1e-2
    y = ops.linear(x, w, b, ops.EPI_F32)
    assert rel(y, ref) < 2e-3
    y = ops.linear(x, w, b, ops.EPI_GELU_TANH_BF16)
    assert rel(y, torch.nn.functional.gelu(ref, approximate="tanh")) < 1e-2
    y = ops.linear(x, w, b, ops.EPI_GELU_ERF_BF16)
    assert rel(y, torch.nn.functional.gelu(ref)) < 1e-2
    y = ops.linear(x, w, b, ops.EPI_SILU_F32)
    assert rel(y, torch.nn.functional.silu(ref)) < 2e-3
    # gated residual, 3 "batch rows" of the CFG batch
    B = 3
    rpb = (M + B - 1) // B
    res = torch.randn(M, N, device=dev)
    gate = torch.randn(B, N, device=dev)
    g_rows = gate[torch.arange(M, device=dev) // rpb]
    out = res.clone()
    ops.linear(x, w, b, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=rpb)
    # the residual consumes the bf16-rounded Linear output, as the reference under autocast (1B:677-678)
    assert rel(out, res + ref.bfloat16().float() * g_rows) < 2e-3


@pytest.mark.parametrize("kernel", [0, 2, 3], ids=["auto", "persistent", "persistent192"])
@pytest.mark.parametrize("M,N", [(1000, 1536), (777, 640), (513, 520), (64512 // 8, 1536)])
def test_gemm_bf16_epilogue_exact(kernel, M, N):
    """The bf16 row epilogue's element placement and bias, bit-exact: small-integer operands make every product and
    sum exact in fp32, so the only rounding is the final bf16 one (RNE on both sides).  N = 640 puts a 128-column
    partial tile in the last column (one wave on the accumulator path, the other on the LDS-strip path), N = 520 a
    ragged one; M leaves partial row tiles."""
    from stableavatar_amd import ops
    K = 256
    x = torch.randint(-3, 4, (M, K), device=dev).bfloat16()
    w = torch.randint(-3, 4, (N, K), device=dev).bfloat16()
    b = torch.randint(-50, 51, (N,), device=dev).float()
    ref = (x.float() @ w.float().t() + b).bfloat16()
    y = ops.linear(x, w, b, ops.EPI_BF16, kernel=kernel)
    assert torch.equal(y, ref)
    y = ops.linear(x, w, None, ops.EPI_BF16, kernel=kernel)
    assert torch.equal(y, (x.float() @ w.float().t()).bfloat16())


@pytest.mark.parametrize("kernel", [0, 1, 2, 3], ids=["auto", "pingpong", "persistent", "persistent192"])
@pytest.mark.parametrize("M,N,K", [(300, 520, 256), (257, 130, 128), (1000, 1536, 1536), (600, 300, 2304)])
def test_gemm_kernels(kernel, M, N, K):
    """Both shipped GEMM schedules (per-call selection, sa_gemm_bf16_ex) on ragged M/N tiles, every
    epilogue, vs torch fp32."""
    from stableavatar_amd import ops
    kw = dict(kernel=kernel)
    x = torch.randn(M, K + 64, device=dev).bfloat16()[:, 32:32 + K]  # strided rows
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev)
    ref = x.float() @ w.float().t() + b
    assert rel(ops.linear(x, w, b, ops.EPI_BF16, **kw), ref) < 1e-2
    assert rel(ops.linear(x, w, b, ops.EPI_F32, **kw), ref) < 2e-3
    assert rel(ops.linear(x, w, b, ops.EPI_GELU_TANH_BF16, **kw), torch.nn.functional.gelu(ref, approximate="tanh")) < 1e-2
    B = 3
    rpb = (M + B - 1) // B
    res = torch.randn(M, N, device=dev)
    gate = torch.randn(B, N, device=dev)
    out = res.clone()
    ops.linear(x, w, b, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=rpb, **kw)
    assert rel(out, res + ref.bfloat16().float() * gate[torch.arange(M, device=dev) // rpb]) < 2e-3
    a = torch.randn(2, 300, K, device=dev).bfloat16()
    bb = torch.randn(2, 200, K, device=dev).bfloat16()
    o = torch.empty(2, 300, 200, device=dev)
    ops.bmm_nt(a, bb, o)
    assert rel(o, a.float() @ bb.float().transpose(1, 2)) < 2e-3


@pytest.mark.parametrize("M,N,K", [(1000, 384, 1536), (64512 // 8, 1536, 1536), (300, 130, 256)])
def test_gemm_transposed_output(M, N, K):
    """EPI_BF16_T (the QKV GEMM's V^T output in natural key order): C^T[n, m] = bf16(x @ w^T + b)[m, n] vs the
    row-major epilogue, ragged M / N tiles; the pad columns past M are left untouched"""
    from stableavatar_amd import ops
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / math.sqrt(K)).bfloat16()
    b = torch.randn(N, device=dev)
    Rv = (M + 63) // 64 * 64
    out = torch.full((N, Rv), 7.0, device=dev, dtype=torch.bfloat16)
    ops.linear(x, w, b, ops.EPI_BF16_T, out=out)
    y = ops.linear(x, w, b, ops.EPI_BF16)
    print(f"EPI_BF16_T vs EPI_BF16 bit-identical: {torch.equal(out[:, :M].t(), y)}")
    assert rel(out[:, :M].t(), y) < 1e-3
    assert rel(out[:, :M].t(), x.float() @ w.float().t() + b) < 1e-2
    assert (out[:, M:] == 7.0).all()
    # P32: the rows of each 32-row chunk in the attention's P order = kbench.vt_layout(y, 3)
    from stableavatar_amd.kbench import vt_layout
    outp = torch.zeros(N, Rv + 64, device=dev, dtype=torch.bfloat16)  # vt_layout's width: ceil64(M) + 64
    ops.linear(x, w, b, ops.EPI_BF16_TP32, out=outp)
    assert torch.equal(outp, vt_layout(out[:, :M].t().contiguous(), 3))


def test_gemm_persistent_rejects_k192():
    """the persistent kernel needs K % 128 == 0: an explicit request is refused, auto falls back"""
    from stableavatar_amd import ops
    from stableavatar_amd._lib import KernelError
    x = torch.randn(64, 192, device=dev).bfloat16()
    w = torch.randn(64, 192, device=dev).bfloat16()
    with pytest.raises(KernelError):
        ops.linear(x, w, None, ops.EPI_F32, kernel=2)
    assert rel(ops.linear(x, w, None, ops.EPI_F32), x.float() @ w.float().t()) < 2e-3


def test_gemm_strided_input_and_batched():
    from stableavatar_amd import ops
    big = torch.randn(200, 320, device=dev).bfloat16()
    x = big[:, 64:256]  # row stride 320, K = 192
    w = torch.randn(130, 192, device=dev).bfloat16()
    y = ops.linear(x, w, None, ops.EPI_F32)
    assert rel(y, x.float() @ w.float().t()) < 2e-3
    a = torch.randn(3, 100, 128, device=dev).bfloat16()
    bb = torch.randn(3, 70, 128, device=dev).bfloat16()
    out = torch.empty(3, 100, 70, device=dev)
    ops.bmm_nt(a, bb, out)
    assert rel(out, a.float() @ bb.float().transpose(1, 2)) < 2e-3


def _ref_attn(q, k, v, scale):
    s = (q.float() @ k.float().t()) * scale
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("kernel", [1, 2], ids=["wg256", "wg128"])
@pytest.mark.parametrize("Lq,Lk", [(300, 300), (512, 257), (1024, 17), (64, 512), (256, 1000)])
def test_attention_segments(Lq, Lk, kernel):
    from stableavatar_amd import ops
    B, H, D = 2, 3, 128
    q = torch.randn(B * Lq, H * D + 64, device=dev).bfloat16()[:, :H * D]  # strided rows
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, B, Lq, H, kernel=kernel)
    for b in range(B):
        for h in range(H):
            ref = _ref_attn(q[b * Lq:(b + 1) * Lq, h * D:(h + 1) * D], k[b * Lk:(b + 1) * Lk, h * D:(h + 1) * D],
                            v[b * Lk:(b + 1) * Lk, h * D:(h + 1) * D], D ** -0.5)
            assert rel(o[b * Lq:(b + 1) * Lq, h * D:(h + 1) * D], ref) < 1e-2, (b, h)
    # accumulate mode adds onto the existing output
    o2 = o.clone()
    ops.attention(q, k, v, o2, segs, B, Lq, H, accumulate=True, kernel=kernel)
    assert rel(o2, 2 * o.float()) < 1e-2


@pytest.mark.parametrize("kernel", [3], ids=["v6t_vt_perm32"])
@pytest.mark.parametrize("B,Lq,Lk", [(2, 300, 320), (2, 512, 256), (1, 256, 1000), (3, 64, 64), (1, 256, 128)])
def test_attention_vt_kernels(kernel, B, Lq, Lk):
    """the self-attention form that reads V as V^T [H*128, Rv] (kernel 3: keys permuted per 32 as P) vs fp32 torch,
    incl. a ragged last key block and accumulate"""
    from stableavatar_amd import ops
    from stableavatar_amd.kbench import vt_layout
    H, D = 3, 128
    q = torch.randn(B * Lq, H * D + 64, device=dev).bfloat16()[:, :H * D]
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    vt = vt_layout(v, 3)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, vt, o, segs, B, Lq, H, kernel=kernel)
    for b in range(B):
        for h in range(H):
            sl = slice(h * D, (h + 1) * D)
            ref = _ref_attn(q[b * Lq:(b + 1) * Lq, sl], k[b * Lk:(b + 1) * Lk, sl], v[b * Lk:(b + 1) * Lk, sl], D ** -0.5)
            assert rel(o[b * Lq:(b + 1) * Lq, sl], ref) < 1e-2, (b, h)
    o2 = o.clone()
    ops.attention(q, k, vt, o2, segs, B, Lq, H, accumulate=True, kernel=kernel)
    assert rel(o2, 2 * o.float()) < 1e-2


@pytest.mark.parametrize("kernel", [3], ids=["v6t_vt_perm32"])
def test_attention_vt_spike_rescale(kernel):
    """the rescale branch of the V^T form"""
    from stableavatar_amd import ops
    from stableavatar_amd.kbench import vt_layout
    L, D = 512, 128
    q = torch.randn(L, D, device=dev).bfloat16()
    k = torch.randn(L, D, device=dev).bfloat16()
    k[400] = q[5] * 4
    k[440] = q[9] * 4
    k[33] = q[20] * 2
    ramp = torch.linspace(0.2, 3.0, L, device=dev)[:, None]
    k[:, :] = (k.float() + ramp * q[17].float()).bfloat16()
    v = torch.randn(L, D, device=dev).bfloat16()
    o = torch.empty_like(q)
    segs = torch.tensor([[0, L, 0, L]], dtype=torch.int32, device=dev)
    ops.attention(q, k, vt_layout(v, 3), o, segs, 1, L, 1, kernel=kernel)
    ref = _ref_attn(q, k, v, D ** -0.5)
    assert rel(o, ref) < 1e-2
    for r in (5, 9, 17, 20):
        assert rel(o[r], ref[r]) < 1e-2, r


def test_attention_vocal_grouping():
    """per-frame grouping of 1B:575-586: q rows of frame f attend to that frame's 17 keys"""
    from stableavatar_amd import ops
    B, F, G, Lv, H, D = 2, 3, 64, 17, 2, 128
    q = torch.randn(B * F * G, H * D, device=dev).bfloat16()
    k = torch.randn(B * F * Lv, H * D, device=dev).bfloat16()
    v = torch.randn(B * F * Lv, H * D, device=dev).bfloat16()
    o = torch.empty_like(q)
    segs = torch.tensor([[i * G, G, i * Lv, Lv] for i in range(B * F)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, B * F, G, H)
    for i in range(B * F):
        for h in range(H):
            sl = slice(h * D, (h + 1) * D)
            ref = _ref_attn(q[i * G:(i + 1) * G, sl], k[i * Lv:(i + 1) * Lv, sl], v[i * Lv:(i + 1) * Lv, sl], D ** -0.5)
            assert rel(o[i * G:(i + 1) * G, sl], ref) < 1e-2


@pytest.mark.parametrize("kernel", [1, 2], ids=["wg256", "wg128"])
def test_attention_spike_rescale(kernel):
    """force the online-softmax rescale branch: late keys with huge scores, in the first and the second
    32-key half of a block, and a ramp that rescales block after block"""
    from stableavatar_amd import ops
    L, D = 512, 128
    q = torch.randn(L, D, device=dev).bfloat16()
    k = torch.randn(L, D, device=dev).bfloat16()
    k[400] = q[5] * 4   # key 16 of block 6: first half
    k[440] = q[9] * 4   # key 56 of block 6: second half
    k[33] = q[9] * 2    # second half of the first block
    ramp = torch.linspace(0.2, 3.0, L, device=dev)[:, None]
    k[:, :] = (k.float() + ramp * q[17].float()).bfloat16()  # query 17's scores rise across the keys
    v = torch.randn(L, D, device=dev).bfloat16()
    o = torch.empty_like(q)
    segs = torch.tensor([[0, L, 0, L]], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, 1, L, 1, kernel=kernel)
    ref = _ref_attn(q, k, v, D ** -0.5)
    assert rel(o, ref) < 1e-2
    for r in (5, 9, 17):
        assert rel(o[r], ref[r]) < 1e-2, r


X3_KERNELS = pytest.mark.parametrize("x3k", ["1", "0"], ids=["w4", "w8"])  # SA_X3_W4


@X3_KERNELS
@pytest.mark.parametrize("tok_offset", [0, 256])
def test_attention_cross3(tok_offset, x3k, monkeypatch):
    """fused text + image + per-frame vocal cross-attention (1B:556-603) vs fp32 torch with the
    reference's bf16 sum (bf16(text) + bf16(img)) + bf16(vocal); every kernel (SA_X3_KERNEL)"""
    monkeypatch.setenv("SA_X3_W4", x3k)
    from stableavatar_amd import ops
    B, H, D, tpf, F, nper, tl, il = 2, 2, 128, 256, 3, 17, 512, 257
    Lq = F * tpf - tok_offset
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    kvt = torch.randn(B * tl, 2 * H * D, device=dev).bfloat16()
    kvi = torch.randn(B * il, 2 * H * D, device=dev).bfloat16()
    kvv = torch.randn(B * F * nper, 2 * H * D, device=dev).bfloat16()
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    HD = H * D
    ops.attention_cross3(q, kvt[:, :HD], kvt[:, HD:], tl, kvi[:, :HD], kvi[:, HD:], il, kvv[:, :HD], kvv[:, HD:],
                         nper, tpf, F, o, B, Lq, H, tok_offset=tok_offset)
    sc = D ** -0.5
    for b in range(B):
        for h in range(H):
            sl, sv = slice(h * D, (h + 1) * D), slice(HD + h * D, HD + (h + 1) * D)
            qq = q[b * Lq:(b + 1) * Lq, sl]
            t = _ref_attn(qq, kvt[b * tl:(b + 1) * tl, sl], kvt[b * tl:(b + 1) * tl, sv], sc).bfloat16()
            i = _ref_attn(qq, kvi[b * il:(b + 1) * il, sl], kvi[b * il:(b + 1) * il, sv], sc).bfloat16()
            vo = torch.empty(Lq, D, device=dev)
            for r0 in range(0, Lq, 64):
                f = (tok_offset + r0) // tpf
                kr = slice((b * F + f) * nper, (b * F + f + 1) * nper)
                vo[r0:r0 + 64] = _ref_attn(qq[r0:r0 + 64], kvv[kr, sl], kvv[kr, sv], sc)
            ref = (t + i) + vo.bfloat16()
            assert rel(o[b * Lq:(b + 1) * Lq, sl], ref) < 1e-2, (b, h)


def _nan_tail(rows, cols, pad=96):
    """[rows, cols] bf16 random rows followed by `pad` rows of NaN in the same allocation"""
    big = torch.full((rows + pad, cols), float("nan"), device=dev, dtype=torch.bfloat16)
    big[:rows] = torch.randn(rows, cols, device=dev).bfloat16()
    return big, big[:rows]


@pytest.mark.parametrize("kernel", [1, 2], ids=["wg256", "wg128"])
def test_attention_tail_block_stays_inside_segment(kernel):
    """a partial last key block must not read the rows past its segment (the block offset in
    soffset is outside the buffer range check): K/V rows past the last segment are NaN, the output must
    match fp32 torch over the segment's keys only"""
    from stableavatar_amd import ops
    B, H, D, Lq, Lk = 2, 2, 128, 200, 257
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    _, k = _nan_tail(B * Lk, H * D)
    _, v = _nan_tail(B * Lk, H * D)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, o, segs, B, Lq, H, kernel=kernel)
    assert torch.isfinite(o.float()).all()
    b = B - 1
    for h in range(H):
        sl = slice(h * D, (h + 1) * D)
        ref = _ref_attn(q[b * Lq:(b + 1) * Lq, sl], k[b * Lk:(b + 1) * Lk, sl], v[b * Lk:(b + 1) * Lk, sl], D ** -0.5)
        assert rel(o[b * Lq:(b + 1) * Lq, sl], ref) < 1e-2, h


def test_attention_vt_ragged_batch_stays_inside_allocation():
    """V^T kernel (3) with B = 2 segments of Lk = 96 keys (Lk = 32 mod 64, so the second segment's last 64-key block
    ends at column 96 + 128 = 224, past ceil64(B * Lk) = 192): V^T sized as the DiT allocates it (ceil64(M) + 64
    columns, kbench.vt_layout), zero pad, NaN right after the allocation -- the output must be finite and match fp32
    torch (a ceil64(M)-wide V^T let the last d-row of the last head read 64 bytes past the buffer)"""
    from stableavatar_amd import ops
    from stableavatar_amd.kbench import vt_layout
    B, H, D, Lq, Lk = 2, 2, 128, 100, 96
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    vt0 = vt_layout(v, 3)
    assert vt0.shape[1] == (B * Lk + 63) // 64 * 64 + 64
    big = torch.full((vt0.numel() + 4096,), float("nan"), device=dev, dtype=torch.bfloat16)
    big[:vt0.numel()] = vt0.flatten()
    vt = big[:vt0.numel()].view(vt0.shape)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    ops.attention(q, k, vt, o, segs, B, Lq, H, kernel=ops.ATTN_VT_P32)
    assert torch.isfinite(o.float()).all()
    for b in range(B):
        for h in range(H):
            sl = slice(h * D, (h + 1) * D)
            ref = _ref_attn(q[b * Lq:(b + 1) * Lq, sl], k[b * Lk:(b + 1) * Lk, sl], v[b * Lk:(b + 1) * Lk, sl],
                            D ** -0.5)
            assert rel(o[b * Lq:(b + 1) * Lq, sl], ref) < 1e-2, (b, h)
    # the default V^T output of ops.linear(EPI_BF16_TP32) has the same width and a zeroed pad
    x = torch.randn(B * Lk, 256, device=dev).bfloat16()
    w = torch.randn(H * D, 256, device=dev).bfloat16()
    vt2 = ops.linear(x, w, torch.zeros(H * D, device=dev), ops.EPI_BF16_TP32)
    torch.cuda.synchronize()
    assert vt2.shape == vt0.shape and torch.count_nonzero(vt2[:, B * Lk:]).item() == 0


@X3_KERNELS
def test_attention_cross3_tail_blocks_stay_inside_sources(x3k, monkeypatch):
    """fused cross-attention with every source's K/V followed by NaN rows: the image stream's last block (257 =
    4 x 64 + 1 keys) and the vocal half block (17 of 32 keys) of the last batch row / last frame must read
    zeros past their source, not the NaN that follows"""
    monkeypatch.setenv("SA_X3_W4", x3k)
    from stableavatar_amd import ops
    B, H, D, tpf, F, nper, tl, il = 2, 2, 128, 256, 2, 17, 512, 257
    HD = H * D
    Lq = F * tpf
    q = torch.randn(B * Lq, HD, device=dev).bfloat16()
    _, kvt = _nan_tail(B * tl, 2 * HD)
    _, kvi = _nan_tail(B * il, 2 * HD)
    _, kvv = _nan_tail(B * F * nper, 2 * HD)
    o = torch.empty(B * Lq, HD, device=dev, dtype=torch.bfloat16)
    ops.attention_cross3(q, kvt[:, :HD], kvt[:, HD:], tl, kvi[:, :HD], kvi[:, HD:], il, kvv[:, :HD], kvv[:, HD:],
                         nper, tpf, F, o, B, Lq, H)
    assert torch.isfinite(o.float()).all()
    sc = D ** -0.5
    b = B - 1
    for h in range(H):
        sl, sv = slice(h * D, (h + 1) * D), slice(HD + h * D, HD + (h + 1) * D)
        qq = q[b * Lq:(b + 1) * Lq, sl]
        t = _ref_attn(qq, kvt[b * tl:(b + 1) * tl, sl], kvt[b * tl:(b + 1) * tl, sv], sc).bfloat16()
        i = _ref_attn(qq, kvi[b * il:(b + 1) * il, sl], kvi[b * il:(b + 1) * il, sv], sc).bfloat16()
        vo = torch.empty(Lq, D, device=dev)
        for f in range(F):
            kr = slice((b * F + f) * nper, (b * F + f + 1) * nper)
            vo[f * tpf:(f + 1) * tpf] = _ref_attn(qq[f * tpf:(f + 1) * tpf], kvv[kr, sl], kvv[kr, sv], sc)
        assert rel(o[b * Lq:(b + 1) * Lq, sl], (t + i) + vo.bfloat16()) < 1e-2, h


@pytest.mark.parametrize("D,H,segs", [
    (192, 8, [(0, 32, 0, 1024), (32, 32, 1024, 1024), (64, 17, 2048, 1000)]),  # vocal projector (1B)
    (64, 12, [(0, 299, 0, 299)]),                                              # wav2vec2 self-attention
    (80, 16, [(0, 257, 0, 257)]),                                              # CLIP ViT-H/14
    (256, 2, [(0, 40, 0, 130), (40, 1, 130, 3)]),
    (64, 2, [(0, 70, 0, 5000)]),                                               # > 4096 keys (tiled kernel)
    (640, 8, [(0, 17, 0, 300)]),                                               # vocal projector (14B)
])
@pytest.mark.parametrize("nsplit", [1, None, 3, 16], ids=["unsplit", "auto", "split3", "split16"])
def test_attention_small(D, H, segs, nsplit):
    """sa_attn_small (the head dims sa_attn_fwd does not take) vs torch fp32 per segment and head,
    ragged query / key counts (tiled kernel for D <= 256, one wave per query above); split: sa_attn_small_split
    (keys of each query chunk over several workgroups + merge; splits past a short segment's keys are empty)."""
    from stableavatar_amd import ops
    if D > 256 and nsplit not in (1, None):
        pytest.skip("key split: tiled kernel (D <= 256) only")
    nq = max(a + b for a, b, _, _ in segs)
    nk = max(c + d for _, _, c, d in segs)
    q = torch.randn(nq, H * D, device=dev).bfloat16()
    kv = torch.randn(nk, 2 * H * D, device=dev).bfloat16()
    k, v = kv[:, :H * D], kv[:, H * D:]
    o = torch.full((nq, H * D), float("nan"), device=dev, dtype=torch.bfloat16)
    st = torch.tensor(segs, dtype=torch.int32, device=dev)
    ops.attention_small(q, k, v, o, st, len(segs), max(b for _, b, _, _ in segs), max(d for *_, d in segs), H, D,
                        nsplit=nsplit)
    for q0, ql, k0, kl in segs:
        for h in range(H):
            sl = slice(h * D, (h + 1) * D)
            ref = _ref_attn(q[q0:q0 + ql, sl], k[k0:k0 + kl, sl], v[k0:k0 + kl, sl], D ** -0.5)
            assert rel(o[q0:q0 + ql, sl], ref) < 1e-2, (q0, h)


def test_layernorm_modulate():
    from stableavatar_amd import ops
    M, C, B = 1000, 1536, 2
    rpb = 500
    x = torch.randn(M, C, device=dev) * 3 + 1
    shift = torch.randn(B, C, device=dev)
    scale = torch.randn(B, C, device=dev)
    out = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    ops.layernorm_mod(x, out, 1e-6, shift=shift, scale=scale, rows_per_batch=rpb)
    ln = torch.nn.functional.layer_norm(x, (C,), eps=1e-6)
    bi = torch.arange(M, device=dev) // rpb
    ref = ln * (1 + scale[bi]) + shift[bi]
    assert rel(out, ref) < 5e-3
    w = torch.randn(C, device=dev)
    bb = torch.randn(C, device=dev)
    out32 = torch.empty(M, C, device=dev)
    ops.layernorm_mod(x, out32, 1e-5, weight=w, bias=bb)
    assert rel(out32, torch.nn.functional.layer_norm(x, (C,), w, bb, 1e-5)) < 1e-5
    gate = torch.randn(B, C, device=dev)
    ops.layernorm_mod(x, out32, 1e-6, shift=shift, scale=scale, gate=gate, rows_per_batch=rpb)
    assert rel(out32, x + ref * gate[bi]) < 1e-5
    # width 1280 (CLIP MLPProj) exercises the partial-chunk path
    x2 = torch.randn(100, 1280, device=dev)
    o2 = torch.empty(100, 1280, device=dev)
    ops.layernorm_mod(x2, o2, 1e-5, weight=w[:1280], bias=bb[:1280])
    assert rel(o2, torch.nn.functional.layer_norm(x2, (1280,), w[:1280], bb[:1280], 1e-5)) < 1e-5


def _rope_ref(x, F, H, W, L, d=128):
    """restatement of 1B:223-231 + 295-323 on one batch row x [L, n, d] (fp64 freqs)"""
    def params(dim):
        f = torch.outer(torch.arange(1024, dtype=torch.float64),
                        1.0 / torch.pow(10000, torch.arange(0, dim, 2, dtype=torch.float64) / dim))
        return torch.polar(torch.ones_like(f), f)
    freqs = torch.cat([params(d - 4 * (d // 6)), params(2 * (d // 6)), params(2 * (d // 6))], 1)
    c = d // 2
    fr = freqs.split([c - 2 * (c // 3), c // 3, c // 3], 1)
    n = x.shape[1]
    S = F * H * W
    xi = torch.view_as_complex(x[:S].double().reshape(S, n, -1, 2))
    fi = torch.cat([fr[0][:F].view(F, 1, 1, -1).expand(F, H, W, -1), fr[1][:H].view(1, H, 1, -1).expand(F, H, W, -1),
                    fr[2][:W].view(1, 1, W, -1).expand(F, H, W, -1)], -1).reshape(S, 1, -1)
    out = torch.view_as_real(xi * fi.to(xi.device)).flatten(2)
    return torch.cat([out, x[S:].double()]).float(), freqs


def test_qk_rmsnorm_rope():
    from stableavatar_amd import ops
    from stableavatar_amd.transformer import rope_table
    F, H, W, B, C = 3, 4, 6, 2, 1536
    L = F * H * W + 8  # padded tokens are normalised but not rotated
    qkv = torch.randn(B * L, 3 * C, device=dev).bfloat16()
    wq = torch.randn(C, device=dev)
    wk = torch.randn(C, device=dev)
    x = qkv.clone()
    rope = rope_table(128).to(dev)
    ops.qk_rmsnorm_rope(x, 0, C, wq, wk, C, 1e-6, rope=rope, rows_per_batch=L, grid=(F, H, W), n_frame_pairs=22,
                        n_height_pairs=21)
    for part, w in ((0, wq), (1, wk)):
        src = qkv[:, part * C:(part + 1) * C].float()
        nrm = src * torch.rsqrt(src.pow(2).mean(-1, keepdim=True) + 1e-6) * w
        for b in range(B):
            ref, _ = _rope_ref(nrm[b * L:(b + 1) * L].view(L, 12, 128).cpu(), F, H, W, L)
            got = x[b * L:(b + 1) * L, part * C:(part + 1) * C].float().cpu()
            assert rel(got, ref.reshape(L, C)) < 5e-3
    assert torch.equal(x[:, 2 * C:], qkv[:, 2 * C:])


@pytest.mark.parametrize("tok_offset", [0, 37])
def test_qk_rmsnorm_rope_pair_matches_generic(tok_offset, monkeypatch):
    """The fused q+k kernel (C=1536, D=128) agrees with the generic per-tensor kernel to one bf16 ulp,
    incl. an SP token offset and padded (unrotated) rows."""
    from stableavatar_amd import ops
    from stableavatar_amd.transformer import rope_table
    F, H, W, C = 3, 4, 6, 1536
    L = F * H * W + 8
    qkv = torch.randn(2 * L, 3 * C, device=dev).bfloat16()
    wq, wk = torch.randn(C, device=dev), torch.randn(C, device=dev)
    rope = rope_table(128).to(dev)
    outs = []
    for generic in (False, True):
        if generic:
            monkeypatch.setenv("SA_QK_GENERIC", "1")
        x = qkv.clone()
        ops.qk_rmsnorm_rope(x, 0, C, wq, wk, C, 1e-6, rope=rope, rows_per_batch=L, tok_offset=tok_offset,
                            grid=(F, H, W), n_frame_pairs=22, n_height_pairs=21)
        torch.cuda.synchronize()
        outs.append(x)
    # same math; FMA contraction may differ, so an element may round to the neighbouring bf16 value
    diff = (outs[0].float() - outs[1].float()).abs()
    assert rel(outs[0].float(), outs[1].float()) < 1e-3
    assert (diff > 0).float().mean().item() < 0.05
    assert (diff <= outs[1].float().abs() * 2 ** -7 + 1e-6).all()


def test_patchify_roundtrip():
    from stableavatar_amd import ops
    B, F, H, W = 3, 2, 8, 12
    lat = torch.randn(1, 16, 5, H, W, device=dev).bfloat16()
    y = torch.randn(B, 20, F, H, W, device=dev).bfloat16()
    L = F * (H // 2) * (W // 2) + 5
    Kp = 192
    cols = torch.empty(B, L, Kp, device=dev, dtype=torch.bfloat16)
    ops.patch_im2col(lat, y, B, F, H, W, cols, Kp, L, x_frame_offset=2, x_batch_broadcast=True)
    xin = torch.cat([lat[:, :, 2:2 + F].expand(B, -1, -1, -1, -1), y], 1).float()  # [B,36,F,H,W]
    wconv = torch.randn(7, 36, 1, 2, 2, device=dev)
    ref = torch.nn.functional.conv3d(xin, wconv, stride=(1, 2, 2)).flatten(2).transpose(1, 2)
    got = cols[:, :F * (H // 2) * (W // 2), :144].float() @ wconv.flatten(1).t()
    assert rel(got, ref) < 1e-5
    assert cols[:, F * (H // 2) * (W // 2):].abs().sum() == 0
    # unpatchify of a [B, L, 64] head output
    ho = torch.randn(B, L, 64, device=dev).bfloat16()
    out = torch.empty(B, 16, F, H, W, device=dev)
    ops.unpatchify(ho.view(B * L, 64), L, B, 16, F, H, W, out)
    for b in range(B):
        u = ho[b, :F * (H // 2) * (W // 2)].float().view(F, H // 2, W // 2, 1, 2, 2, 16)
        u = torch.einsum("fhwpqrc->cfphqwr", u).reshape(16, F, H, W)
        assert torch.equal(out[b], u)


def test_small_kernels():
    from stableavatar_amd import ops
    t = torch.tensor([1000.0, 995.87, 24.41], device=dev)
    e = torch.empty(3, 256, device=dev)
    ops.timestep_embed(t, 256, e)
    pos = t.double().cpu()
    sinus = torch.outer(pos, torch.pow(10000, -torch.arange(128).double().div(128)))
    ref = torch.cat([torch.cos(sinus), torch.sin(sinus)], 1).float()
    assert (e.cpu() - ref).abs().max() < 1e-5
    W = torch.randn(9216, 1536, device=dev).bfloat16()
    b = torch.randn(9216, device=dev)
    x = torch.randn(3, 1536, device=dev)
    out = torch.empty(3, 9216, device=dev)
    ops.small_linear_f32(x, W, b, out, act_in=1)
    assert rel(out, torch.nn.functional.silu(x) @ W.float().t() + b) < 1e-5
    mod = torch.randn(4, 6, 1536, device=dev)
    e0 = torch.randn(3, 6, 1536, device=dev)
    o = torch.empty(4, 3, 6, 1536, device=dev)
    ops.mod_add(mod, e0, o)
    assert torch.equal(o, mod[:, None] + e0[None])
    src = torch.randn(10, 1536, device=dev)
    idx = torch.tensor([3, -1, 0, 9], dtype=torch.int32, device=dev)
    g = torch.empty(4, 1536, device=dev)
    ops.gather_rows(src, idx, g)
    assert torch.equal(g[0], src[3]) and g[1].abs().sum() == 0 and torch.equal(g[3], src[9])


def test_flow_step_blend():
    from stableavatar_amd import ops
    C, T, Fw, H, W = 16, 30, 21, 8, 8
    lat = torch.randn(1, C, T, H, W, device=dev).bfloat16()
    pred = torch.randn(1, C, T, H, W, device=dev).bfloat16()
    noise = torch.randn(3, C, Fw, H, W, device=dev).bfloat16()
    start, ov = 6, 15
    wts = torch.arange(ov, device=dev, dtype=torch.float32) / (ov - 1)
    pred0 = pred.clone()
    ops.flow_step(lat, pred, noise, start, -0.0042, 5.0, 3.0, ov, start + ov, wts, True)
    u, d, c = noise.chunk(3)
    v = u + 5.0 * (d - u) + 3.0 * (c - d)
    x = lat[:, :, start:start + Fw].float() + (-0.0042) * v.float()
    wb = wts.bfloat16().view(1, 1, ov, 1, 1).float()
    x[:, :, :ov] = x[:, :, :ov] * wb + pred0[:, :, start:start + ov].float() * (1 - wb)
    assert rel(pred[:, :, start:start + Fw], x) < 1e-2
    assert torch.equal(pred[:, :, :start], pred0[:, :, :start])


@pytest.mark.parametrize("B,Lq,Lk,N,D", [(2, 300, 300, 3, 128), (1, 1024, 257, 12, 128), (3, 40, 17, 8, 192),
                                         (2, 64, 100, 4, 64)])
def test_attention_op_seam_drop_in(B, Lq, Lk, N, D):
    """stableavatar_amd.attention.attention == the reference's SDPA branch (1B:158-207): q/k/v
    [B, L, N, D] bf16, scale 1/sqrt(D) whatever softmax_scale says, q_lens/k_lens only warn."""
    import warnings
    from stableavatar_amd.attention import attention
    q = torch.randn(B, Lq, N, D, device=dev).bfloat16()
    k = torch.randn(B, Lk, N, D, device=dev).bfloat16()
    v = torch.randn(B, Lk, N, D, device=dev).bfloat16()
    ref = torch.nn.functional.scaled_dot_product_attention(q.float().transpose(1, 2), k.float().transpose(1, 2),
                                                           v.float().transpose(1, 2)).transpose(1, 2)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        out = attention(q, k, v, q_lens=torch.full((B,), Lq), k_lens=None, softmax_scale=0.5)
    assert any("Padding mask" in str(x.message) for x in w)
    assert out.shape == (B, Lq, N, D) and out.dtype == torch.bfloat16
    assert rel(out, ref) < 1e-2
    with pytest.raises(NotImplementedError):
        attention(q, k, v, causal=True)


@pytest.mark.parametrize("in_bf16", [False, True])
def test_layernorm_shared_modulation_bit_identical(in_bf16):
    """layernorm_mod_shared_kernel (8 / 16 rows per workgroup sharing the modulation vectors through LDS) vs the
    one-row-per-wave kernel: bit-identical in every mode the DiT uses (AdaLN modulate, affine, gated residual)"""
    import os
    from stableavatar_amd import ops
    M, C, B, rpb = 1040, 1536, 2, 528  # 1040 = 65 x 16; rows_per_batch % 16 == 0
    x = torch.randn(M, C, device=dev) * 3 + 1
    if in_bf16:
        x = x.bfloat16()
    shift, scale, gate = (torch.randn(B, C, device=dev) for _ in range(3))
    w, bb = torch.randn(C, device=dev), torch.randn(C, device=dev)
    modes = [dict(shift=shift, scale=scale, rows_per_batch=rpb, dt=torch.bfloat16),
             dict(weight=w, bias=bb, dt=torch.bfloat16), dict(weight=w, bias=bb, dt=torch.float32)]
    if not in_bf16:
        modes.append(dict(shift=shift, scale=scale, gate=gate, rows_per_batch=rpb, dt=torch.float32))
    for mode in modes:
        kw = dict(mode)
        dt = kw.pop("dt")
        outs = []
        for nw in ("0", "8", "16"):
            o = torch.empty(M, C, device=dev, dtype=dt)
            os.environ["SA_LN_SHARED"] = nw
            try:
                ops.layernorm_mod(x, o, 1e-6, **kw)
            finally:
                os.environ.pop("SA_LN_SHARED", None)
            torch.cuda.synchronize()
            outs.append(o)
        assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]), sorted(kw)


@pytest.mark.parametrize("q_len,tok_offset", [(21504, 0), (21504 - 300, 256)], ids=["config2", "ragged"])
def test_attention_cross3_kernels_bit_identical_fullsize(q_len, tok_offset, monkeypatch):
    """the 4-wave and 8-wave cross-attention kernels give the same output bytes at the config-2 shape (3 CFG rows x
    12 heads x 84 query tiles) and with a ragged last tile, whose rows past q_len stay untouched"""
    from stableavatar_amd import ops
    B, H, D, nper, nfr, tl, il = 3, 12, 128, 32, 21, 512, 257
    tpf = 21504 // nfr
    HD = H * D
    torch.manual_seed(3)
    q = torch.randn(B * q_len, HD, device=dev).bfloat16()
    kvt = torch.randn(B * tl, 2 * HD, device=dev).bfloat16()
    kvi = torch.randn(B * il, 2 * HD, device=dev).bfloat16()
    kvv = torch.randn(B * nfr * nper, 2 * HD, device=dev).bfloat16()
    outs = {}
    for k in ("1", "0"):
        monkeypatch.setenv("SA_X3_W4", k)
        o = torch.full((B * q_len + 64, HD), 7.0, device=dev, dtype=torch.bfloat16)
        ops.attention_cross3(q, kvt[:, :HD], kvt[:, HD:], tl, kvi[:, :HD], kvi[:, HD:], il, kvv[:, :HD], kvv[:, HD:],
                             nper, tpf, nfr, o[:B * q_len], B, q_len, H, tok_offset=tok_offset)
        torch.cuda.synchronize()
        assert (o[B * q_len:] == 7.0).all(), k
        outs[k] = o[:B * q_len]
    assert torch.isfinite(outs["1"].float()).all()
    assert torch.equal(outs["0"], outs["1"])
    # one row per (batch row, head) against fp32 torch
    sc = D ** -0.5
    for b in range(B):
        r = b * q_len + (q_len - 1 if b == B - 1 else 1234)
        f = (tok_offset + r - b * q_len) // tpf
        for h in (0, H - 1):
            sl, sv = slice(h * D, (h + 1) * D), slice(HD + h * D, HD + (h + 1) * D)
            qq = q[r:r + 1, sl]
            t = _ref_attn(qq, kvt[b * tl:(b + 1) * tl, sl], kvt[b * tl:(b + 1) * tl, sv], sc).bfloat16()
            i = _ref_attn(qq, kvi[b * il:(b + 1) * il, sl], kvi[b * il:(b + 1) * il, sv], sc).bfloat16()
            kr = slice((b * nfr + f) * nper, (b * nfr + f + 1) * nper)
            vo = _ref_attn(qq, kvv[kr, sl], kvv[kr, sv], sc).bfloat16()
            assert rel(outs["1"][r:r + 1, sl], (t + i) + vo) < 1e-2, (b, h)
