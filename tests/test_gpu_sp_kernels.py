"""The three kernels that carry the sequence-parallel exchange with no copy pass (stableavatar_amd/sp.py,
SURVEY.md §8 row a18; the seam is usp_attn_forward, wan/dist/wan_xfuser.py:72-115):

* sa_qkv_pack -- the Q/K/V RMSNorm + RoPE writing per-destination slabs -- against the in-place
  sa_qk_rmsnorm_rope followed by a torch scatter: bit-identical (same arithmetic, different stores);
* sa_attn_fwd_map -- the attention storing by output row map -- against the plain attention scattered by
  torch: bit-identical;
* sa_gemm_bf16_panels -- the O-projection reading column panels -- against the same GEMM on the
  contiguous matrix: bit-identical (same K order).
Runs on the MI355X only."""
import pytest
import torch

from stableavatar_amd import ops, sp

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("C,H,world,rank", [(1536, 12, 1, 0), (1536, 12, 2, 1), (1536, 12, 8, 5), (5120, 40, 8, 3),
                                            (1536, 12, 3, 2)])
def test_qkv_pack_matches_inplace_norm_and_scatter(C, H, world, rank):
    from stableavatar_amd.transformer import rope_table
    B, D = 3, 128
    F, Hh, W = 3, 4, 5                       # 60 tokens; the SP pad rows past them are normalised, not rotated
    Lc = sp.padded_len(F * Hh * W, world) // world
    plan = sp.make_plan(world, rank, H)
    ex = sp.UlyssesExchange(plan, B, Lc, D, dev)
    qkv = torch.randn(B * Lc, 3 * C, device=dev).bfloat16()
    wq, wk = torch.randn(C, device=dev), torch.randn(C, device=dev)
    rope = rope_table(D).to(dev)
    rope_kw = dict(rope=rope, rows_per_batch=Lc, tok_offset=rank * Lc, grid=(F, Hh, W), head_dim=D,
                   n_frame_pairs=D // 2 - 2 * (D // 6), n_height_pairs=D // 6)
    ref = qkv.clone()
    ops.qk_rmsnorm_rope(ref, 0, C, wq, wk, C, 1e-6, **rope_kw)
    hgd = C // plan.G
    outs = []
    for per_row in (False, True):
        for t in [ex.q, ex.kv] + list(ex.sq.values()) + list(ex.skv.values()):
            t.fill_(float("nan"))
        if per_row:
            for b in range(B):
                ops.qkv_pack(qkv[b * Lc:(b + 1) * Lc], wq, wk, C, 1e-6, ex.table, plan.G, plan.R, plan.part,
                             b_offset=b, **rope_kw)
        else:
            ops.qkv_pack(qkv, wq, wk, C, 1e-6, ex.table, plan.G, plan.R, plan.part, **rope_kw)
        torch.cuda.synchronize()
        r3 = ref.view(B, Lc, 3, plan.G, hgd)
        for d, (qd, kd) in ex.slabs.items():
            g = d % plan.G
            if qd is not None:
                assert torch.equal(qd, r3[:, :, 0, g]), d
            assert torch.equal(kd[..., :hgd], r3[:, :, 1, g]) and torch.equal(kd[..., hgd:], r3[:, :, 2, g]), d
        outs.append([t.clone() for t in (ex.q, ex.kv)])
    # rows of the attention inputs the pack does not own stay untouched (NaN), the own chunk is filled
    qv = outs[0][0].view(B, plan.G, Lc, hgd)
    assert not qv[:, plan.group].isnan().any()
    if plan.G > 1:
        assert qv[:, (plan.group + 1) % plan.G].isnan().all()


@pytest.mark.parametrize("kernel", [1, 2], ids=["wg256", "wg128"])
def test_attention_output_row_map(kernel):
    B, Lq, Lk, H, D = 2, 300, 257, 3, 128
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    o = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    ops.attention(q, k, v, o, segs, B, Lq, H, kernel=kernel)
    rows = torch.randperm(3 * B * Lq, device=dev)[:B * Lq].to(torch.int32)
    big = torch.full((3 * B * Lq, H * D), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.attention(q, k, v, big, segs, B, Lq, H, kernel=kernel, o_rows=rows)
    torch.cuda.synchronize()
    assert torch.equal(big[rows.long()], o)
    untouched = torch.ones(3 * B * Lq, dtype=torch.bool, device=dev)
    untouched[rows.long()] = False
    assert big[untouched].isnan().all()
    # a segment with no keys writes its zeros through the map as well
    segs0 = torch.tensor([[0, Lq, 0, 0]], dtype=torch.int32, device=dev)
    ops.attention(q, k, v, big, segs0, 1, Lq, H, kernel=kernel, o_rows=rows)
    assert (big[rows[:Lq].long()] == 0).all()


@pytest.mark.parametrize("M,N,pc,G,rows_per_batch", [(1000, 1536, 384, 4, 334), (771, 1536, 768, 2, 257),
                                                      (512, 5120, 640, 8, 256), (300, 1536, 1536, 1, 100)])
def test_gemm_column_panels(M, N, pc, G, rows_per_batch):
    """the O-projection over the exchange's panel buffer equals the GEMM over the contiguous rows, bit for bit,
    also for a slice of rows (the per-CFG-row O-projection of the pipelined schedule)"""
    K = pc * G
    a = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=dev)
    gate = torch.randn(-(-M // rows_per_batch), N, device=dev)
    Mp = M + 37                                # panels further apart than their rows
    pan = torch.full((G * Mp, pc), float("nan"), device=dev, dtype=torch.bfloat16)
    pan.view(G, Mp, pc)[:, :M] = a.view(M, G, pc).transpose(0, 1)
    res = torch.randn(M, N, device=dev)
    ref = res.clone()
    ops.linear(a, w, bias, ops.EPI_RES_F32, out=ref, residual=ref, gate=gate, rows_per_batch=rows_per_batch)
    out = res.clone()
    ops.linear(pan[:M], w, bias, ops.EPI_RES_F32, out=out, residual=out, gate=gate, rows_per_batch=rows_per_batch,
               a_panels=(pc, Mp * pc))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    r0, r1 = rows_per_batch, 2 * rows_per_batch
    out2 = res.clone()
    ref2 = res.clone()
    ops.linear(a[r0:r1], w, bias, ops.EPI_RES_F32, out=ref2[r0:r1], residual=ref2[r0:r1], gate=gate[1:2],
               rows_per_batch=rows_per_batch)
    ops.linear(pan[r0:r1], w, bias, ops.EPI_RES_F32, out=out2[r0:r1], residual=out2[r0:r1], gate=gate[1:2],
               rows_per_batch=rows_per_batch, a_panels=(pc, Mp * pc))
    torch.cuda.synchronize()
    assert torch.equal(out2, ref2)
    if G > 1:
        with pytest.raises(ValueError):  # panels running past the buffer
            ops.linear(pan[:M], w, bias, ops.EPI_RES_F32, out=out, residual=out,
                       a_panels=(pc, 2 * Mp * pc))
