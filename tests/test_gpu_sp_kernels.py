"""The three kernels that carry the sequence-parallel exchange with no copy pass (stableavatar_amd/sp.py,
SURVEY.md §8 row a18; the seam is usp_attn_forward, wan/dist/wan_xfuser.py:72-115):

* sa_qkv_pack -- the Q/K/V RMSNorm + RoPE writing per-destination slabs -- against the in-place
  sa_qk_rmsnorm_rope followed by a torch scatter: bit-identical (same arithmetic, different stores);
* sa_attn_fwd_map -- the attention storing by output row map -- against the plain attention scattered by
  torch: bit-identical; sa_attn_fwd_split (the last tiles as two key halves + merge) against fp32 torch;
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


def _ref_attn(q, k, v, scale):
    s = (q.float() @ k.float().t()) * scale
    return torch.softmax(s, -1) @ v.float()


@pytest.mark.parametrize("Lk", [777, 50, 128], ids=["ragged", "one_block_empty_half", "two_blocks"])
@pytest.mark.parametrize("split", [1, 7, 36])
def test_attention_key_split(Lk, split):
    """sa_attn_fwd_split: the last `split` of 36 tiles (3 segments x 3 heads x 4 query blocks) as two key halves +
    the log-sum-exp merge, output by row map and accumulated: vs fp32 torch, and the unsplit tiles bit-identical to
    the plain launch"""
    B, Lq, H, D = 3, 1000, 3, 128
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    rows = torch.randperm(2 * B * Lq, device=dev)[:B * Lq].to(torch.int32)
    plain = torch.full((2 * B * Lq, H * D), float("nan"), device=dev, dtype=torch.bfloat16)
    ops.attention(q, k, v, plain, segs, B, Lq, H, kernel=1, o_rows=rows)
    o = torch.full_like(plain, float("nan"))
    ops.attention(q, k, v, o, segs, B, Lq, H, o_rows=rows, split_tiles=split)
    torch.cuda.synchronize()
    got, ref_p = o[rows.long()].view(B, Lq, H, D), plain[rows.long()].view(B, Lq, H, D)
    for b in range(B):
        for h in range(H):
            ref = _ref_attn(q.view(B, Lq, H, D)[b, :, h], k.view(B, Lk, H, D)[b, :, h], v.view(B, Lk, H, D)[b, :, h],
                            D ** -0.5)
            assert ((got[b, :, h].float() - ref).norm() / ref.norm()).item() < 1e-2, (b, h)
    # tiles in launch order (segment, head, query block); the first 36 - split are the plain kernel's
    nqb = 4
    for t in range(36 - split):
        b, h, qb = t // (H * nqb), (t // nqb) % H, t % nqb
        sl = slice(qb * 256, min((qb + 1) * 256, Lq))
        assert torch.equal(got[b, sl, h], ref_p[b, sl, h]), t
    assert (o.isnan().any(1) == ~torch.isin(torch.arange(2 * B * Lq, device=dev), rows.long())).all()
    acc = o.clone()
    ops.attention(q, k, v, acc, segs, B, Lq, H, o_rows=rows, split_tiles=split, accumulate=True)
    assert ((acc[rows.long()].float() - 2 * o[rows.long()].float()).norm() / o[rows.long()].float().norm()) < 1e-2


def test_attention_key_split_sp_shape():
    """the Ulysses N = 8 per-rank launch (3 rows x 10 752 queries x 3 heads over 21 504 keys = 378 tiles): the split
    policy picks the tiles past the first round over the CUs, and the split launch matches the plain one"""
    B, Lq, Lk, H, D = 3, 10752, 21504, 3, 128
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    n_tiles = B * H * (Lq // 256)
    split = ops.attn_tail_split(0, n_tiles, q_dev := torch.device(dev))
    if n_cu == 256:
        assert split == 122
        # per-row launches on concurrent streams: only the last row's launch holds the tail
        assert [ops.attn_tail_split(b * n_tiles // 3, n_tiles // 3, q_dev) for b in range(3)] == [0, 0, 122]
    if not split:
        pytest.skip(f"no tail split on {n_cu} CUs")
    q = torch.randn(B * Lq, H * D, device=dev).bfloat16()
    k = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    v = torch.randn(B * Lk, H * D, device=dev).bfloat16()
    segs = torch.tensor([[b * Lq, Lq, b * Lk, Lk] for b in range(B)], dtype=torch.int32, device=dev)
    plain = torch.empty(B * Lq, H * D, device=dev, dtype=torch.bfloat16)
    ops.attention(q, k, v, plain, segs, B, Lq, H, kernel=1)
    o = torch.empty_like(plain)
    ops.attention(q, k, v, o, segs, B, Lq, H, split_tiles=split)
    torch.cuda.synchronize()
    rel = ((o.float() - plain.float()).norm() / plain.float().norm()).item()
    assert rel < 5e-3, rel
    tiles_plain = n_tiles - split  # whole tiles are the plain kernel's, bit for bit
    ov, pv = o.view(B, Lq, H, D), plain.view(B, Lq, H, D)
    for t in (0, tiles_plain - 1):
        b, h, qb = t // (H * 42), (t // 42) % H, t % 42
        assert torch.equal(ov[b, qb * 256:(qb + 1) * 256, h], pv[b, qb * 256:(qb + 1) * 256, h])


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
