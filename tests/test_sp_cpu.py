"""Sequence-parallel exchange (stableavatar_amd/sp.py) on CPU with gloo, world sizes 2/3/4/8.

Pins the identity the reference's SP path is meant to hold (xfuser row): attention
over the token-sharded, head-exchanged layout equals single-device full attention (1B:158-207 SDPA),
plus the single-GPU frame grouping of the per-frame vocal attention and the head all-gather.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stableavatar_amd import sp


def _rendezvous_file():
    """a fresh rendezvous file for the process group (file:// init: no TCP port to race for -- a port picked free and
    released can be taken before the store listens on it, EADDRINUSE)"""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="sa_rdv_"), "store")


def _sdpa(q, k, v):
    # q [B, Lq, h, D], k/v [B, Lk, h, D] -> [B, Lq, h, D], fp32 softmax(QK^T/sqrt(D))V
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / q.shape[-1] ** 0.5
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v)


def _pack(ex, mine, plan):
    """test-side restatement of sa_qkv_pack's scatter (the norm / RoPE aside): head group g of this rank's
    q to destination my_part*G + g, of k | v to every r*G + g -- through the same slab views the device
    table names"""
    B, Lc = mine.shape[:2]
    hg = plan.hg
    for d, (qd, kd) in ex.slabs.items():
        g = d % plan.G
        grp = mine[:, :, :, g * hg:(g + 1) * hg].reshape(B, Lc, 3, -1)
        if qd is not None:
            assert d // plan.G == plan.part
            qd.copy_(grp[:, :, 0])
        else:
            assert d // plan.G != plan.part
        kd.copy_(torch.cat([grp[:, :, 1], grp[:, :, 2]], -1))


def _worker(rank, world, port, B, Lp, H, D, q_ret, loopback=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)
        qkv = torch.randn(B, Lp, 3, H, D, generator=g)
        ref = _sdpa(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])          # [B, Lp, H, D]
        plan = sp.make_plan(world, rank, H)
        Lc = Lp // world
        mine = qkv[:, rank * Lc:(rank + 1) * Lc]                          # [B, Lc, 3, H, D]
        hg, G = plan.hg, plan.G
        res = []
        for rows in ([list(range(B))], [[b] for b in range(B)]):          # batched / per CFG row
            ex = sp.UlyssesExchange(plan, B, Lc, D, "cpu", dtype=torch.float32, loopback=loopback)
            assert (rank in ex.remote) == loopback
            # the pack table is the slab views' addresses and strides (elements)
            for d, (qd, kd) in ex.slabs.items():
                t = ex.table[d].tolist()
                assert t[3:] == [kd.data_ptr(), kd.stride(1), kd.stride(0)]
                assert t[:3] == ([0, 0, 0] if qd is None else [qd.data_ptr(), qd.stride(1), qd.stride(0)])
            _pack(ex, mine, plan)
            for r in rows:
                ex.heads(r).wait()
            Lq = ex.Lq
            assert Lq == Lp // plan.R
            # the attention inputs: query part's tokens (head group g) and all keys
            qpart = qkv[:, plan.part * Lq:(plan.part + 1) * Lq, 0, plan.group * hg:(plan.group + 1) * hg]
            assert torch.equal(ex.q.view(B, Lq, hg, D), qpart)
            kvh = ex.kv.view(B, Lp, 2, hg, D)
            assert torch.equal(kvh[:, :, 0], qkv[:, :, 1, plan.group * hg:(plan.group + 1) * hg])
            o = _sdpa(ex.q.view(B, Lq, hg, D), kvh[:, :, 0], kvh[:, :, 1]).reshape(B * Lq, hg * D)
            ex.obuf[ex.omap.long()] = o                                   # the attention's row-mapped store
            for r in rows:
                ex.tokens(r).wait()
            a0, (pc, ps) = ex.panels()
            assert pc == hg * D and ps == B * Lc * hg * D and a0.data_ptr() == ex.pan.data_ptr()
            att = ex.pan.view(G, B, Lc, hg, D).permute(1, 2, 0, 3, 4).reshape(B, Lc, H, D)
            res.append(att)
        err = (res[0] - ref[:, rank * Lc:(rank + 1) * Lc]).abs().max().item()
        assert torch.equal(res[0], res[1])
        full = sp.gather_tokens(res[0].reshape(B * Lc, H * D).contiguous(), B, Lc, world)  # 1B:1150-1152
        err = max(err, (full.view(B, Lp, H, D) - ref).abs().max().item())
        q_ret.put((rank, err, plan.G, plan.R))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,loopback", [(2, 12, False), (3, 12, False), (4, 12, False), (8, 12, False),
                                               (8, 40, False), (1, 12, True), (2, 12, True), (8, 12, True)])
def test_ulysses_exchange_matches_full_attention(world, H, loopback):
    """12 heads: the 1.3B model (N = 8 is U4 x 2 query parts); 40 heads: the 14B model (N = 8 is U8).  loopback:
    each rank's own chunk also goes through the transport (to itself), the layout the degree-1 RCCL test runs"""
    B, D = 3, 16
    Lp = sp.padded_len(48, world)
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, Lp, H, D, qret, loopback)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qret.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, G, R in res:
        assert err < 1e-5, (rank, err)
        assert G * R == world and H % G == 0


def test_plan_shapes():
    assert (sp.make_plan(8, 5, 12).G, sp.make_plan(8, 5, 12).R) == (4, 2)
    assert (sp.make_plan(2, 1, 12).G, sp.make_plan(2, 1, 12).R) == (2, 1)
    assert (sp.make_plan(4, 0, 12).G, sp.make_plan(4, 0, 12).R) == (4, 1)
    assert (sp.make_plan(8, 3, 40).G, sp.make_plan(8, 3, 40).R) == (8, 1)  # 14B: Ulysses 8
    assert sp.padded_len(21504, 8) == 21504 and sp.padded_len(21505, 8) == 21512


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_vocal_segments_use_global_frames(world):
    """Union over ranks of the local segments == the single-GPU grouping q.view(B*F, -1) (1B:576)."""
    B, n_fr, nper, G = 3, 21, 17, 1024
    Lp = n_fr * G
    Lc = Lp // world
    seen = {}
    for r in range(world):
        for q0, ql, k0, kl in sp.vocal_segments(B, Lp, Lc, r, n_fr, nper):
            b = q0 // Lc
            for t in range(q0 - b * Lc, q0 - b * Lc + ql):
                gt = r * Lc + t
                seen[(b, gt)] = (k0, kl)
    assert len(seen) == B * Lp
    for (b, gt), (k0, kl) in seen.items():
        assert k0 == (b * n_fr + gt // G) * nper and kl == nper


@pytest.mark.parametrize("world,S,n_fr", [(8, 84, 21), (3, 80, 5), (8, 80, 5), (16, 84, 21)])
def test_vocal_segments_with_sp_pads(world, S, n_fr):
    """S not a multiple of the degree: the tokens < S keep the single-GPU frame t // (S / F); the pad tokens
    past S (Lp - S of them, queries only) join the last frame; every local row is covered exactly once."""
    B, nper = 3, 17
    G = S // n_fr
    Lp = sp.padded_len(S, world)
    Lc = Lp // world
    seen = {}
    for r in range(world):
        for q0, ql, k0, kl in sp.vocal_segments(B, S, Lc, r, n_fr, nper):
            assert ql > 0 and kl == nper
            b = q0 // Lc
            for t in range(q0 - b * Lc, q0 - b * Lc + ql):
                assert (b, r * Lc + t) not in seen
                seen[(b, r * Lc + t)] = k0
    assert len(seen) == B * Lp
    for (b, gt), k0 in seen.items():
        assert k0 == (b * n_fr + min(gt // G, n_fr - 1)) * nper


def _slots_worker(rank, world, port, q_ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        n_win, S = 5, 33
        rounds = -(-n_win // world)
        buf = torch.full((rounds * world, S), -1.0)
        pend = []
        for j in range(rounds):  # the window-parallel schedule of pipeline._denoise_window_parallel
            k = j * world + rank
            if k < n_win:
                buf[k] = torch.arange(S, dtype=torch.float32) + 100 * k
            pend.append(sp.all_gather_slots(buf[j * world:(j + 1) * world], rank))
        for p in pend:
            p.wait()
        ok = all(torch.equal(buf[k], torch.arange(S, dtype=torch.float32) + 100 * k) for k in range(n_win))
        q_ret.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_window_parallel_slot_gather(world):
    """Every rank ends with every window's slot (5 windows: uneven rounds for both world sizes)."""
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_slots_worker, args=(r, world, port, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qret.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res), res
