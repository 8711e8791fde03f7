"""Sequence-parallel DiT forward on the HIP path, pinned to the reference's own outputs: gloo ranks sharing one
MI355X (host-staged exchange) at world 2, 4 and 8 run the goldens of tests/golden/dit_small.npz (12 heads: U2, U4,
and at 8 the U4 x 2 query-split layout) and, at world 8, the 14B-width model (40 heads: U8) against
dit14_small.npz, with the same tolerance as the single-GPU golden tests (rel-L2 <= 2e-2, cosine >= 0.9995).  Each
run also matches the same process's single-GPU forward to 1e-3.  Cases: 'full' (80 tokens), 'short' (the padded
last window), 'wide' (120 tokens); at world 8 the 80- and 84-token sequences are padded to a multiple of the
degree (SP pads are queries only).  All four exchange schedules run (sync batched; per-row with per-row attention;
per-row Q/K/V exchanges with one batched attention; every CFG row through the whole block on its own stream).  On RCCL the box's one GPU allows a single rank
(two RCCL ranks cannot share a device), so the RCCL tests run at degree 1 with loopback transfers (each rank's own
chunk sent to itself): every send / receive, stream wait and all-gather of the exchange executes on RCCL."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

sys.path.insert(0, HERE)
from mp_util import collect  # noqa: E402

pytestmark = pytest.mark.gpu


def _rendezvous_file():
    """a fresh rendezvous file for the process group (file:// init: no TCP port to race for -- a port picked free and
    released can be taken before the store listens on it, EADDRINUSE)"""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="sa_rdv_"), "store")


def _stats(out, ref):
    a, b = out.double().flatten(), torch.as_tensor(ref).double().flatten()
    return ((a - b).norm() / b.norm()).item(), (a @ b / (a.norm() * b.norm())).item()


def _worker(rank, world, port, model, qret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        res = []
        if model == "1.3B":
            from test_gpu_dit import make_model, run
            from golden_cases import DIT_SMALL, dit_inputs
            m = make_model(DIT_SMALL)
            g = np.load(os.path.join(HERE, "golden", "dit_small.npz"))
            cases = [(c, dit_inputs(DIT_SMALL, c), g[f"{c}_out"]) for c in ("full", "short", "wide")]
        else:
            from stableavatar_amd import synthetic
            from stableavatar_amd.transformer import WanTransformer3DFantasy14BModel, param_shapes
            from golden_cases import DIT14_SMALL, dit14_inputs
            cfg = dict(DIT14_SMALL, vocal="14B")
            m = WanTransformer3DFantasy14BModel(**{k: v for k, v in cfg.items() if k not in ("seed", "vocal")})
            m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), cfg["seed"]))
            m = m.cuda()
            cases = [("dit14", dict(dit14_inputs(cfg), n_frames=81),
                      np.load(os.path.join(HERE, "golden", "dit14_small.npz"))["out"])]

            def run(mm, inp):
                with torch.no_grad():
                    o = mm(x=inp["x"].cuda(), t=inp["t"].cuda(), context=[c.cuda() for c in inp["context"]],
                           seq_len=inp["seq_len"], clip_fea=inp["clip_fea"].cuda(), y=inp["y"].cuda(),
                           vocal_embeddings=inp["vocal"].cuda())
                torch.cuda.synchronize()
                return o.float().cpu()
        for name, inp, gold in cases:
            m.disable_multi_gpus_inference()
            single = run(m, inp)
            es_gold, _ = _stats(single, gold)
            m.enable_multi_gpus_inference()
            # one batched exchange / per-row exchanges + per-row attention / per-row Q/K/V exchanges + batched attention
            for ov in ("0", "2", "3", "4"):
                os.environ["SA_SP_OVERLAP"] = ov
                par = run(m, inp)
                e_single = ((par - single).norm() / single.norm()).item()
                e_gold, c_gold = _stats(par, gold)
                res.append((name, ov, e_single, e_gold, c_gold, bool(torch.isfinite(par).all()),
                            tuple(par.shape) == tuple(gold.shape), es_gold))
        qret.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,model", [(2, "1.3B"), (4, "1.3B"), (8, "1.3B"), (8, "14B")])
def test_sp_matches_reference_golden(world, model):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(procs, qret, world, timeout=540)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, rows in res:
        for name, ov, e_single, e_gold, c_gold, finite, shape_ok, es_gold in rows:
            print(f"world {world} {model} rank {rank} {name} overlap {ov}: vs golden rel {e_gold:.2e} cos "
                  f"{c_gold:.6f}, vs single-GPU {e_single:.1e} (single-GPU vs golden {es_gold:.2e})")
            assert finite and shape_ok, (rank, name)
            assert e_gold < 2e-2 and c_gold > 0.9995, (rank, name, ov, e_gold, c_gold)
            assert es_gold < 2e-2, (rank, name, es_gold)
            assert e_single < 1e-3, (rank, name, ov, e_single)


def _shared_rows_worker(rank, world, port, qret):
    """forward_window(shared_rows=True) on the Ulysses path: the first block's self-attention half for CFG row 0
    through the exchange, copied to the other rows -- equal to computing every row, in every schedule"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        from test_gpu_dit import make_model
        from golden_cases import DIT_SMALL
        from stableavatar_amd import synthetic
        from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
        m = make_model(DIT_SMALL)
        dev = "cuda"
        lat = synthetic.seeded_normal((1, 16, 5, 8, 8), 401).to(dev).bfloat16()
        y = WanI2VTalkingInferenceLongPipeline.mask_latents(synthetic.seeded_normal((1, 16, 5, 8, 8), 402).to(dev),
                                                            17).bfloat16()
        ctx = [synthetic.seeded_normal((20, 64), 403).to(dev)] * 2 + [synthetic.seeded_normal((25, 64), 404).to(dev)]
        clip = synthetic.seeded_normal((1, 257, 1280), 405).expand(3, -1, -1).contiguous().to(dev)
        a = synthetic.seeded_normal((1, 39, 768), 406).to(dev)
        voc = torch.cat([torch.zeros_like(a), a, a])
        t = torch.tensor([937.5], device=dev)
        m.enable_multi_gpus_inference()
        res = []
        for ov in ("0", "2", "3", "4"):
            os.environ["SA_SP_OVERLAP"] = ov
            outs = []
            with torch.no_grad():
                for shared in (False, True):
                    outs.append(m.forward_window(lat, 0, True, 3, t, ctx, 80, clip, y, voc, 17,
                                                 shared_rows=shared).float().cpu())
            res.append((ov, torch.equal(outs[0], outs[1]), bool(torch.isfinite(outs[0]).all())))
        qret.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 4])
def test_sp_shared_cfg_rows_first_block_once(world):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_shared_rows_worker, args=(r, world, port, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(procs, qret, world, timeout=360)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, rows in res:
        for ov, same, finite in rows:
            print(f"world {world} rank {rank} overlap {ov}: shared first block bit-identical {same}")
            assert finite and same, (rank, ov)


def _rccl_worker(port, overlap, qret):
    """RCCL (backend "nccl") process group of ONE rank with the SP path forced on, in loopback mode
    (UlyssesExchange(loopback=True)): this rank's own token chunk goes through the point-to-point transport to
    itself, so every Q/K/V and head-output transfer of the layer is a real dist.P2POp in a batch_isend_irecv group
    on ProcessGroupNCCL's stream, with the caller's stream waiting on it (sp.Pending) -- the sends / receives that
    run over xGMI at N = 2/4/8 -- and the head output goes through all_gather_into_tensor.  Without loopback the
    degree-1 exchange has no remote rank and sends nothing; that run is checked too."""
    os.environ["SA_SP_OVERLAP"] = overlap
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from test_gpu_dit import make_model, run
    from golden_cases import DIT_SMALL, dit_inputs
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="file://" + port, rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        m = make_model(DIT_SMALL)
        res = []
        for case in ("full", "short"):
            inp = dit_inputs(DIT_SMALL, case)
            m.disable_multi_gpus_inference()
            single = run(m, inp)
            for loop in (False, True):
                m.enable_multi_gpus_inference(loopback=loop)
                assert dist.get_backend() == "nccl" and m._sp_enabled
                par = run(m, inp)
                ex = m._sp_ex[1]
                res.append((case, loop, torch.equal(par, single), ((par - single).norm() / single.norm()).item(),
                            ex.loopback, len(ex.remote)))
        qret.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", ["0", "2", "3", "4"],
                         ids=["batched", "per_row_async", "row_exchange_batched_attn", "row_streams"])
def test_sp_rccl_path_degree1(overlap):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_rendezvous_file(), overlap, qret))
    p.start()
    res = collect([p], qret, 1)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    for case, loop, same, err, ex_loop, n_remote in res:
        print(f"RCCL degree 1 overlap {overlap} {case} loopback {loop}: bit-identical {same} (rel {err:.1e})")
        assert ex_loop == loop and n_remote == (1 if loop else 0)
        assert same, (case, loop, err)


def _rccl_shared_rows_worker(port, qret):
    """the CFG rows' shared first block on RCCL (degree 1, loopback): row 0's Q/K/V and head outputs through real
    P2P ops, in the one-stream and per-row-stream schedules, vs the single-GPU forward computing every row"""
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from test_gpu_dit import make_model
    from golden_cases import DIT_SMALL
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="file://" + port, rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        m = make_model(DIT_SMALL)
        dev = "cuda"
        lat = synthetic.seeded_normal((1, 16, 5, 8, 8), 501).to(dev).bfloat16()
        y = WanI2VTalkingInferenceLongPipeline.mask_latents(synthetic.seeded_normal((1, 16, 5, 8, 8), 502).to(dev),
                                                            17).bfloat16()
        ctx = [synthetic.seeded_normal((20, 64), 503).to(dev)] * 2 + [synthetic.seeded_normal((25, 64), 504).to(dev)]
        clip = synthetic.seeded_normal((1, 257, 1280), 505).expand(3, -1, -1).contiguous().to(dev)
        a = synthetic.seeded_normal((1, 39, 768), 506).to(dev)
        voc = torch.cat([torch.zeros_like(a), a, a])
        t = torch.tensor([937.5], device=dev)

        def fwd(shared):
            with torch.no_grad():
                o = m.forward_window(lat, 0, True, 3, t, ctx, 80, clip, y, voc, 17, shared_rows=shared).float()
            torch.cuda.synchronize()
            return o.cpu()
        m.disable_multi_gpus_inference()
        single = fwd(False)
        m.enable_multi_gpus_inference(loopback=True)
        res = []
        for ov in ("0", "4"):
            os.environ["SA_SP_OVERLAP"] = ov
            res.append((ov, torch.equal(fwd(True), single)))
        qret.put(res)
    finally:
        dist.destroy_process_group()


def test_sp_rccl_shared_rows_degree1():
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_rccl_shared_rows_worker, args=(_rendezvous_file(), qret))
    p.start()
    res = collect([p], qret, 1)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    for ov, same in res:
        print(f"RCCL degree 1 loopback, shared first block, overlap {ov}: bit-identical {same}")
        assert same, ov


def _rccl_fullsize_worker(port, overlap, qret):
    """config-2 size on the RCCL transport: a 1-layer full-width 1.3B DiT (dim 1536, 12 heads, ffn 8960) at the
    512^2 x 81f shape (L = 21 504 tokens, B = 3 CFG rows), Ulysses at degree 1 with loopback transfers (every Q/K/V
    and head-output slab of the layer -- 3 x 21 504 tokens -- moved by RCCL P2P ops to this rank itself) in the
    given exchange schedule, vs the single-GPU forward of the same process"""
    os.environ["SA_SP_OVERLAP"] = overlap
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from golden_cases import DIT_FULL
    from stableavatar_amd import synthetic
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="file://" + port, rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        dev = "cuda"
        cfg = dict(DIT_FULL, num_layers=1)
        m = WanTransformer3DFantasyModel(**cfg)
        m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), 54))
        m = m.to(dev)
        L = 21504
        lat = synthetic.seeded_normal((1, 16, 21, 64, 64), 531)
        x = torch.cat([lat] * 3).to(dev).bfloat16()
        y = synthetic.seeded_normal((3, 20, 21, 64, 64), 532).to(dev).bfloat16()
        ctx = [c.to(dev) for c in [synthetic.seeded_normal((24, 4096), 533)] * 2 +
               [synthetic.seeded_normal((31, 4096), 534)]]
        clip = synthetic.seeded_normal((1, 257, 1280), 535).expand(3, -1, -1).contiguous().to(dev)
        a = synthetic.seeded_normal((1, 167, 768), 536)
        voc = torch.cat([torch.zeros_like(a), a, a]).to(dev)
        t = torch.full((3,), 937.5, device=dev)

        def fwd():
            with torch.no_grad():
                o = m(x=x, t=t, context=ctx, seq_len=L, clip_fea=clip, y=y, vocal_embeddings=voc,
                      video_sample_n_frames=81).float()
            torch.cuda.synchronize()
            return o
        m.disable_multi_gpus_inference()
        single = fwd()
        m.enable_multi_gpus_inference(loopback=True)
        assert dist.get_backend() == "nccl" and m._sp_enabled
        par = fwd()
        ex = m._sp_ex[1]
        qret.put([(torch.equal(par, single), ((par - single).norm() / single.norm()).item(), ex.loopback,
                   len(ex.remote), tuple(ex.q.shape))])
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("overlap", ["4", "0"], ids=["row_streams", "batched"])
def test_sp_rccl_fullsize_degree1(overlap):
    """BASELINE config 2's shape through the RCCL exchange (degree 1, loopback): bit-identical to one GPU"""
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_rccl_fullsize_worker, args=(_rendezvous_file(), overlap, qret))
    p.start()
    res = collect([p], qret, 1, timeout=360)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    same, err, ex_loop, n_remote, qshape = res[0]
    print(f"RCCL degree 1 loopback, config-2 shape (L = 21504, B = 3, q slab {qshape}), overlap {overlap}: "
          f"bit-identical {same} (rel {err:.1e})")
    assert ex_loop and n_remote == 1
    assert same, err


def _rccl_dp_vae_worker(port, qret):
    """window parallelism's async all_gather_into_tensor (sp.all_gather_slots) on a one-rank RCCL group, and the VAE
    decode's causal-cache wavefront over 3 virtual ranks whose hand-offs are RCCL transfers to this rank itself"""
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="file://" + port, rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        from golden_cases import PIPE
        from stableavatar_amd import synthetic
        from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
        from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
        from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes, param_shapes as vae_shapes
        from test_gpu_window_dp import _run
        dcfg = PIPE["dit"]
        dit = WanTransformer3DFantasyModel(**{k: v for k, v in dcfg.items() if k != "seed"})
        dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), dcfg["seed"]))
        pipe = WanI2VTalkingInferenceLongPipeline(transformer=dit.cuda())
        single = _run(pipe, 9, False)
        par = _run(pipe, 9, True)
        res = {"window_dp": (bool(torch.equal(single, par)), float((single.float() - par.float()).abs().max()))}
        v = AutoencoderKLWan(dim=32)
        v.load_state_dict(synthetic.fill_state_dict(dict(vae_shapes(dim=32), **encoder_param_shapes(dim=32)), 24))
        v = v.cuda()
        z = synthetic.seeded_normal((16, 7, 8, 8), 424).cuda()
        with torch.no_grad():
            vs = v.decode_clip(z, post=True).cpu()
            v.enable_multi_gpus_inference(loopback_ranks=3)
            vp = v.decode_clip(z, post=True, chunk=2).cpu()
        torch.cuda.synchronize()
        res["vae_loopback"] = (bool(torch.equal(vs, vp)), float((vs - vp).abs().max()), v.decode_loopback)
        qret.put(res)
    finally:
        dist.destroy_process_group()


def test_rccl_window_dp_and_vae_loopback_degree1():
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_rccl_dp_vae_worker, args=(_rendezvous_file(), qret))
    p.start()
    res = collect([p], qret, 1, timeout=300)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    print(res)
    assert res["window_dp"][0], res
    assert res["vae_loopback"][0] and res["vae_loopback"][2] == 3, res


def _split_rank_worker(qret):
    """one Ulysses rank of N = 8 at the config-2 shape (3 rows x 2 688 tokens, 2 full-width blocks) with the transfers
    stubbed out (the exchange buffers hold the same seeded values in both runs): the self-attention launches with
    their tail split into key halves (the default: ops.attn_tail_split, schedule 4 splits the last row's launch and runs
    every row on the 8-wave kernel; schedule 0 splits the batched launch) against SA_ATTN_SPLIT=0"""
    import torch
    from golden_cases import DIT_FULL
    from stableavatar_amd import ops, sp, synthetic
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    dev = "cuda"
    cfg = dict(DIT_FULL, num_layers=2)
    m = WanTransformer3DFantasyModel(**cfg)
    m.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), 61))
    m = m.to(dev)
    sp._p2p = lambda sends, recvs, group: sp.Pending(None)
    sp.gather_tokens = lambda local, B, Lc, world, group=None: torch.zeros(B * world * Lc, local.shape[1],
                                                                             device=local.device, dtype=local.dtype)
    m.sp_group, m.sp_world_size, m.sp_world_rank, m._sp_enabled = None, 8, 5, True
    g = torch.Generator(device=dev).manual_seed(0)
    lat = torch.randn(1, 16, 21, 64, 64, device=dev, generator=g).bfloat16()
    y = torch.randn(3, 20, 21, 64, 64, device=dev, generator=g).bfloat16()
    ctx = [torch.randn(n, 4096, device=dev, generator=g) for n in (120, 120, 60)]
    clip = torch.randn(3, 257, 1280, device=dev, generator=g)
    voc = torch.randn(3, 167, 768, device=dev, generator=g)
    t = torch.tensor([990.0], device=dev)
    res = []
    with torch.no_grad():
        for ov in ("4", "0"):
            os.environ["SA_SP_OVERLAP"] = ov
            outs = []
            for split in ("0", "1"):
                os.environ["SA_ATTN_SPLIT"] = split
                m.forward_window(lat, 0, True, 3, t, ctx, 21504, clip, y, voc, 81)  # builds the exchange
                ex = m._sp_ex[1]
                gb = torch.Generator(device=dev).manual_seed(1)
                for buf in (ex.q, ex.kv, ex.obuf):
                    buf.normal_(generator=gb)
                m.forward_window(lat, 0, True, 3, t, ctx, 21504, clip, y, voc, 81)
                # this rank's residual stream after the blocks (the stubbed all-gather returns zeros for the output)
                outs.append(next(iter(m._ws.values())).x.clone())
            torch.cuda.synchronize()
            n_split = ops.attn_tail_split(0, 3 * 3 * 42, torch.device(dev))
            a, b = outs[0].double(), outs[1].double()  # stubbed transfers: large values, norms in fp64
            rel = ((b - a).norm() / a.norm()).item()
            res.append((ov, rel, bool(torch.isfinite(outs[1]).all()), n_split, bool(torch.isfinite(outs[0]).all())))
    qret.put(res)


@pytest.mark.timeout(400)
def test_sp_rank_attention_key_split_n8_shape():
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_split_rank_worker, args=(qret,))
    p.start()
    res = collect([p], qret, 1, timeout=360)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    for ov, rel, finite, n_split, finite0 in res:
        print(f"N = 8 rank shape, schedule {ov}: key-split tail ({n_split} tiles) vs unsplit rel {rel:.2e} "
              f"(finite: split {finite}, unsplit {finite0})")
        assert finite and finite0 and rel < 5e-3, (ov, rel)
