"""Window-parallel denoising: the sliding windows of every step spread over
the ranks, noise predictions all-gathered, blend replicated.  2 ranks sharing one MI355X (gloo,
host-staged gather) must reproduce the single-GPU loop BIT-EXACTLY, with 3 windows per step (an
uneven split: rank 1 idles in the second round)."""
import math
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

sys.path.insert(0, HERE)
from mp_util import collect  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(pipe, T, steps, window_parallel):
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    from golden_cases import PIPE
    P = PIPE
    fpb = (P["clip_length"] - 1) // 4 + 1
    g = torch.Generator().manual_seed(5)
    lat = torch.randn(1, 16, T, 8, 8, generator=g)
    y = torch.randn(3, 20, fpb, 8, 8, generator=g)
    ctx = [torch.randn(12, 64, generator=g), torch.randn(12, 64, generator=g), torch.randn(9, 64, generator=g)]
    clip = torch.randn(1, 257, 1280, generator=g).expand(3, -1, -1).contiguous()
    feats = {}
    for (s, e, _) in window_schedule(T, fpb, P["overlap"]):
        a = synthetic.fake_wav2vec_features(torch.randn(1, 20 * 640, generator=g))
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a]).cuda()
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(steps, device="cuda")
    pipe.window_group = None
    if window_parallel:
        pipe.enable_window_parallel()
    seq_len = math.ceil(8 * 8 / 4 * fpb)
    with torch.no_grad():
        out = pipe.denoise(lat.cuda(), y.cuda(), [c.cuda() for c in ctx], clip.cuda(), feats, sched.timesteps,
                           sched.sigmas, clip_length=P["clip_length"], seq_len=seq_len, overlap=P["overlap"],
                           text_guide_scale=3.0, audio_guide_scale=5.0)
    torch.cuda.synchronize()
    return out.cpu()


def _worker(rank, world, port, qret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from golden_cases import PIPE
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dcfg = PIPE["dit"]
        dit = WanTransformer3DFantasyModel(**{k: v for k, v in dcfg.items() if k != "seed"})
        dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), dcfg["seed"]))
        pipe = WanI2VTalkingInferenceLongPipeline(transformer=dit.cuda())
        single = _run(pipe, 9, 3, False)
        par = _run(pipe, 9, 3, True)
        qret.put((rank, bool(torch.equal(single, par)), float((single.float() - par.float()).abs().max())))
    finally:
        dist.destroy_process_group()


def test_window_parallel_bit_exact():
    from stableavatar_amd.pipeline import window_schedule
    assert len(window_schedule(9, 5, 2)) == 3
    world = 2
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(procs, qret, world)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, same, mx in res:
        assert same, (rank, mx)
