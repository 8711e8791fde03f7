"""Window-parallel denoising: the sliding windows of every step spread over
the ranks, noise predictions all-gathered, blend replicated.  Ranks sharing one MI355X (gloo, host-staged
gather) must reproduce the single-GPU loop BIT-EXACTLY: 2 ranks x 3 windows per step (rank 1 idles in the
second round) and 3 ranks x 8 windows per step (26 latent frames, uneven last round); the 8-window run is also
checked against the CPU oracle's restatement of the reference loop (oracle/pipeline.py, pinned to the
reference's __call__ goldens) at the pipeline tolerance (latents rel-L2 <= 3e-2); 8 ranks x 17 windows per step
(53 latent frames) is config 5's rank count, also against the oracle loop; and config 5's LENGTH: T_lat 251 (1 001
video frames) with the reference's 81-frame windows at overlap 10 = 22 windows per step over 8 ranks (SURVEY.md §8(d)
config 5), on the small 8x8-latent DiT, bit-exact vs one GPU and against the oracle loop."""
import math
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

sys.path.insert(0, HERE)
from mp_util import collect  # noqa: E402

pytestmark = pytest.mark.gpu

STEPS = 3


def _rendezvous_file():
    """a fresh rendezvous file for the process group (file:// init: no TCP port to race for -- a port picked free and
    released can be taken before the store listens on it, EADDRINUSE)"""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="sa_rdv_"), "store")


def _inputs(T, clip_length=17):
    fpb = (clip_length - 1) // 4 + 1
    g = torch.Generator().manual_seed(5)
    lat = torch.randn(1, 16, T, 8, 8, generator=g)
    y = torch.randn(3, 20, fpb, 8, 8, generator=g)
    ctx = [torch.randn(12, 64, generator=g), torch.randn(12, 64, generator=g), torch.randn(9, 64, generator=g)]
    ctx[1] = ctx[0]
    clip = torch.randn(1, 257, 1280, generator=g).expand(3, -1, -1).contiguous()
    audio = 0.1 * torch.randn((1 + 4 * (T - 1)) * 640 + 320, generator=g)  # 1 + 4 (T - 1) video frames
    return lat, y, ctx, clip, audio


def _run(pipe, T, window_parallel, clip_length=17, overlap=2):
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import audio_window, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
    fpb = (clip_length - 1) // 4 + 1
    lat, y, ctx, clip, audio = _inputs(T, clip_length)
    feats = {}
    for (s, e, _) in window_schedule(T, fpb, overlap):
        a = synthetic.fake_wav2vec_features(audio[audio_window(s, e, T, 640, audio.shape[0])][None])
        feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a]).cuda()
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(STEPS, device="cuda")
    pipe.window_group = None
    if window_parallel:
        pipe.enable_window_parallel()
    seq_len = math.ceil(8 * 8 / 4 * fpb)
    with torch.no_grad():
        out = pipe.denoise(lat.cuda(), y.cuda(), [c.cuda() for c in ctx], clip.cuda(), feats, sched.timesteps,
                           sched.sigmas, clip_length=clip_length, seq_len=seq_len, overlap=overlap,
                           text_guide_scale=3.0, audio_guide_scale=5.0)
    torch.cuda.synchronize()
    return out.cpu()


def _worker(rank, world, port, T, qret, clip_length=17, overlap=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    import torch.distributed as dist
    from golden_cases import PIPE
    from stableavatar_amd import synthetic
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        dcfg = PIPE["dit"]
        dit = WanTransformer3DFantasyModel(**{k: v for k, v in dcfg.items() if k != "seed"})
        dit.load_state_dict(synthetic.fill_state_dict(param_shapes(dcfg), dcfg["seed"]))
        pipe = WanI2VTalkingInferenceLongPipeline(transformer=dit.cuda())
        single = _run(pipe, T, False, clip_length, overlap)
        par = _run(pipe, T, True, clip_length, overlap)
        qret.put((rank, bool(torch.equal(single, par)), float((single.float() - par.float()).abs().max()),
                  par if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def _oracle_loop(T, clip_length=17, overlap=2):
    """the reference loop (pipeline:703-790) restated on the CPU with the oracle DiT"""
    from oracle import dit as odit
    from oracle import pipeline as opipe
    from stableavatar_amd import synthetic
    from golden_cases import PIPE
    P = PIPE
    Pd = synthetic.fill_state_dict(odit.param_shapes(P["dit"]), P["dit"]["seed"])
    lat, y, ctx, clip, audio = _inputs(T, clip_length)

    def dit(x, t, context, seq_len, yy, clip_fea, vocal, n):
        return odit.forward(Pd, P["dit"], x.to(torch.bfloat16).float(), t, context, seq_len, clip_fea,
                            yy.to(torch.bfloat16).float(), vocal, n)

    enc = lambda s: synthetic.fake_wav2vec_features(torch.as_tensor(s)[None])  # noqa: E731
    with torch.no_grad():
        return opipe.denoise(dit, lat.to(torch.bfloat16).float(), y, ctx, clip, audio, enc,
                             num_inference_steps=STEPS, clip_length=clip_length, num_frames=clip_length,
                             height=64, width=64, overlap=overlap, text_guide_scale=3.0, audio_guide_scale=5.0)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,T,clip_length,overlap", [(2, 9, 17, 2), (3, 26, 17, 2), (8, 53, 17, 2),
                                                         (8, 251, 81, 10)])
def test_window_parallel_bit_exact(world, T, clip_length, overlap):
    """(8, 53): config 5's rank count, 17 windows per step (3 rounds over 8 ranks, 1 window in the last);
    (8, 251, 81, 10): config 5's length -- 1 001 frames in 81-frame windows at overlap 10, 22 windows per step
    (pipeline:714-789), 3 rounds over 8 ranks with 6 windows in the last"""
    from stableavatar_amd.pipeline import window_schedule
    n_win = len(window_schedule(T, (clip_length - 1) // 4 + 1, overlap))
    assert n_win == {9: 3, 26: 8, 53: 17, 251: 22}[T]
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, qret, clip_length, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(procs, qret, world, timeout=540)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, same, mx, _ in res:
        assert same, (rank, mx)
    if T >= 26:
        par = next(r[3] for r in res if r[0] == 0).float()
        ref = _oracle_loop(T, clip_length, overlap)
        e = ((par - ref).norm() / ref.norm()).item()
        print(f"window-parallel {world} ranks, {n_win} windows/step: vs oracle loop rel-L2 {e:.2e}")
        assert e <= 3e-2, e
