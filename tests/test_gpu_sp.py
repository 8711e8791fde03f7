"""Sequence-parallel DiT forward on the HIP path: 2 ranks (gloo, host-staged exchange) sharing one
MI355X must reproduce the single-GPU forward.  Token chunks of 40 = 2.5 latent frames exercise the
global-frame vocal grouping (SURVEY.md App. A.2 fix), the 'short' window the padded tail."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case, overlap, qret):
    os.environ["SA_SP_OVERLAP"] = overlap
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from test_gpu_dit import make_model, run
    from golden_cases import DIT_SMALL, dit_inputs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = make_model(DIT_SMALL)
        inp = dit_inputs(DIT_SMALL, case)
        single = run(m, inp)
        m.enable_multi_gpus_inference()
        par = run(m, inp)
        err = ((par - single).norm() / single.norm()).item()
        qret.put((rank, err, bool(torch.isfinite(par).all())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,overlap", [("full", "0"), ("short", "0"), ("full", "2"), ("short", "2")])
def test_sp2_matches_single_gpu(case, overlap):
    world = 2
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, overlap, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = [qret.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, err, finite in res:
        assert finite and err < 1e-3, (rank, err)
