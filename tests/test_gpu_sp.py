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

sys.path.insert(0, HERE)
from mp_util import collect  # noqa: E402

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
    res = collect(procs, qret, world)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, err, finite in res:
        assert finite and err < 1e-3, (rank, err)


def _rccl_worker(port, overlap, qret):
    """RCCL (backend "nccl") process group of ONE rank with the SP path forced on: every Ulysses
    exchange is a real async all_to_all_single on ProcessGroupNCCL's stream (a self-copy at degree 1)
    with the deferred unpack (sp.Pending), and the head output goes through all_gather_into_tensor -
    the code that runs over xGMI at N = 2/4/8, here on the one GPU of the box."""
    os.environ["SA_SP_OVERLAP"] = overlap
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from test_gpu_dit import make_model, run
    from golden_cases import DIT_SMALL, dit_inputs
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        m = make_model(DIT_SMALL)
        inp = dit_inputs(DIT_SMALL, "full")
        single = run(m, inp)
        m.enable_multi_gpus_inference()
        assert dist.get_backend() == "nccl" and m._sp_enabled
        par = run(m, inp)
        qret.put((torch.equal(par, single), ((par - single).norm() / single.norm()).item()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", ["0", "2"], ids=["batched", "per_row_async"])
def test_sp_rccl_path_degree1(overlap):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), overlap, qret))
    p.start()
    same, err = collect([p], qret, 1)[0]
    p.join(timeout=120)
    assert p.exitcode == 0
    assert same, err
