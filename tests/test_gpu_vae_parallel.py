"""Multi-rank VAE decode (second half): rank r decodes the r-th contiguous run of
latent frames, receiving every causal conv's 2-frame cache from rank r-1 and passing its own to rank r+1
(wan_vae.py:27-36 cache_x, :549-574 per-frame loop), then one gather.  2 and 3 ranks sharing one MI355X
(gloo, host-staged P2P) must reproduce the single-GPU decode BIT-EXACTLY, including per-rank runs split
into sub-chunks (chunk 2) and a first run of a single latent frame (3 ranks over 4 frames)."""
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


def _rendezvous_file():
    """a fresh rendezvous file for the process group (file:// init: no TCP port to race for -- a port picked free and
    released can be taken before the store listens on it, EADDRINUSE)"""
    import tempfile
    return os.path.join(tempfile.mkdtemp(prefix="sa_rdv_"), "store")


def _worker(rank, world, port, T, chunk, qret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    import torch.distributed as dist
    from stableavatar_amd import synthetic
    from stableavatar_amd.vae import AutoencoderKLWan, encoder_param_shapes, param_shapes
    dist.init_process_group("gloo", init_method="file://" + port, rank=rank, world_size=world)
    try:
        v = AutoencoderKLWan(dim=32)
        v.load_state_dict(synthetic.fill_state_dict(dict(param_shapes(dim=32), **encoder_param_shapes(dim=32)), 24))
        v = v.cuda()
        z = synthetic.seeded_normal((16, T, 8, 8), 424).cuda()
        with torch.no_grad():
            single = v.decode_clip(z, post=True).cpu()
            v.enable_multi_gpus_inference()
            par = v.decode_clip(z, post=True, chunk=chunk).cpu()
        torch.cuda.synchronize()
        qret.put((rank, tuple(par.shape), bool(torch.equal(single, par)), float((single - par).abs().max())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T,chunk", [(2, 7, None), (2, 7, 2), (3, 4, None)])
def test_vae_decode_multi_rank_bit_exact(world, T, chunk):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    port = _rendezvous_file()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, chunk, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = collect(procs, qret, world)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, shape, same, mx in res:
        assert shape == (3, 1 + 4 * (T - 1), 64, 64)
        assert same, (rank, mx)
