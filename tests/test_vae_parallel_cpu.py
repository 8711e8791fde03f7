"""The multi-rank VAE decode's hand-off protocol on CPU (gloo, world 2 and 3): every rank walks the same
sequence of causal-cache points, takes each cache from rank r-1 and passes its update to rank r+1, in order;
skipped points forward the previous cache; the frame gather returns every rank's block in rank order."""
import os
import tempfile
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from mp_util import collect  # noqa: E402


def _store():
    """a file:// rendezvous path (nothing to bind: no free port picked and released)"""
    fd, path = tempfile.mkstemp(prefix="sa_store_")
    os.close(fd)
    os.unlink(path)
    return path


def _worker(rank, world, store, qret):
    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    try:
        from stableavatar_amd.vae import _all_gather, _ChainState, _SeqState
        # 3 "frames" per rank at every cache point; the update keeps the last two; rank r's frames hold r
        like = torch.zeros(3, 2, 2, 4, dtype=torch.bfloat16)
        x = torch.full_like(like, float(rank + 1))
        st = _ChainState(dist.group.WORLD, rank, world)
        seen = []
        for sub in range(2):  # two sub-chunks per rank: only the first receives, only the last sends
            st.begin(sub == 0, sub == 1)
            for k in range(12):
                if k == 5:
                    st.skip(k, like)
                    continue
                p = st.get(k, like)
                seen.append(None if p is None else float(p.float().mean()))
                st.put(k, (x + sub)[-2:].clone())
        st.finish()
        seq = _SeqState()
        seq.put(0, x)
        assert seq.get(0, like) is x and seq.get(1, like) is None
        g = _all_gather(torch.full((2, 3), float(rank)), world, dist.group.WORLD)
        qret.put((rank, seen, g.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_chain_protocol(world):
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    store = _store()
    procs = [ctx.Process(target=_worker, args=(r, world, store, qret)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(collect(procs, qret, world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, seen, g in res:
        first = seen[:11]  # sub-chunk 0 (11 cache points, one skipped)
        if rank == 0:
            assert all(v is None for v in first)
        else:
            # rank r-1's LAST sub-chunk (sub = 1) sent frames of value (r - 1) + 1 + 1 = r + 1
            assert all(v == float(rank + 1) for v in first), (rank, first)
        assert seen[11:] == [float(rank + 1)] * 11  # sub-chunk 1 reads sub-chunk 0's local caches
        assert g == [[[float(i)] * 3] * 2 for i in range(world)]


def _loop_worker(store, n, qret):
    dist.init_process_group("gloo", init_method="file://" + store, rank=0, world_size=1)
    try:
        import collections
        from stableavatar_amd.vae import _LoopbackChain
        like = torch.zeros(3, 2, 2, 4, dtype=torch.bfloat16)
        fifo = collections.deque()
        out = []
        for v in range(n):  # the virtual ranks, decoded in turn on the one rank
            x = torch.full_like(like, float(v + 1))
            st = _LoopbackChain(dist.group.WORLD, v, n, fifo)
            seen = []
            for sub in range(2):
                st.begin(sub == 0, sub == 1)
                for k in range(12):
                    if k == 5:
                        st.skip(k, like)
                        continue
                    p = st.get(k, like)
                    seen.append(None if p is None else float(p.float().mean()))
                    st.put(k, (x + sub)[-2:].clone())
            st.finish()
            out.append((v, seen))
        qret.put((out, len(fifo)))
    finally:
        dist.destroy_process_group()


def test_chain_protocol_loopback():
    """3 virtual ranks on ONE rank (AutoencoderKLWan.enable_multi_gpus_inference(loopback_ranks=3)): the same
    hand-off sequence as 3 real ranks, every cache passed through a transfer to the rank itself"""
    ctx = mp.get_context("spawn")
    qret = ctx.Queue()
    p = ctx.Process(target=_loop_worker, args=(_store(), 3, qret))
    p.start()
    (res, left), = collect([p], qret, 1)
    p.join(timeout=60)
    assert p.exitcode == 0 and left == 0
    for v, seen in res:
        first = seen[:11]
        assert all(x is None for x in first) if v == 0 else all(x == float(v + 1) for x in first), (v, first)
        assert seen[11:] == [float(v + 1)] * 11
