"""Probe: can two RCCL ranks share the box's one GPU?  (If yes, the multi-rank RCCL paths -- Ulysses all-to-all,
the VAE cache hand-off P2P -- can be tested on a 1-GPU box.)  Prints one line per rank and exits 0 either way."""
import os
import sys

import torch
import torch.multiprocessing as mp


def _w(rank, store):
    import torch.distributed as dist
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", init_method="file://" + store, rank=rank, world_size=2,
                                device_id=torch.device("cuda:0"))
        x = torch.full((4,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce ok {x.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        print(f"rank {rank}: failed {type(e).__name__}: {str(e)[:300]}", flush=True)


if __name__ == "__main__":
    import tempfile
    store = os.path.join(tempfile.mkdtemp(prefix="sa_rccl_probe_"), "store")  # file:// rendezvous: nothing to bind
    mp.start_processes(_w, args=(store,), nprocs=2, join=True, start_method="spawn")
    sys.exit(0)
