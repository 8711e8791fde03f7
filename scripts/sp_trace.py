"""One RCCL rank with the sequence-parallel path on (argv[1] == "sp"), on with loopback transfers ("loop": the rank's
own chunk sent to itself through batch_isend_irecv, so the RCCL send / receive kernels run) or off ("single"): two
DiT forwards of the small golden model, for a rocprofv3 kernel trace of each mode -- the SP run must add no copy
kernels (the exchange is pack / row-mapped attention / column-panel O-projection only).
usage: rocprofv3 --kernel-trace --stats -d <dir> -o run -- python scripts/sp_trace.py sp|single|loop"""
import os
import sys
import tempfile

import torch
import torch.distributed as dist

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from test_gpu_dit import make_model, run  # noqa: E402
from golden_cases import DIT_SMALL, dit_inputs  # noqa: E402

torch.cuda.set_device(0)
store = os.path.join(tempfile.mkdtemp(prefix="sa_sp_trace_"), "store")  # file:// rendezvous: nothing to bind
dist.init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1,
                        device_id=torch.device("cuda:0"))
try:
    m = make_model(DIT_SMALL)
    if sys.argv[1] in ("sp", "loop"):
        m.enable_multi_gpus_inference(loopback=sys.argv[1] == "loop")
    inp = dit_inputs(DIT_SMALL, "full")
    outs = [run(m, inp) for _ in range(2)]
    print(sys.argv[1], "sp_enabled", m._sp_enabled, "loopback", getattr(m, "_sp_loopback", False), "checksum",
          outs[1].double().abs().sum().item())
finally:
    dist.destroy_process_group()
