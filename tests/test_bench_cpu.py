"""bench.py's multi-process orchestration on CPU (gloo, world 2), with a stand-in workload in place of
the HIP clip: rank/world handling, the barrier-bracketed timing with the max over ranks, the SP default
for N > 1 with the extra `replicas` key, the per-row attention-span accounting and the JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _Ev:
    """stands in for a torch.cuda.Event pair: elapsed_time in ms"""

    def __init__(self, ms):
        self.ms = ms

    def elapsed_time(self, other):
        return other.ms - self.ms


class FakeClip:
    """CPU stand-in with ClipWorkload's interface: a small all-reduce per step in SP layout (the data
    path collective), none in replicas layout; attention spans as the per-row SP path records them
    (three rows of 1/3 each, 2 ms apiece -> 6 ms per whole launch)."""

    def __init__(self, args, dev, rank, world):
        self.args, self.rank, self.world = args, rank, world
        self.fpb = (args.frames - 1) // 4 + 1
        self.h = args.size // 8
        self.seq_len = self.fpb * (self.h // 2) ** 2
        self.T = self.fpb
        self.wins = [(0, self.fpb, self.fpb)]
        self.out_frames = args.frames
        self.layout = None
        self.events = None
        self.steps_run = 0

    def set_layout(self, layout):
        self.layout = layout

    def step(self):
        x = torch.full((4,), float(self.rank + 1))
        if self.layout == "sp":
            dist.all_reduce(x)
        if self.events is not None:
            for _ in range(3):
                self.events.append((_Ev(0.0), _Ev(2.0), 1 / 3))
        self.steps_run += 1
        return torch.zeros(3, self.out_frames, 8, 8)

    def check(self, video):
        assert video.shape[1] == self.out_frames

    def start_events(self):
        self.events = []

    def attention_launch_ms(self):  # per-launch mean and the CFG-batch share of one launch, as ClipWorkload
        ev, self.events = self.events, None
        return sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev), sum(f for _, _, f in ev) / len(ev)

    def n_fwd(self):
        return self.args.sample_steps * len(self.wins)


def _worker(rank, world, store, argv, path):
    # a file:// rendezvous: nothing to bind, so no port is picked and released (a race with other listeners)
    os.environ.update(SA_DIST_INIT_METHOD="file://" + store, RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    out = open(path + f".{rank}", "w")
    sys.stdout = out
    try:
        bench.main(argv, work_factory=FakeClip, device="cpu")
    finally:
        out.close()


def _run(world, argv, tmp_path):
    path = str(tmp_path / "bench")
    mp.start_processes(_worker, args=(world, str(tmp_path / "store"), argv, path), nprocs=world, join=True,
                       start_method="spawn")
    lines = [open(path + f".{r}").read().strip() for r in range(world)]
    assert all(not ln for ln in lines[1:]), "only rank 0 prints"
    return json.loads(lines[0])


def test_bench_sp_default_world2(tmp_path):
    j = _run(2, ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-encode"], tmp_path)
    assert j["n_gpus"] == 2 and j["steps"] == 2 and j["warmup"] == 1
    assert j["scaling"] == "strong" and j["config"]["parallelism"] == "ulysses2"
    assert j["config"]["global_batch"] == 3
    assert j["value"] > 0 and j["ms_per_step"] > 0
    # one clip of 81 frames per step, over all ranks; ms_per_step is rounded to 0.1 ms, so the stand-in's
    # sub-millisecond steps are bracketed by the rounding interval
    ms = j["ms_per_step"]
    assert j["value"] * max(ms - 0.05, 0) / 1e3 * 0.99 <= 81 <= j["value"] * (ms + 0.05) / 1e3 * 1.01
    # per-row launches (1/3 of the batch, 2 ms each): the roofline is quoted per launch, flop = this
    # rank's half of one CFG row (the achieved rate is the same as per whole-batch launch)
    assert j["roofline"]["launch_ms"] == 2.0 and j["roofline"]["launch_share_of_cfg_batch"] == round(1 / 3, 4)
    assert abs(j["roofline"]["flop_per_launch"] - 4.0 * 3 * 12 * 21504 ** 2 * 128 / 2 / 3) < 1e3
    assert j["replicas"]["scaling"] == "weak" and j["replicas"]["parallelism"] == "replicas2"
    for k in ("metric", "unit", "higher_is_better", "vs_baseline", "dtype", "data", "config", "roofline",
              "cpu_baseline"):
        assert k in j


def test_bench_replicas_mode_world2(tmp_path):
    j = _run(2, ["--gpus", "2", "--steps", "1", "--warmup", "0", "--mode", "replicas", "--no-cpu-baseline",
                 "--no-encode"], tmp_path)
    assert j["scaling"] == "weak" and j["config"]["parallelism"] == "replicas2"
    assert j["config"]["global_batch"] == 6 and "replicas" not in j


def test_bench_parse_defaults():
    a = bench.parse([])
    assert a.gpus == 1 and a.mode == "sp" and a.steps >= 1
    assert bench.parse(["--window-dp"]).mode == "window-dp"
    assert bench.cpu_cores() >= 1 and isinstance(bench.cpu_model(), str)


def test_bench_cpu_baseline_child_world1(capsys):
    """N = 1: the CPU baseline runs in a child process started before the GPU work, is collected after the
    warmup (never inside the timed region) and lands in the JSON with the thread count it used; the
    JSON records the time budget."""
    rc = bench.main(["--steps", "1", "--warmup", "1", "--size", "64", "--frames", "17", "--no-cpu-config1",
                     "--no-encode"], work_factory=FakeClip, device="cpu")
    assert rc == 0
    j = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    c = j["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1
    assert "1 of 30 DiT blocks at B=3,L=80" in c["sample"]
    assert c["config_1"]["value"] is None and c["config_1"]["skipped"] == "not run"
    assert j["time_budget"]["budget_s"] == 540.0 and j["time_budget"]["elapsed_s"] > 0


def test_bench_cpu_baseline_deadline(tmp_path):
    """A child still running past the deadline is ended once its mandatory config-2 leg is in."""
    import subprocess
    import time as _t
    cb = bench.CpuBaseline.__new__(bench.CpuBaseline)
    cb.path, cb.log, cb.killed = str(tmp_path / "c.jsonl"), str(tmp_path / "c.log"), False
    with open(cb.path, "w") as f:
        f.write(json.dumps({"leg": "config2", "t_block": 1.0, "t_vae_frame": 0.5, "L": 80, "threads": 3}) + "\n")
        f.write(json.dumps({"leg": "config1_step", "i": 0, "s": 2.0, "dit_forwards": 2}) + "\n")
    cb.proc = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    t0 = _t.time()
    cb.wait(deadline=_t.time(), required_by=_t.time() + 30)
    assert cb.killed and _t.time() - t0 < 15
    r = cb.result(n_fwd=50, out_frames=81, size=512)
    assert r["cores"] == 3 and abs(r["value"] - 81 / (50 * 30 * 1.0 + 81 * 0.5)) < 1e-5
    assert r["config_1"]["skipped"] == "not finished within the time budget" and r["config_1"]["steps_done"] == 1
    # with the (first-timed) config-1 decode in, k measured steps give a partial, extrapolated config-1 number
    with open(cb.path, "a") as f:
        f.write(json.dumps({"leg": "config1_decode", "s": 3.0, "frames": 21}) + "\n")
        f.write(json.dumps({"leg": "config1_step", "i": 1, "s": 4.2, "dit_forwards": 4}) + "\n")
    c1 = cb.result(n_fwd=50, out_frames=81, size=512)["config_1"]
    assert c1["steps_run"] == 2 and abs(c1["value"] - 21 / (5 * 2.1 + 3.0)) < 1e-4 and "2 of 5" in c1["partial"]
    cb.cleanup()
