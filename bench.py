"""StableAvatar hot-path benchmark on MI355X: denoised frames/s for one 512x512x81-frame
audio-driven clip (BASELINE.json configs[1]): 50 sliding-window x 3-way-CFG DiT denoising steps of
the Wan-2.1 1.3B StableAvatar model + the 3-D causal VAE decode to 81 frames.

One bench "step" = one whole clip (50 DiT forwards at B=3, L=21504 + 50 fused CFG/Euler steps +
VAE decode), inputs resident in HBM.  `python bench.py --gpus N --steps K --warmup W`.

N = 1: one clip on one GPU.  N > 1 (one process per GPU; torch.distributed.run sets RANK/WORLD_SIZE,
and without it this script starts that launcher itself before touching the GPU):
  --mode sp (default)   ONE clip, Ulysses sequence parallel over all ranks on RCCL (BASELINE config 3,
                        strong scaling); the JSON also carries `replicas` = one clip per rank timed in
                        the same processes (--replica-steps, 0 to skip)
  --mode replicas       one clip per rank, no data-path collective (weak scaling)
  --mode window-dp      one long clip (--video-frames) with its sliding windows spread over the ranks
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "denoised frames/sec, Wan-1.3B 512²×81f audio-driven, 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15  # dense bf16 MFMA, MI355X_MICROARCH.md
ATTN_KERNEL_NAME = "attn_fwd_v6_kernel"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--frames", type=int, default=81)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--sample-steps", type=int, default=50)
    p.add_argument("--overlap", type=int, default=15)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-cpu-config1", action="store_true",
                   help="skip the config-1 run of the CPU oracle inside cpu_baseline")
    p.add_argument("--cpu-config1-steps", type=int, default=1,
                   help="sampling steps of the config-1 CPU oracle run actually executed (1..5; the rest of the 5 "
                        "are extrapolated from the measured per-step time; 5 = fully end to end)")
    p.add_argument("--no-encode", action="store_true", help="skip the (untimed) VAE encode measurement")
    p.add_argument("--no-dit14", action="store_true",
                   help="skip the (untimed) per-block measurement of the 14B model at config 4's 720p geometry")
    p.add_argument("--mode", choices=("sp", "replicas", "window-dp"), default=None,
                   help="N>1 layout (default sp); ignored at N=1")
    p.add_argument("--sp", action="store_true", help="alias of --mode sp")
    p.add_argument("--window-dp", action="store_true", help="alias of --mode window-dp")
    p.add_argument("--replica-steps", type=int, default=1,
                   help="sp mode: clips per rank of the extra replicas measurement (0 = skip)")
    p.add_argument("--video-frames", type=int, default=None,
                   help="length of the generated video (default: --frames, i.e. one window); e.g. 165 = the "
                        "examples/case-1 shape (42 latent frames, 5 windows per step at overlap 15)")
    a = p.parse_args(argv)
    if a.mode is None:
        a.mode = "window-dp" if a.window_dp else "sp"
    return a


def launch_workers(args, argv) -> int:
    """--gpus N > 1 without a launcher: start torch.distributed.run as a CHILD process (this process
    has not touched the GPU and stays the parent) and return its exit code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------------------------ CPU baseline

def cpu_cores() -> int:
    """Cores this process may use: the affinity mask, capped by a cgroup-v2 CPU quota and by the
    OMP_NUM_THREADS share the host sets (the GPU box's per-GPU CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(size, frames, sample_steps, n_fwd, out_frames, config1=True, config1_steps=1):
    """The CPU oracle (oracle/, fp32 restatement of the reference) on this host's cores:
    (a) config 2, bounded sample: one of the 30 DiT blocks at the full shape + the VAE decoder on one
        latent frame, extrapolated to the clip (n_fwd forwards x 30 blocks + out_frames frames);
    (b) config 1 (BASELINE.json configs[0]): the restated pipeline with the full 30-layer DiT at 256x256
        clip 17 (2 windows per step) + the full VAE decode of the 21-frame video; config1_steps of its 5
        sampling steps run (5 = end to end), the others extrapolated at the measured per-step time."""
    from oracle import dit as odit
    from oracle import vae as ovae
    from stableavatar_amd import synthetic
    threads = cpu_cores()
    torch.set_num_threads(threads)
    h = size // 8
    T = (frames - 1) // 4 + 1
    L = T * (h // 2) ** 2
    cfg = dict(odit.CONFIG_1_3B, num_layers=1)
    P = synthetic.fill_state_dict({k: v for k, v in odit.param_shapes(cfg).items() if k.startswith("blocks.0.")}, 0)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, L, 1536, generator=g)
    e0 = torch.randn(3, 6, 1536, generator=g) * 0.1
    ctx = torch.randn(3, 769, 1536, generator=g)
    voc = torch.randn(3, T, 17, 1536, generator=g)
    grid = [(T, h // 2, h // 2)] * 3
    with torch.no_grad():
        t0 = time.time()
        odit.block(P, "blocks.0", x, e0, grid, odit.model_freqs(128), ctx, voc, T, 12)
        t_block = time.time() - t0
        Pv = synthetic.fill_state_dict(ovae.param_shapes(), 1)
        z = torch.randn(1, 16, 1, h, h, generator=g)
        t0 = time.time()
        ovae.decode(Pv, z)
        t_vae_frame = time.time() - t0
    del P, x, ctx, voc
    t_clip = n_fwd * 30 * t_block + out_frames * t_vae_frame
    out = {"value": round(out_frames / t_clip, 6), "unit": "frames/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
           "sample": f"oracle fp32 (oracle/dit.py, oracle/vae.py) on {threads} threads: 1 of 30 DiT blocks at "
                     f"B=3,L={L} ({t_block:.1f}s) + VAE decode of 1 latent frame at {size}x{size} "
                     f"({t_vae_frame:.1f}s), extrapolated to {n_fwd} forwards x 30 blocks + {out_frames} frames "
                     f"= {t_clip:.0f}s per clip"}
    if config1:
        out["config_1"] = cpu_config1(Pv, config1_steps)
    return out


def cpu_config1(Pv, run_steps=5):
    """BASELINE config 1 on the CPU oracle: the full 30-layer DiT (synthetic weights) through the
    restated sliding-window loop (oracle/pipeline.py) + the full VAE decode; encoders excluded (once
    per call).  run_steps of the 5 sampling steps are executed (the denoise loop takes
    the first run_steps sigmas of the 5-step schedule); the remaining steps cost the measured per-step
    time."""
    from oracle import dit as odit
    from oracle import pipeline as opipe
    from oracle import vae as ovae
    from stableavatar_amd import synthetic
    cfg = dict(odit.CONFIG_1_3B)
    Pd = synthetic.fill_state_dict(odit.param_shapes(cfg), 41)
    size, clip_length, steps, overlap, audio_frames = 256, 17, 5, 2, 24
    run_steps = max(1, min(steps, run_steps))
    T = (audio_frames - 1) // 4 + 1
    lat0 = synthetic.seeded_normal((1, 16, T, size // 8, size // 8), 301)
    y = synthetic.seeded_normal((3, 20, (clip_length - 1) // 4 + 1, size // 8, size // 8), 302)
    ctx = [synthetic.seeded_normal((24, 4096), 303)] * 2 + [synthetic.seeded_normal((31, 4096), 304)]
    clip = synthetic.seeded_normal((1, 257, 1280), 305).expand(3, -1, -1).contiguous()
    audio = synthetic.seeded_normal((audio_frames * 640,), 306, 0.1)
    n_fwd = [0]

    def dit(x, t, context, seq_len, yy, clip_fea, vocal, n):
        n_fwd[0] += 1
        return odit.forward(Pd, cfg, x, t, context, seq_len, clip_fea, yy, vocal, n)

    enc = lambda s: synthetic.fake_wav2vec_features(torch.as_tensor(s)[None])  # noqa: E731
    with torch.no_grad():
        t0 = time.time()
        lat = opipe.denoise(dit, lat0, y, ctx, clip, audio, enc, num_inference_steps=steps, clip_length=clip_length,
                            num_frames=clip_length, height=size, width=size, overlap=overlap, text_guide_scale=3.0,
                            audio_guide_scale=5.0, max_steps=run_steps)
        t_denoise = time.time() - t0
        t1 = time.time()
        video = ovae.decode(Pv, lat)
        t_decode = time.time() - t1
    n_out = video.shape[2]
    total = t_denoise * steps / run_steps + t_decode
    return {"value": round(n_out / total, 5), "unit": "frames/s", "seconds": round(total, 1),
            "denoise_s_measured": round(t_denoise, 1), "decode_s": round(t_decode, 1), "steps_run": run_steps,
            "dit_forwards_run": n_fwd[0], "frames": n_out,
            "workload": f"Wan-1.3B 30 layers {size}x{size}, clip {clip_length}, {audio_frames} frames of audio "
                        f"(T_lat {T}, 2 windows/step), {steps} steps, fp32, + VAE decode"
                        + ("" if run_steps == steps else f"; {run_steps} of {steps} steps run, the rest extrapolated")}


# ------------------------------------------------------------------------------------------------ GPU workload

def build(dev, seed=0):
    from stableavatar_amd import synthetic
    from stableavatar_amd.transformer import WanTransformer3DFantasyModel, param_shapes
    from stableavatar_amd.vae import AutoencoderKLWan
    from stableavatar_amd.vae import encoder_param_shapes, param_shapes as vae_shapes
    cfg = dict(model_type="i2v", dim=1536, ffn_dim=8960, freq_dim=256, text_dim=4096, in_dim=36, out_dim=16,
               num_heads=12, num_layers=30, text_len=512)
    dit = WanTransformer3DFantasyModel(**cfg).to(dev)
    dit.load_state_dict(synthetic.fill_state_dict(param_shapes(cfg), seed, backend="torch", device=dev))
    vae = AutoencoderKLWan().to(dev)
    vae.load_state_dict(synthetic.fill_state_dict(dict(vae_shapes(), **encoder_param_shapes()), seed + 1,
                                                  backend="torch", device=dev))
    return dit, vae


def make_inputs(dev, frames, size, seed, video_frames=None):
    T = ((video_frames or frames) - 1) // 4 + 1
    fpb = (frames - 1) // 4 + 1
    h = size // 8
    g = torch.Generator().manual_seed(seed)
    latents = torch.randn(1, 16, T, h, h, generator=g).to(dev).bfloat16()  # CPU noise, injected (App. A.13)
    gd = torch.Generator(device=dev).manual_seed(seed + 1)
    y = torch.randn(3, 20, fpb, h, h, device=dev, generator=gd).bfloat16()
    ctx = [torch.randn(n, 4096, device=dev, generator=gd) for n in (126, 126, 48)]
    ctx[1] = ctx[0]
    clip = torch.randn(1, 257, 1280, device=dev, generator=gd).expand(3, -1, -1).contiguous()
    n_audio = ((frames + 3) * 640 - 400) // 320 + 1  # wav2vec tokens of the window's audio slice
    a = torch.randn(1, n_audio, 768, device=dev, generator=gd)
    return latents, y, ctx, clip, a


class ClipWorkload:
    """One audio-driven clip per step: the denoise loop (pipeline.denoise) + VAE decode."""

    def __init__(self, args, dev, rank, world):
        from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, window_schedule
        from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler
        self.args, self.dev, self.rank, self.world = args, dev, rank, world
        self.dit, self.vae = build(dev, seed=0)
        self.sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
        self.sched.set_timesteps(args.sample_steps, device=dev)
        self.pipe = WanI2VTalkingInferenceLongPipeline(vae=self.vae, transformer=self.dit, scheduler=self.sched)
        self.fpb = (args.frames - 1) // 4 + 1
        self.h = args.size // 8
        self.seq_len = math.ceil(self.h * self.h / 4 * self.fpb)
        self.window_schedule = window_schedule
        self.set_layout("single")

    def set_layout(self, layout):
        """single | sp | replicas | window-dp: model / pipeline parallel state + this rank's inputs."""
        self.layout = layout
        self.dit.disable_multi_gpus_inference()
        self.pipe.disable_window_parallel()
        if layout == "sp":  # Ulysses DiT + the VAE decode split over the ranks
            self.dit.enable_multi_gpus_inference()
            self.pipe._decode_group_sync()
        elif layout == "window-dp":  # windows + the VAE decode split over the ranks
            self.pipe.enable_window_parallel()
        shared = layout in ("sp", "window-dp")  # one clip over all ranks
        a = self.args
        self.latents, self.y, self.ctx, self.clip, au = make_inputs(self.dev, a.frames, a.size,
                                                                    seed=42 + (0 if shared else self.rank),
                                                                    video_frames=a.video_frames)
        self.T = self.latents.shape[2]
        self.wins = self.window_schedule(self.T, self.fpb, a.overlap)
        self.feats = {(s, e): torch.cat([torch.zeros_like(au), au, au]) for (s, e, _) in self.wins}
        self.out_frames = 1 + 4 * (self.T - 1)

    def step(self):
        a = self.args
        lat = self.pipe.denoise(self.latents, self.y, self.ctx, self.clip, self.feats, self.sched.timesteps,
                                self.sched.sigmas, clip_length=a.frames, seq_len=self.seq_len, overlap=a.overlap,
                                text_guide_scale=3.0, audio_guide_scale=5.0)
        return self.vae.decode_clip(lat[0].float(), post=True)

    def check(self, video):
        assert video.shape[1] == self.out_frames and torch.isfinite(video).all()

    def start_events(self):
        self.dit._events = []

    def attention_launch_ms(self):
        """(mean duration of one self-attention launch, the share of the CFG batch one launch covers), from
        HIP events on the launching stream (per-row launches -- the per-row stream loop, per-row SP -- cover
        1/3 of the batch each)"""
        ev, self.dit._events = self.dit._events or [], None
        if not ev:
            return None, 1.0
        tot = sum(e0.elapsed_time(e1) for e0, e1, _ in ev)
        share = sum(f for _, _, f in ev) / len(ev)
        return tot / len(ev), share

    def n_fwd(self):
        return self.args.sample_steps * len(self.wins)


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def barrier(world, dev):
    sync(dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        sync(dev)


def timed(work, steps, warmup, world, dev, events=False):
    """W untimed warmup steps, then EXACTLY K steps between barriers; the max over ranks."""
    with torch.no_grad():
        for _ in range(warmup):
            work.step()
        barrier(world, dev)
        if events:
            work.start_events()
        t0 = time.perf_counter()
        out = None
        for _ in range(steps):
            out = work.step()
        barrier(world, dev)
        dt = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    return dt, out


def vae_encode_ms(vae, frames, size, dev):
    from stableavatar_amd import flops
    ref = torch.zeros(1, 3, frames, size, size, device=dev)
    ref[:, :, 0].uniform_(-1, 1)
    with torch.no_grad():
        vae.encode(ref)
        sync(dev)
        te = time.perf_counter()
        lat_y = vae.encode(ref)[0].mode()
        sync(dev)
        te = time.perf_counter() - te
    assert tuple(lat_y.shape) == (1, 16, (frames - 1) // 4 + 1, size // 8, size // 8)
    ef = flops.vae_encode_flops(frames, size, size)
    return {"ms": round(te * 1e3, 1), "tflop": round(ef / 1e12, 2), "tflops_per_s": round(ef / te / 1e12, 1),
            "note": "AutoencoderKLWan.encode of the reference frame + zeros, once per call; outside the timed "
                    "region and the metric (SURVEY.md §8(d))"}


def attn_traffic(seq_len, layout):
    """HBM bytes per self-attention launch from the committed rocprofv3 PMC passes, when they were
    taken on the kernel this build runs at this shape (else None)."""
    tpath = os.path.join(ROOT, "profiles", "pmc_attn_traffic.json")
    if layout != "single" or seq_len != 21504 or not os.path.exists(tpath):
        return None, None
    with open(tpath) as f:
        tj = json.load(f)
    if not tj.get("kernel", "").startswith(ATTN_KERNEL_NAME):
        return None, None
    return tj["hbm_bytes_per_launch"], f"profiles/pmc_attn_traffic.json ({tj.get('source', 'rocprofv3 --pmc')})"


def run(args, world, rank, dev, work_factory=ClipWorkload):
    """The measurement; returns the JSON dict on rank 0 (None elsewhere)."""
    from stableavatar_amd import flops
    from stableavatar_amd import sp
    layout = "single" if world == 1 else args.mode
    work = work_factory(args, dev, rank, world)
    work.set_layout(layout)
    dt, video = timed(work, args.steps, args.warmup, world, dev, events=True)
    work.check(video)
    attn_ms, attn_share = work.attention_launch_ms()
    seq_len = work.seq_len
    attn_flop = flops.self_attention_flops(B=3, L=seq_len) * attn_share
    parallelism = {"single": "single", "replicas": f"replicas{world}", "window-dp": f"windows{world}"}.get(layout)
    if layout == "sp":
        plan = sp.make_plan(world, rank, 12)
        attn_flop /= world  # this rank's (head group, query part) share
        parallelism = f"ulysses{plan.G}" + (f"x{plan.R}qsplit" if plan.R > 1 else "")
    shared = layout in ("sp", "window-dp")
    frames_total = (1 if shared else world) * work.out_frames * args.steps
    value = frames_total / dt
    n_fwd = work.n_fwd()
    path_flop = n_fwd * flops.dit_forward_flops(B=3, L=seq_len, n_frames=work.fpb) + \
        flops.vae_decode_flops(work.T, work.h, work.h)
    replicas = None
    if layout == "sp" and args.replica_steps > 0:
        work.set_layout("replicas")
        rdt, rvideo = timed(work, args.replica_steps, 0, world, dev)
        work.check(rvideo)
        replicas = {"value": round(world * work.out_frames * args.replica_steps / rdt, 4), "unit": "frames/s",
                    "steps": args.replica_steps, "ms_per_step": round(rdt / args.replica_steps * 1e3, 1),
                    "scaling": "weak", "parallelism": f"replicas{world}",
                    "note": "one independent clip per rank in the same processes (no data-path collective)"}
    enc = None
    if not args.no_encode and rank == 0 and hasattr(work, "vae"):
        enc = vae_encode_ms(work.vae, args.frames, args.size, dev)
    dit14 = None
    if world == 1 and not args.no_dit14 and hasattr(work, "dit"):
        from stableavatar_amd.kbench import bench_dit14
        dit14 = dict(bench_dit14(), note="BASELINE config 4's model (Wan-14B StableAvatar widths: dim 5120, 40 heads, "
                                         "ffn 13824) at 720x1280, 81 frames (L = 75 600, B = 3) on one GPU: forwards "
                                         "with 1 and 2 blocks, one block's time from their difference, the 40-block "
                                         "forward projected; outside the timed region and the metric")
    if rank != 0:
        return None
    traffic, traffic_src = attn_traffic(seq_len, layout)
    achieved = attn_flop / (attn_ms * 1e-3) if attn_ms else None
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.size, args.frames, args.sample_steps, n_fwd, work.out_frames,
                           config1=not args.no_cpu_config1, config1_steps=args.cpu_config1_steps)
    n_win = len(work.wins)
    out = {"metric": METRIC, "value": round(value, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 1), "higher_is_better": True,
           "scaling": "strong" if shared else "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random-init weights by name-keyed seed; synthetic text/CLIP/wav2vec features "
                   "and conditioning latents; CPU-generated initial noise)",
           "config": {"workload": f"Wan-1.3B StableAvatar {args.size}x{args.size}x{work.out_frames}f"
                                  + (f" ({n_win} windows of {args.frames}f, overlap {args.overlap})"
                                     if work.out_frames != args.frames else "")
                                  + f", {args.sample_steps} steps, CFG x3, single audio clip, VAE decode",
                      "global_batch": 3 * (1 if shared else world), "seq_len": seq_len,
                      "dit_forwards_per_clip": n_fwd, "parallelism": parallelism},
           "roofline": {"bound": "mfma", "kernel": f"{ATTN_KERNEL_NAME} (self-attention, flash, D=128)",
                        "achieved": round(achieved / 1e12, 1) if achieved else None, "peak": PEAK_BF16 / 1e12,
                        "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16, 4) if achieved else None,
                        "traffic": round(traffic * attn_share) if traffic else None, "traffic_source": traffic_src,
                        "algorithmic_bytes": round(4 * 3 * seq_len * 1536 * 2 * attn_share),
                        "launch_share_of_cfg_batch": round(attn_share, 4),
                        "launch_ms": round(attn_ms, 3) if attn_ms else None, "flop_per_launch": attn_flop},
           "path_mfma_frac": round(path_flop * args.steps / dt / PEAK_BF16 / (world if shared else 1), 4),
           "cpu_baseline": cpu, "vae_encode": enc, "config_4_dit14": dit14}
    if replicas is not None:
        out["replicas"] = replicas
    return out


def main(argv=None, work_factory=ClipWorkload, device=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.sp:
        args.mode = "sp"
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_workers(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if device is None:
        dev = torch.device(f"cuda:{local}")
        torch.cuda.set_device(dev)
    else:
        dev = torch.device(device)
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            if dev.type == "cuda":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo")
    out = run(args, world, rank, dev, work_factory)
    if out is not None:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
