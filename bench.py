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

import time

# the time budget counts from process start: taken before `import torch`, which can take 1-2 minutes on a fresh
# box while the image pages in (the driver's clock runs through it)
T0 = time.time()

import argparse  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "denoised frames/sec, Wan-1.3B 512²×81f audio-driven, 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15  # dense bf16 MFMA, MI355X_MICROARCH.md
ATTN_KERNEL_NAME = "attn_fwd_v6t_kernel"  # the V^T form (round 5); profiles/pmc_attn_traffic.json must name it


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
    p.add_argument("--cpu-config1-steps", type=int, default=5,
                   help="sampling steps of the config-1 CPU oracle run actually executed (1..5; the rest of the 5 "
                        "are extrapolated from the measured per-step time; 5 = fully end to end)")
    p.add_argument("--no-encode", action="store_true", help="skip the (untimed) VAE encode measurement")
    p.add_argument("--dit14", action="store_true",
                   help="also time (untimed extra) one block of the 14B model at config 4's 720p geometry")
    p.add_argument("--no-dit14", action="store_true", help=argparse.SUPPRESS)  # the default since round 3
    p.add_argument("--time-budget", type=float, default=540.0,
                   help="seconds from process start within which the untimed extras must end (the driver kills "
                        "the run at 600 s): the CPU baseline's config-1 leg, the VAE encode and --dit14 are "
                        "skipped, and say so in the JSON, when they would not fit")
    p.add_argument("--cpu-child", type=str, default=None, help=argparse.SUPPRESS)  # internal: CPU baseline process
    p.add_argument("--vae-parallel", dest="vae_parallel", action="store_true", default=True,
                   help="N>1 sp / window-dp: split the VAE decode over the ranks (the default since round 4: a "
                        "wavefront of causal-cache hand-offs, bit-identical to one GPU)")
    p.add_argument("--no-vae-parallel", dest="vae_parallel", action="store_false",
                   help="every rank decodes the whole clip, as the reference does (wan_inference_long_pipeline.py"
                        ":793-796)")
    p.add_argument("--replica-warmup", type=int, default=1,
                   help="sp mode: untimed replicas clips per rank after the layout switch, before the timed ones")
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
    has not touched the GPU and stays the parent) and return its exit code.  --standalone: the launcher's
    c10d rendezvous binds its TCPStore on port 0 itself and the workers share that store (MASTER_PORT = the
    store's port), so no port is picked free and released before use (a race with any other listener)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", os.path.abspath(__file__), *argv]
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


def _emit(path, rec):
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")


def cpu_child(args):
    """`bench.py --cpu-child PATH`: the CPU baseline in its own process, started by the N = 1 bench before it
    touches the GPU so that it runs during the (untimed) warmup clips and has ended before the timed region
    starts.  No GPU use here.  Each finished leg is appended to PATH as one JSON line:
    (a) config 2, bounded sample: one of the 30 DiT blocks at the full shape + the VAE decoder on one latent
        frame (the parent extrapolates them to the clip: forwards x 30 blocks + output frames);
    (b) config 1 (BASELINE.json configs[0]): the full VAE decode of the 21-frame video's latent shape (timed
        first: one line), then the restated pipeline with the full 30-layer DiT at 256x256, clip 17 (2 windows
        per step), one line per sampling step and one at the end (a time budget that ends the child early
        leaves k measured steps + the decode, reported as a partial, extrapolated config-1 number)."""
    from oracle import dit as odit
    from oracle import pipeline as opipe
    from oracle import vae as ovae
    from stableavatar_amd import synthetic
    path = args.cpu_child
    threads = max(1, cpu_cores() - 1)  # one core stays with the GPU process's launch thread
    torch.set_num_threads(threads)
    size, frames = args.size, args.frames
    h = size // 8
    T = (frames - 1) // 4 + 1
    L = T * (h // 2) ** 2
    cfg = dict(odit.CONFIG_1_3B, num_layers=1)
    # timing-only weights (synthetic.timing_state_dict: the rule's scales, tiled from one seeded block), so that the
    # 1.7 G-parameter fills do not eat into the time the child has before the timed region starts
    P = synthetic.timing_state_dict({k: v for k, v in odit.param_shapes(cfg).items() if k.startswith("blocks.0.")}, 0)
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
        Pv = synthetic.timing_state_dict(ovae.param_shapes(), 1)
        z = torch.randn(1, 16, 1, h, h, generator=g)
        t0 = time.time()
        ovae.decode(Pv, z)
        t_vae_frame = time.time() - t0
    del P, x, ctx, voc
    _emit(path, {"leg": "config2", "t_block": t_block, "t_vae_frame": t_vae_frame, "L": L, "threads": threads})
    if args.no_cpu_config1:
        return 0
    # config 1: the 30-layer DiT (synthetic weights) through the restated sliding-window loop + the full decode;
    # encoders excluded (once per call)
    cfg = dict(odit.CONFIG_1_3B)
    Pd = synthetic.timing_state_dict(odit.param_shapes(cfg), 41)
    size1, clip_length, steps, overlap, audio_frames = 256, 17, 5, 2, 24
    run_steps = max(1, min(steps, args.cpu_config1_steps))
    T1 = (audio_frames - 1) // 4 + 1
    lat0 = synthetic.seeded_normal((1, 16, T1, size1 // 8, size1 // 8), 301)
    y = synthetic.seeded_normal((3, 20, (clip_length - 1) // 4 + 1, size1 // 8, size1 // 8), 302)
    ctx1 = [synthetic.seeded_normal((24, 4096), 303)] * 2 + [synthetic.seeded_normal((31, 4096), 304)]
    clip = synthetic.seeded_normal((1, 257, 1280), 305).expand(3, -1, -1).contiguous()
    audio = synthetic.seeded_normal((audio_frames * 640,), 306, 0.1)
    n_fwd = [0]

    def dit(xx, t, context, seq_len, yy, clip_fea, vocal, n):
        n_fwd[0] += 1
        return odit.forward(Pd, cfg, xx, t, context, seq_len, clip_fea, yy, vocal, n)

    enc = lambda s: synthetic.fake_wav2vec_features(torch.as_tensor(s)[None])  # noqa: E731
    # the decode of the clip's latent shape is timed first (a conv stack: its cost does not depend on the
    # latent values), so that a time budget ending the denoise loop early still leaves a measured decode and
    # k measured sampling steps to report (CpuBaseline.result)
    with torch.no_grad():
        t1 = time.time()
        video = ovae.decode(Pv, torch.zeros_like(lat0))
        t_decode = time.time() - t1
    n_out = video.shape[2]
    _emit(path, {"leg": "config1_decode", "s": t_decode, "frames": n_out})
    t0 = time.time()
    step_cb = lambda i: _emit(path, {"leg": "config1_step", "i": i, "s": time.time() - t0,  # noqa: E731
                                     "dit_forwards": n_fwd[0]})
    with torch.no_grad():
        opipe.denoise(dit, lat0, y, ctx1, clip, audio, enc, num_inference_steps=steps, clip_length=clip_length,
                      num_frames=clip_length, height=size1, width=size1, overlap=overlap, text_guide_scale=3.0,
                      audio_guide_scale=5.0, max_steps=run_steps, step_callback=step_cb)
        t_denoise = time.time() - t0
    total = t_denoise * steps / run_steps + t_decode
    _emit(path, {"leg": "config1", "value": round(n_out / total, 5), "unit": "frames/s", "seconds": round(total, 1),
                 "denoise_s_measured": round(t_denoise, 1), "decode_s": round(t_decode, 1), "steps_run": run_steps,
                 "dit_forwards_run": n_fwd[0], "frames": n_out, "threads": threads,
                 "workload": f"Wan-1.3B 30 layers {size1}x{size1}, clip {clip_length}, {audio_frames} frames of audio "
                             f"(T_lat {T1}, 2 windows/step), {steps} steps, fp32, + VAE decode (timed first on the "
                             f"latent shape)"
                             + ("" if run_steps == steps else
                                f"; {run_steps} of {steps} steps run, the rest extrapolated")})
    return 0


class CpuBaseline:
    """The parent's handle on the CPU-baseline child process (see cpu_child)."""

    def __init__(self, args):
        import tempfile
        fd, self.path = tempfile.mkstemp(prefix="sa_cpu_baseline_", suffix=".jsonl")
        os.close(fd)
        self.log = self.path[:-6] + ".log"
        argv = [sys.executable, os.path.abspath(__file__), "--cpu-child", self.path, "--size", str(args.size),
                "--frames", str(args.frames), "--cpu-config1-steps", str(args.cpu_config1_steps)]
        if args.no_cpu_config1:
            argv.append("--no-cpu-config1")
        self.t_start = time.time()
        with open(self.log, "w") as lf:
            self.proc = subprocess.Popen(argv, stdout=lf, stderr=subprocess.STDOUT)
        self.killed = False

    def records(self):
        try:
            with open(self.path) as f:
                return [json.loads(ln) for ln in f if ln.strip()]
        except (OSError, ValueError):
            return []

    def _has(self, leg):
        return any(r["leg"] == leg for r in self.records())

    def wait(self, deadline, required_by):
        """wait for the child to end; past `deadline` (time.time()) end it, but never before the config-2 leg
        is in (bounded by `required_by`)"""
        last = 0.0
        while self.proc.poll() is None:
            now = time.time()
            if now - last > 30:
                legs = [r["leg"] for r in self.records()]
                progress(f"waiting for the CPU baseline child ({len(legs)} records: {legs[-1] if legs else '-'})")
                last = now
            if now > deadline and (self._has("config2") or now > required_by):
                self.proc.terminate()
                try:
                    self.proc.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    self.proc.kill()
                    self.proc.wait()
                self.killed = True
                break
            time.sleep(0.5)
        return self.proc.returncode

    def result(self, n_fwd, out_frames, size):
        recs = self.records()
        c2 = next((r for r in recs if r["leg"] == "config2"), None)
        if c2 is None:
            tail = ""
            try:
                with open(self.log) as f:
                    tail = f.read()[-400:]
            except OSError:
                pass
            return {"value": None, "error": f"CPU baseline child ended without a result (rc {self.proc.returncode})",
                    "log_tail": tail}
        t_clip = n_fwd * 30 * c2["t_block"] + out_frames * c2["t_vae_frame"]
        th = c2["threads"]
        out = {"value": round(out_frames / t_clip, 6), "unit": "frames/s", "cores": th, "kind": "port",
               "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
               "sample": f"oracle fp32 (oracle/dit.py, oracle/vae.py) on {th} threads (one core of this process's "
                         f"share left to the GPU launch thread; run during the untimed warmup clips, so it shares the "
                         f"host with the GPU process's launch thread, and ended before the timed region): 1 of 30 DiT blocks at B=3,L={c2['L']} ({c2['t_block']:.1f}s) + VAE "
                         f"decode of 1 latent frame at {size}x{size} ({c2['t_vae_frame']:.1f}s), extrapolated to "
                         f"{n_fwd} forwards x 30 blocks + {out_frames} frames = {t_clip:.0f}s per clip"}
        c1 = next((r for r in recs if r["leg"] == "config1"), None)
        if c1 is not None:
            c1 = {k: v for k, v in c1.items() if k != "leg"}
        else:
            steps = [r for r in recs if r["leg"] == "config1_step"]
            dec = next((r for r in recs if r["leg"] == "config1_decode"), None)
            step_s = [round(b["s"] - a, 1) for a, b in zip([0.0] + [s["s"] for s in steps], steps)]
            why = "not finished within the time budget" if self.killed else "not run" if not steps else \
                "child ended early"
            if dec is not None and steps:
                # k of the 5 sampling steps measured (each 2 windows = 2 full DiT forwards) + the measured
                # decode: the remaining steps extrapolated at the measured mean step time
                t_step = steps[-1]["s"] / len(steps)
                total = 5 * t_step + dec["s"]
                c1 = {"value": round(dec["frames"] / total, 5), "unit": "frames/s", "seconds": round(total, 1),
                      "steps_run": len(steps), "step_s": step_s, "decode_s": round(dec["s"], 1),
                      "frames": dec["frames"], "threads": c2["threads"],
                      "partial": f"{len(steps)} of 5 sampling steps measured ({why}); the rest extrapolated at the "
                                 f"measured mean step time"}
            else:
                c1 = {"value": None, "skipped": why, "steps_done": len(steps), "step_s": step_s}
        out["config_1"] = c1
        return out

    def cleanup(self):
        if self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()
        for p in (self.path, self.log):
            try:
                os.remove(p)
            except OSError:
                pass


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
    # conditioning as the pipeline builds it (wan_inference_long_pipeline.py:693-700): the first-frame mask + the VAE
    # latents of the reference frame and zeros (synthetic here), tripled for the CFG rows
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline
    ref_lat = torch.randn(1, 16, fpb, h, h, device=dev, generator=gd)
    y = WanI2VTalkingInferenceLongPipeline.mask_latents(ref_lat, frames).bfloat16()
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
        if layout == "sp":  # Ulysses DiT
            self.dit.enable_multi_gpus_inference()
        elif layout == "window-dp":  # the windows of each step over the ranks
            self.pipe.enable_window_parallel()
        # --vae-parallel: the decode split over the ranks of a shared clip (else every rank decodes it whole)
        self.pipe.enable_vae_parallel(getattr(self.args, "vae_parallel", False) and layout in ("sp", "window-dp"))
        self.pipe._decode_group_sync()
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

    def _forward_once(self):
        s, e, _ = self.wins[0]
        tt = torch.as_tensor(self.sched.timesteps[0], dtype=torch.float32, device=self.dev).reshape(1)
        return self.dit.forward_window(self.latents, s, True, 3, tt, self.ctx, self.seq_len, self.clip,
                                       self.y[:, :, :e - s], self.feats[(s, e)], self.args.frames)

    def sp_check(self):
        """The N > 1 sequence-parallel run checks itself: one DiT forward of the clip's first window (B = 3, the
        full sequence) through the Ulysses exchange and through the single-GPU layout on every rank, which must
        agree bit for bit (the SP path reproduces the single-GPU forward); plus the SP output's
        checksum must be the same on every rank (every rank holds the whole noise prediction)."""
        import torch.distributed as dist
        with torch.no_grad():
            o_sp = self._forward_once().clone()
            self.dit.disable_multi_gpus_inference()
            o1 = self._forward_once()
            self.dit.enable_multi_gpus_inference()
            sync(self.dev)
            eq = bool(torch.equal(o_sp, o1))
            rel = ((o_sp.float() - o1.float()).norm() / o1.float().norm()).item()
            ck = o_sp.view(torch.int16).to(torch.float64).sum()
            t = torch.tensor([0.0 if eq else 1.0, rel, ck.item(), -ck.item()], dtype=torch.float64, device=self.dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return {"forward_bit_identical_to_single_gpu": t[0].item() == 0.0, "max_rel_l2_vs_single_gpu": t[1].item(),
                "ranks_agree": t[2].item() == -t[3].item(),
                "note": "one DiT forward of the clip's first window (B=3, L=%d) via the Ulysses exchange vs the "
                        "single-GPU layout, on every rank (max over ranks); ranks_agree: the SP outputs' checksums "
                        "are equal on all ranks" % self.seq_len}

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


def progress(msg):
    """one line on stderr (stdout carries only the JSON line): keeps a long run visibly alive"""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.time() - T0:6.1f}s] {msg}", file=sys.stderr, flush=True)


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def barrier(world, dev):
    sync(dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        sync(dev)


class ClockSampler:
    """The GPU's graphics clock sampled every `period` s on a thread while the timed clips run (amdsmi: the SMU
    metrics table's average gfx clock where the driver exposes it, else the current SCLK).  The device is matched
    to this process's GPU by PCI bus id.  Reports mean / min / max MHz, or the reason it could not read."""

    def __init__(self, dev, period=0.25):
        import threading
        self.period, self.samples, self.field, self.error = period, [], None, None
        self._stop = threading.Event()
        self._thr = None
        self._read = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self._smi = amdsmi
            props = torch.cuda.get_device_properties(dev)
            bus = getattr(props, "pci_bus_id", None)
            handles = amdsmi.amdsmi_get_processor_handles()
            h = None
            for x in handles:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(x)  # "dddd:bb:dd.f"
                if bus is not None and int(bdf.split(":")[1], 16) == int(bus):
                    h = x
            if h is None and len(handles) == 1:
                h = handles[0]
            if h is None:
                raise RuntimeError(f"no amdsmi device with PCI bus {bus} among {len(handles)}")
            self._h = h
            self._read = self._probe()
        except Exception as e:  # noqa: BLE001 -- a missing clock reading never fails the bench
            self.error = f"{type(e).__name__}: {e}"[:200]

    def _probe(self):
        smi, h = self._smi, self._h
        try:
            m = smi.amdsmi_get_gpu_metrics_info(h)
            for key in ("average_gfxclk_frequency", "current_gfxclk"):
                v = m.get(key)
                if isinstance(v, (int, float)) and 0 < v < 10000:
                    self.field = f"gpu_metrics.{key}"
                    return lambda: smi.amdsmi_get_gpu_metrics_info(h)[key]
            v = m.get("current_gfxclks")
            if isinstance(v, (list, tuple)) and any(isinstance(x, (int, float)) and 0 < x < 10000 for x in v):
                self.field = "gpu_metrics.current_gfxclks (mean over XCDs)"

                def rd():
                    xs = [x for x in smi.amdsmi_get_gpu_metrics_info(h)["current_gfxclks"]
                          if isinstance(x, (int, float)) and 0 < x < 10000]
                    return sum(xs) / len(xs)
                return rd
        except Exception:  # noqa: BLE001
            pass
        self.field = "clock_info.GFX.clk"
        return lambda: smi.amdsmi_get_clock_info(h, smi.AmdSmiClkType.GFX)["clk"]

    def _loop(self):
        while not self._stop.wait(self.period):
            try:
                self.samples.append(float(self._read()))
            except Exception as e:  # noqa: BLE001
                self.error = f"{type(e).__name__}: {e}"[:200]
                return

    def start(self):
        if self._read is not None:
            import threading
            self._thr = threading.Thread(target=self._loop, daemon=True)
            self._thr.start()

    def stop(self):
        if self._thr is not None:
            self._stop.set()
            self._thr.join(timeout=5)
        try:
            if self._read is not None:
                self._smi.amdsmi_shut_down()
        except Exception:  # noqa: BLE001
            pass
        s = self.samples
        if not s:
            return {"mean_mhz": None, "error": self.error or "no samples", "source": self.field}
        return {"mean_mhz": round(sum(s) / len(s)), "min_mhz": round(min(s)), "max_mhz": round(max(s)),
                "samples": len(s), "period_s": self.period, "source": f"amdsmi {self.field}"}


def timed(work, steps, warmup, world, dev, events=False, before_timed=None):
    """W untimed warmup steps, then EXACTLY K steps between barriers; the max over ranks.
    before_timed(warmup_seconds) runs after the warmup, before the opening barrier.  events=True: the
    self-attention events (roofline) and the SCLK samples of the timed clips are recorded, and the per-kernel-class
    HIP events (ktimer: one event after every library launch) on the LAST WARMUP clip, so that the timed region
    carries no per-launch event but the self-attention's (work.kernels)."""
    kt = clk = None
    if events:
        from stableavatar_amd.ktimer import KernelTimer
        kt = KernelTimer() if dev.type == "cuda" and os.environ.get("SA_BENCH_KTIMER", "1") != "0" else None
        clk = ClockSampler(dev) if dev.type == "cuda" and int(os.environ.get("RANK", "0")) == 0 else None
    kt_ms = None
    with torch.no_grad():
        tw = time.perf_counter()
        for i in range(warmup):
            ti = time.perf_counter()
            if kt is not None and i == warmup - 1:
                with kt:
                    work.step()
                    sync(dev)
                kt_ms = (time.perf_counter() - ti) * 1e3
            else:
                work.step()
                sync(dev)
            progress(f"warmup {i + 1}/{warmup} {time.perf_counter() - tw:.1f}s")
        tw = time.perf_counter() - tw
        if before_timed is not None:
            before_timed(tw)
        barrier(world, dev)
        if events:
            work.start_events()
            if clk is not None:
                clk.start()
        t0 = time.perf_counter()
        out = None
        for i in range(steps):
            out = work.step()
            if steps > 1 and i + 1 < steps:  # no sync: the clips stay queued back to back
                progress(f"timed {i + 1}/{steps} queued {time.perf_counter() - t0:.1f}s")
        barrier(world, dev)
        dt = time.perf_counter() - t0
        progress(f"timed {steps} steps {dt:.1f}s")
        if events:
            rec = kt.summary(1) if (kt is not None and kt_ms is not None) else {}
            if rec:
                rec["frac_of_clip_ms"] = round(rec["sum_ms_per_clip"] / kt_ms, 4)
                rec["clip_ms"] = round(kt_ms, 1)
            rec["sclk"] = clk.stop() if clk is not None else None
            rec["note"] = ("per-kernel-class device time of the last (untimed) warmup clip from one HIP event after "
                           "every library launch on its stream (the interval since the stream's previous event, so "
                           "each class includes the kernel boundary in front of it); sclk: sampled over the timed "
                           "clips, which carry no per-launch events besides the self-attention's (roofline)")
            work.kernels = rec
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
    if ATTN_KERNEL_NAME not in tj.get("kernel", ""):
        return None, None
    return tj["hbm_bytes_per_launch"], f"profiles/pmc_attn_traffic.json ({tj.get('source', 'rocprofv3 --pmc')})"


POST_RESERVE_S = 6.0  # after the timed region: result assembly, JSON, process-group teardown (~1 s measured, r03)


def run(args, world, rank, dev, work_factory=ClipWorkload, cpu=None):
    """The measurement; returns the JSON dict on rank 0 (None elsewhere).  `cpu`: the CpuBaseline child
    (N = 1), collected after the warmup so it never overlaps the timed region."""
    from stableavatar_amd import flops
    from stableavatar_amd import sp
    budget_end = T0 + args.time_budget
    skipped = []
    layout = "single" if world == 1 else args.mode
    work = work_factory(args, dev, rank, world)
    work.set_layout(layout)

    def collect_cpu(t_warm):
        if cpu is None:
            return
        per_step = t_warm / args.warmup if args.warmup > 0 else None
        if per_step is None:  # no warmup to size the timed region by: the mandatory config-2 leg only
            deadline = time.time()
        else:
            deadline = budget_end - args.steps * per_step - POST_RESERVE_S
        cpu.wait(deadline, required_by=time.time() + 180.0)

    dt, video = timed(work, args.steps, args.warmup, world, dev, events=True, before_timed=collect_cpu)
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
    sp_check = None
    if layout == "sp" and world > 1 and hasattr(work, "sp_check"):
        sp_check = work.sp_check()
        progress(f"sp check: {sp_check}")
    replicas = None
    if layout == "sp" and args.replica_steps > 0:
        # the layout switch changes the DiT's per-rank token count (workspaces, segment tables): untimed
        # warmup clips first
        est = (dt / args.steps) * world * (args.replica_steps + args.replica_warmup)
        if time.time() + est < budget_end:
            work.set_layout("replicas")
            rdt, rvideo = timed(work, args.replica_steps, args.replica_warmup, world, dev)
            work.check(rvideo)
            replicas = {"value": round(world * work.out_frames * args.replica_steps / rdt, 4), "unit": "frames/s",
                        "steps": args.replica_steps, "warmup": args.replica_warmup,
                        "ms_per_step": round(rdt / args.replica_steps * 1e3, 1),
                        "scaling": "weak", "parallelism": f"replicas{world}",
                        "note": "one independent clip per rank in the same processes (no data-path collective)"}
        else:
            skipped.append("replicas (would not fit the time budget)")
    enc = None
    if not args.no_encode and rank == 0 and hasattr(work, "vae"):
        if time.time() + 10.0 < budget_end:
            enc = vae_encode_ms(work.vae, args.frames, args.size, dev)
        else:
            skipped.append("vae_encode (time budget)")
    dit14 = None
    if world == 1 and args.dit14 and hasattr(work, "dit"):
        if time.time() + 40.0 < budget_end:
            from stableavatar_amd.kbench import bench_dit14
            dit14 = dict(bench_dit14(), note="BASELINE config 4's model (Wan-14B StableAvatar widths: dim 5120, 40 "
                                             "heads, ffn 13824) at 720x1280, 81 frames (L = 75 600, B = 3) on one "
                                             "GPU: forwards with 1 and 2 blocks, one block's time from their "
                                             "difference, the 40-block forward projected; outside the timed region "
                                             "and the metric")
        else:
            skipped.append("config_4_dit14 (time budget)")
    if rank != 0:
        return None
    traffic, traffic_src = attn_traffic(seq_len, layout)
    achieved = attn_flop / (attn_ms * 1e-3) if attn_ms else None
    cpu_res = None
    if cpu is not None:
        cpu_res = cpu.result(n_fwd, work.out_frames, args.size)
        c1 = cpu_res.get("config_1") or {}
        if c1.get("value", 0) is None:
            skipped.append("cpu_baseline.config_1 (" + c1["skipped"] + ")")
        elif "partial" in c1:
            skipped.append("cpu_baseline.config_1 steps (" + c1["partial"] + ")")
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
                      "dit_forwards_per_clip": n_fwd, "parallelism": parallelism,
                      "vae_decode": "split over the ranks" if (shared and world > 1 and args.vae_parallel)
                      else "whole clip on every rank" if world > 1 else "one GPU"},
           "roofline": {"bound": "mfma", "kernel": f"{ATTN_KERNEL_NAME} (self-attention, flash, D=128, V^T operand)",
                        "achieved": round(achieved / 1e12, 1) if achieved else None, "peak": PEAK_BF16 / 1e12,
                        "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16, 4) if achieved else None,
                        "traffic": round(traffic * attn_share) if traffic else None, "traffic_source": traffic_src,
                        "algorithmic_bytes": round(4 * 3 * seq_len * 1536 * 2 * attn_share),
                        "launch_share_of_cfg_batch": round(attn_share, 4),
                        "launch_ms": round(attn_ms, 3) if attn_ms else None, "flop_per_launch": attn_flop},
           "path_mfma_frac": round(path_flop * args.steps / dt / PEAK_BF16 / (world if shared else 1), 4),
           "cpu_baseline": cpu_res, "vae_encode": enc, "config_4_dit14": dit14,
           "time_budget": {"budget_s": args.time_budget, "elapsed_s": round(time.time() - T0, 1),
                           "skipped": skipped}}
    if replicas is not None:
        out["replicas"] = replicas
    if sp_check is not None:
        out["sp_check"] = sp_check
    if getattr(work, "kernels", None):
        out["kernels"] = work.kernels
    return out


def main(argv=None, work_factory=ClipWorkload, device=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.cpu_child:
        return cpu_child(args)
    if args.sp:
        args.mode = "sp"
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_workers(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        # the N > 1 sequence-parallel schedule runs each CFG row on its own stream beside RCCL's: enough hardware
        # queues (HIP default 4) that the row streams and the transport do not share one; set before any HIP call
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = CpuBaseline(args)  # started before this process touches the GPU (a plain child, no exec of ours)
    try:
        if device is None:
            dev = torch.device(f"cuda:{local}")
            torch.cuda.set_device(dev)
        else:
            dev = torch.device(device)
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                # env:// from the launcher by default; SA_DIST_INIT_METHOD (e.g. file://...) binds atomically for
                # launches without one (the CPU tests)
                init = os.environ.get("SA_DIST_INIT_METHOD")
                kw = dict(init_method=init, rank=rank, world_size=world) if init else {}
                if dev.type == "cuda":
                    dist.init_process_group("nccl", device_id=dev, **kw)
                else:
                    dist.init_process_group("gloo", **kw)
        out = run(args, world, rank, dev, work_factory, cpu=cpu)
        if out is not None:
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            dist.destroy_process_group()
    finally:
        if cpu is not None:
            cpu.cleanup()
    return 0


if __name__ == "__main__":
    sys.exit(main())
