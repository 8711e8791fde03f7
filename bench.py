"""StableAvatar hot-path benchmark on MI355X: denoised frames/s for one 512x512x81-frame
audio-driven clip (BASELINE.json configs[1]): 50 sliding-window x 3-way-CFG DiT denoising steps of
the Wan-2.1 1.3B StableAvatar model + the 3-D causal VAE decode to 81 frames.

One bench "step" = one whole clip (50 DiT forwards at B=3, L=21504 + 50 fused CFG/Euler steps +
VAE decode), inputs resident in HBM.  `python bench.py --gpus N --steps K --warmup W`; for N>1 it is
launched by torch.distributed.run, one process per GPU: by default every rank denoises its own clip
(replicas, weak scaling); with --sp all ranks denoise ONE clip with Ulysses sequence parallelism over
RCCL (strong scaling).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "denoised frames/sec, Wan-1.3B 512²×81f audio-driven, 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15  # dense bf16 MFMA, MI355X_MICROARCH.md


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--frames", type=int, default=81)
    p.add_argument("--size", type=int, default=512)
    p.add_argument("--sample-steps", type=int, default=50)
    p.add_argument("--overlap", type=int, default=15)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-encode", action="store_true", help="skip the (untimed) VAE encode measurement")
    p.add_argument("--sp", action="store_true",
                   help="N>1: one clip sequence-parallel over all ranks (Ulysses, strong scaling) instead of "
                        "one clip per rank (replicas, weak scaling)")
    p.add_argument("--window-dp", action="store_true",
                   help="N>1: one long clip with its sliding windows spread over the ranks (window parallelism, "
                        "strong scaling; use with --video-frames)")
    p.add_argument("--video-frames", type=int, default=None,
                   help="length of the generated video (default: --frames, i.e. one window); e.g. 165 = the "
                        "examples/case-1 shape (42 latent frames, 5 windows per step at overlap 15)")
    return p.parse_args()


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


def cpu_baseline(size, frames, sample_steps, n_fwd=None, out_frames=None):
    """Time the CPU oracle (fp32 restatement, oracle/) on a bounded sample of the same workload:
    one of the 30 DiT blocks at the full config-2 shape and the VAE decoder on one latent frame,
    then extrapolate to the clip (50 steps x 30 blocks + 81-frame decode)."""
    from oracle import dit as odit
    from oracle import vae as ovae
    from stableavatar_amd import synthetic
    threads = min(16, os.cpu_count() or 1)
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
    n_fwd = n_fwd or sample_steps
    out_frames = out_frames or frames
    t_clip = n_fwd * 30 * t_block + out_frames * t_vae_frame
    return {"value": round(out_frames / t_clip, 6), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle fp32: 1 of 30 DiT blocks at B=3,L={L} ({t_block:.1f}s) + VAE decode of 1 latent "
                      f"frame at {size}x{size} ({t_vae_frame:.1f}s), extrapolated to {n_fwd} forwards x 30 "
                      f"blocks + {out_frames} frames = {t_clip:.0f}s per clip"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from stableavatar_amd import flops
    from stableavatar_amd.pipeline import WanI2VTalkingInferenceLongPipeline, window_schedule
    from stableavatar_amd.scheduler import FlowMatchEulerDiscreteScheduler

    sp_mode = args.sp and world > 1
    wdp = args.window_dp and world > 1
    if sp_mode and wdp:
        raise SystemExit("--sp and --window-dp are exclusive")
    dit, vae = build(dev, seed=0)
    if sp_mode:
        dit.enable_multi_gpus_inference()
    latents, y, ctx, clip, a = make_inputs(dev, args.frames, args.size, seed=42 + (0 if sp_mode or wdp else rank),
                                           video_frames=args.video_frames)
    sched = FlowMatchEulerDiscreteScheduler(1000, shift=5.0)
    sched.set_timesteps(args.sample_steps, device=dev)
    pipe = WanI2VTalkingInferenceLongPipeline(vae=vae, transformer=dit, scheduler=sched)
    if wdp:
        pipe.enable_window_parallel()
    T = latents.shape[2]
    fpb = (args.frames - 1) // 4 + 1
    feats = {(s, e): torch.cat([torch.zeros_like(a), a, a]) for (s, e, _) in window_schedule(T, fpb, args.overlap)}
    h = args.size // 8
    seq_len = math.ceil(h * h / 4 * fpb)

    def clip_step():
        lat = pipe.denoise(latents, y, ctx, clip, feats, sched.timesteps, sched.sigmas, clip_length=args.frames,
                           seq_len=seq_len, overlap=args.overlap, text_guide_scale=3.0, audio_guide_scale=5.0)
        return vae.decode_clip(lat[0].float(), post=True)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            torch.cuda.synchronize()

    with torch.no_grad():
        for _ in range(args.warmup):
            clip_step()
        barrier()
        dit._events = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            video = clip_step()
        barrier()
        dt = time.perf_counter() - t0
        events = dit._events
        dit._events = None
    out_frames = 1 + 4 * (T - 1)
    assert video.shape[1] == out_frames and torch.isfinite(video).all()
    enc = None
    if not args.no_encode:  # once-per-call VAE encode of reference frame + zeros (pipeline:679-692), untimed
        ref = torch.zeros(1, 3, args.frames, args.size, args.size, device=dev)
        ref[:, :, 0].uniform_(-1, 1)
        with torch.no_grad():
            vae.encode(ref)
            torch.cuda.synchronize()
            te = time.perf_counter()
            lat_y = vae.encode(ref)[0].mode()
            torch.cuda.synchronize()
            te = time.perf_counter() - te
        assert tuple(lat_y.shape) == (1, 16, (args.frames - 1) // 4 + 1, args.size // 8, args.size // 8)
        ef = flops.vae_encode_flops(args.frames, args.size, args.size)
        enc = {"ms": round(te * 1e3, 1), "tflop": round(ef / 1e12, 2), "tflops_per_s": round(ef / te / 1e12, 1),
               "note": "AutoencoderKLWan.encode of the reference frame + zeros, once per call; outside the timed "
                       "region and the metric (SURVEY.md §8(d))"}
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    attn_ms = sum(e0.elapsed_time(e1) for e0, e1 in events) / max(len(events), 1)
    attn_flop = flops.self_attention_flops(B=3, L=seq_len)
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", "pmc_attn_traffic.json")
    if os.path.exists(tpath) and not args.sp and seq_len == 21504:
        with open(tpath) as f:
            tj = json.load(f)
        traffic = tj["hbm_bytes_per_launch"]
        traffic_src = f"profiles/pmc_attn_traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, {tj['kernel'][:60]})"
    parallelism = f"replicas{world}" if world > 1 else "single"
    if wdp:
        parallelism = f"windows{world}"
    if sp_mode:
        from stableavatar_amd import sp
        plan = sp.make_plan(world, rank, 12)
        attn_flop /= world  # this rank's (head group, query part) share
        parallelism = f"ulysses{plan.G}" + (f"x{plan.R}qsplit" if plan.R > 1 else "")
    achieved = attn_flop / (attn_ms * 1e-3)
    n_fwd = args.sample_steps * len(window_schedule(T, fpb, args.overlap))
    path_flop = n_fwd * flops.dit_forward_flops(B=3, L=seq_len, n_frames=fpb) + flops.vae_decode_flops(T, h, h)
    frames_total = (1 if sp_mode or wdp else world) * out_frames * args.steps
    value = frames_total / dt
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.size, args.frames, args.sample_steps, n_fwd, out_frames)
        out = {"metric": METRIC, "value": round(value, 4), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 1), "higher_is_better": True,
               "scaling": "strong" if sp_mode or wdp else "weak", "vs_baseline": None, "dtype": "bf16",
               "data": "synthetic (random-init weights by name-keyed seed; synthetic text/CLIP/wav2vec features "
                       "and conditioning latents; CPU-generated initial noise)",
               "config": {"workload": f"Wan-1.3B StableAvatar {args.size}x{args.size}x{out_frames}f"
                                      + (f" ({len(window_schedule(T, fpb, args.overlap))} windows of {args.frames}f,"
                                         f" overlap {args.overlap})" if out_frames != args.frames else "")
                                      + f", {args.sample_steps} steps, CFG x3, single audio clip, VAE decode",
                          "global_batch": 3 * (1 if sp_mode or wdp else world), "seq_len": seq_len,
                          "dit_forwards_per_clip": n_fwd, "parallelism": parallelism},
               "roofline": {"bound": "mfma", "kernel": "attn_fwd (self-attention, flash, D=128)",
                            "achieved": round(achieved / 1e12, 1), "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s",
                            "frac": round(achieved / PEAK_BF16, 4), "traffic": traffic, "traffic_source": traffic_src,
                            "algorithmic_bytes": 4 * 3 * seq_len * 1536 * 2,
                            "launch_ms": round(attn_ms, 3), "flop_per_launch": attn_flop},
               "path_mfma_frac": round(path_flop * args.steps / dt / PEAK_BF16 / (world if sp_mode or wdp else 1), 4),
               "cpu_baseline": cpu, "vae_encode": enc}
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
