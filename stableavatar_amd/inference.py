"""``inference.py`` of the reference (CLI flags inference.py:238-409, main() :412-578) on the MI355X drop-ins.

Same flags and defaults, plus ``--device`` / ``--dtype``; the components are this package's HIP modules:
``WanT5EncoderModel`` and ``CLIPModel`` (encoders.py), ``AutoencoderKLWan`` (vae.py),
``WanTransformer3DFantasyModel`` (transformer.py), ``FlowMatchEulerDiscreteScheduler`` (scheduler.py) and
``WanI2VTalkingInferenceLongPipeline`` (pipeline.py) and ``Wav2Vec2Model`` (wav2vec.py, the audio encoder on the
HIP kernels, reading the same transformers model directory); the tokenizer and the wav2vec2 processor come from
``transformers`` as in the reference.  wav2vec2 features are computed once per window and reused across steps.

Flag mapping:
* ``--ulysses_degree`` x ``--ring_degree`` > 1 (under torchrun, RCCL): the transformer's sequence parallelism
  over all ranks (``enable_multi_gpus_inference``); the head split is gcd(12, N) groups x N / gcd query parts
  (stableavatar_amd/sp.py), which replaces xfuser's Ulysses x ring layout with the same rank count;
  ``--window_parallel`` instead spreads the sliding windows over the ranks;
* ``--GPU_memory_mode``: ``model_full_load`` as the reference; ``model_cpu_offload_and_qfloat8`` stores the DiT
  weights as float8_e4m3fn (fp8_optimization.py:29-43, 'modulation' excluded) and upcasts them at pack time;
  the CPU-offload modes keep the models resident (288 GB of HBM holds every model) and say so;
* ``--enable_teacache`` / ``--teacache_threshold`` / ``--num_skip_start_steps`` / ``--teacache_offload``:
  ``transformer.enable_teacache`` with the reference's coefficient table;
* ``--fsdp_dit`` / ``--t5_fsdp`` / ``--t5_cpu`` / ``--offload_model``: accepted, no effect (the 3.5 GB DiT is
  replicated).
Audio is read with scipy (16-bit / float WAV, channels averaged, polyphase resampling to 16 kHz) where the
reference uses librosa.load (soxr resampler): sample values differ slightly.  The video is written as
``video_without_audio.mp4`` when imageio is importable, else as PNG frames + ``video.npy`` (the reference's
save_videos_grid needs imageio / cv2).
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np
import torch

NEGATIVE_PROMPT = ("色调艳丽，过曝，静态，细节模糊不清，字幕，风格，作品，画作，画面，静止，整体发灰，最差质量，低质量，JPEG压缩残留，丑陋的，"
                   "残缺的，多余的手指，画得不好的手部，画得不好的脸部，畸形的，毁容的，形态畸形的肢体，手指融合，静止不动的画面，杂乱的背景，"
                   "三条腿，背景人很多，倒着走")  # inference.py:546


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="StableAvatar inference on MI355X (HIP kernels)")
    p.add_argument("--input_perturbation", type=float, default=0)
    p.add_argument("--pretrained_model_name_or_path", type=str, default=None, required=True)
    p.add_argument("--transformer_path", type=str, default=None)
    p.add_argument("--revision", type=str, default=None)
    p.add_argument("--variant", type=str, default=None)
    p.add_argument("--output_dir", type=str)
    p.add_argument("--width", type=int, default=512)
    p.add_argument("--height", type=int, default=512)
    p.add_argument("--validation_prompts", type=str, default="The protagonist is singing", nargs="+")
    p.add_argument("--pretrained_wav2vec_path", type=str)
    p.add_argument("--validation_reference_path", type=str)
    p.add_argument("--validation_driven_audio_path", type=str)
    p.add_argument("--offload_model", action="store_true")
    p.add_argument("--ulysses_degree", type=int, default=1)
    p.add_argument("--ring_degree", type=int, default=1)
    p.add_argument("--t5_fsdp", action="store_true", default=False)
    p.add_argument("--t5_cpu", action="store_true", default=False)
    p.add_argument("--fsdp_dit", action="store_true")
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--motion_frame", type=int, default=25)
    p.add_argument("--sample_steps", type=int, default=None)
    p.add_argument("--sample_shift", type=float, default=None)
    p.add_argument("--sample_text_guide_scale", type=float, default=5.0)
    p.add_argument("--sample_audio_guide_scale", type=float, default=4.0)
    p.add_argument("--overlap_window_length", type=int, default=10)
    p.add_argument("--config_path", type=str, default=None)
    p.add_argument("--enable_teacache", action="store_true")
    p.add_argument("--teacache_threshold", type=float, default=0.10)
    p.add_argument("--num_skip_start_steps", type=int, default=5)
    p.add_argument("--teacache_offload", action="store_true")
    p.add_argument("--GPU_memory_mode", type=str, default="model_full_load",
                   help="[model_full_load, sequential_cpu_offload, model_cpu_offload_and_qfloat8, model_cpu_offload]")
    p.add_argument("--clip_sample_n_frames", type=int, default=81)
    p.add_argument("--overlapping_weight_scheme", type=str, default="uniform", help="[uniform, log]")
    # MI355X build additions
    p.add_argument("--device", type=str, default=None, help="default cuda:LOCAL_RANK")
    p.add_argument("--dtype", type=str, default="bf16", choices=("bf16",), help="DiT compute dtype (as the reference)")
    p.add_argument("--window_parallel", action="store_true",
                   help="multi-GPU: spread the sliding windows of each step over the ranks instead of sequence "
                        "parallelism (long clips, SURVEY.md §8(e))")
    p.add_argument("--vae_parallel", action="store_true",
                   help="multi-GPU: split the VAE decode over the ranks (a wavefront of causal-cache hand-offs); "
                        "off by default: every rank decodes the whole clip, as the reference does")
    args = p.parse_args(argv)
    if args.window_parallel and args.enable_teacache:
        # checked before any model is loaded (the pipeline would raise at its first denoise step)
        p.error("--window_parallel cannot be combined with --enable_teacache: TeaCache's skip decisions follow the "
                "sequence of forwards one process runs (cache_utils.py:59-80), which window parallelism changes")
    if args.window_parallel and (args.ulysses_degree > 1 or args.ring_degree > 1):
        p.error("--window_parallel and --ulysses_degree/--ring_degree > 1 are alternative multi-GPU layouts")
    return args


def prompt_text(prompts):
    """--validation_prompts uses nargs='+'.  The reference passes the list on as a batch of prompts
    (inference.py:544-546 -> pipeline:608-611), but its context list then holds 3k entries against a CFG batch of 3
    latents, which only works for k = 1 (one quoted prompt).  Several words given unquoted are joined into that
    one prompt here, with a warning."""
    if isinstance(prompts, str):
        return prompts
    prompts = list(prompts)
    if len(prompts) > 1:
        import warnings
        warnings.warn(f"--validation_prompts got {len(prompts)} arguments; they are joined into one prompt (the "
                      "reference's pipeline takes one prompt per audio clip: quote the prompt)")
    return " ".join(prompts)


def load_config(path):
    import yaml
    with open(path) as f:
        return yaml.safe_load(f)


def load_audio(path, sr=16000):
    """librosa.load(path, sr=16000) equivalent: mono float32 in [-1, 1] at `sr` Hz."""
    from math import gcd

    from scipy.io import wavfile
    from scipy.signal import resample_poly
    rate, data = wavfile.read(path)
    if data.dtype == np.int16:
        x = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:
        x = data.astype(np.float32) / 2147483648.0
    elif data.dtype == np.uint8:
        x = (data.astype(np.float32) - 128.0) / 128.0
    else:
        x = data.astype(np.float32)
    if x.ndim == 2:
        x = x.mean(axis=1)
    if rate != sr:
        g = gcd(rate, sr)
        x = resample_poly(x, sr // g, rate // g).astype(np.float32)
    return x, sr


def save_video(sample, output_dir, fps=25):
    """sample [1, 3, F, H, W] in [0, 1] (pipeline .videos)."""
    os.makedirs(output_dir, exist_ok=True)
    frames = (sample[0].permute(1, 2, 3, 0).clamp(0, 1).numpy() * 255).round().astype(np.uint8)  # [F, H, W, 3]
    try:
        import imageio
        path = os.path.join(output_dir, "video_without_audio.mp4")
        imageio.mimsave(path, list(frames), fps=fps)
        return path
    except ImportError:
        from PIL import Image
        d = os.path.join(output_dir, "animated_images")
        os.makedirs(d, exist_ok=True)
        for i, fr in enumerate(frames):
            Image.fromarray(fr).save(os.path.join(d, f"frame_{i:05d}.png"))
        np.save(os.path.join(output_dir, "video.npy"), sample.numpy())
        return d


def convert_model_weight_to_float8(model, exclude_module_name=("modulation",)):
    """fp8_optimization.py:29-43: parameters outside the excluded modules stored as float8_e4m3fn."""
    for name, p in model.named_parameters():
        if not any(e in name for e in exclude_module_name) and p.dim() >= 2:
            p.data = p.data.to(torch.float8_e4m3fn)


def main(argv=None):
    args = parse_args(argv)
    from transformers import AutoTokenizer, Wav2Vec2Processor

    from .wav2vec import Wav2Vec2Model

    from .encoders import CLIPModel, WanT5EncoderModel
    from .pipeline import WanI2VTalkingInferenceLongPipeline
    from .scheduler import FlowMatchEulerDiscreteScheduler
    from .teacache import get_teacache_coefficients
    from .transformer import WanTransformer3DFantasyModel
    from .vae import AutoencoderKLWan

    config = load_config(args.config_path)
    multi = args.ulysses_degree > 1 or args.ring_degree > 1 or args.window_parallel
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device(args.device or f"cuda:{local_rank}")
    torch.cuda.set_device(device)
    rank = 0
    if multi:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=device)
        rank = dist.get_rank()
        if not args.window_parallel:
            assert dist.get_world_size() == args.ring_degree * args.ulysses_degree, \
                "number of GPUs(%d) should be equal to ring_degree * ulysses_degree." % dist.get_world_size()
    weight_dtype = torch.bfloat16
    fps = 25
    root = args.pretrained_model_name_or_path
    tk = config["text_encoder_kwargs"]
    tokenizer = AutoTokenizer.from_pretrained(os.path.join(root, tk.get("tokenizer_subpath", "tokenizer")))
    text_encoder = WanT5EncoderModel.from_pretrained(os.path.join(root, tk.get("text_encoder_subpath", "text_encoder")),
                                                     additional_kwargs=tk, low_cpu_mem_usage=True,
                                                     torch_dtype=weight_dtype).eval()
    vk = config["vae_kwargs"]
    vae = AutoencoderKLWan.from_pretrained(os.path.join(root, vk.get("vae_subpath", "vae")), additional_kwargs=vk)
    wav2vec_processor = Wav2Vec2Processor.from_pretrained(args.pretrained_wav2vec_path)
    wav2vec = Wav2Vec2Model.from_pretrained(args.pretrained_wav2vec_path).to(device)
    ik = config["image_encoder_kwargs"]
    clip_image_encoder = CLIPModel.from_pretrained(os.path.join(root, ik.get("image_encoder_subpath", "image_encoder")),
                                                   transformer_additional_kwargs=ik).eval()
    trk = config["transformer_additional_kwargs"]
    transformer3d = WanTransformer3DFantasyModel.from_pretrained(
        os.path.join(root, trk.get("transformer_subpath", "transformer")),
        transformer_additional_kwargs=dict(trk), low_cpu_mem_usage=False, torch_dtype=weight_dtype)
    if args.transformer_path is not None:
        print(f"From checkpoint: {args.transformer_path}")
        state_dict = torch.load(args.transformer_path, map_location="cpu", weights_only=True)
        state_dict = state_dict["state_dict"] if "state_dict" in state_dict else state_dict
        m, u = transformer3d.load_state_dict(state_dict, strict=False)
        print(f"missing keys: {len(m)}, unexpected keys: {len(u)}")
    sk = dict(config.get("scheduler_kwargs", {}))
    if args.sample_shift is not None:
        sk["shift"] = args.sample_shift
    scheduler = FlowMatchEulerDiscreteScheduler(**{k: v for k, v in sk.items() if k in (
        "num_train_timesteps", "shift", "use_dynamic_shifting", "base_shift", "max_shift", "base_image_seq_len",
        "max_image_seq_len")})
    pipeline = WanI2VTalkingInferenceLongPipeline(tokenizer=tokenizer, text_encoder=text_encoder, vae=vae,
                                                  transformer=transformer3d, clip_image_encoder=clip_image_encoder,
                                                  scheduler=scheduler, wav2vec_processor=wav2vec_processor,
                                                  wav2vec=wav2vec)
    if args.GPU_memory_mode == "model_cpu_offload_and_qfloat8":
        convert_model_weight_to_float8(transformer3d, exclude_module_name=["modulation"])
    elif args.GPU_memory_mode in ("sequential_cpu_offload", "model_cpu_offload"):
        print(f"GPU_memory_mode={args.GPU_memory_mode}: models stay resident in HBM on MI355X (no offload)")
    pipeline.to(device=device)
    text_encoder.to(device)
    clip_image_encoder.to(device)
    if multi:
        if args.window_parallel:
            pipeline.enable_window_parallel()
        else:
            transformer3d.enable_multi_gpus_inference()
        pipeline.enable_vae_parallel(args.vae_parallel)
    if args.enable_teacache:
        coefficients = get_teacache_coefficients(root)
        if coefficients is not None:
            print(f"Enable TeaCache with threshold {args.teacache_threshold} and skip the first "
                  f"{args.num_skip_start_steps} steps.")
            pipeline.transformer.enable_teacache(coefficients, args.sample_steps, args.teacache_threshold,
                                                 num_skip_start_steps=args.num_skip_start_steps,
                                                 offload=args.teacache_offload)
    seed = args.seed if args.seed is not None else 0
    generator = torch.Generator(device=device).manual_seed(seed)
    clip_n = args.clip_sample_n_frames
    video_length = int((clip_n - 1) // vae.config.temporal_compression_ratio *
                       vae.config.temporal_compression_ratio) + 1 if clip_n != 1 else 1
    sr = 16000
    vocal_input, _ = load_audio(args.validation_driven_audio_path, sr=sr)
    prompt = prompt_text(args.validation_prompts)
    with torch.no_grad():
        sample = pipeline(prompt, num_frames=video_length, negative_prompt=NEGATIVE_PROMPT, height=args.height,
                          width=args.width, guidance_scale=6.0, generator=generator,
                          num_inference_steps=args.sample_steps, text_guide_scale=args.sample_text_guide_scale,
                          audio_guide_scale=args.sample_audio_guide_scale, vocal_input_values=vocal_input,
                          motion_frame=args.motion_frame, fps=fps, sr=sr,
                          cond_file_path=args.validation_reference_path, seed=seed,
                          overlap_window_length=args.overlap_window_length,
                          overlapping_weight_scheme=args.overlapping_weight_scheme, clip_length=clip_n).videos
    out = None
    if rank == 0:
        out = save_video(sample, args.output_dir, fps=fps)
        print(f"saved {tuple(sample.shape)} -> {out}")
    if multi:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
    sys.exit(0)
