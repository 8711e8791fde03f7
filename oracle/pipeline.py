"""ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

CPU restatement of the sliding-window, 3-way-CFG denoise loop of
WanI2VTalkingInferenceLongPipeline.__call__ (wan/pipeline/wan_inference_long_pipeline.py:703-796)
and of the FlowMatchEulerDiscreteScheduler it drives (diffusers 0.30.1, absent offline: restated
from its published algorithm — parity of the sigma table is pinned only by this restatement, see
DESIGN.md "parity unpinned" note).  The reference's infinite loop on a clip of exactly one window
(App. A.1) is fixed here: a first window that reaches the end is the last one.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def flow_sigmas(num_inference_steps, shift=5.0, num_train_timesteps=1000):
    """FlowMatchEulerDiscreteScheduler(shift).set_timesteps(n) -> (timesteps [n], sigmas [n+1]).
    __init__ shifts linspace(1, N)/N once to get sigma_max/min; set_timesteps re-applies the shift."""
    N = num_train_timesteps
    s = np.linspace(1, N, N, dtype=np.float32)[::-1].copy() / N
    s = torch.from_numpy(s)
    s = shift * s / (1 + (shift - 1) * s)
    smax, smin = s[0].item(), s[-1].item()
    t = np.linspace(smax * N, smin * N, num_inference_steps)
    sig = t / N
    sig = shift * sig / (1 + (shift - 1) * sig)
    sig = torch.from_numpy(sig).to(torch.float32)
    return sig * N, torch.cat([sig, torch.zeros(1)])


def window_schedule(infer_length, frames_per_batch, overlap):
    """Sequence of (index_start, index_end, index_previous_end) windows of one denoise step
    (pipeline:709-789), with the single-window hang fixed."""
    if infer_length < frames_per_batch:
        raise ValueError(f"clip has {infer_length} latent frames < one window ({frames_per_batch}); "
                         "the reference decodes all-zero latents here (App. A.1)")
    out = []
    start, end = 0, frames_per_batch
    prev_end = end
    last = end == infer_length  # the reference never terminates in this case
    while end <= infer_length:
        out.append((start, end, prev_end))
        if last:
            break
        if end != infer_length:
            prev_end = end
            start = start + (frames_per_batch - overlap)
            if start + frames_per_batch < infer_length:
                end = start + frames_per_batch
            else:
                end = infer_length
                last = True
    return out


def overlap_weights(overlap, scheme="uniform"):
    """pipeline:757-766."""
    if scheme == "uniform":
        return torch.tensor([j / (overlap - 1) for j in range(overlap)], dtype=torch.float32)
    w = torch.linspace(0, 1, overlap)
    w = torch.log1p(w * (torch.exp(torch.tensor(1.0)) - 1))
    return (w - w.min()) / (w.max() - w.min())


def audio_window(index_start, index_end, infer_length, audio_token_per_frame, max_audio_index):
    """pipeline:718-724: sample indices of the audio slice for one window."""
    a0 = index_start * 4 * audio_token_per_frame
    if index_end == infer_length:
        return [ii % max_audio_index for ii in range(a0, max_audio_index)]
    frames = (index_end - index_start) * 4
    return [ii % max_audio_index for ii in range(a0, a0 + frames * audio_token_per_frame)]


def denoise(dit, latents, y, context, clip_ctx, audio, audio_encoder, *, num_inference_steps, clip_length,
            num_frames, height, width, overlap, text_guide_scale, audio_guide_scale, sr=16000, fps=25,
            scheme="uniform", shift=5.0, patch=(1, 2, 2), max_steps=None, step_callback=None):
    """Restated loop of pipeline:703-790.  `dit(x, t, context, seq_len, y, clip_fea, vocal, n)` is the
    denoiser; `audio_encoder(samples [n]) -> [1, tokens, 768]`.  Returns latents_all (fp32 holding
    bf16-rounded values like the reference, :771,:776)."""
    frames_per_batch = (clip_length - 1) // 4 + 1
    atpf = int(sr / fps)
    max_audio = audio.shape[0]
    timesteps, sigmas = flow_sigmas(num_inference_steps, shift)
    infer_length = latents.size(2)
    latents_all = latents.clone()
    tgt_f = (num_frames - 1) // 4 + 1
    seq_len = math.ceil((width // 8) * (height // 8) / (patch[1] * patch[2]) * tgt_f)
    wts = overlap_weights(overlap, scheme) if overlap > 0 else None
    for i, t in enumerate(timesteps):
        if max_steps is not None and i >= max_steps:
            break
        pred = torch.zeros_like(latents_all)
        for (s, e, pe) in window_schedule(infer_length, frames_per_batch, overlap):
            idx = [ii % latents_all.shape[2] for ii in range(s, e)]
            lat = latents_all[:, :, idx].clone()
            sub = audio[audio_window(s, e, infer_length, atpf, max_audio)]
            a = audio_encoder(sub)
            a = torch.cat([torch.zeros_like(a), a, a], 0)
            nf = lat.size(2)
            noise = dit(torch.cat([lat] * 3), t.expand(3), context, seq_len, y[:, :, :nf], clip_ctx, a, clip_length)
            u, d, c = noise.chunk(3)
            v = u + audio_guide_scale * (d - u) + text_guide_scale * (c - d)
            lat = (lat.float() + (sigmas[i + 1] - sigmas[i]) * v).to(v.dtype)
            if s != 0 and i != 0:
                w = wts.view(1, 1, overlap, 1, 1).to(lat.dtype)
                oi = [ii % lat.shape[2] for ii in range(overlap)]
                pi = [ii % latents_all.shape[2] for ii in range(pe - overlap, pe)]
                lat[:, :, oi] = lat[:, :, oi] * w + pred[:, :, pi] * (1 - w)
            lat = lat.to(torch.bfloat16)
            for k in range(nf):
                pred[:, :, (s + k) % pred.shape[2]] = lat[:, :, k].to(pred.dtype)
        latents_all = pred
        if step_callback is not None:  # progress of a timed run (bench.py's CPU baseline)
            step_callback(i)
    return latents_all
