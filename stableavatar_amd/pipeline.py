"""Drop-in WanI2VTalkingInferenceLongPipeline for MI355X (reference:
wan/pipeline/wan_inference_long_pipeline.py).

Same constructor and `__call__` arguments.  The hot path -- the sliding-window x 3-way-CFG denoise
loop (:703-790) and the VAE decode (:793-796, :424-430) -- runs on the HIP kernels:
WanTransformer3DFantasyModel.forward_window per window, then ONE fused sa_flow_step kernel per
window for CFG combine + Euler step + overlap blend + scatter.  The once-per-call encoders (T5,
CLIP, VAE-encode of the reference frame) are called exactly as the reference does when given, or
their outputs can be passed directly (`prompt_embeds`/`negative_prompt_embeds`, `clip_context`,
`y`).  wav2vec features depend only on the audio slice of a window, so they are computed once per
window and reused across steps (the reference recomputes them every step, :727-729).

Fixes the reference's infinite loop when the clip is exactly one window.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import ops


def window_schedule(infer_length, frames_per_batch, overlap):
    """(index_start, index_end, index_previous_end) of each window of one step (:709-789)."""
    if infer_length < frames_per_batch:
        raise ValueError(f"clip has {infer_length} latent frames < one window ({frames_per_batch}); "
                         "the reference decodes all-zero latents in this case")
    out = []
    start, end = 0, frames_per_batch
    prev_end = end
    last = end == infer_length
    while end <= infer_length:
        out.append((start, end, prev_end))
        if last:
            break
        prev_end = end
        start = start + (frames_per_batch - overlap)
        if start + frames_per_batch < infer_length:
            end = start + frames_per_batch
        else:
            end = infer_length
            last = True
    return out


def overlap_weights(overlap, scheme="uniform"):
    """:757-766."""
    if scheme == "uniform":
        return torch.tensor([j / (overlap - 1) for j in range(overlap)], dtype=torch.float32)
    if scheme == "log":
        w = torch.linspace(0, 1, overlap)
        w = torch.log1p(w * (torch.exp(torch.tensor(1.0)) - 1))
        return (w - w.min()) / (w.max() - w.min())
    raise ValueError(f"unknown overlapping_weight_scheme {scheme}")


def audio_window(index_start, index_end, infer_length, audio_token_per_frame, max_audio_index):
    """:718-724."""
    a0 = index_start * 4 * audio_token_per_frame
    if index_end == infer_length:
        return [ii % max_audio_index for ii in range(a0, max_audio_index)]
    frames = (index_end - index_start) * 4
    return [ii % max_audio_index for ii in range(a0, a0 + frames * audio_token_per_frame)]


class WanI2VPipelineTalkingInferenceLongOutput:
    def __init__(self, videos):
        self.videos = videos


class WanI2VTalkingInferenceLongPipeline:
    def __init__(self, tokenizer=None, text_encoder=None, vae=None, transformer=None, clip_image_encoder=None,
                 scheduler=None, wav2vec_processor=None, wav2vec=None):
        self.tokenizer, self.text_encoder, self.vae, self.transformer = tokenizer, text_encoder, vae, transformer
        self.clip_image_encoder, self.scheduler = clip_image_encoder, scheduler
        self.wav2vec_processor, self.wav2vec = wav2vec_processor, wav2vec
        self.vae_encoder = None  # optional module with .encode() for the reference frame (§8(f))
        self.window_group = None  # set by enable_window_parallel()
        self.device = torch.device("cuda")

    def enable_window_parallel(self, group=None):
        """Split the sliding windows of every step over the ranks of ``group`` (default: the
        torch.distributed world, RCCL).  All windows of a step read only latents_all (:726), so
        each rank runs the DiT on windows k = rank, rank + N, ..; the noise predictions are
        all-gathered (one async collective per round of N windows, overlapping the next round's
        forward) and every rank applies the CFG / Euler / blend steps of all windows in the
        reference order -- bit-identical latents on every rank and to the single-GPU loop."""
        import torch.distributed as dist
        self._check_window_parallel(self.transformer)
        self.window_group = group if group is not None else dist.group.WORLD
        return self

    def disable_window_parallel(self):
        self.window_group = None
        return self

    def enable_vae_parallel(self, on=True):
        """Opt-in: decode the clip over the ranks the denoise loop runs on (window parallelism or the
        transformer's sequence-parallel group) -- a wavefront of causal-cache hand-offs, 1/N of the frames per
        rank + one gather, bit-identical to the single-GPU decode.  Off by default: every rank decodes the
        whole clip, as the reference does (:793-796)."""
        self.vae_parallel = bool(on)
        return self

    vae_parallel = False

    def _decode_group_sync(self):
        """point the VAE's decode group at the ranks of the denoise loop when enable_vae_parallel() is on"""
        t = self.transformer
        if self.vae is None or not hasattr(self.vae, "decode_group"):
            return
        grp = None
        if self.vae_parallel:
            import torch.distributed as dist
            if self.window_group is not None:
                grp = self.window_group
            elif getattr(t, "_sp_enabled", False):
                grp = t.sp_group if t.sp_group is not None else dist.group.WORLD
        if grp is None:
            if self.vae.decode_group is not None:
                self.vae.disable_multi_gpus_inference()
        elif self.vae.decode_group is not grp:
            self.vae.enable_multi_gpus_inference(grp)

    @staticmethod
    def _check_window_parallel(transformer):
        if transformer is None:
            return
        if getattr(transformer, "sp_world_size", 1) > 1:
            raise RuntimeError("window parallelism and sequence parallelism over the same ranks would deadlock "
                               "(each rank runs different windows while SP needs all ranks in every forward); "
                               "use one of them")
        if getattr(transformer, "teacache", None) is not None:
            raise RuntimeError("window parallelism cannot be combined with TeaCache: its skip decisions and reused "
                               "residual follow the sequence of forwards one process runs (cache_utils.py:59-80), "
                               "which window parallelism changes (rank r sees windows r, r+N, ..)")

    def to(self, device=None, **_):
        if device is not None:
            self.device = torch.device(device)
        for m in (self.transformer, self.vae):
            if m is not None:
                m.to(self.device)
        return self

    # ---------------------------------------------------------------- once-per-call inputs

    def _prompt_embeds(self, prompt, max_sequence_length):
        """_get_t5_prompt_embeds (:236-278): trimmed per mask length."""
        ids = self.tokenizer([prompt], padding="max_length", max_length=max_sequence_length, truncation=True,
                             add_special_tokens=True, return_tensors="pt")
        seq_len = int(ids.attention_mask.gt(0).sum())
        emb = self.text_encoder(ids.input_ids.to(self.device), attention_mask=ids.attention_mask.to(self.device))[0]
        return emb[0, :seq_len]

    def _audio_features(self, samples, sr):
        inp = self.wav2vec_processor(samples, sampling_rate=sr, return_tensors="pt").input_values
        dev = next(self.wav2vec.parameters()).device if any(True for _ in self.wav2vec.parameters()) else "cpu"
        return self.wav2vec(inp.to(dev)).last_hidden_state

    def _conditioning(self, cond_file_path, height, width, clip_length, dtype):
        """:665-700: CLIP context and y = cat(mask, VAE.encode(ref + zeros))."""
        from PIL import Image
        img = Image.open(cond_file_path).convert("RGB").resize([width, height])
        t = torch.from_numpy(np.array(img)).permute(2, 0, 1).float() / 255
        t = (t - 0.5) * 2
        clip = self.clip_image_encoder([t.to(self.device, dtype)[:, None]])
        clip = torch.cat([clip] * 3)
        enc = self.vae_encoder if self.vae_encoder is not None else self.vae
        frames = torch.zeros(1, 3, clip_length, height, width, device=self.device)
        frames[:, :, :1] = t.to(self.device)[None, :, None]
        lat = enc.encode(frames)[0].mode()
        return clip, self.mask_latents(lat, clip_length)

    @staticmethod
    def mask_latents(masked_video_latents, clip_length, cfg=True):
        """:693-700: 4-channel first-frame mask + reference latents, tripled for CFG."""
        h, w = masked_video_latents.shape[-2:]
        dev = masked_video_latents.device
        msk = torch.ones(1, clip_length, h, w, device=dev)
        msk[:, 1:] = 0
        msk = torch.cat([torch.repeat_interleave(msk[:, 0:1], repeats=4, dim=1), msk[:, 1:]], dim=1)
        msk = msk.view(1, msk.shape[1] // 4, 4, h, w).transpose(1, 2).float()
        n = 3 if cfg else 1
        return torch.cat([torch.cat([msk] * n), torch.cat([masked_video_latents] * n)], dim=1)

    # ---------------------------------------------------------------- hot path

    def denoise(self, latents, y, context, clip_context, window_features, timesteps, sigmas, *, clip_length,
                seq_len, overlap, text_guide_scale, audio_guide_scale, scheme="uniform", callback=None):
        """The denoise loop of :703-790 on the GPU.  latents: bf16 [1, 16, T, H, W] (initial noise);
        window_features: {(start, end): [3, n_audio, 768]} (zero row first, :737).  Returns the
        final latents_all (bf16)."""
        dev = latents.device
        if hasattr(self.transformer, "invalidate_context"):
            self.transformer.invalidate_context()  # text / image K/V are rebuilt once for this call's inputs
        fpb = (clip_length - 1) // 4 + 1
        T = latents.shape[2]
        wins = window_schedule(T, fpb, overlap)
        wts = overlap_weights(overlap, scheme).to(dev) if overlap and overlap > 1 else None
        cfg = y.shape[0] == 3
        # a copy: the two ping-pong buffers are written in turn, and the caller's noise tensor must survive the
        # call (the reference's scheduler.step returns new tensors, :754)
        lat = latents.to(torch.bfloat16, copy=True).contiguous()
        pred = torch.empty_like(lat)
        yb = y.to(device=dev, dtype=torch.bfloat16).contiguous()
        # the CFG rows' DiT inputs are equal when y's rows are (mask_latents triples one row, :693-700; the latents
        # are tripled at :730 and t expanded at :733): the DiT then runs its first block's self-attention half once
        # (forward_window shared_rows); checked once per call.  SA_CFG_SHARED=0 computes every row (A/B)
        self._shared_rows = (cfg and os.environ.get("SA_CFG_SHARED", "1") != "0"
                             and bool((yb[1:] == yb[:1]).all()))
        sig = [float(s) for s in sigmas]
        if self.window_group is not None:
            return self._denoise_window_parallel(lat, pred, yb, context, clip_context, window_features, timesteps,
                                                 sig, wins, wts, cfg, fpb, clip_length, seq_len, overlap,
                                                 text_guide_scale, audio_guide_scale, callback)
        for i, t in enumerate(timesteps):
            pred.zero_()
            tt = torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(1)
            for (s, e, pe) in wins:
                Fw = e - s
                noise = self.transformer.forward_window(lat, s, True, 3 if cfg else 1, tt, context, seq_len,
                                                        clip_context, yb[:, :, :Fw], window_features[(s, e)],
                                                        clip_length, shared_rows=self._shared_rows)
                blend = s != 0 and i != 0
                ops.flow_step(lat, pred, noise, s, sig[i + 1] - sig[i], audio_guide_scale or 0.0,
                              text_guide_scale or 0.0, overlap if blend else 0, pe, wts if blend else None, blend)
            lat, pred = pred, lat
            if callback is not None:
                callback(i, t, lat)
        return lat

    def _denoise_window_parallel(self, lat, pred, yb, context, clip_context, window_features, timesteps, sig, wins,
                                 wts, cfg, fpb, clip_length, seq_len, overlap, text_guide_scale, audio_guide_scale,
                                 callback):
        import torch.distributed as dist

        from . import sp
        self._check_window_parallel(self.transformer)  # the transformer may have changed since enable
        grp = self.window_group
        N, r = dist.get_world_size(grp), dist.get_rank(grp)
        dev = lat.device
        R = 3 if cfg else 1
        C, H, W = lat.shape[1], lat.shape[3], lat.shape[4]
        rounds = -(-len(wins) // N)
        slots = torch.empty(rounds * N, R * C * fpb * H * W, device=dev, dtype=torch.bfloat16)

        def view(k):
            Fw = wins[k][1] - wins[k][0]
            return slots[k, :R * C * Fw * H * W].view(R, C, Fw, H, W)

        for i, t in enumerate(timesteps):
            pred.zero_()
            tt = torch.as_tensor(t, dtype=torch.float32, device=dev).reshape(1)
            pend = []
            for j in range(rounds):
                k = j * N + r
                if k < len(wins):
                    s, e, _ = wins[k]
                    self.transformer.forward_window(lat, s, True, R, tt, context, seq_len, clip_context,
                                                    yb[:, :, :e - s], window_features[(s, e)], clip_length,
                                                    out=view(k), shared_rows=self._shared_rows)
                pend.append(sp.all_gather_slots(slots[j * N:(j + 1) * N], r, grp))
            for p_ in pend:
                p_.wait()
            for k, (s, e, pe) in enumerate(wins):
                blend = s != 0 and i != 0
                ops.flow_step(lat, pred, view(k), s, sig[i + 1] - sig[i], audio_guide_scale or 0.0,
                              text_guide_scale or 0.0, overlap if blend else 0, pe, wts if blend else None, blend)
            lat, pred = pred, lat
            if callback is not None:
                callback(i, t, lat)
        return lat

    @torch.no_grad()
    def __call__(self, prompt=None, negative_prompt=None, height=480, width=720, video=None, mask_video=None,
                 num_frames=81, num_inference_steps=50, timesteps=None, guidance_scale=6, num_videos_per_prompt=1,
                 eta=0.0, generator=None, latents=None, prompt_embeds=None, negative_prompt_embeds=None,
                 output_type="numpy", return_dict=False, callback_on_step_end=None, attention_kwargs=None,
                 callback_on_step_end_tensor_inputs=["latents"], clip_image=None, max_sequence_length=512,
                 text_guide_scale=None, audio_guide_scale=None, vocal_input_values=None, motion_frame=None, fps=None,
                 sr=None, cond_file_path=None, seed=None, overlap_window_length=None,
                 overlapping_weight_scheme="uniform", clip_length=81, y=None, clip_context=None):
        if height % 8 or width % 8:
            raise ValueError(f"`height` and `width` have to be divisible by 8 but are {height} and {width}.")
        cfg = guidance_scale > 1.0
        if cfg and (text_guide_scale is None or audio_guide_scale is None):
            raise ValueError("the talking pipeline's CFG needs text_guide_scale and audio_guide_scale (:736-753)")
        dev = self.device
        if prompt_embeds is None:
            prompt_embeds = self._prompt_embeds(prompt, max_sequence_length)
        if cfg and negative_prompt_embeds is None:
            negative_prompt_embeds = self._prompt_embeds(negative_prompt or "", max_sequence_length)
        pe = prompt_embeds[0] if prompt_embeds.dim() == 3 else prompt_embeds
        context = [negative_prompt_embeds[0] if negative_prompt_embeds.dim() == 3 else negative_prompt_embeds] * 2 \
            + [pe] if cfg else [pe]
        context = [c.to(dev) for c in context]
        fpb = (clip_length - 1) // 4 + 1
        atpf = int(sr / fps)
        max_audio = len(vocal_input_values)
        total_frames = int(max_audio / atpf)
        self.scheduler.set_timesteps(num_inference_steps, device=dev, mu=1)
        ts, sg = self.scheduler.timesteps, self.scheduler.sigmas
        T = (total_frames - 1) // 4 + 1
        shape = (1, 16, T, height // 8, width // 8)
        if latents is None:
            latents = torch.randn(shape, generator=generator, device=dev, dtype=torch.bfloat16)
        latents = latents.to(dev)
        if y is None or clip_context is None:
            clip_context, y = self._conditioning(cond_file_path, height, width, clip_length, torch.float32)
        tgt_f = (num_frames - 1) // 4 + 1
        seq_len = math.ceil((width // 8) * (height // 8) / 4 * tgt_f)
        feats = {}
        for (s, e, _) in window_schedule(T, fpb, overlap_window_length):
            sub = vocal_input_values[audio_window(s, e, T, atpf, max_audio)]
            a = self._audio_features(sub, sr).to(dev).float()
            feats[(s, e)] = torch.cat([torch.zeros_like(a), a, a]) if cfg else a
        lat = self.denoise(latents, y.to(dev), context, clip_context.to(dev), feats, ts, sg, clip_length=clip_length,
                           seq_len=seq_len, overlap=overlap_window_length, text_guide_scale=text_guide_scale,
                           audio_guide_scale=audio_guide_scale, scheme=overlapping_weight_scheme)
        if output_type == "latent":
            video = lat.float()
        else:
            self._decode_group_sync()
            video = torch.stack([self.vae.decode_clip(u.float(), post=True) for u in lat]).cpu()
        return WanI2VPipelineTalkingInferenceLongOutput(videos=video)
