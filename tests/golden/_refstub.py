"""Minimal stand-ins for the `diffusers` symbols the reference modules import, so that
/root/reference can be imported on CPU in the survey/build container to GENERATE golden vectors
(SURVEY.md Appendix B).  Used only by gen_golden.py; never imported by tests, the package,
smoke() or bench.py, and never shipped to the GPU box as a dependency."""
import contextlib
import functools
import inspect
import logging
import sys
import types

import numpy as np
import torch

REF = "/root/reference"


def _mod(n):
    m = types.ModuleType(n)
    sys.modules[n] = m
    return m


class FlowMatchEulerDiscreteScheduler:
    """Restated diffusers 0.30.x FlowMatchEulerDiscreteScheduler (package absent offline:
    parity of this piece is unpinned by any reference test)."""
    order = 1

    def __init__(self, num_train_timesteps=1000, shift=1.0, use_dynamic_shifting=False, **_):
        N = num_train_timesteps
        s = torch.from_numpy(np.linspace(1, N, N, dtype=np.float32)[::-1].copy() / N)
        s = shift * s / (1 + (shift - 1) * s)
        self.N, self.shift = N, shift
        self.timesteps = s * N
        self.sigmas = s
        self.sigma_min, self.sigma_max, self._step_index = s[-1].item(), s[0].item(), None
        self.config = types.SimpleNamespace(num_train_timesteps=N, shift=shift, use_dynamic_shifting=False)

    def set_timesteps(self, num_inference_steps=None, device=None, mu=None, **_):
        t = np.linspace(self.sigma_max * self.N, self.sigma_min * self.N, num_inference_steps)
        s = t / self.N
        s = self.shift * s / (1 + (self.shift - 1) * s)
        s = torch.from_numpy(s).to(dtype=torch.float32, device=device)
        self.timesteps = s * self.N
        self.sigmas = torch.cat([s, s.new_zeros(1)])
        self._step_index = None

    def step(self, model_output, timestep, sample, return_dict=True, **_):
        if self._step_index is None:
            idx = (self.timesteps == timestep).nonzero()
            self._step_index = idx[1 if len(idx) > 1 else 0].item()
        sample = sample.to(torch.float32)
        out = sample + (self.sigmas[self._step_index + 1] - self.sigmas[self._step_index]) * model_output
        out = out.to(model_output.dtype)
        self._step_index += 1
        return (out,)


def install():
    if "diffusers" in sys.modules and getattr(sys.modules["diffusers"], "_sa_stub", False):
        return
    import transformers  # noqa: F401  (probes torchvision before the stubs below)

    d = _mod("diffusers")
    d._sa_stub = True
    cu = _mod("diffusers.configuration_utils")

    class ConfigMixin:
        @classmethod
        def from_config(cls, config, **kw):
            p = set(inspect.signature(cls.__init__).parameters) - {"self"}
            return cls(**{k: v for k, v in {**config, **kw}.items() if k in p})

    def register_to_config(fn):
        @functools.wraps(fn)
        def w(self, *a, **kw):
            fn(self, *a, **kw)
            b = inspect.signature(fn).bind(self, *a, **kw)
            b.apply_defaults()
            cfg = dict(b.arguments)
            cfg.pop("self")
            self.config = types.SimpleNamespace(**cfg)
        return w

    cu.ConfigMixin, cu.register_to_config = ConfigMixin, register_to_config
    _mod("diffusers.loaders")
    _mod("diffusers.loaders.single_file_model").FromOriginalModelMixin = type("F", (), {})
    _mod("diffusers.models")

    class ModelMixin(torch.nn.Module):
        @property
        def dtype(self):
            return next(self.parameters()).dtype

        @property
        def device(self):
            return next(self.parameters()).device

    _mod("diffusers.models.modeling_utils").ModelMixin = ModelMixin
    ut = _mod("diffusers.utils")
    ut.is_torch_version = lambda *a: True
    ut.logging = types.SimpleNamespace(get_logger=logging.getLogger)

    class BaseOutput:
        def __init__(self, **kw):
            self.__dict__.update(kw)

    ut.BaseOutput = BaseOutput
    ut.replace_example_docstring = lambda doc: (lambda f: f)
    _mod("diffusers.utils.accelerate_utils").apply_forward_hook = lambda f: f
    _mod("diffusers.utils.torch_utils").randn_tensor = (
        lambda shape, generator=None, device=None, dtype=None: torch.randn(shape, generator=generator,
                                                                            dtype=dtype).to(device))
    _mod("diffusers.models.autoencoders")
    vae = _mod("diffusers.models.autoencoders.vae")

    class DecoderOutput:
        def __init__(self, sample):
            self.sample = sample

    class DiagonalGaussianDistribution:
        def __init__(self, h):
            self.mean, self.logvar = torch.chunk(h, 2, dim=1)

        def mode(self):
            return self.mean

    vae.DecoderOutput, vae.DiagonalGaussianDistribution = DecoderOutput, DiagonalGaussianDistribution

    class AutoencoderKLOutput:
        def __init__(self, latent_dist):
            self.latent_dist = latent_dist

        def __getitem__(self, i):
            return [self.latent_dist][i]

    _mod("diffusers.models.modeling_outputs").AutoencoderKLOutput = AutoencoderKLOutput
    _mod("diffusers.models.embeddings").get_1d_rotary_pos_embed = None
    d.FlowMatchEulerDiscreteScheduler = FlowMatchEulerDiscreteScheduler
    _mod("diffusers.schedulers").FlowMatchEulerDiscreteScheduler = FlowMatchEulerDiscreteScheduler
    cb = _mod("diffusers.callbacks")
    cb.MultiPipelineCallbacks = type("MultiPipelineCallbacks", (), {})
    cb.PipelineCallback = type("PipelineCallback", (), {})
    _mod("diffusers.image_processor").VaeImageProcessor = lambda **kw: None
    _mod("diffusers.video_processor").VideoProcessor = lambda **kw: None
    _mod("diffusers.pipelines")

    class _PB:
        def update(self):
            pass

    class DiffusionPipeline:
        def register_modules(self, **kw):
            for k, v in kw.items():
                setattr(self, k, v)

        @property
        def _execution_device(self):
            return torch.device("cpu")

        def progress_bar(self, total=None):
            return contextlib.nullcontext(_PB())

        def maybe_free_model_hooks(self):
            pass

    _mod("diffusers.pipelines.pipeline_utils").DiffusionPipeline = DiffusionPipeline
    for n in ("skimage", "skimage.color", "torchvision", "torchvision.transforms",
              "torchvision.transforms.functional"):
        if n not in sys.modules:
            _mod(n)
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
    sys.modules["skimage"].color = sys.modules["skimage.color"]
    if REF not in sys.path:
        sys.path.insert(0, REF)
    wu = types.ModuleType("wan.utils")
    wu.__path__ = [REF + "/wan/utils"]
    import wan  # noqa: F401
    sys.modules["wan.utils"] = wu
