"""ctypes binding of libstableavatar_hip.so (the C ABI declared in include/stableavatar_hip.h).

The product path has no fallback: if the library is missing or a symbol is absent, `lib()` raises.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("SA_LIB", PKG / "libstableavatar_hip.so"))
HEADER = PKG.parent / "include" / "stableavatar_hip.h"

# argument codes: p = pointer, i = int32, l = int64, f = float
SIGNATURES = {
    "sa_gemm_bf16": "pllpllpplliiiiipllplip",
    "sa_gemm_bf16_ex": "pllpllpplliiiiipllpliiip",
    "sa_gemm_bf16_panels": "pllpllpplliiiiipllpliiillp",
    "sa_gemm_panel_slack_rows": "",
    "sa_attn_fwd": "pppppiiiillllfip",
    "sa_attn_fwd_ex": "pppppiiiillllfiip",
    "sa_attn_fwd_map": "pppppiiiillllfiipp",
    "sa_attn_fwd_split": "pppppiiiillllfipiplp",
    "sa_layernorm_mod": "pliplipppplpiiifp",
    "sa_qk_rmsnorm_rope": "pliippiiifpiiiiiiip",
    "sa_qkv_pack": "plppiiifpiiiiiiipiiiip",
    "sa_patch_im2col": "plllipllliiiiipiip",
    "sa_unpatchify": "pliiiiiipip",
    "sa_timestep_embed": "piipp",
    "sa_small_linear_f32": "pliplppliiiip",
    "sa_mod_add": "ppllpiiiip",
    "sa_attn_small": "pppppiiiiillllfp",
    "sa_attn_small_split": "pppppiiiiillllfiplp",
    "sa_attn_cross3": "plpplipplippliiiipliiifp",
    "sa_flow_step": "pppiiiilifffiipip",
    "sa_gather_rows": "plpipllp",
    "sa_fill_f32": "plfp",
    "sa_cast_f32_bf16": "pplp",
    "sa_conv3d_cl": "piiiiippiiiiippiipp",
    "sa_vae_rmsnorm_silu": "pppliip",
    "sa_vae_input": "pilpppip",
    "sa_vae_output": "piilpip",
    "sa_conv3d_cl_down": "piiiiippiipp",
    "sa_vae_latent_out": "piilpppp",
    "sa_softmax_rows": "plpllifp",
    "sa_transpose_bf16": "pllplliiip",
    "sa_t5_rmsnorm": "pliplpiifp",
    "sa_t5_softmax_bias": "plpliiiipppp",
    "sa_t5_geglu": "plpllip",
    "sa_clip_preprocess": "piiipippp",
    "sa_clip_patch_im2col": "piiipip",
    "sa_cast_bf16_f32": "pplp",
    "sa_w2v_conv0_gn_gelu": "pipiiippfpip",
    "sa_conv1d_im2col": "pliiiiiiipiip",
    "sa_add_f32_bf16": "plpliip",
}
_CT = {"p": ctypes.c_void_p, "i": ctypes.c_int32, "l": ctypes.c_int64, "f": ctypes.c_float}

_lib = None
# a ktimer.KernelTimer while a measurement records per-kernel-class time (bench.py); None otherwise
_timer = None


def header_symbols() -> list[str]:
    """Function names declared in include/stableavatar_hip.h."""
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*int\s+(sa_\w+)\s*\(", txt, flags=re.M)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # torch first: its wheel bundles libamdhip64.so.7; if this library were dlopened before torch, the
    # soname would bind to /opt/rocm's copy and torch would then map a second HIP runtime, whose
    # streams and allocations ours cannot use (launches fail with hipErrorNoDevice)
    import torch  # noqa: F401
    if not LIB_PATH.exists():
        raise RuntimeError(f"libstableavatar_hip.so not built ({LIB_PATH}); run __graft_entry__.build()")
    L = ctypes.CDLL(str(LIB_PATH))
    for name in header_symbols():
        fn = getattr(L, name)  # AttributeError = missing export -> loud failure
        sig = SIGNATURES[name]
        fn.argtypes = [_CT[c] for c in sig]
        fn.restype = ctypes.c_int
    _lib = L
    return L


class KernelError(RuntimeError):
    pass


def call(name: str, *args):
    fn = getattr(lib(), name)
    t = _timer
    if t is not None:
        t.before(name, args)
    rc = fn(*args)
    if t is not None:
        t.after(name, args)
    if rc != 0:
        kind = "bad argument" if rc == 1 else f"launch failure (hipError {rc - 2000})"
        raise KernelError(f"{name}: {kind} (rc={rc})")
