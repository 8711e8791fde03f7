"""C-ABI checks that need no GPU: the library builds/loads, exports every symbol declared in
include/stableavatar_hip.h, and the ctypes signatures match the header's parameter lists."""
import re
import subprocess

import pytest

from stableavatar_amd import _lib


def _header_decls():
    txt = _lib.HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    out = {}
    for m in re.finditer(r"\bint\s+(sa_\w+)\s*\(([^)]*)\)\s*;", txt, flags=re.S):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip() and p.strip() != "void"]
        codes = ""
        for p in params:
            if "*" in p:
                codes += "p"
            elif p.startswith("int64_t"):
                codes += "l"
            elif p.startswith("float"):
                codes += "f"
            elif p.startswith("int"):
                codes += "i"
            else:
                raise AssertionError(f"unknown param type: {p}")
        out[m.group(1)] = codes
    return out


def test_signatures_match_header():
    decls = _header_decls()
    assert decls, "no declarations parsed"
    assert set(decls) == set(_lib.header_symbols())
    for name, codes in decls.items():
        assert _lib.SIGNATURES.get(name) == codes, (name, codes, _lib.SIGNATURES.get(name))


def test_library_exports_every_symbol():
    if not _lib.LIB_PATH.exists():
        pytest.skip("library not built (run __graft_entry__.build())")
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (sa_\w+)", nm))
    missing = set(_lib.header_symbols()) - exported
    assert not missing, missing
    L = _lib.lib()  # torch's HIP runtime first, then the library (see _lib.lib)
    for name in _lib.header_symbols():
        assert getattr(L, name) is not None


def test_bad_arguments_are_rejected_without_gpu_work():
    """argument validation happens before any HIP call: NULL pointers return rc=1"""
    if not _lib.LIB_PATH.exists():
        pytest.skip("library not built")
    L = _lib.lib()
    assert L.sa_gemm_bf16(None, 64, 0, None, 64, 0, None, None, 64, 0, 1, 1, 64, 1, 0, None, 0, 0, None, 0, 0,
                          None) == 1
    assert L.sa_attn_fwd(None, None, None, None, None, 1, 1, 1, 128, 128, 128, 128, 128, 1.0, 0, None) == 1
    with pytest.raises(_lib.KernelError):
        _lib.call("sa_fill_f32", None, 10, 0.0, None)


def test_encoder_entry_points_reject_bad_arguments():
    """VAE-encode entry points (sa_conv3d_cl_down, sa_vae_latent_out) validate before launching."""
    if not _lib.LIB_PATH.exists():
        pytest.skip("library not built")
    L = _lib.lib()
    one = 16  # any non-null host address: rejected before it is dereferenced
    assert L.sa_conv3d_cl_down(None, 1, 8, 8, 32, 1, one, one, 32, 96, one, None) == 1      # null input
    assert L.sa_conv3d_cl_down(one, 1, 8, 8, 32, 3, one, one, 32, 96, one, None) == 1       # unknown mode
    assert L.sa_conv3d_cl_down(one, 1, 7, 8, 32, 1, one, one, 32, 96, one, None) == 1       # odd H for stride 2
    assert L.sa_conv3d_cl_down(one, 1, 8, 8, 3, 1, one, one, 32, 96, one, None) == 1        # Cin % 32
    assert L.sa_vae_latent_out(None, 32, 16, 64, one, one, one, None) == 1
    assert L.sa_vae_latent_out(one, 16, 16, 64, one, one, one, None) == 1                   # 2*Cz > C_stride


def test_gemm_rejects_empty_k_without_gpu_work():
    """K <= 0 is refused at the ABI: the persistent GEMM's bias preload (inline-asm loads retired by the first K step's
    counted wait) relies on every tile running at least one K step (scripts/bpre_audit.py)"""
    if not _lib.LIB_PATH.exists():
        pytest.skip("library not built")
    import ctypes
    L = _lib.lib()
    buf = ctypes.create_string_buffer(4096)
    p = ctypes.addressof(buf) + (-ctypes.addressof(buf)) % 16  # 16-byte aligned, never dereferenced on this path
    for K in (0, -128):
        assert L.sa_gemm_bf16(p, 128, 0, p, 128, 0, None, p, 64, 0, 64, 64, K, 1, 0, None, 0, 0, None, 0, 0,
                              None) == 1


@pytest.mark.timeout(600)
def test_bias_preload_disassembly_audit():
    """no compiler instruction copies, spills or reads the inline-asm bias preload registers before the
    first K step's counted vmcnt wait, in every bf16 / GELU persistent-GEMM instantiation (gfx950 disassembly)"""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "bpre_audit.py")], capture_output=True, text=True)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.count(": OK") >= 8
