"""In-tree build of libstableavatar_hip.so (gfx950) with hipcc; no cmake, no JIT cache.

`python -m stableavatar_amd.build` (or __graft_entry__.build()) compiles every csrc/*.hip to an
object under build/ in parallel and links them into stableavatar_amd/libstableavatar_hip.so,
which travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "obj"
LIB = PKG / "libstableavatar_hip.so"
ARCH = os.environ.get("SA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
          f"-I{CSRC}", f"-I{PKG.parent / 'include'}"]


# per-source extra flags (none at present: -fno-slp-vectorize on attention.hip was measured slower,
# it pushes the 16x16x32 attention into scratch spills and costs the 32x32x16 one 4 %)
EXTRA: dict[str, list[str]] = {}


def _compile(src: Path) -> Path:
    obj = BUILD / (src.stem + ".o")
    deps = [src, *CSRC.glob("*.h"), Path(__file__)]
    if obj.exists() and all(obj.stat().st_mtime >= d.stat().st_mtime for d in deps if d.exists()):
        return obj
    cmd = [HIPCC, *CFLAGS, *EXTRA.get(src.stem, []), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr}")
    return obj


def build(verbose: bool = True) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with cf.ThreadPoolExecutor(max_workers=max(jobs, 1)) as ex:
        objs = list(ex.map(_compile, srcs))
    if LIB.exists() and all(LIB.stat().st_mtime >= o.stat().st_mtime for o in objs):
        if verbose:
            print(f"[build] up to date: {LIB}")
        return LIB
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[build] linked {LIB} from {len(objs)} objects")
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
