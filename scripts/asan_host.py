"""Host-side AddressSanitizer run of the C-ABI library (SURVEY.md §5 "Race detection / sanitizers").

Every csrc/*.hip is compiled with AddressSanitizer on the host side only (`-Xarch_host -fsanitize=address`: GPU ASan
is not available on this pool; the device code is built as usual and never launched here) and linked into one
executable with a driver generated from
include/stableavatar_hip.h: every entry point is called with NULL pointers (and positive sizes), then the
argument-validation paths that run host-side loops (GEMM column panels, transposed-output strides, attention
kernel selection, cross-attention frame checks) with fake, never-dereferenced device addresses.  Each call must
return SA_ERR_ARG before any HIP call; ASan aborts the run on any host memory error in that code.

usage: python scripts/asan_host.py   (exit 0 = clean; build products under build/asan/, git-ignored)"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "stableavatar_amd" / "csrc"
HEADER = ROOT / "include" / "stableavatar_hip.h"
OUT = ROOT / "build" / "asan"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O1", "-g", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Xarch_host", "-fsanitize=address",
         "-Xarch_host", "-fno-omit-frame-pointer", f"-I{CSRC}", f"-I{ROOT / 'include'}"]


def decls():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = []
    for m in re.finditer(r"\bint\s+(sa_\w+)\s*\(([^)]*)\)\s*;", txt, flags=re.S):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip() and p.strip() != "void"]
        out.append((m.group(1), params))
    return out


def null_call(name, params):
    args = []
    for p in params:
        if "*" in p:
            args.append("nullptr")
        elif p.startswith("int64_t"):
            args.append("64")
        elif p.startswith("float"):
            args.append("1.0f")
        else:
            args.append("1")
    return f"{name}({', '.join(args)})"


# argument-validation paths with non-null (fake, 256-B aligned, never dereferenced) device addresses
EXTRA = r'''
  void* P = (void*)0x100000;  // fake device address: the calls below must reject before touching it
  // GEMM: K not a multiple of 64; lda not a multiple of 8; a column-panel A whose panel count overflows the map
  CHECK(sa_gemm_bf16(P, 64, 0, P, 64, 0, nullptr, P, 64, 0, 64, 64, 96, 1, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr), 1);
  CHECK(sa_gemm_bf16(P, 63, 0, P, 64, 0, nullptr, P, 64, 0, 64, 64, 64, 1, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr), 1);
  CHECK(sa_gemm_bf16_panels(P, 1536, 0, P, 1536, 0, nullptr, P, 1536, 0, 8064, 1536, 1536, 1, 3, nullptr, 0, 0,
                            nullptr, 0, 0, 0, 0, 384, 1, nullptr), 1);   // residual epilogue without a residual
  CHECK(sa_gemm_bf16_panels(P, 1536, 0, P, 1536, 0, nullptr, P, 1536, 0, 8064, 1536, 1536, 2, 0, nullptr, 0, 0,
                            nullptr, 0, 0, 0, 0, 384, 8064L * 1536, nullptr), 1);  // panels need batch 1
  CHECK(sa_gemm_bf16_panels(P, 1536, 0, P, 1536, 0, nullptr, P, 1536, 0, 8064, 1536, 1536, 1, 0, nullptr, 0, 0,
                            nullptr, 0, 0, 0, 0, 100, 8064L * 1536, nullptr), 1);  // panel width % 64
  CHECK(sa_gemm_bf16_ex(P, 64, 0, P, 64, 0, nullptr, P, 60, 0, 64, 64, 128, 1, 7, nullptr, 0, 0, nullptr, 0, 0, 0,
                        0, nullptr), 1);  // transposed P32 output: ldc < M rounded to 32
  CHECK(sa_gemm_bf16_ex(P, 64, 0, P, 64, 0, nullptr, P, 64, 0, 64, 64, 128, 1, 0, nullptr, 0, 0, nullptr, 0, 0, 99,
                        0, nullptr), 1);  // unknown kernel id
  // attention: head_dim 64; unaligned strides; V^T kernel with a stride not a multiple of 64; kernel id past the last
  int32_t segs[4] = {0, 64, 0, 64};
  CHECK(sa_attn_fwd(P, P, P, P, segs, 1, 64, 1, 64, 128, 128, 128, 128, 1.0f, 0, nullptr), 1);
  CHECK(sa_attn_fwd(P, P, P, P, segs, 1, 64, 1, 128, 130, 128, 128, 128, 1.0f, 0, nullptr), 1);
  CHECK(sa_attn_fwd_ex(P, P, P, P, segs, 1, 64, 1, 128, 128, 128, 96, 128, 1.0f, 0, 3, nullptr), 1);
  CHECK(sa_attn_fwd_ex(P, P, P, P, segs, 1, 64, 1, 128, 128, 128, 128, 128, 1.0f, 0, 9, nullptr), 1);
  // fused cross-attention: tokens per frame not a multiple of 256; the frames do not cover the queries
  CHECK(sa_attn_cross3(P, 1536, P, P, 3072, 512, P, P, 3072, 257, P, P, 3072, 32, 1000, 21, 0, P, 1536, 3, 21000, 12,
                       1.0f, nullptr), 1);
  CHECK(sa_attn_cross3(P, 1536, P, P, 3072, 512, P, P, 3072, 257, P, P, 3072, 32, 1024, 2, 0, P, 1536, 3, 21504, 12,
                       1.0f, nullptr), 1);
  CHECK(sa_gemm_panel_slack_rows(), 256);
'''


def driver_source():
    lines = ["#include <cstdio>", "#include <cstdint>", '#include "stableavatar_hip.h"',
             "static int fails = 0;",
             "#define CHECK(call, want) do { int rc_ = (call); if (rc_ != (want)) { "
             "std::printf(\"FAIL %s -> %d (want %d)\\n\", #call, rc_, (want)); ++fails; } } while (0)",
             "int main() {"]
    n = 0
    for name, params in decls():
        if not params:
            continue
        lines.append(f"  CHECK({null_call(name, params)}, 1);")
        n += 1
    lines.append(EXTRA)
    lines.append(f'  std::printf("asan_host: %d null-argument calls + validation paths, %d failures\\n", {n}, fails);')
    lines.append("  return fails ? 1 : 0;")
    lines.append("}")
    return "\n".join(lines) + "\n"


def build():
    OUT.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))

    def comp(src):
        obj = OUT / (src.stem + ".o")
        deps = [src, CSRC / "common.h", HEADER, Path(__file__)]
        if not (obj.exists() and all(obj.stat().st_mtime >= d.stat().st_mtime for d in deps)):
            subprocess.run([HIPCC, *FLAGS, "-c", str(src), "-o", str(obj)], check=True, capture_output=True, text=True)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(comp, srcs))
    drv = OUT / "driver.cpp"
    drv.write_text(driver_source())
    exe = OUT / "asan_host"
    subprocess.run([HIPCC, *FLAGS, "-x", "hip", "-c", str(drv), "-o", str(OUT / "driver.o")], check=True,
                   capture_output=True, text=True)
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-Xarch_host", "-fsanitize=address", str(OUT / "driver.o"),
                        *map(str, objs),
                        "-o", str(exe)], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"link failed:\n{r.stderr[-3000:]}")
    return exe


def run():
    exe = build()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    return subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)


if __name__ == "__main__":
    r = run()
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-4000:])
    sys.exit(r.returncode)
