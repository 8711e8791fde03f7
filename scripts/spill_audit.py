"""Per-kernel register use and spills of every csrc/*.hip (hipcc -Rpass-analysis=kernel-resource-usage, gfx950).
usage: python scripts/spill_audit.py [source stems...]  -> one line per kernel; exits 1 if any VGPR spills to scratch"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "stableavatar_amd" / "csrc"


def audit(stem):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{CSRC}",
                        f"-I{ROOT / 'include'}", "-c", str(CSRC / f"{stem}.hip"), "-o", "/tmp/_spill_audit.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"kernel": re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", v)[:60]}
            out.append(cur)
        elif cur is not None:
            cur[k] = v
    return out


if __name__ == "__main__":
    stems = sys.argv[1:] or sorted(p.stem for p in CSRC.glob("*.hip"))
    bad = 0
    for s in stems:
        for k in audit(s):
            sp = int(k.get("VGPRs Spill", 0))
            bad += sp > 0
            print(f"{s:12s} {k['kernel']:60s} vgpr {k.get('VGPRs')} agpr {k.get('AGPRs')} "
                  f"spill {sp} sgpr_spill {k.get('SGPRs Spill')} occ {k.get('Occupancy [waves/SIMD]')}")
    sys.exit(1 if bad else 0)
