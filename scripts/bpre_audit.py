"""Disassembly audit of the bf16 GEMM epilogue's bias preload: s8_bias_preload issues the tile's bias loads
as inline-asm buffer_load_dwordx4 into bpre[0..7], which hipcc does not count (cdna_hip_programming.md §5.7 item 1); the
first K step's counted vmcnt wait retires them.  Correctness needs that NO compiler instruction between the loads and
that wait reads, writes, copies or spills a bpre register.  This compiles gemm.hip for gfx950 (--save-temps), finds
every preload group in every kernel, and scans to the first s_waitcnt vmcnt: any instruction outside an asm statement
naming a bpre VGPR there (a copy, a spill or a use) is a violation, except on the K loop's zero-trip path, which the ABI
makes dead (K <= 0 is rejected).
usage: python scripts/bpre_audit.py  -> one line per kernel with a preload; exit 1 on a violation or if none found"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "stableavatar_amd" / "csrc"
LOAD = re.compile(r"^\s*buffer_load_dwordx4 v\[(\d+):(\d+)\], v\d+, s\[\d+:\d+\], 0 offen\s*$")
VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs_of(line):
    out = set()
    for a, b, c in VREG.findall(line):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


def _scan(asm_lines, start, regs, labels):
    """(violations, zero-trip reads) on every control-flow path from line `start` to the first s_waitcnt vmcnt
    (s_branch followed, s_cbranch both ways).  A read of a bpre register reached without any MFMA on the path is the
    K loop's zero-trip path (nk == 0), dead at run time: the ABI rejects K <= 0 (sa_gemm_bf16_panels / _ex)."""
    viol, zero_trip, work, seen = [], [], [(start, False)], set()
    n = len(asm_lines)
    while work:
        k, mfma = work.pop()
        in_asm = False
        while k < n and (k, mfma) not in seen:
            seen.add((k, mfma))
            t = asm_lines[k].strip()
            if ";;#ASMSTART" in t:
                in_asm = True
            elif ";;#ASMEND" in t:
                in_asm = False
            elif t.startswith("s_endpgm"):
                break
            elif t and not t.startswith(";") and not t.startswith("."):
                if t.startswith("s_waitcnt") and "vmcnt" in t:
                    break
                if t.startswith("v_mfma"):
                    mfma = True
                if t.startswith("s_branch "):
                    k = labels[t.split()[1]]
                    continue
                if t.startswith("s_cbranch"):
                    work.append((labels[t.split()[1]], mfma))
                elif not in_asm and regs & regs_of(t):
                    (viol if mfma else zero_trip).append(t)
            k += 1
    return viol, zero_trip


def audit(asm_lines):
    """-> list of (kernel, bpre registers, violations, loads).  A preload group is 8 consecutive asm statements
    buffer_load_dwordx4 ... offen (no lds) with the address arithmetic of the later loads between them (checked against
    the registers already loaded); after the 8th load every control-flow path is scanned to its first s_waitcnt vmcnt."""
    labels = {}
    for k, ln in enumerate(asm_lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = k
    res, kern = [], None
    i, n = 0, len(asm_lines)
    while i < n:
        ln = asm_lines[i]
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            kern = m.group(1)
        if not (";;#ASMSTART" in ln and i + 1 < n and LOAD.match(asm_lines[i + 1])):
            i += 1
            continue
        regs, cnt, viol, in_asm = set(), 0, [], False
        k = i
        while k < n and cnt < 8:
            t = asm_lines[k].strip()
            if ";;#ASMSTART" in t:
                in_asm = True
            elif ";;#ASMEND" in t:
                in_asm = False
            elif t and not t.startswith(";") and not t.startswith("."):
                lm = LOAD.match(asm_lines[k])
                if in_asm and lm:
                    a, b = map(int, lm.groups())
                    regs.update(range(a, b + 1))
                    cnt += 1
                elif t.startswith("s_") and ("branch" in t or "waitcnt" in t):
                    break  # not a straight-line group
                elif t.startswith("scratch_") or (not in_asm and regs & regs_of(t)):
                    viol.append(t)
            k += 1
        if cnt == 8:
            v2, zt = _scan(asm_lines, k, regs, labels)
            res.append((kern, sorted(regs), viol + v2, cnt, len(zt)))
        i = k
    return res


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{CSRC}",
                            f"-I{ROOT / 'include'}", "-c", str(CSRC / "gemm.hip"), "-o", f"{td}/g.o", "--save-temps"],
                           capture_output=True, text=True, cwd=td)
        if r.returncode:
            print(r.stderr[-2000:])
            sys.exit(2)
        s = next(Path(td).glob("gemm-hip-amdgcn-amd-amdhsa-gfx950.s")).read_text().split("\n")
    res = audit(s)
    bad = 0
    for kern, regs, viol, cnt, zt in res:
        print(f"{kern[:70]:70s} {cnt} loads, bpre {len(regs)} VGPRs, {zt} reads on the zero-trip path: "
              f"{'OK' if not viol else 'VIOLATION ' + '; '.join(viol[:3])}")
        bad += bool(viol) or cnt != 8
    if not res:
        print("no bias preload group found")
    sys.exit(1 if bad or not res else 0)
