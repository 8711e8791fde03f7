"""Host-side AddressSanitizer run of the C-ABI library's argument validation (SURVEY.md §5 "Race detection /
sanitizers"): scripts/asan_host.py builds every csrc/*.hip with -Xarch_host -fsanitize=address and runs a driver
that calls each entry point of include/stableavatar_hip.h with NULL pointers plus the host-side validation paths;
every call must be rejected (SA_ERR_ARG) before any HIP call, with no ASan report.  No GPU."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="hipcc not available")
def test_asan_host_validation_paths():
    r = subprocess.run([sys.executable, str(ROOT / "scripts" / "asan_host.py")], capture_output=True, text=True,
                       timeout=1200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
    assert "AddressSanitizer" not in r.stderr
