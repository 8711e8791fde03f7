#!/bin/bash
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hbl -o run -- \
  python scripts/hipblaslt_probe.py > gpurun_out/hbl.log 2>&1
rc=$?; cat gpurun_out/hbl.log | grep -v amdgpu.ids; exit $rc
