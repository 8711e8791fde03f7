#!/bin/bash
# SP schedules: gloo world 2/4/8 + 14B vs goldens, RCCL degree-1 loopback, then per-rank compute by schedule
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4s}
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_sp.py \
  > gpurun_out/sp_tests_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error|overlap 4" gpurun_out/sp_tests_$TAG.log | tail -20; echo "sp tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_SPRC_MODES=${MODES:-2,3,4} timeout -k 10 400 python scripts/sp_rank_compute.py 1 2 4 8 > gpurun_out/sprc_$TAG.jsonl 2>&1
rc=$?; cat gpurun_out/sprc_$TAG.jsonl | grep -v amdgpu; exit $rc
