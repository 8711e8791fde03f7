#!/bin/bash
# SP: the GPU SP / DiT tests (gloo world 2/4/8 + 14B U8 vs the goldens, RCCL degree-1 loopback), then the per-rank
# compute with transfers stubbed (schedule 4) at N = 1, 2, 4, 8.  usage: scripts/r6_sp.sh <tag>
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 900 gpurun_out/sp_tests_$tag.log python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_sp.py tests/test_gpu_dit.py tests/test_gpu_dit14.py
rc=$?; grep -E "passed|failed" gpurun_out/sp_tests_$tag.log | tail -3; echo "sp tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_SPRC_MODES=${MODES:-4} scripts/gpustep.sh 500 gpurun_out/sprc_$tag.jsonl python -u scripts/sp_rank_compute.py 1 2 4 8
rc=$?; grep -v amdgpu gpurun_out/sprc_$tag.jsonl; exit $rc
