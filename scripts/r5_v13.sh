#!/bin/bash
# V^T attention kernel tests (v6t, v12, v13) then the attention A/B (kbench attnvar) on the same box
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "vt_" > gpurun_out/ktests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/ktests_$TAG.log; echo "ktests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=${AVARS:-3,5} timeout -k 10 300 python -u -m stableavatar_amd.kbench attnvar > gpurun_out/kb_attn_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_attn_$TAG.jsonl; exit $rc
