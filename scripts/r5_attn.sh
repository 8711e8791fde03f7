#!/bin/bash
# round 5: attention kernel tests (incl. V^T forms, NaN-tail) + the config-2 attention A/B
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "attention or transposed" > gpurun_out/ktests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/ktests_$TAG.log; echo "ktests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=${AVARS:-1,3,4} timeout -k 10 300 python -u -m stableavatar_amd.kbench attnvar > gpurun_out/kb_attn_$TAG.jsonl 2>&1
rc=$?; cat gpurun_out/kb_attn_$TAG.jsonl | grep -v amdgpu.ids; echo "kbench rc=$rc"; exit $rc
