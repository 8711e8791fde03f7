#!/bin/bash
# v13 ping-pong on 32x32x16 MFMAs (kernel 8, V^T in P16 order) vs v6t (kernel 3): V^T kernel tests, then
# kbench attnvar in two processes (error vs fp32 on sampled rows; not bit-identical to kernel 3: fp32 row sums)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5v15}
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "v15 or v14" --timeout 60 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/tests_$TAG.log | tail -12; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  SA_KB_AVARS=3,8 timeout -k 10 200 python -u -m stableavatar_amd.kbench attnvar 2>>gpurun_out/attn_v15_$TAG.err | tail -1 >> gpurun_out/attn_v15_$TAG.jsonl
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
cat gpurun_out/attn_v15_$TAG.jsonl
