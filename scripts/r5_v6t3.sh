#!/bin/bash
# self-attention on a 3-stage K/V ring (kernel 6) vs v6t (kernel 3): the V^T kernel tests, then kbench attnvar
# (config-2 launch, interleaved in one process, bit-identity vs kernel 3) in two processes
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5z}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "vt_kernels or vt_spike" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  SA_KB_AVARS=3,6 timeout -k 10 200 python -u -m stableavatar_amd.kbench attnvar 2>>gpurun_out/attn_v6t3_$TAG.err | tail -1 >> gpurun_out/attn_v6t3_$TAG.jsonl
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
cat gpurun_out/attn_v6t3_$TAG.jsonl
