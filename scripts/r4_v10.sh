#!/bin/bash
# v10 self-attention: kernel tests, then an interleaved A/B against v6 (kbench attnvar, config-2 launch)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-v10}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k attention \
  > gpurun_out/t_$TAG.log 2>&1
rc=$?; grep -E "passed|failed|Error" gpurun_out/t_$TAG.log | tail -5; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=${AVARS:-1,3} timeout -k 10 300 python -m stableavatar_amd.kbench attnvar > gpurun_out/kb_$TAG.jsonl 2> gpurun_out/kb_$TAG.err
rc=$?; cat gpurun_out/kb_$TAG.jsonl; tail -3 gpurun_out/kb_$TAG.err; exit $rc
