#!/bin/bash
# cross-attention after the spill fix (runtime ring slot) + the persistent kernel: kernel tests, then kbench cross3
# for SA_X3_KERNEL = 1 (4 waves), 2 (8 waves), 3 (persistent) of this tree vs the previous library (build_ab/prev,
# 4-wave kernel that spilled 152 VGPRs); interleaved processes, two rounds
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5p}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "cross3 or transposed" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for rnd in 1 2; do
  for v in prev 1 2 3; do
    if [ $v = prev ]; then export SA_LIB=build_ab/prev/libstableavatar_hip.so; unset SA_X3_KERNEL; else unset SA_LIB; export SA_X3_KERNEL=$v; fi
    timeout -k 10 120 python -u -m stableavatar_amd.kbench cross3 2>>gpurun_out/x3p_$TAG.err | sed "s/^{/{\"variant\": \"$v\", \"round\": $rnd, /" >> gpurun_out/x3p_$TAG.jsonl
    rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
cat gpurun_out/x3p_$TAG.jsonl
