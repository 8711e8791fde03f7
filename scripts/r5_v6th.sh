#!/bin/bash
# self-attention with the K/V DMA issued by waves 4-7 only (kernel 7) vs v6t (kernel 3): V^T kernel tests, kbench
# attnvar (two processes), and the barrier / DMA-wait anatomy of both from the SA_V6T_STAMPS build
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "vt_kernels or vt_spike" --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  SA_KB_AVARS=3,7 timeout -k 10 200 python -u -m stableavatar_amd.kbench attnvar 2>>gpurun_out/attn_v6th_$TAG.err | tail -1 >> gpurun_out/attn_v6th_$TAG.jsonl
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
for k in 3 7; do
  SA_STAMPS_KERNEL=$k SA_LIB=build_ab/v6tstamps/libstableavatar_hip.so timeout -k 10 200 python -u scripts/v6t_stamps.py >> gpurun_out/attn_v6th_$TAG.jsonl 2>>gpurun_out/attn_v6th_$TAG.err
  rc=$?; [ $rc -ne 0 ] && exit $rc
done
cat gpurun_out/attn_v6th_$TAG.jsonl
