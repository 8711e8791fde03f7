#!/bin/bash
# attention kernel tests (V^T forms incl. the ping-pong v13) + attention A/B, then the GEMM s10 A/B
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "vt_" > gpurun_out/ktests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/ktests_$TAG.log; echo "ktests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=${AVARS:-3,5} timeout -k 10 300 python -u -m stableavatar_amd.kbench attnvar > gpurun_out/kb_attn_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_attn_$TAG.jsonl; echo "kb attn rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_KB_GVARS=${GVARS:-6,10} SA_KB_SHAPES=${SHAPES:-qkv,cross_q,ffn_up,o_proj} timeout -k 10 400 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_gemm_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_gemm_$TAG.jsonl; exit $rc
