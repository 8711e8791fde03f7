#!/bin/bash
# GEMM A/B: s9 (kernel 6), s9 192-row (7), s10 deferred epilogue (10), s9 no-epilogue (8, 9) at the config-2 shapes
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5f}
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "gemm" > gpurun_out/gtests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gtests_$TAG.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
SA_KB_GVARS=${GVARS:-6,10,9} SA_KB_SHAPES=${SHAPES:-qkv,cross_q,ffn_up,o_proj} timeout -k 10 400 python -u -m stableavatar_amd.kbench gemmvar > gpurun_out/kb_gemm_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/kb_gemm_$TAG.jsonl; exit $rc
