#!/bin/bash
# bf16 GEMM epilogue v2 (bias preloaded at the tile's top, no strip write->read wait) vs the round-4 form (SA_EPI_V2=0
# build): GEMM GPU tests on the default (v2) library, then kbench gemmvar in alternating processes
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5e2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_sp_kernels.py -m gpu -x -q -k "gemm or linear" --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
export SA_KB_SHAPES=${SHAPES:-qkv,cross_q,ffn_up} SA_KB_GVARS=0
for r in 1 2; do
  timeout -k 10 200 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/gemm_epiv2_$TAG.err | sed "s/^{/{\"lib\": \"v2\", /" >> gpurun_out/gemm_epiv2_$TAG.jsonl || exit 1
  SA_LIB=build_ab/epiv1/libstableavatar_hip.so timeout -k 10 200 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/gemm_epiv2_$TAG.err | sed 's/^{/{"lib": "v1", /' >> gpurun_out/gemm_epiv2_$TAG.jsonl || exit 1
done
cat gpurun_out/gemm_epiv2_$TAG.jsonl || true
SA_LIB=build_ab/gstamps/libstableavatar_hip.so timeout -k 10 300 python -u scripts/gemm_stamps.py > gpurun_out/gemm_stamps_$TAG.jsonl 2>> gpurun_out/gemm_epiv2_$TAG.err
cat gpurun_out/gemm_stamps_$TAG.jsonl
