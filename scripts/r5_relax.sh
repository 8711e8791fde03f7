#!/bin/bash
# relaxed first-step wait after a full-tile bf16 epilogue (default) vs the step's normal wait (SA_EPI_RELAX=0 build):
# GEMM GPU tests on the default library, kbench gemmvar in alternating processes, then the stamps build
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5rx}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_sp_kernels.py tests/test_gpu_dit.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
export SA_KB_SHAPES=qkv,cross_q,ffn_up SA_KB_GVARS=0
for r in 1 2; do
  timeout -k 10 200 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/gemm_relax_$TAG.err | sed 's/^{/{"lib": "relax", /' >> gpurun_out/gemm_relax_$TAG.jsonl || exit 1
  SA_LIB=build_ab/norelax/libstableavatar_hip.so timeout -k 10 200 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/gemm_relax_$TAG.err | sed 's/^{/{"lib": "norelax", /' >> gpurun_out/gemm_relax_$TAG.jsonl || exit 1
done
cat gpurun_out/gemm_relax_$TAG.jsonl
SA_LIB=build_ab/gstamps/libstableavatar_hip.so timeout -k 10 300 python -u scripts/gemm_stamps.py > gpurun_out/gemm_stamps_$TAG.jsonl 2>> gpurun_out/gemm_relax_$TAG.err
cat gpurun_out/gemm_stamps_$TAG.jsonl
