#!/bin/bash
# V^T GEMM epilogue with 16-byte stores: the transposed-output kernel tests, then kbench gemmvar of the V^T shape
# (and cross-Q, the same shape with a row-major bf16 output) for this tree vs the previous library (build_ab/prev)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5t}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
export SA_KB_GVARS=0 SA_KB_SHAPES=v_t,cross_q
for rnd in 1 2; do
  for lib in default prev; do
    if [ $lib = default ]; then unset SA_LIB; else export SA_LIB=build_ab/$lib/libstableavatar_hip.so; fi
    timeout -k 10 180 python -u -m stableavatar_amd.kbench gemmvar 2>>gpurun_out/vt16_$TAG.err | sed "s/^{/{\"lib\": \"$lib\", \"round\": $rnd, /" >> gpurun_out/vt16_$TAG.jsonl
    rc=$?; [ $rc -ne 0 ] && exit $rc
  done
done
cat gpurun_out/vt16_$TAG.jsonl
