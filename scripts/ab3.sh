#!/bin/bash
set -u
mkdir -p gpurun_out
tag=${1:-ab3}
scripts/gpustep.sh 300 gpurun_out/t_$tag.log python -m pytest tests/test_gpu_kernels.py -q; rc=$?; echo "tests v3 rc=$rc"
[ $rc -ne 0 ] && exit $rc
SA_GEMM_VARIANT=4 scripts/gpustep.sh 300 gpurun_out/t4_$tag.log python -m pytest tests/test_gpu_kernels.py -q -k gemm; rc=$?; echo "tests v4 rc=$rc"
[ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/kb_$tag.log python -m stableavatar_amd.kbench gemmvar attnvar; echo "kb rc=$?"
