#!/bin/bash
set -u
mkdir -p gpurun_out
tag=${1:-ab4}
SA_ATTN_VARIANT=5 scripts/gpustep.sh 300 gpurun_out/t_$tag.log python -m pytest tests/test_gpu_kernels.py tests/test_gpu_dit.py -q; rc=$?; echo "tests v5 rc=$rc"
[ $rc -eq 99 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/kb_$tag.log python -m stableavatar_amd.kbench attnvar; echo "kb rc=$?"
