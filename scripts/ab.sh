#!/bin/bash
# A/B pass: kernel tests of the candidate variants, kernel timings, attention HBM traffic.
set -u
mkdir -p gpurun_out
tag=${1:-ab}
SA_GEMM_VARIANT=4 scripts/gpustep.sh 300 gpurun_out/t_$tag.log python -m pytest tests/test_gpu_kernels.py tests/test_gpu_dit.py -q; rc=$?; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/kb_$tag.log python -m stableavatar_amd.kbench gemmvar attnvar; rc=$?; echo "kb rc=$rc"
[ $rc -ne 0 ] && exit $rc
scripts/pmc_attn.sh
