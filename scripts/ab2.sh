#!/bin/bash
set -u
mkdir -p gpurun_out
tag=${1:-ab2}
scripts/gpustep.sh 400 gpurun_out/t_$tag.log python -m pytest tests/test_gpu_kernels.py tests/test_gpu_dit.py -q; rc=$?; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
SA_CROSS3=1 scripts/gpustep.sh 300 gpurun_out/kbd1_$tag.log python -m stableavatar_amd.kbench dit; echo "dit cross3 rc=$?"
SA_CROSS3=0 scripts/gpustep.sh 300 gpurun_out/kbd0_$tag.log python -m stableavatar_amd.kbench dit; echo "dit 3-launch rc=$?"
scripts/pmc_sq.sh
