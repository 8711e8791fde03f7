#!/bin/bash
# cross-attention: kernel tests, then the config-2 launch (kbench cross3) with the in-tree library and with abl/x3old
# (the previous body, one block-body copy per ring slot), alternating processes, 3 rounds
set -u
mkdir -p gpurun_out
scripts/gpustep.sh 600 gpurun_out/t_x3_r6e.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dit.py -m gpu -x -v --timeout 300 --timeout-method thread -k "cross3 or fused_cross"
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_x3_r6e.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  scripts/gpustep.sh 200 gpurun_out/x3_new_$i.log python -u -m stableavatar_amd.kbench cross3 || exit 1
  SA_LIB=abl/x3old/libstableavatar_hip.so scripts/gpustep.sh 200 gpurun_out/x3_old_$i.log python -u -m stableavatar_amd.kbench cross3 || exit 1
done
grep -h kernel gpurun_out/x3_new_*.log | sed 's/^/new /'; grep -h kernel gpurun_out/x3_old_*.log | sed 's/^/old /'
