set -u
mkdir -p gpurun_out
scripts/gpustep.sh 600 gpurun_out/t_x3.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 300 --timeout-method thread -k "attention or cross or dit_block_fullsize or ragged" || { tail -30 gpurun_out/t_x3.log; exit 1; }
tail -2 gpurun_out/t_x3.log
for i in 1 2; do
  SA_LIB=build_ab/lib_head.so scripts/gpustep.sh 300 gpurun_out/x3_head_$i.log python -u -m stableavatar_amd.kbench cross3 || exit 1
  scripts/gpustep.sh 300 gpurun_out/x3_new_$i.log python -u -m stableavatar_amd.kbench cross3 || exit 1
done
grep -h kernel gpurun_out/x3_*.log
