set -u
mkdir -p gpurun_out
scripts/gpustep.sh 600 gpurun_out/t_r6b.log python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread -k "attention or transposed"
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_r6b.log; [ $rc -ne 0 ] && exit $rc
SA_KB_AVARS=3,4 scripts/gpustep.sh 300 gpurun_out/kb_attn_r6b.log python -u -m stableavatar_amd.kbench attnvar
rc=$?; echo "kb rc=$rc"; tail -2 gpurun_out/kb_attn_r6b.log; exit $rc
