set -u
mkdir -p gpurun_out
true || scripts/gpustep.sh 600 gpurun_out/t_ah.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -v -x --timeout 300 --timeout-method thread -k "gemm or cross3" || { tail -30 gpurun_out/t_ah.log; exit 1; }
tail -3 gpurun_out/t_ah.log
true || SA_LIB=build_ab/lib_ah16.so scripts/gpustep.sh 600 gpurun_out/t_ah16.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -m gpu -v -x --timeout 300 --timeout-method thread -k "gemm" || { tail -30 gpurun_out/t_ah16.log; exit 1; }
tail -3 gpurun_out/t_ah16.log
SA_KB_GVARS=2 SA_KB_SHAPES=o_proj,ffn_down,cross_q scripts/ab_libs.sh ah "build_ab/lib_head.so build_ab/lib_ah8.so build_ab/lib_ah12.so build_ab/lib_ah16.so" gemmvar cross3 ditvar
