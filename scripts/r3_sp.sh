#!/bin/bash
# round-3 fused SP exchange check: kernel bit-identity, SP vs goldens (gloo ranks on one GPU + RCCL degree 1),
# then (optional, $1 == full) PMC traffic of bench.py's own launches and the case-1 windowed bench
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_sp_kernels.py tests/test_gpu_sp.py tests/test_gpu_kernels.py tests/test_gpu_dit.py tests/test_gpu_dit14.py \
  -x -v --timeout 300 --timeout-method thread > gpurun_out/t_sp_r3k.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_sp_r3k.log; [ $rc -ne 0 ] && exit $rc
[ "${1:-}" != full ] && exit 0
scripts/pmc_bench.sh; rc=$?; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 500 gpurun_out/bench_case1_r3j.log python -u bench.py --video-frames 165 --steps 1 --warmup 1 \
  --no-cpu-baseline; rc=$?; echo "case1 rc=$rc"; tail -c 1200 gpurun_out/bench_case1_r3j.log; exit $rc
