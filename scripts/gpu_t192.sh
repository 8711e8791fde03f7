#!/bin/bash
# 192-row persistent GEMM tiles: GEMM / SP numerics, 192 vs 256 rows at the config-2 shapes, per-rank SP compute
set -u
mkdir -p gpurun_out
tag=${1:-t192}
scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_sp.py tests/test_gpu_sp_kernels.py -m gpu -v -x --timeout 600 --timeout-method thread -k "gemm or sp" || { tail -30 gpurun_out/t_$tag.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1
SA_KB_GVARS=2,3 scripts/gpustep.sh 400 gpurun_out/kb_$tag.jsonl python -u -m stableavatar_amd.kbench gemmvar || exit 1
grep kernel gpurun_out/kb_$tag.jsonl
scripts/gpustep.sh 400 gpurun_out/sprank_$tag.jsonl python -u scripts/sp_rank_compute.py 1 2 4 8 || exit 1
tail -1 gpurun_out/sprank_$tag.jsonl
