#!/bin/bash
# V^T Ulysses exchange: kernel tests (chunked V^T attention, q/k pack), SP tests (incl. V^T vs V-rows bit identity),
# then the per-rank compute at N = 1, 2, 4, 8 (schedules 4 and 0).  usage: scripts/r6_vt.sh <tag>
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 600 gpurun_out/vt_kern_$tag.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp_kernels.py tests/test_gpu_kernels.py -k "attention or pack or transposed"
rc=$?; grep -E "passed|failed" gpurun_out/vt_kern_$tag.log | tail -2; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 1200 gpurun_out/vt_sp_$tag.log python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_sp.py
rc=$?; grep -E "passed|failed|V\^T exchange" gpurun_out/vt_sp_$tag.log | tail -12; echo "sp tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
SA_SPRC_MODES=${MODES:-4,0} scripts/gpustep.sh 500 gpurun_out/sprc_$tag.jsonl python -u scripts/sp_rank_compute.py 1 2 4 8
rc=$?; grep -v amdgpu gpurun_out/sprc_$tag.jsonl | grep -v summary; exit $rc
