#!/bin/bash
# Key-split attention for the SP per-rank shapes: kernel tests, SP tests, then the per-rank compute at N = 1, 8
# (schedules 4 and 0) with the split off and on.  usage: scripts/r6_split.sh <tag>
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 600 gpurun_out/split_kern_$tag.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp_kernels.py
rc=$?; grep -E "passed|failed" gpurun_out/split_kern_$tag.log | tail -2; echo "kernel tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 1200 gpurun_out/split_sp_$tag.log python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_sp.py
rc=$?; grep -E "passed|failed" gpurun_out/split_sp_$tag.log | tail -2; echo "sp tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for sw in 0 1 0 1; do
  SA_ATTN_SPLIT=$sw SA_SPRC_MODES=4,0 scripts/gpustep.sh 400 gpurun_out/sprc_split${sw}_$tag.jsonl python -u scripts/sp_rank_compute.py 8 1 || exit 1
  echo "split=$sw"; grep sp_rank_forward gpurun_out/sprc_split${sw}_$tag.jsonl | grep -v summary
done
