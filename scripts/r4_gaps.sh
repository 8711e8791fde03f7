#!/bin/bash
# Per-rank forward at SP degree 8 (exchanges stubbed): host enqueue time vs GPU time, and a kernel trace whose
# in-forward idle time (scripts/gap_analysis.py) bounds what a HIP graph of the forward could recover.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4gap}
SA_SPRC_MODES=${MODES:-4,1} timeout -k 10 300 python scripts/sp_rank_compute.py 1 8 > gpurun_out/sprc_$TAG.jsonl 2>&1
rc=$?; grep -v amdgpu gpurun_out/sprc_$TAG.jsonl; [ $rc -ne 0 ] && exit $rc
for md in ${TRACE_MODES:-4 1}; do
  SA_SPRC_MODES=$md timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap_$TAG/m$md \
    -o tr -- python scripts/sp_rank_compute.py 8 > gpurun_out/gap_${TAG}_m$md.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/gap_${TAG}_m$md.log; exit $rc; }
  f=$(ls gpurun_out/gap_$TAG/m$md/*/tr_kernel_trace.csv gpurun_out/gap_$TAG/m$md/tr_kernel_trace.csv 2>/dev/null | tail -1)
  echo "mode $md trace $f"; python scripts/gap_analysis.py "$f" | tail -2
done
