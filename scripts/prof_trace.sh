#!/bin/bash
# rocprofv3 kernel trace of one clip (after one warmup clip) -> gpurun_out/trace_<tag>/ ; per-shape summary
# with scripts/trace_shapes.py.  usage: scripts/prof_trace.sh <tag> [extra bench args]
set -u
mkdir -p gpurun_out
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$tag -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-encode "$@" > gpurun_out/trace_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/trace_$tag.log
f=$(find gpurun_out/trace_$tag -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/trace_shapes.py "$f" 45 > gpurun_out/trace_${tag}_shapes.txt && cat gpurun_out/trace_${tag}_shapes.txt | head -50
exit $rc
