#!/bin/bash
# kernel traces of one RCCL rank with the SP path on / off (scripts/sp_trace.py)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in single sp; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sptrace_$mode -o run -- \
    python scripts/sp_trace.py $mode > gpurun_out/sptrace_$mode.log 2>&1
  rc=$?; echo "$mode rc=$rc"; tail -2 gpurun_out/sptrace_$mode.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
