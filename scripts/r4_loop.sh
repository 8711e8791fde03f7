#!/bin/bash
# round 4: the RCCL loopback exchange (degree 1) under a kernel trace, single vs sp vs loop
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for mode in single loop; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4trace_$mode -o run -- \
    python scripts/sp_trace.py $mode > gpurun_out/r4trace_$mode.log 2>&1
  rc=$?; echo "$mode rc=$rc"; tail -2 gpurun_out/r4trace_$mode.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
