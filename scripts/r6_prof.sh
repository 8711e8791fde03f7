#!/bin/bash
# rocprofv3 kernel trace + stats of one bench clip (the summary committed under profiles/r06/)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r6 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-encode > gpurun_out/prof_r6.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_r6.log | cut -c1-300; find gpurun_out/prof_r6 -name "*stats*" | head; exit $rc
