#!/bin/bash
# GPU check used between edits: tests (failures reported, not fatal), bench, rocprof, extra kbench.
# Stops at the first GPU fault / abort / timeout (gpustep exit 99).
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 700 gpurun_out/t_$tag.log python -m pytest tests -m gpu -q; rc=$?; echo "tests rc=$rc"
[ $rc -eq 99 ] && exit 99
scripts/gpustep.sh 300 gpurun_out/bench_$tag.log python bench.py; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run -- python bench.py > gpurun_out/prof_$tag.log 2>&1
echo "prof rc=$?"
[ -n "${2:-}" ] && scripts/gpustep.sh 300 gpurun_out/kbx_$tag.log python -m stableavatar_amd.kbench $2
echo done
