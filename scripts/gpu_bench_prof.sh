#!/bin/bash
# optional pytest -k subset, then the default bench (JSON line) and a rocprofv3 kernel-trace/stats run of
# one clip.  usage: scripts/gpu_bench_prof.sh <tag> [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=${1:-x}
if [ -n "${2:-}" ]; then
  scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 600 --timeout-method thread -k "$2"
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t_$tag.log; [ $rc -ne 0 ] && exit $rc
fi
scripts/gpustep.sh 900 gpurun_out/bench_$tag.log python -u bench.py; rc=$?; echo "bench rc=$rc"
tail -2 gpurun_out/bench_$tag.log; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-encode --no-dit14 > gpurun_out/prof_$tag.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
