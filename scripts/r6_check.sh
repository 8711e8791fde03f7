#!/bin/bash
# Round-6 GPU check: the -m gpu suite (optionally a -k subset), smoke(), a short bench and a rocprofv3 kernel-stats
# run of one clip.  Stops at the first fault (scripts/gpustep.sh).  usage: scripts/r6_check.sh <tag> [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=${1:-x}
if [ -n "${2:-}" ]; then
  scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -x -v -rP --timeout 600 --timeout-method thread -k "$2"
else
  scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -x -v -rP --timeout 600 --timeout-method thread
fi
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_$tag.log; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 300 gpurun_out/smoke_$tag.log python -c "import __graft_entry__ as g; g.smoke()"
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
scripts/gpustep.sh 400 gpurun_out/bench_$tag.log python -u bench.py --steps 3 --warmup 2 --no-cpu-config1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$tag.log; exit $rc
