#!/bin/bash
# round-5 baseline: the -m gpu suite + smoke, then a short bench (2 timed clips) on the same box
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/suite_$TAG.log; echo "suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-config1 --no-encode > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 gpurun_out/bench_$TAG.json; exit $rc
