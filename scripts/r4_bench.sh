#!/bin/bash
# the driver's bench command (JSON line), then a rocprofv3 kernel-trace/stats run of one clip
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4}
if [ -z "${NOBENCH:-}" ]; then
  timeout -k 10 590 python3 bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_$TAG.err; cut -c1-400 gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "${NOPROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-encode > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof_$TAG.log | cut -c1-300; exit $rc
fi
exit 0
