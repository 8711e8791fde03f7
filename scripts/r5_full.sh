#!/bin/bash
# round-5 full record: -m gpu suite + smoke, a bench run (driver-style line), and the rocprofv3 kernel-trace summary
# of one more bench run on the same box
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5m}
STEPS=${STEPS:-3}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/suite_$TAG.log; echo "suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python3 bench.py --gpus 1 --steps $STEPS --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --gpus 1 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?; echo "prof rc=$rc"; find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -3; exit $rc
