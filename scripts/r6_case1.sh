#!/bin/bash
# BASELINE config 2 (ii): the examples/case-1 shape -- 168 audio frames -> T_lat 42 -> 165 video frames, 81-frame windows at
# overlap 15 (5 windows per step) -- through bench.py on one GPU.  usage: scripts/r6_case1.sh <tag>
set -u
mkdir -p gpurun_out
tag=${1:-x}
scripts/gpustep.sh 900 gpurun_out/bench_case1_$tag.log python -u bench.py --video-frames 165 --steps 2 --warmup 1 --no-cpu-config1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_case1_$tag.log; exit $rc
