#!/bin/bash
# GPU tests (all -m gpu, stop after 3 failures or at any GPU fault) then one default bench run.
# usage: scripts/gpu_check.sh <tag> [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=${1:-x}
kexpr=${2:-}
if [ -n "$kexpr" ]; then
  scripts/gpustep.sh 1500 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 600 --timeout-method thread -k "$kexpr"
else
  scripts/gpustep.sh 1500 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 3 --timeout 600 --timeout-method thread
fi
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_$tag.log; [ $rc -eq 99 ] && exit $rc
scripts/gpustep.sh 900 gpurun_out/bench_$tag.log python -u bench.py; rc2=$?; echo "bench rc=$rc2"
tail -3 gpurun_out/bench_$tag.log
exit $(( rc > rc2 ? rc : rc2 ))
