#!/bin/bash
# Round-3 GPU check: the full GPU suite, a short bench (CPU baseline child included), then the RCCL
# two-ranks-on-one-GPU probe.  Stops at the first fault.  usage: scripts/r3_check.sh <tag> [pytest -k expr]
set -u
mkdir -p gpurun_out
tag=${1:-x}
kexpr=${2:-}
if [ -n "$kexpr" ]; then
  scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 5 --timeout 600 --timeout-method thread -k "$kexpr"
else
  scripts/gpustep.sh 900 gpurun_out/t_$tag.log python -u -m pytest tests -m gpu -v -rP --maxfail 5 --timeout 600 --timeout-method thread
fi
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/t_$tag.log | tail -1; [ $rc -eq 99 ] && exit 99
scripts/gpustep.sh 500 gpurun_out/bench_$tag.log python bench.py --steps 2 --warmup 2
rc2=$?; echo "bench rc=$rc2"; tail -c 600 gpurun_out/bench_$tag.log; [ $rc2 -eq 99 ] && exit 99
timeout -k 10 120 python scripts/rccl_probe.py > gpurun_out/probe_$tag.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe_$tag.log | tail -5
exit $rc
